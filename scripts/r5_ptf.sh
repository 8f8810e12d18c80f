#!/bin/bash
# round-5 c2cur: pending_to_front without a per-push allocation (stream.current GPU tests first), the c2cur
# line and its kernel statistics
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream_current.py tests/test_gpu_snapshot.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5ptf_tests.log 2>&1 || { tail -30 gpurun_out/r5ptf_tests.log; exit 1; }
tail -2 gpurun_out/r5ptf_tests.log
timeout -k 10 300 python3 -u bench.py --workload c2cur --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r5ptf_c2cur.json 2>gpurun_out/r5ptf_c2cur.err || { echo "c2cur failed"; tail -5 gpurun_out/r5ptf_c2cur.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c2cur', '%.3e' % d['value'], round(d['ms_per_step'],3))" gpurun_out/r5ptf_c2cur.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r5ptf -o run -- python3 bench.py --workload c2cur --steps 3 --warmup 1 --no-cpu-baseline --no-pcie > /dev/null 2>/tmp/r5ptf.err || { echo prof failed; tail -5 /tmp/r5ptf.err; exit 1; }
python3 - /tmp/r5ptf > gpurun_out/r5ptf_c2cur_kernel_stats.txt <<'PY'
import csv, sys, glob
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)
for r in csv.DictReader(open(f[0])):
    if "at::native" in r["Name"]: continue
    print(f"{r['Name'].split('(')[0][:70]:70s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.1f} us")
PY
head -8 gpurun_out/r5ptf_c2cur_kernel_stats.txt
echo done
