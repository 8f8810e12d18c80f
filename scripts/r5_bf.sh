#!/bin/bash
# round-5 C3 / c3all: the quirk-check filter in LDS and the simpler sum chain (sliding GPU tests first)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_sliding_minmax.py tests/test_gpu_scale.py tests/test_gpu_sliding_expired.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5bf_tests.log 2>&1 || { tail -30 gpurun_out/r5bf_tests.log; exit 1; }
tail -2 gpurun_out/r5bf_tests.log
for w in c3 c3all; do
  timeout -k 10 300 python3 -u bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r5bf_$w.json 2>gpurun_out/r5bf_$w.err || { echo "$w failed"; tail -5 gpurun_out/r5bf_$w.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], '%.3e' % d['value'], round(d['ms_per_step'],3))" gpurun_out/r5bf_$w.json $w
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r5bf -o run -- python3 bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --no-pcie > /dev/null 2>/tmp/r5bf.err || { echo prof failed; tail -5 /tmp/r5bf.err; exit 1; }
python3 - /tmp/r5bf > gpurun_out/r5bf_c3_kernel_stats.txt <<'PY'
import csv, sys, glob
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)
for r in csv.DictReader(open(f[0])):
    if "at::native" in r["Name"]: continue
    print(f"{r['Name'].split('(')[0][:70]:70s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.1f} us")
PY
head -6 gpurun_out/r5bf_c3_kernel_stats.txt
echo done
