#!/bin/bash
# round-5: stream.current row values as one record per row (k_sc_walk)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_stream_current.py \
  tests/test_gpu_parity.py tests/test_gpu_snapshot.py tests/test_gpu_rate.py > gpurun_out/r5sc_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|error" gpurun_out/r5sc_tests.log | head -20; tail -30 gpurun_out/r5sc_tests.log; exit 1; }
tail -2 gpurun_out/r5sc_tests.log
timeout -k 10 300 python -u bench.py --workload c2cur --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r5sc_c2cur.json 2>gpurun_out/r5sc.err || { echo "c2cur failed"; tail -5 gpurun_out/r5sc.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c2cur', '%.3e' % d['value'], d['ms_per_step'])" gpurun_out/r5sc_c2cur.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r5sc -o run --output-format csv -- python3 bench.py --workload c2cur --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2>/tmp/r5sc.err || { echo "prof failed"; exit 1; }
python3 - /tmp/r5sc > gpurun_out/r5sc_kernel_stats.txt <<'PY'
import csv, sys, glob
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)
for r in csv.DictReader(open(f[0])):
    if "at::native" in r["Name"]:
        continue
    print(f"{r['Name'].split('(')[0][:70]:70s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.1f} us")
PY
head -8 gpurun_out/r5sc_kernel_stats.txt
echo done
