#!/bin/bash
# round-5 c3all: wave-per-key expired-output replay (k_slx_wkey)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P=/tmp/r5slx
rm -rf $P && mkdir -p $P
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sliding_expired.py tests/test_gpu_partition.py tests/test_gpu_snapshot.py > gpurun_out/r5slx_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|error" gpurun_out/r5slx_tests.log | head -20; tail -40 gpurun_out/r5slx_tests.log; exit 1; }
tail -3 gpurun_out/r5slx_tests.log
timeout -k 10 300 python -u bench.py --workload c3all --steps 6 --warmup 2 > gpurun_out/r5slx_bench.json 2>gpurun_out/r5slx.err || { echo "c3all failed"; tail -5 gpurun_out/r5slx.err; exit 1; }
echo "c3all $(python3 -c "import json;d=json.load(open('gpurun_out/r5slx_bench.json'));print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_step'])")"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/c3all -o run -- python3 bench.py --workload c3all --steps 3 --warmup 1 > /dev/null 2>$P/c3.err || { echo "c3all prof failed"; tail -5 $P/c3.err; exit 1; }
python3 - $P/c3all > gpurun_out/r5slx_kernel_stats.txt <<'PY'
import csv, sys, glob
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)
for r in csv.DictReader(open(f[0])):
    if "at::native" in r["Name"]:
        continue
    print(f"{r['Name'].split('(')[0][:70]:70s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.1f} us")
PY
head -10 gpurun_out/r5slx_kernel_stats.txt
echo done
