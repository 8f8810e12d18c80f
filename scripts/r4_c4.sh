#!/bin/bash
# round-4 C4 pass: ext-timeout parity, C4 bench (+ host timing), C4 kernel stats (summaries only)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P=/tmp/r4c4
rm -rf $P && mkdir -p $P
timeout -k 10 600 python -u -m pytest -q -rf --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ext.py \
  "tests/test_gpu_parity.py::test_reference_kat_on_gpu" tests/test_gpu_aggregation.py > gpurun_out/r4c4_tests.log 2>&1; rc=$?
tail -8 gpurun_out/r4c4_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc"; exit 1; fi
timeout -k 10 300 python -u bench.py --workload c4 --steps 10 --warmup 3 > gpurun_out/r4c4_bench.json 2>/dev/null || { echo c4 bench failed; exit 1; }
cat gpurun_out/r4c4_bench.json
SH_TIMING=1 timeout -k 10 300 python -u bench.py --workload c4 --steps 20 --warmup 3 --no-cpu-baseline > /dev/null 2> gpurun_out/r4c4_timing.txt || { echo c4 timing failed; exit 1; }
grep "sh timing" gpurun_out/r4c4_timing.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/c4 -o run --output-format csv -- python3 bench.py --workload c4 --steps 5 --warmup 2 --no-cpu-baseline > /dev/null 2>$P/c4.err || { echo "c4 prof failed"; tail $P/c4.err; exit 1; }
python3 - $P/c4 > gpurun_out/r4c4_kernel_stats.txt <<'PY'
import csv, sys, glob
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)
for r in csv.DictReader(open(f[0])):
    if "at::native" in r["Name"]:
        continue
    print(f"{r['Name'].split('(')[0][:70]:70s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.1f} us")
PY
head -14 gpurun_out/r4c4_kernel_stats.txt
echo done
