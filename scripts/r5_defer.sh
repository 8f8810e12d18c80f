#!/bin/bash
# round-5 C3: k_sl_wkey's row stores one chunk late (default lib) vs at once (exp lib, SH_WK_NODEFER); the
# sliding GPU tests on the default lib first
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_sliding_minmax.py tests/test_gpu_scale.py tests/test_gpu_sliding_expired.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5df_tests.log 2>&1 || { tail -30 gpurun_out/r5df_tests.log; exit 1; }
tail -2 gpurun_out/r5df_tests.log
for v in "" _exp; do
  SH_LIB=$PWD/siddhi_amd/libsiddhi_hip$v.so timeout -k 10 300 python3 -u bench.py --workload c3 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r5df_c3$v.json 2>gpurun_out/r5df_c3$v.err || { echo "c3 $v failed"; tail -5 gpurun_out/r5df_c3$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], '%.3e' % d['value'], round(d['ms_per_step'],3))" gpurun_out/r5df_c3$v.json "c3$v"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r5df -o run -- python3 bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --no-pcie > /dev/null 2>/tmp/r5df.err || { echo prof failed; tail -5 /tmp/r5df.err; exit 1; }
python3 - /tmp/r5df > gpurun_out/r5df_c3_kernel_stats.txt <<'PY'
import csv, sys, glob
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)
for r in csv.DictReader(open(f[0])):
    print(f"{r['Name'].split('(')[0][:70]:70s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.1f} us")
PY
head -6 gpurun_out/r5df_c3_kernel_stats.txt
echo done
