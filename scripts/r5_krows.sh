#!/bin/bash
# round-5 C3: per-event rows of k_sl_wkey in key order, gathered by the emission through the inverse rank
# list (libsiddhi_hip_krows.so, SH_SL_KROWS=1): sliding GPU tests on that library, then c3 on both
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SH_LIB=$PWD/siddhi_amd/libsiddhi_hip_krows.so timeout -k 10 600 python -u -m pytest tests/test_gpu_sliding_minmax.py tests/test_gpu_scale.py tests/test_gpu_sliding_expired.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5kr_tests.log 2>&1 || { tail -30 gpurun_out/r5kr_tests.log; exit 1; }
tail -2 gpurun_out/r5kr_tests.log
for v in "" _krows; do
  SH_LIB=$PWD/siddhi_amd/libsiddhi_hip$v.so timeout -k 10 300 python3 -u bench.py --workload c3 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r5kr_c3$v.json 2>gpurun_out/r5kr_c3$v.err || { echo "c3 $v failed"; tail -5 gpurun_out/r5kr_c3$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], '%.3e' % d['value'], round(d['ms_per_step'],3))" gpurun_out/r5kr_c3$v.json "c3$v"
done
echo done
