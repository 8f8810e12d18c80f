#!/bin/bash
# round-5: k_sl_wkey at 4 waves / SIMD and k_slx_wkey's rolling staging — sliding GPU tests, then c3 / c3all
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_sliding_expired.py tests/test_gpu_sliding_minmax.py tests/test_gpu_scale.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5stg_tests.log 2>&1 || { tail -30 gpurun_out/r5stg_tests.log; exit 1; }
tail -2 gpurun_out/r5stg_tests.log
for w in c3 c3all; do
  timeout -k 10 300 python3 -u bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r5stg_$w.json 2>gpurun_out/r5stg_$w.err || { echo "$w failed"; tail -5 gpurun_out/r5stg_$w.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], '%.3e' % d['value'], round(d['ms_per_step'],3))" gpurun_out/r5stg_$w.json $w
done
echo done
