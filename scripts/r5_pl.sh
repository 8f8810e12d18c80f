#!/bin/bash
# round-5: partition lanes without per-slot counting (offsets from the sorted slots)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_partition.py \
  tests/test_gpu_snapshot.py tests/test_gpu_rate.py tests/test_gpu_ext.py tests/test_gpu_parity.py tests/test_gpu_sliding_minmax.py tests/test_gpu_sliding_expired.py tests/test_gpu_shard.py > gpurun_out/r5pl_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|error" gpurun_out/r5pl_tests.log | head -20; tail -30 gpurun_out/r5pl_tests.log; exit 1; }
tail -2 gpurun_out/r5pl_tests.log
for w in plb plg c3 c3all; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r5pl_$w.json 2>gpurun_out/r5pl.err || { echo "$w failed"; tail -5 gpurun_out/r5pl.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], '%.3e' % d['value'], d['ms_per_step'])" gpurun_out/r5pl_$w.json $w
done
echo done
