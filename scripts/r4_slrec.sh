#!/bin/bash
# wave-aggregated slot counts: sliding + partition parity, then the lane benches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q -x -rf --timeout 300 --timeout-method thread -m gpu tests/test_gpu_partition.py tests/test_gpu_aggregation.py \
  tests/test_gpu_ext.py tests/test_gpu_sliding_minmax.py tests/test_gpu_parity.py tests/test_gpu_snapshot.py tests/test_gpu_rate.py tests/test_gpu_shard.py tests/test_gpu_shard_snapshot.py tests/test_gpu_scale.py > gpurun_out/r4s_tests.log 2>&1 || { tail -30 gpurun_out/r4s_tests.log; exit 1; }
tail -2 gpurun_out/r4s_tests.log
for w in plb plg c3; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r4s_$w.json 2>/dev/null || { echo "$w failed"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], '%.3e' % d['value'], d['ms_per_step'])" gpurun_out/r4s_$w.json $w
done
echo done
