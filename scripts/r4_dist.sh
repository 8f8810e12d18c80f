#!/bin/bash
# round-4 multi-process rehearsal on one GPU: the two-process gloo tests, then bench --gpus 2 over gloo
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q -rf --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dist.py tests/test_gpu_dist_more.py > gpurun_out/r4d_tests.log 2>&1; rc=$?
tail -5 gpurun_out/r4d_tests.log
if [ $rc -ne 0 ]; then echo "dist tests rc=$rc"; exit 1; fi
for w in c2 c4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
    bench.py --gpus 2 --backend gloo --workload $w --steps 3 --warmup 1 > gpurun_out/r4d_${w}_x2.json 2> gpurun_out/r4d_${w}_x2.err || { echo "$w x2 failed"; tail -20 gpurun_out/r4d_${w}_x2.err; exit 1; }
  cat gpurun_out/r4d_${w}_x2.json
done
echo done
