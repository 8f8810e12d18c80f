#!/bin/bash
# round-5: compact (20-byte) shard records — the multi-GPU parity suites on one GPU
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_shard.py \
  tests/test_gpu_shard_pipeline.py tests/test_gpu_dist.py tests/test_gpu_shard_snapshot.py tests/test_gpu_shard_agg.py \
  tests/test_gpu_ext.py > gpurun_out/r5sh_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|error" gpurun_out/r5sh_tests.log | head -20; tail -30 gpurun_out/r5sh_tests.log; exit 1; }
tail -3 gpurun_out/r5sh_tests.log
echo done
