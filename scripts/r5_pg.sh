#!/bin/bash
# round-5: partitioned lengthBatch(L, true) grouped by other columns (lane 3, k_pg_sc_*)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_partition.py \
  tests/test_gpu_snapshot.py tests/test_gpu_rate.py tests/test_gpu_stream_current.py > gpurun_out/r5pg_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|error" gpurun_out/r5pg_tests.log | head -20; tail -30 gpurun_out/r5pg_tests.log; exit 1; }
tail -3 gpurun_out/r5pg_tests.log
echo done
