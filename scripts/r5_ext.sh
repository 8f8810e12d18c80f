#!/bin/bash
# round-5 externalTimeBatch replaceTimestampWithBatchEndTime: ext suite, KATs on the GPU, snapshot suite
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ext.py \
  "tests/test_gpu_parity.py::test_reference_kat_on_gpu" tests/test_gpu_snapshot.py tests/test_gpu_rate.py \
  > gpurun_out/r5ext_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|error" gpurun_out/r5ext_tests.log | head -20; tail -40 gpurun_out/r5ext_tests.log; exit 1; }
tail -3 gpurun_out/r5ext_tests.log
echo done
