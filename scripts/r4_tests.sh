#!/bin/bash
# round-4 GPU parity of the partition lanes, limiters, checkpoints and externalTime(Batch) lanes
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -q -rf --timeout 300 --timeout-method thread -m gpu tests/test_gpu_partition.py \
  tests/test_gpu_snapshot.py tests/test_gpu_ext.py tests/test_gpu_rate.py "tests/test_gpu_parity.py::test_reference_kat_on_gpu" \
  > gpurun_out/r4t.log 2>&1; rc=$?
tail -30 gpurun_out/r4t.log
exit $rc
