#!/bin/bash
# round-5 first check: the new tests (NULL unread columns, C1 at configuration size and by digest), the
# default bench line with its new `pcie` leg, the C1 line with its digest
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ingest.py \
  tests/test_gpu_headline.py "tests/test_gpu_parity.py::test_c1_full_size_matches_oracle" \
  > gpurun_out/r5_t1.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|error" gpurun_out/r5_t1.log | head -20; tail -30 gpurun_out/r5_t1.log; exit 1; }
tail -3 gpurun_out/r5_t1.log
timeout -k 10 400 python -u bench.py > gpurun_out/r5_bench.json 2> gpurun_out/r5_bench.err || { echo bench failed; tail gpurun_out/r5_bench.err; exit 1; }
cat gpurun_out/r5_bench.json
timeout -k 10 300 python -u bench.py --workload c1 --steps 10 --warmup 3 > gpurun_out/r5_c1.json 2> gpurun_out/r5_c1.err || { echo c1 bench failed; tail gpurun_out/r5_c1.err; exit 1; }
cat gpurun_out/r5_c1.json
echo done
