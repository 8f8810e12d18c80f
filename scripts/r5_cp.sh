#!/bin/bash
# round-5: lane-strided k_compact_pending — batch-window suites and the C2 / C4 / c2cur lines
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_headline.py \
  tests/test_gpu_parity.py tests/test_gpu_stream_current.py tests/test_gpu_aggregation.py tests/test_gpu_expired.py \
  tests/test_gpu_ingest.py tests/test_gpu_ext.py tests/test_gpu_shard.py tests/test_gpu_sliding_expired.py > gpurun_out/r5cp_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|error" gpurun_out/r5cp_tests.log | head -20; tail -30 gpurun_out/r5cp_tests.log; exit 1; }
tail -2 gpurun_out/r5cp_tests.log
for w in c2 c2cur c4 c1 c3all; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline --no-pcie > gpurun_out/r5cp_$w.json 2>gpurun_out/r5cp.err || { echo "$w failed"; tail -5 gpurun_out/r5cp.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], '%.3e' % d['value'], d['ms_per_step'], d.get('output_sha256_match'))" gpurun_out/r5cp_$w.json $w
done
echo done
