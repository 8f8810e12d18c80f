#!/bin/bash
# round-5 C4 after the speculative band: aggregation parity, C4 bench, host timing, kernel timeline
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P=/tmp/r5c4b
rm -rf $P && mkdir -p $P
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_aggregation.py \
  tests/test_gpu_shard_agg.py > gpurun_out/r5c4b_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|error" gpurun_out/r5c4b_tests.log | head -20; tail -30 gpurun_out/r5c4b_tests.log; exit 1; }
tail -3 gpurun_out/r5c4b_tests.log
timeout -k 10 300 python -u bench.py --workload c4 --steps 20 --warmup 3 > gpurun_out/r5c4b_bench.json 2>gpurun_out/r5c4b_bench.err || { echo "c4 failed"; tail -5 gpurun_out/r5c4b_bench.err; exit 1; }
cat gpurun_out/r5c4b_bench.json
SH_TIMING=1 timeout -k 10 300 python -u bench.py --workload c4 --steps 20 --warmup 3 > /dev/null 2> gpurun_out/r5c4b_timing.txt || { echo c4 timing failed; exit 1; }
grep "sh timing" gpurun_out/r5c4b_timing.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $P/c4t -o run -- python3 bench.py --workload c4 --steps 4 --warmup 2 > /dev/null 2>$P/c4t.err || { echo "c4 trace failed"; tail -5 $P/c4t.err; exit 1; }
python3 scripts/timeline.py $P/c4t k_boundaries > gpurun_out/r5c4b_timeline.txt 2>&1 || echo "timeline failed"
tail -3 gpurun_out/r5c4b_timeline.txt
echo done
