#!/bin/bash
# round-5 C4 probe: the pair-table rebuild / truncated lane blob tests, C4 at several push sizes and band
# rows, host timing marks, a kernel timeline of the default C4 push
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P=/tmp/r5c4
rm -rf $P && mkdir -p $P
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  "tests/test_gpu_partition.py::test_partitioned_time_group_by_other_pair_churn" \
  "tests/test_gpu_snapshot.py::test_truncated_partition_lane_blob_leaves_query_unchanged" \
  tests/test_gpu_snapshot.py > gpurun_out/r5c4_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|error" gpurun_out/r5c4_tests.log | head -20; tail -30 gpurun_out/r5c4_tests.log; exit 1; }
tail -3 gpurun_out/r5c4_tests.log
for cfg in "4194304 8" "8388608 16" "16777216 32" "33554432 32"; do
  set -- $cfg
  SH_AGG_BAND_ROWS=$2 timeout -k 10 300 python -u bench.py --workload c4 --batch $1 --steps 8 --warmup 3 > gpurun_out/r5c4_b$1_r$2.json 2>gpurun_out/r5c4_b$1.err || { echo "c4 $1 failed"; tail -5 gpurun_out/r5c4_b$1.err; exit 1; }
  echo "batch $1 rows $2: $(python3 -c "import json;d=json.load(open('gpurun_out/r5c4_b$1_r$2.json'));print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_step'])")"
done
SH_TIMING=1 timeout -k 10 300 python -u bench.py --workload c4 --steps 20 --warmup 3 > /dev/null 2> gpurun_out/r5c4_timing.txt || { echo c4 timing failed; exit 1; }
grep "sh timing" gpurun_out/r5c4_timing.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $P/c4t -o run -- python3 bench.py --workload c4 --steps 4 --warmup 2 > /dev/null 2>$P/c4t.err || { echo "c4 trace failed"; tail -5 $P/c4t.err; exit 1; }
python3 scripts/timeline.py $P/c4t k_minmax_i64 > gpurun_out/r5c4_timeline.txt 2>&1 || echo "timeline failed"
tail -3 gpurun_out/r5c4_timeline.txt
echo done
