#!/bin/bash
# round-4 check: the GPU tests touched this round, the C2 / C3 bench lines and a kernel trace of C2
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_snapshot.py::test_partition_lanes_checkpoint tests/test_gpu_partition.py \
  tests/test_gpu_headline.py tests/test_gpu_ingest.py "tests/test_gpu_parity.py::test_reference_kat_on_gpu" \
  "tests/test_gpu_parity.py::test_c3_sliding_dictionary_keys" tests/test_gpu_parity.py::test_c2_split_sweep_and_counting_split tests/test_gpu_parity.py::test_c2_split_sweep_bucket_overflow_falls_back tests/test_gpu_scale.py::test_c3_time_10s_10k_keys_1k_resident_per_key \
  > gpurun_out/r4_t1.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|error" gpurun_out/r4_t1.log | head -20; tail -30 gpurun_out/r4_t1.log; exit 1; }
tail -3 gpurun_out/r4_t1.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r4_bench.json 2> gpurun_out/r4_bench.err || { echo bench failed; tail gpurun_out/r4_bench.err; exit 1; }
cat gpurun_out/r4_bench.json
timeout -k 10 300 python -u bench.py --workload c3 --steps 5 --warmup 2 > gpurun_out/r4_c3.json 2> gpurun_out/r4_c3.err || { echo c3 bench failed; tail gpurun_out/r4_c3.err; exit 1; }
cat gpurun_out/r4_c3.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4_c3prof -o c3 -- python3 bench.py --workload c3 --steps 3 --warmup 1 > gpurun_out/r4_c3prof.log 2>&1 || { echo c3 prof failed; tail gpurun_out/r4_c3prof.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r4_trace -o trace -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/r4_trace.log 2>&1 || { echo trace failed; tail gpurun_out/r4_trace.log; exit 1; }
echo done
