#!/bin/bash
# A/B of the one-sweep split against the two-pass split on the C2 bench, plus their parity tests
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py::test_c2_split_sweep_and_counting_split tests/test_gpu_parity.py::test_c2_split_sweep_bucket_overflow_falls_back \
  tests/test_gpu_headline.py > gpurun_out/r4_sw_t.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r4_sw_t.log; exit 1; }
tail -2 gpurun_out/r4_sw_t.log
for v in 0 1 0 1; do
  SH_SWEEP=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r4_sw_$v.json 2>/dev/null || { echo bench failed; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r4_sw_$v.json'));print('sweep=$v', round(d['value']/1e9,2), 'Gev/s', round(d['ms_per_step'],3), 'ms', d.get('output_sha256_match'))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4_sw_prof -o c2 -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r4_sw_prof.log 2>&1 || { echo prof failed; exit 1; }
echo done
