#!/bin/bash
# round-4 profiles: C2 / C3 / C4 kernel stats + a C4 kernel trace, and the PMC passes of C2 and C3
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sliding_minmax.py \
  "tests/test_gpu_parity.py::test_c3_sliding_dictionary_keys" tests/test_gpu_scale.py::test_c3_time_10s_10k_keys_1k_resident_per_key \
  tests/test_gpu_snapshot.py tests/test_gpu_ext.py -k "not group_lanes and not lanes_rate and not partitioned_ext and not partitioned_external" > gpurun_out/r4p_t.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r4p_t.log; exit 1; }
tail -1 gpurun_out/r4p_t.log
# partition lanes grouped by another column (lane 3): assertion failures are reported, faults end the run
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_partition.py \
  tests/test_gpu_snapshot.py::test_partition_group_lanes_checkpoint "tests/test_gpu_parity.py::test_reference_kat_on_gpu[partition_lengthBatch_group_by_other_all]" \
  tests/test_gpu_rate.py::test_partition_lanes_rate tests/test_gpu_rate.py::test_partition_lanes_keyed_rate_refused_for_other_group_keys \
  tests/test_gpu_snapshot.py::test_partition_lanes_rate_checkpoint "tests/test_gpu_ext.py::test_partitioned_ext" \
  tests/test_gpu_ext.py::test_partitioned_ext_checkpoint tests/test_gpu_ext.py::test_partitioned_external_time \
  tests/test_gpu_ext.py::test_partitioned_external_time_checkpoint \
  > gpurun_out/r4p_lane3.log 2>&1; rc=$?
tail -15 gpurun_out/r4p_lane3.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "lane3 tests rc=$rc"; exit 1; fi
for w in plb plg; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 5 --warmup 2 > gpurun_out/r4p_$w.json 2>gpurun_out/r4p_$w.err || { echo "$w bench failed"; tail -5 gpurun_out/r4p_$w.err; exit 1; }
  cat gpurun_out/r4p_$w.json
done
SH_PL_SORT=1 timeout -k 10 300 python -u bench.py --workload plb --steps 5 --warmup 2 > gpurun_out/r4p_plb_sorted.json 2>gpurun_out/r4p_plbs.err || { echo "plb sorted bench failed"; tail -5 gpurun_out/r4p_plbs.err; exit 1; }
cat gpurun_out/r4p_plb_sorted.json
for v in 0 1 0 1; do
  SH_SL_RECORDS_SEQ=$v timeout -k 10 300 python -u bench.py --workload c3 --steps 5 --warmup 2 > gpurun_out/r4p_c3seq_$v.json 2>/dev/null || { echo c3 seq bench failed; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r4p_c3seq_$v.json'));print('records_seq=$v', round(d['value']/1e9,3), 'Gev/s', round(d['ms_per_step'],2), 'ms')"
done
timeout -k 10 300 python -u bench.py --workload c4 --steps 10 --warmup 3 > gpurun_out/r4p_c4.json 2>/dev/null || { echo c4 bench failed; exit 1; }
cat gpurun_out/r4p_c4.json
for w in c2 c3 c4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4p_$w -o $w -- python3 bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r4p_$w.log 2>&1 || { echo "$w prof failed"; tail gpurun_out/r4p_$w.log; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r4p_c4trace -o c4 -- python3 bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r4p_c4trace.log 2>&1 || { echo "c4 trace failed"; exit 1; }
for w in c2 c3; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $ctr -d gpurun_out/r4p_${w}_$ctr -o pmc -- python3 bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r4p_${w}_$ctr.log 2>&1 || { echo "$w $ctr failed"; exit 1; }
  done
done
echo done
