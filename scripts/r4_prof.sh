#!/bin/bash
# round-4 GPU evidence: partition-lane parity, lane benches, C2 / C3 / C4 kernel stats (summaries only:
# the raw rocprofv3 output stays in /tmp on the box), a C4 kernel timeline, C2 / C3 PMC traffic
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P=/tmp/r4p
rm -rf $P && mkdir -p $P
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_partition.py \
  tests/test_gpu_snapshot.py tests/test_gpu_ext.py tests/test_gpu_rate.py tests/test_gpu_sliding_minmax.py \
  "tests/test_gpu_parity.py::test_reference_kat_on_gpu" > gpurun_out/r4p_tests.log 2>&1; rc=$?
tail -25 gpurun_out/r4p_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc"; exit 1; fi
for w in plb plg; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 5 --warmup 2 > gpurun_out/r4p_$w.json 2>gpurun_out/r4p_$w.err || { echo "$w bench failed"; tail -5 gpurun_out/r4p_$w.err; exit 1; }
  cat gpurun_out/r4p_$w.json
done
timeout -k 10 300 python -u bench.py --workload c4 --steps 10 --warmup 3 > gpurun_out/r4p_c4.json 2>/dev/null || { echo c4 bench failed; exit 1; }
cat gpurun_out/r4p_c4.json
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r4p_c2.json 2>gpurun_out/r4p_c2.err || { echo c2 bench failed; exit 1; }
cat gpurun_out/r4p_c2.json
for w in c2 c3 c4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/$w -o run --output-format csv -- python3 bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r4p_${w}_prof.json 2>$P/$w.err || { echo "$w prof failed"; tail $P/$w.err; exit 1; }
  python3 - $P/$w > gpurun_out/r4p_${w}_kernel_stats.txt <<'PY'
import csv, sys, glob
d = sys.argv[1]
f = glob.glob(d + "/**/run_kernel_stats.csv", recursive=True)
for r in csv.DictReader(open(f[0])):
    if "at::native" in r["Name"]:
        continue
    print(f"{r['Name'].split('(')[0][:70]:70s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.1f} us")
PY
done
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $P/c4t -o run -- python3 bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2>$P/c4t.err || { echo "c4 trace failed"; exit 1; }
python3 scripts/timeline.py $P/c4t k_minmax_i64 > gpurun_out/r4p_c4_timeline.txt 2>&1 || echo "timeline failed"
for w in c2 c3; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $ctr -d $P/${w}_$ctr -o run --output-format csv -- python3 bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2>$P/${w}_$ctr.err || { echo "$w $ctr failed"; exit 1; }
  done
  python3 scripts/pmc_summary.py "$(ls $P/${w}_FETCH_SIZE/*/run_counter_collection.csv $P/${w}_FETCH_SIZE/run_counter_collection.csv 2>/dev/null | head -1)" \
    "$(ls $P/${w}_WRITE_SIZE/*/run_counter_collection.csv $P/${w}_WRITE_SIZE/run_counter_collection.csv 2>/dev/null | head -1)" > gpurun_out/r4p_${w}_pmc.json || echo "$w pmc summary failed"
done
du -sh gpurun_out
echo done
