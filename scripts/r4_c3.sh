#!/bin/bash
# C3 after the stream-order rows of the keyed replay: parity, bench, kernel stats, PMC
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P=/tmp/r4c3 && rm -rf $P && mkdir -p $P
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sliding_minmax.py \
  tests/test_gpu_parity.py -k "sliding or c3 or minmax or ext" tests/test_gpu_ext.py \
  tests/test_gpu_scale.py::test_c3_time_10s_10k_keys_1k_resident_per_key > gpurun_out/r4c3_t.log 2>&1 || { tail -30 gpurun_out/r4c3_t.log; exit 1; }
tail -2 gpurun_out/r4c3_t.log
timeout -k 10 300 python -u bench.py --workload c3 --steps 5 --warmup 2 > gpurun_out/r4c3_bench.json 2>$P/b.err || { tail $P/b.err; exit 1; }
cat gpurun_out/r4c3_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/kt -o run --output-format csv -- python3 bench.py --workload c3 --steps 5 --warmup 2 --no-cpu-baseline > /dev/null 2>$P/kt.err || { echo prof failed; exit 1; }
python3 - $P/kt > gpurun_out/r4c3_kernel_stats.txt <<'PY'
import csv, sys, glob
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)
for r in csv.DictReader(open(f[0])):
    if "at::native" not in r["Name"]:
        print(f"{r['Name'].split('(')[0][:70]:70s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.1f} us")
PY
head -8 gpurun_out/r4c3_kernel_stats.txt
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d $P/$ctr -o run --output-format csv -- python3 bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2>$P/$ctr.err || { echo "$ctr failed"; exit 1; }
done
F=$(python3 -c "import glob,sys;print(glob.glob(sys.argv[1]+'/**/run_counter_collection.csv',recursive=True)[0])" $P/FETCH_SIZE)
W=$(python3 -c "import glob,sys;print(glob.glob(sys.argv[1]+'/**/run_counter_collection.csv',recursive=True)[0])" $P/WRITE_SIZE)
python3 scripts/pmc_summary.py "$F" "$W" > gpurun_out/r4c3_pmc.json
echo done
