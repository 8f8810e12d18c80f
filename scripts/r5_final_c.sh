#!/bin/bash
# round-5 closing evidence (3/3): kernel statistics of C2 / C3 / C4 / c3all and the C2 PMC traffic
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P=/tmp/r5f
rm -rf $P && mkdir -p $P
for w in c2 c3 c4 c3all; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/$w -o run --output-format csv -- python3 bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline --no-pcie > /dev/null 2>$P/$w.err || { echo "$w prof failed"; tail $P/$w.err; exit 1; }
  python3 - $P/$w > gpurun_out/r5f_${w}_kernel_stats.txt <<'PY'
import csv, sys, glob
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)
for r in csv.DictReader(open(f[0])):
    if "at::native" in r["Name"]:
        continue
    print(f"{r['Name'].split('(')[0][:70]:70s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.1f} us")
PY
  head -4 gpurun_out/r5f_${w}_kernel_stats.txt
done
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d $P/c2_$ctr -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pcie > /dev/null 2>$P/c2_$ctr.err || { echo "c2 $ctr failed"; exit 1; }
done
F=$(python3 -c "import glob,sys;print(glob.glob(sys.argv[1]+'/**/run_counter_collection.csv',recursive=True)[0])" $P/c2_FETCH_SIZE)
W=$(python3 -c "import glob,sys;print(glob.glob(sys.argv[1]+'/**/run_counter_collection.csv',recursive=True)[0])" $P/c2_WRITE_SIZE)
python3 scripts/pmc_summary.py "$F" "$W" > gpurun_out/r5f_c2_pmc.json || echo "c2 pmc summary failed"
head -c 1500 gpurun_out/r5f_c2_pmc.json
echo done
