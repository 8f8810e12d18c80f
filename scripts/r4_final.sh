#!/bin/bash
# round-4 closing evidence: the whole GPU suite, every bench line, C2 / C4 kernel stats, C4 PMC traffic
# (summaries only: raw rocprofv3 output stays in /tmp on the box)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P=/tmp/r4f
rm -rf $P && mkdir -p $P
timeout -k 10 1000 python -u -m pytest tests -q -rf -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4f_tests.log 2>&1; rc=$?
tail -6 gpurun_out/r4f_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc"; exit 1; fi
timeout -k 10 300 python -u bench.py > gpurun_out/r4f_c2.json 2>gpurun_out/r4f_c2.err || { echo c2 bench failed; tail -5 gpurun_out/r4f_c2.err; exit 1; }
cat gpurun_out/r4f_c2.json
for w in c3 c4 ext c1 c5 plb plg c2all c2cur c3all; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r4f_$w.json 2>/dev/null || { echo "$w bench failed"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], '%.3e' % d['value'], d['ms_per_step'])" gpurun_out/r4f_$w.json $w
done
for w in c2 c4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/$w -o run --output-format csv -- python3 bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline > /dev/null 2>$P/$w.err || { echo "$w prof failed"; tail $P/$w.err; exit 1; }
  python3 - $P/$w > gpurun_out/r4f_${w}_kernel_stats.txt <<'PY'
import csv, sys, glob
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)
for r in csv.DictReader(open(f[0])):
    if "at::native" in r["Name"]:
        continue
    print(f"{r['Name'].split('(')[0][:70]:70s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.1f} us")
PY
done
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d $P/c4_$ctr -o run --output-format csv -- python3 bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2>$P/c4_$ctr.err || { echo "c4 $ctr failed"; exit 1; }
done
F=$(python3 -c "import glob,sys;print(glob.glob(sys.argv[1]+'/**/run_counter_collection.csv',recursive=True)[0])" $P/c4_FETCH_SIZE)
W=$(python3 -c "import glob,sys;print(glob.glob(sys.argv[1]+'/**/run_counter_collection.csv',recursive=True)[0])" $P/c4_WRITE_SIZE)
python3 scripts/pmc_summary.py "$F" "$W" > gpurun_out/r4f_c4_pmc.json || echo "c4 pmc summary failed"
du -sh gpurun_out
echo done
