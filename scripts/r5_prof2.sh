#!/bin/bash
# round-5: kernel statistics of the plb / plg / c2cur lines
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P=/tmp/r5p2
rm -rf $P && mkdir -p $P
for w in plb c2cur; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/$w -o run --output-format csv -- python3 bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2>$P/$w.err || { echo "$w prof failed"; tail $P/$w.err; exit 1; }
  python3 - $P/$w > gpurun_out/r5p2_${w}_kernel_stats.txt <<'PY'
import csv, sys, glob
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)
for r in csv.DictReader(open(f[0])):
    if "at::native" in r["Name"]:
        continue
    print(f"{r['Name'].split('(')[0][:70]:70s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.1f} us {float(r['TotalDurationNs'])/1e6:9.2f} ms")
PY
  echo "== $w"; head -14 gpurun_out/r5p2_${w}_kernel_stats.txt
done
echo done
