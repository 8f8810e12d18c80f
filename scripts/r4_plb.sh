#!/bin/bash
# smoke, then the partition lanes' kernel stats (plb / plg)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4_smoke.log 2>&1 || { tail gpurun_out/r4_smoke.log; exit 1; }
tail -1 gpurun_out/r4_smoke.log
for w in plb plg; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/$w -o run -- python3 bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2>/tmp/$w.err || { tail /tmp/$w.err; exit 1; }
  python3 - /tmp/$w > gpurun_out/r4_${w}_kernel_stats.txt <<'PY'
import csv, sys, glob
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)
for r in csv.DictReader(open(f[0])):
    if "at::native" in r["Name"]:
        continue
    print(f"{r['Name'].split('(')[0][:90]:90s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.1f} us")
PY
  head -16 gpurun_out/r4_${w}_kernel_stats.txt
done
echo done
