#!/bin/bash
# round-5 C4 probe: the pair-table rebuild / truncated lane blob tests, C4 at several push sizes and band
# rows, host timing marks, a kernel timeline of the default C4 push
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P=/tmp/r5c4
rm -rf $P && mkdir -p $P
for cfg in "1048576 2" "2097152 4" "1048576 4"; do
  set -- $cfg
  SH_AGG_BAND_ROWS=$2 timeout -k 10 300 python -u bench.py --workload c4 --batch $1 --steps 8 --warmup 3 > gpurun_out/r5c4_b$1_r$2.json 2>gpurun_out/r5c4_b$1.err || { echo "c4 $1 failed"; tail -5 gpurun_out/r5c4_b$1.err; exit 1; }
  echo "batch $1 rows $2: $(python3 -c "import json;d=json.load(open('gpurun_out/r5c4_b$1_r$2.json'));print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_step'])")"
done
SH_TIMING=1 timeout -k 10 300 python -u bench.py --workload c4 --steps 20 --warmup 3 > /dev/null 2> gpurun_out/r5c4_timing.txt || { echo c4 timing failed; exit 1; }
grep "sh timing" gpurun_out/r5c4_timing.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/c4t -o run -- python3 bench.py --workload c4 --steps 4 --warmup 2 > /dev/null 2>$P/c4t.err || { echo "c4 trace failed"; tail -5 $P/c4t.err; exit 1; }
python3 scripts/timeline.py $P/c4t k_minmax_i64 > gpurun_out/r5c4_timeline.txt 2>&1 || echo "timeline failed"
tail -3 gpurun_out/r5c4_timeline.txt
python3 - $P/c4t > gpurun_out/r5c4_kernel_stats.txt <<'PY'
import csv, sys, glob
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)
for r in csv.DictReader(open(f[0])):
    if "at::native" in r["Name"]:
        continue
    print(f"{r['Name'].split('(')[0][:70]:70s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.1f} us {float(r['TotalDurationNs'])/1e3:10.1f}")
PY
head -30 gpurun_out/r5c4_kernel_stats.txt
echo done
