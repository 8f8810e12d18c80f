#!/bin/bash
# Per-kernel times of the C2 bench (rocprofv3 kernel trace) -> gpurun_out/<tag>/stats.txt
# usage (on the GPU box, repo root): scripts/kstats.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-k}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > "$OUT/bench.json" 2> "$OUT/kt.err" || exit $?
python3 - "$OUT" <<'PY' > "$OUT/stats.txt"
import csv, sys, glob
f = glob.glob(sys.argv[1] + "/kt/**/run_kernel_stats.csv", recursive=True) + glob.glob(sys.argv[1] + "/kt/run_kernel_stats.csv")
rows = list(csv.DictReader(open(f[0])))
for r in rows:
    n = r["Name"]
    if "at::native" in n:
        continue
    print(f"{n.split('(')[0][:70]:70s} {r['Calls']:>4} {float(r['AverageNs'])/1e3:9.1f} us")
PY
cat "$OUT/bench.json" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'ms/step', d['ms_per_step'])"
cat "$OUT/stats.txt"
python3 scripts/timeline.py "$OUT/kt" > "$OUT/timeline.txt" 2>&1 && tail -1 "$OUT/timeline.txt"
