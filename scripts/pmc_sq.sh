#!/bin/bash
# One SQ counter pass over the bench (C2, or BENCH_ARGS): scripts/pmc_sq.sh <tag> <counters...> (<= 8 SQ)
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/sq" -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/b.json" 2> "$OUT/err" || exit $?
python3 - "$OUT" <<'PY'
import csv, sys, glob, collections, re
f = glob.glob(sys.argv[1] + "/sq/**/run_counter_collection.csv", recursive=True)
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f[0])):
    k = re.sub(r"\(.*", "", r["Kernel_Name"])
    if "shd::" not in k: continue
    acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k[:40], " ".join(f"{c[3:]}={sum(v)/len(v):.3g}" for c, v in sorted(d.items())))
PY
