#!/bin/bash
# SQ counters of the C2 bench kernels (one pass; 8 SQ slots) -> gpurun_out/<tag>/pmc
set -o pipefail
TAG=${1:-pmc}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
    -d "$OUT/sq" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/b.json" 2> "$OUT/err" || exit $?
python3 - "$OUT" <<'PY'
import csv, sys, glob, collections, re
f = glob.glob(sys.argv[1] + "/sq/**/run_counter_collection.csv", recursive=True)
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f[0])):
    k = re.sub(r"\(.*", "", r["Kernel_Name"])
    if "shd::" not in k: continue
    acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k[:60], {c: f"{sum(v)/len(v):.3g}" for c, v in sorted(d.items())})
PY
