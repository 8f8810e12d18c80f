#!/bin/bash
# Bench + rocprofv3 evidence for one round, run on the GPU box from the repo root:
#   scripts/profile_bench.sh <tag>
# 1) the default bench line (with cpu_baseline), 2) kernel trace + stats, 3) FETCH_SIZE and
# 4) WRITE_SIZE in separate passes (FETCH_SIZE uses 3 TCC slots, WRITE_SIZE 2; never combined).
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
cat "$OUT/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/kt.json" 2> "$OUT/kt.err" || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/fetch.json" 2> "$OUT/fetch.err" || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/write.json" 2> "$OUT/write.err" || exit $?
echo profile done
python3 scripts/pmc_summary.py "$(ls "$OUT"/fetch/*/run_counter_collection.csv "$OUT"/fetch/run_counter_collection.csv 2>/dev/null | head -1)" \
    "$(ls "$OUT"/write/*/run_counter_collection.csv "$OUT"/write/run_counter_collection.csv 2>/dev/null | head -1)" > "$OUT/pmc.json" || exit $?
python3 - "$OUT" > "$OUT/kernel_stats.txt" <<'PY'
import csv, sys, glob
d = sys.argv[1]
f = glob.glob(d + "/kt/**/run_kernel_stats.csv", recursive=True) + glob.glob(d + "/kt/run_kernel_stats.csv")
for r in csv.DictReader(open(f[0])):
    if "at::native" in r["Name"]:
        continue
    print(f"{r['Name'].split('(')[0][:70]:70s} {r['Calls']:>4} {float(r['AverageNs'])/1e3:9.1f} us")
PY
echo summaries done
