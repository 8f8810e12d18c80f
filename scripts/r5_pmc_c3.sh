#!/bin/bash
# round-5 closing: PMC HBM traffic (FETCH_SIZE, WRITE_SIZE: separate passes) of C3 on the final tree
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P=/tmp/r5pmcf
rm -rf $P && mkdir -p $P
for w in c3; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $ctr -d $P/${w}_$ctr -o run --output-format csv -- python3 bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2>$P/${w}_$ctr.err || { echo "$w $ctr failed"; tail -3 $P/${w}_$ctr.err; exit 1; }
  done
  F=$(python3 -c "import glob,sys;print(glob.glob(sys.argv[1]+'/**/run_counter_collection.csv',recursive=True)[0])" $P/${w}_FETCH_SIZE)
  W=$(python3 -c "import glob,sys;print(glob.glob(sys.argv[1]+'/**/run_counter_collection.csv',recursive=True)[0])" $P/${w}_WRITE_SIZE)
  python3 scripts/pmc_summary.py "$F" "$W" > gpurun_out/r5pmcf_${w}.json || echo "$w pmc summary failed"
  python3 - gpurun_out/r5pmcf_${w}.json $w <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))["kernels"]
# per push: every kernel's bytes x launches / the pushes (the bench's 3 pushes: 1 warm-up + 2 timed)
tot = sum(v["hbm_bytes"] * v["launches"] for v in d.values()) / 3
top = sorted(d.items(), key=lambda kv: -kv[1]["hbm_bytes"] * kv[1]["launches"])[:6]
print(sys.argv[2], "GB per push %.2f" % (tot / 1e9), "; ".join("%s %.2f" % (k.split("<")[0].replace("shd::", ""), v["hbm_bytes"] / 1e9) for k, v in top))
PY
done
echo done
