#!/bin/bash
# round-5 C3: k_sl_wkey timing experiments (x1 no row stores, x2 no quirk check, x3 sequential min/max; timing only)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P=/tmp/r5wk2
rm -rf $P && mkdir -p $P
for v in "" _x1 _x2 _x3; do
  SH_LIB=$PWD/siddhi_amd/libsiddhi_hip$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/k$v -o run -- python3 bench.py --workload c3 --steps 2 --warmup 1 > /dev/null 2>$P/k$v.err || { echo "prof $v failed"; tail -5 $P/k$v.err; exit 1; }
  f=$(ls $P/k$v/*/run_kernel_stats.csv $P/k$v/run_kernel_stats.csv 2>/dev/null | head -1)
  python3 - "$f" "$v" <<'PY' | tee -a gpurun_out/r5wk2_times.txt
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "records" in n or "wkey" in n or "slk_emit" in n:
        print(sys.argv[2] or "default", n.split("(")[0][:50], r["AverageNs"])
PY
done
echo done
