#!/bin/bash
# round-5 c3all: k_slx_wkey timing experiments (exp libraries, never the product) + PMC of the default
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P=/tmp/r5xw
rm -rf $P && mkdir -p $P
for v in "" _x1 _x2 _x3; do
  SH_LIB=$PWD/siddhi_amd/libsiddhi_hip$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/k$v -o run -- python3 bench.py --workload c3all --steps 2 --warmup 1 > /dev/null 2>$P/k$v.err || { echo "prof $v failed"; tail -5 $P/k$v.err; exit 1; }
  f=$(ls $P/k$v/*/run_kernel_stats.csv $P/k$v/run_kernel_stats.csv 2>/dev/null | head -1)
  echo "lib$v $(grep -h k_slx_wkey $f | awk -F, '{print $0}' | python3 -c "import sys,csv;r=list(csv.reader(sys.stdin));print(r[0][3] if r else 'none')")" | tee -a gpurun_out/r5xw_times.txt
done
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d $P/c_$ctr -o run --output-format csv -- python3 bench.py --workload c3all --steps 1 --warmup 1 > /dev/null 2>$P/c_$ctr.err || { echo "$ctr failed"; exit 1; }
done
python3 scripts/pmc_summary.py "$(ls $P/c_FETCH_SIZE/*/run_counter_collection.csv | head -1)" "$(ls $P/c_WRITE_SIZE/*/run_counter_collection.csv | head -1)" > gpurun_out/r5xw_pmc.json || echo "pmc summary failed"
head -c 2500 gpurun_out/r5xw_pmc.json
echo done
