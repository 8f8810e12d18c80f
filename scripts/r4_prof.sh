#!/bin/bash
# round-4 profiles: C2 / C3 / C4 kernel stats + a C4 kernel trace, and the PMC passes of C2 and C3
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for w in c2 c3 c4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4p_$w -o $w -- python3 bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r4p_$w.log 2>&1 || { echo "$w prof failed"; tail gpurun_out/r4p_$w.log; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r4p_c4trace -o c4 -- python3 bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r4p_c4trace.log 2>&1 || { echo "c4 trace failed"; exit 1; }
for w in c2 c3; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $ctr -d gpurun_out/r4p_${w}_$ctr -o pmc -- python3 bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r4p_${w}_$ctr.log 2>&1 || { echo "$w $ctr failed"; exit 1; }
  done
done
echo done
