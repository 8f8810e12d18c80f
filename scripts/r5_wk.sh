#!/bin/bash
# round-5 C3 k_sl_wkey timing experiments (libsiddhi_hip_exp_*.so: parts of the replay skipped; results
# are wrong by construction, only the timing matters) next to the product library
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for lib in "" NOSEQ NOROWS NOPAR; do
  if [ -n "$lib" ]; then export SH_LIB=$GRAFT_REPO_ROOT/siddhi_amd/libsiddhi_hip_exp_$lib.so; else unset SH_LIB; fi
  timeout -k 10 300 python -u bench.py --workload c3 --steps 4 --warmup 2 > gpurun_out/r5wk_$lib.json 2>gpurun_out/r5wk.err || { echo "c3 $lib failed"; tail -5 gpurun_out/r5wk.err; exit 1; }
  echo "lib=${lib:-product} $(python3 -c "import json;d=json.load(open('gpurun_out/r5wk_$lib.json'));print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_step'])")"
done
unset SH_LIB
echo done
