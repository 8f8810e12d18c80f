#!/bin/bash
# round-5: resident waves per SIMD of the wave-per-key replays (libsiddhi_hip_w{4,5,6}.so; timing only)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in "" _w4 _w5 _w6; do
  for w in c3 c3all; do
    SH_LIB=$PWD/siddhi_amd/libsiddhi_hip$v.so timeout -k 10 300 python3 -u bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r5wpe_$w$v.json 2>gpurun_out/r5wpe_$w$v.err || { echo "$w $v failed"; tail -5 gpurun_out/r5wpe_$w$v.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], '%.3e' % d['value'], round(d['ms_per_step'],3), d['roofline']['achieved'])" gpurun_out/r5wpe_$w$v.json "$w${v:-_w3}"
  done
done
echo done
