#!/bin/bash
# round-5 closing evidence (2/3): the default bench line (C2 + host-fed leg + CPU baseline) and every
# secondary line
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u bench.py > gpurun_out/r5f_c2.json 2>gpurun_out/r5f_c2.err || { echo c2 bench failed; tail -5 gpurun_out/r5f_c2.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r5f_c2.json')); print('c2', '%.3e' % d['value'], d['ms_per_step'], d.get('output_sha256_match'), d['pcie']['frac'], d['cpu_baseline']['value'])"
for w in c1 c3 c4 c5 ext c2all c2cur c3all plb plg; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r5f_$w.json 2>gpurun_out/r5f_$w.err || { echo "$w bench failed"; tail -3 gpurun_out/r5f_$w.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], '%.3e' % d['value'], d['ms_per_step'], d.get('output_sha256_match'))" gpurun_out/r5f_$w.json $w
done
echo done
