#!/bin/bash
# round-5 C2 gather emission: batch-window parity suites, headline digests, C2 bench A/B, kernel stats
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P=/tmp/r5c2g
rm -rf $P && mkdir -p $P
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_headline.py \
  tests/test_gpu_parity.py tests/test_gpu_expired.py tests/test_gpu_shard.py tests/test_gpu_aggregation.py \
  tests/test_gpu_keys.py tests/test_gpu_stream_current.py tests/test_gpu_shard_pipeline.py \
  > gpurun_out/r5c2g_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|error" gpurun_out/r5c2g_tests.log | head -20; tail -40 gpurun_out/r5c2g_tests.log; exit 1; }
tail -3 gpurun_out/r5c2g_tests.log
for g in 1 0; do
  SH_EMIT_GATHER=$g timeout -k 10 300 python -u bench.py --steps 20 --warmup 4 --no-cpu-baseline --no-pcie > gpurun_out/r5c2g_$g.json 2>gpurun_out/r5c2g.err || { echo "c2 failed"; tail -5 gpurun_out/r5c2g.err; exit 1; }
  echo "gather=$g $(python3 -c "import json;d=json.load(open('gpurun_out/r5c2g_$g.json'));print(d['value'], d['ms_per_step'], d.get('output_sha256_match'))")"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/c2 -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-pcie > /dev/null 2>$P/c2.err || { echo "c2 prof failed"; tail -5 $P/c2.err; exit 1; }
python3 - $P/c2 > gpurun_out/r5c2g_kernel_stats.txt <<'PY'
import csv, sys, glob
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)
for r in csv.DictReader(open(f[0])):
    if "at::native" in r["Name"]:
        continue
    print(f"{r['Name'].split('(')[0][:70]:70s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.1f} us")
PY
head -12 gpurun_out/r5c2g_kernel_stats.txt
echo done
