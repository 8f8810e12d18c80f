#!/bin/bash
# round-5 C3 / c3all: records without per-slot counting, key offsets from the sorted slots
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P=/tmp/r5c3c
rm -rf $P && mkdir -p $P
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sliding_minmax.py \
  tests/test_gpu_sliding_expired.py "tests/test_gpu_scale.py::test_c3_time_10s_10k_keys_1k_resident_per_key" \
  tests/test_gpu_parity.py tests/test_gpu_snapshot.py tests/test_gpu_shard.py > gpurun_out/r5c3c_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|error" gpurun_out/r5c3c_tests.log | head -20; tail -30 gpurun_out/r5c3c_tests.log; exit 1; }
tail -2 gpurun_out/r5c3c_tests.log
for w in c3 c3all; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 6 --warmup 2 > gpurun_out/r5c3c_${w}_bench.json 2>gpurun_out/r5c3c.err || { echo "$w failed"; tail -5 gpurun_out/r5c3c.err; exit 1; }
  echo "$w $(python3 -c "import json;d=json.load(open('gpurun_out/r5c3c_${w}_bench.json'));print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_step'])")"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/c3 -o run -- python3 bench.py --workload c3 --steps 3 --warmup 1 > /dev/null 2>$P/c3.err || { echo "c3 prof failed"; tail -5 $P/c3.err; exit 1; }
python3 - $P/c3 > gpurun_out/r5c3c_kernel_stats.txt <<'PY'
import csv, sys, glob
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)
for r in csv.DictReader(open(f[0])):
    if "at::native" in r["Name"]:
        continue
    print(f"{r['Name'].split('(')[0][:70]:70s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.1f} us")
PY
head -12 gpurun_out/r5c3c_kernel_stats.txt
echo done
