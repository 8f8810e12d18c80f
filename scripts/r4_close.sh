#!/bin/bash
# closing check on the final tree: whole GPU suite, smoke, default bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -q -rf -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4c_tests.log 2>&1; rc=$?
tail -4 gpurun_out/r4c_tests.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc"; exit 1; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/r4c_bench.json 2>/dev/null || { echo bench failed; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c2', '%.3e' % d['value'], d['ms_per_step'], d.get('output_sha256_match'))" gpurun_out/r4c_bench.json
echo done
