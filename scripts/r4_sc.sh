#!/bin/bash
# stream.current.event flushes built on the device: parity, then the c2cur line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q -x -rf --timeout 300 --timeout-method thread -m gpu tests/test_gpu_stream_current.py \
  tests/test_gpu_parity.py tests/test_gpu_rate.py tests/test_gpu_snapshot.py tests/test_gpu_partition.py > gpurun_out/r4sc_tests.log 2>&1 || { tail -30 gpurun_out/r4sc_tests.log; exit 1; }
tail -2 gpurun_out/r4sc_tests.log
timeout -k 10 300 python -u bench.py --workload c2cur --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r4sc_c2cur.json 2>/dev/null || { echo "c2cur failed"; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c2cur', '%.3e' % d['value'], d['ms_per_step'])" gpurun_out/r4sc_c2cur.json
echo done
