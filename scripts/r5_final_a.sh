#!/bin/bash
# round-5 closing evidence (1/3): the whole GPU suite and smoke()
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 1080 python -u -m pytest tests -q -rf -m gpu --timeout 300 --timeout-method thread > gpurun_out/r5f_tests.log 2>&1; rc=$?
tail -8 gpurun_out/r5f_tests.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc"; exit 1; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5f_smoke.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/r5f_smoke.log; exit 1; }
tail -2 gpurun_out/r5f_smoke.log
echo done
