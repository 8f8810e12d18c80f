#!/bin/bash
# One GPU-box runner for every round's evidence (replaces the per-experiment r4_*/r5_* scripts).
#   scripts/gpu_run.sh TAG STEP [STEP ...]
# STEPs (run in order, each under its own time limit; the first failure ends the call):
#   tests[=EXPR]        pytest -m gpu (optionally -k EXPR) -> gpurun_out/TAG_tests.log
#   smoke               __graft_entry__.smoke()
#   bench[=WL]          bench.py line (default workload, with cpu_baseline) or --workload WL
#   kstats=WL           rocprofv3 --kernel-trace --stats of bench.py --workload WL -> TAG_WL_kernel_stats.txt
#   pmc=WL              FETCH_SIZE and WRITE_SIZE passes (separate runs) -> TAG_WL_pmc.json
#   shard=WL            bench.py --workload WL --shard-loopback G=8 (one-GPU sharded pipeline phases)
#   timeline=WL         kernel trace of 5 steps -> per-step kernel timeline (TL_FIRST = the step's first kernel)
#   htiming=WL          SH_TIMING=1 host-side times between the push's numbered points
# Extra bench arguments: BENCH_ARGS env (e.g. BENCH_ARGS="--steps 10 --warmup 3").
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P=/tmp/gpu_run_$TAG
rm -rf "$P" && mkdir -p "$P"
O=gpurun_out/$TAG
fail() { echo "$1 failed"; [ -f "$2" ] && tail -8 "$2"; exit 1; }
wl_args() { [ -z "$1" ] && echo "" || echo "--workload $1"; }
for step in "$@"; do
  key=${step%%=*}; arg=""; [ "$key" != "$step" ] && arg=${step#*=}
  case $key in
    tests)
      K=(); [ -n "$arg" ] && K=(-k "$arg")
      timeout -k 10 1080 python -u -m pytest tests -q -rf -m gpu "${K[@]}" --timeout 300 --timeout-method thread \
          > "${O}_tests.log" 2>&1 || fail tests "${O}_tests.log"
      tail -3 "${O}_tests.log" ;;
    smoke)
      timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "${O}_smoke.log" 2>&1 || fail smoke "${O}_smoke.log"
      tail -1 "${O}_smoke.log" ;;
    bench)
      n=${arg:-c2}
      extra="--no-cpu-baseline"; [ -z "$arg" ] && extra=""
      timeout -k 10 400 python -u bench.py $(wl_args "$arg") $extra ${BENCH_ARGS:-} > "${O}_${n}_bench.json" 2> "${O}_${n}_bench.err" \
          || fail "bench $n" "${O}_${n}_bench.err"
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d.get('roofline') or {}; print(sys.argv[2], '%.3e' % d['value'], d['ms_per_step'], 'sha', d.get('output_sha256_match'), 'frac', r.get('frac'))" \
          "${O}_${n}_bench.json" "$n" ;;
    kstats)
      n=${arg:-c2}
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$P/kt_$n" -o run --output-format csv -- \
          python3 bench.py $(wl_args "$arg") --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > "$P/kt_$n.json" 2> "$P/kt_$n.err" \
          || fail "kstats $n" "$P/kt_$n.err"
      python3 scripts/kstats.py "$P/kt_$n" > "${O}_${n}_kernel_stats.txt" || fail "kstats summary $n"
      head -8 "${O}_${n}_kernel_stats.txt" ;;
    pmc)
      n=${arg:-c2}
      for ctr in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 150 rocprofv3 --pmc $ctr -d "$P/${n}_$ctr" -o run --output-format csv -- \
            python3 bench.py $(wl_args "$arg") --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > /dev/null 2> "$P/${n}_$ctr.err" \
            || fail "pmc $n $ctr" "$P/${n}_$ctr.err"
      done
      F=$(python3 -c "import glob,sys;print(glob.glob(sys.argv[1]+'/**/run_counter_collection.csv',recursive=True)[0])" "$P/${n}_FETCH_SIZE")
      W=$(python3 -c "import glob,sys;print(glob.glob(sys.argv[1]+'/**/run_counter_collection.csv',recursive=True)[0])" "$P/${n}_WRITE_SIZE")
      python3 scripts/pmc_summary.py "$F" "$W" > "${O}_${n}_pmc.json" || fail "pmc summary $n"
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'GB per push %.3f' % (d['per_push_bytes']/1e9))" "${O}_${n}_pmc.json" "$n" ;;
    timeline)
      n=${arg:-c2}
      first=${TL_FIRST:-k_boundaries}
      timeout -k 10 300 rocprofv3 --kernel-trace -d "$P/tl_$n" -o run --output-format csv -- \
          python3 bench.py $(wl_args "$arg") --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > "$P/tl_$n.json" 2> "$P/tl_$n.err" \
          || fail "timeline $n" "$P/tl_$n.err"
      python3 scripts/timeline.py "$P/tl_$n" "$first" > "${O}_${n}_timeline.txt" || fail "timeline summary $n"
      tail -1 "${O}_${n}_timeline.txt" ;;
    htiming)
      n=${arg:-c2}
      SH_TIMING=1 timeout -k 10 300 python -u bench.py $(wl_args "$arg") --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} \
          > "${O}_${n}_htiming.json" 2> "${O}_${n}_htiming.txt" || fail "htiming $n" "${O}_${n}_htiming.txt"
      grep "sh timing" "${O}_${n}_htiming.txt" | head -12 ;;
    shard)
      n=${arg:-c2}
      timeout -k 10 400 python -u bench.py $(wl_args "$arg") --shard-loopback 8 --steps 5 --warmup 2 --no-cpu-baseline \
          > "${O}_${n}_shard.json" 2> "${O}_${n}_shard.err" || fail "shard $n" "${O}_${n}_shard.err"
      cat "${O}_${n}_shard.json" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo done
