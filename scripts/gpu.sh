#!/bin/bash
# One parameterised GPU-box script (run through gpurun).  Each argument is a
# step; steps run in order, each under its own time limit, and the first
# failure ends the script (no GPU step runs after a failed one).
#
#   tests[=PATHS[@K]]       python -m pytest -m gpu PATHS -k K (default: the whole gpu suite)
#   smoke                   __graft_entry__.smoke()
#   bench=WORKLOAD[,ARGS]   bench.py --workload WORKLOAD ARGS (commas -> spaces)
#                           -> gpurun_out/bench_WORKLOAD.json
#   prof=TAG,WORKLOAD       scripts/profile.sh TAG WORKLOAD (kernel trace + PMC)
#   ab=WORKLOAD,LIB,...     scripts/ab_libs.py A/B of libthrs builds (main | exp/variants names)
#   cpp                     the C++ UTEST port (tests/cpp/unittest_thrs)
#
# e.g. gpurun -- bash scripts/gpu.sh tests smoke bench=c2 bench=c2_sorted,--steps,5
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for step in "$@"; do
  name=${step%%=*}
  arg=""
  [[ "$step" == *=* ]] && arg=${step#*=}
  echo "=== $step ($(date +%T))"
  case $name in
    tests)
      # tests=PATHS[@K_EXPR]: pytest PATHS -k "K_EXPR"
      targs=${arg:-tests}
      kexpr=""
      [[ "$targs" == *@* ]] && { kexpr=${targs#*@}; targs=${targs%%@*}; }
      timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread $targs \
        ${kexpr:+-k "$kexpr"} > gpurun_out/gpu_tests.txt 2>&1
      rc=$?
      tail -4 gpurun_out/gpu_tests.txt
      [ $rc -eq 0 ] || { echo "TESTS FAILED rc=$rc"; grep -E "FAIL|Error|error" gpurun_out/gpu_tests.txt | head -30; exit 1; }
      ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" || { echo "SMOKE FAILED"; exit 1; }
      ;;
    bench)
      wl=${arg%%,*}
      extra=""
      [[ "$arg" == *,* ]] && extra=$(echo "${arg#*,}" | tr ',' ' ')
      timeout -k 10 600 python -u bench.py --workload $wl $extra > gpurun_out/bench_$wl.json 2> gpurun_out/bench_$wl.err \
        || { echo "BENCH $wl FAILED"; tail -20 gpurun_out/bench_$wl.err; exit 1; }
      cat gpurun_out/bench_$wl.json
      ;;
    prof)
      tag=${arg%%,*}
      wl=${arg#*,}
      bash scripts/profile.sh $tag $wl > gpurun_out/prof_$tag.log 2>&1 || { echo "PROFILE FAILED"; tail -20 gpurun_out/prof_$tag.log; exit 1; }
      echo "profile $tag $wl ok"
      ;;
    stats)
      # per-kernel durations of a short bench run (no counters)
      wl=$arg
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats_$wl -o run -- \
        python3 bench.py --workload $wl --steps 3 --warmup 1 --cpu-baseline off --vendor off --ref-gpu off \
        > gpurun_out/stats_$wl.json 2> gpurun_out/stats_$wl.err || { echo "STATS $wl FAILED"; tail -20 gpurun_out/stats_$wl.err; exit 1; }
      cat gpurun_out/stats_$wl.json
      python3 - "$wl" <<'PY'
import csv, glob, sys
wl = sys.argv[1]
for p in glob.glob(f"gpurun_out/stats_{wl}/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        print(f"{r.get('Name','')[:70]:70s} calls={r.get('Calls')} avg_ns={float(r.get('AverageNs', 0)):.0f}")
PY
      ;;
    ab)
      # ab=WORKLOAD,libA,libB,...: interleaved A/B of libthrs builds (scripts/ab_libs.py)
      # (WORKLOAD may carry a key count: c2:268435456)
      wl=${arg%%,*}
      libs=$(echo "${arg#*,}" | tr ',' ' ')
      nopt=""
      [[ "$wl" == *:* ]] && { nopt="--n ${wl#*:}"; wl=${wl%%:*}; }
      timeout -k 10 600 python -u scripts/ab_libs.py --workload $wl $nopt --rounds 6 $libs > gpurun_out/ab_$wl${nopt:+_n}.txt 2>&1 \
        || { echo "AB $wl FAILED"; tail -20 gpurun_out/ab_$wl.txt; exit 1; }
      cat gpurun_out/ab_$wl${nopt:+_n}.txt
      ;;
    cpp)
      timeout -k 10 600 tests/cpp/unittest_thrs > gpurun_out/cpp_tests.txt 2>&1 \
        || { echo "CPP TESTS FAILED"; tail -20 gpurun_out/cpp_tests.txt; exit 1; }
      tail -3 gpurun_out/cpp_tests.txt
      ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo "=== all steps ok ($(date +%T))"
