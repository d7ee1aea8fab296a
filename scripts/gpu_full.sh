#!/bin/bash
# full GPU test suite (incl. large) + default bench + 1-rank RCCL bench, one call
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1000 python -m pytest tests -m gpu -x -q --durations=15 > gpurun_out/full_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -25 gpurun_out/full_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --force-dist --steps 5 --cpu-baseline off > gpurun_out/bench_dist.json 2> gpurun_out/bench_dist.err
rc=$?; echo "bench dist rc=$rc"; cat gpurun_out/bench_dist.json; tail -5 gpurun_out/bench_dist.err
exit $rc
