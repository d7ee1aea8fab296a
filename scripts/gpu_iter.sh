#!/bin/bash
# One build->measure iteration on the GPU box: fast parity tests, then a
# variant sweep.  Usage: bash scripts/gpu_iter.sh [sweep args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m "gpu and not large" -x -q > gpurun_out/iter_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/iter_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python scripts/sweep.py "$@" > gpurun_out/iter_sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; cat gpurun_out/iter_sweep.log | tail -20
exit $rc
