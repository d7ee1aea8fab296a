#!/bin/bash
# quick experiment: interleaved sweep of variants (args passed to sweep.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m "gpu and not large" -x -q -k "matrix or reference_streams" > gpurun_out/exp_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/exp_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/sweep.py "$@" > gpurun_out/exp_sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; grep -v amdgpu.ids gpurun_out/exp_sweep.log | tail -20
exit $rc
