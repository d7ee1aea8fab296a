#!/bin/bash
# tests + sweep + stamps in one GPU call
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m "gpu and not large" -x -q > gpurun_out/iter_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/iter_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/sweep.py --rounds 4 --vendor main w16 w4 > gpurun_out/iter_sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; grep -v amdgpu.ids gpurun_out/iter_sweep.log | tail -20
[ $rc -eq 0 ] || exit $rc
#timeout -k 10 300 python scripts/stamps.py > gpurun_out/stamps.log 2>&1
rc=$?; echo "stamps rc=$rc"; grep -v amdgpu.ids gpurun_out/stamps.log | head -2
