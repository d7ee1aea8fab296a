#!/bin/bash
# full GPU tests (incl. large) on the main build, then main vs variants on every workload
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/wl_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/wl_tests.log
[ $rc -eq 0 ] || exit $rc
for W in c2 c3 c5 k64 c4; do
  timeout -k 10 400 python scripts/sweep.py --workload $W --rounds 4 "$@" > gpurun_out/wl_$W.log 2>&1
  rc=$?; echo "== $W rc=$rc"; grep -v amdgpu gpurun_out/wl_$W.log | tail -4
  [ $rc -eq 0 ] || exit $rc
done
