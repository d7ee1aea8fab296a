#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "hybrid or matrix or streams or cpp_port_of or pairs_stability" > gpurun_out/hyb6_t.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/hyb6_t.log; exit 1; }
tail -1 gpurun_out/hyb6_t.log
for wl in c2 c3; do
  timeout -k 10 300 python -u scripts/sweep.py --rounds 3 --workload $wl > gpurun_out/hyb6_$wl.log 2>&1 || { echo "SWEEP FAILED"; tail -20 gpurun_out/hyb6_$wl.log; exit 1; }
  echo "$wl $(grep main gpurun_out/hyb6_$wl.log)"
  THRS_HYBRID=0 timeout -k 10 300 python -u scripts/sweep.py --rounds 3 --workload $wl > gpurun_out/hyb6_$wl.log 2>&1 || { echo "SWEEP FAILED"; tail -20 gpurun_out/hyb6_$wl.log; exit 1; }
  echo "$wl LSD $(grep main gpurun_out/hyb6_$wl.log)"
done
