#!/bin/bash
# local-sort variants: hybrid parity tests, then C2 with THRS_LOC16 on/off, C3, C4
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "hybrid or cpp_port" > gpurun_out/l16_t.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/l16_t.log; exit 1; }
tail -1 gpurun_out/l16_t.log
for v in 1 0 1 0; do
  THRS_LOC16=$v timeout -k 10 200 python -u scripts/sweep.py --rounds 5 --workload c2 > gpurun_out/l16_c2.log 2>&1 || { echo "SWEEP FAILED"; tail -20 gpurun_out/l16_c2.log; exit 1; }
  echo "c2 loc16=$v $(grep main gpurun_out/l16_c2.log)"
done
for wl in c3 c4; do
  timeout -k 10 200 python -u scripts/sweep.py --rounds 5 --workload $wl > gpurun_out/l16_$wl.log 2>&1 || { echo "SWEEP FAILED"; tail -20 gpurun_out/l16_$wl.log; exit 1; }
  echo "$wl $(grep main gpurun_out/l16_$wl.log)"
done
