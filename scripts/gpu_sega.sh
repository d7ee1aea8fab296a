#!/bin/bash
# segmented second-digit pass: hybrid parity tests, then C2/C3/C4 with THRS_SEGA on/off
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  -k "hybrid" > gpurun_out/sega_t.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/sega_t.log; exit 1; }
tail -1 gpurun_out/sega_t.log
for wl in c2 c3 c4; do
  for sg in 1 0 1 0; do
    THRS_SEGA=$sg timeout -k 10 200 python -u scripts/sweep.py --rounds 4 --workload $wl > gpurun_out/sega_$wl.log 2>&1 || { echo "SWEEP FAILED"; tail -20 gpurun_out/sega_$wl.log; exit 1; }
    echo "$wl sega=$sg $(grep main gpurun_out/sega_$wl.log)"
  done
done
