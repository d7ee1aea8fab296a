#!/bin/bash
# hybrid vs LSD for the given workloads (sweep.py, one process per setting)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for wl in ${WLS:-c4}; do
  for hy in 1 0; do
    THRS_HYBRID=$hy timeout -k 10 300 python -u scripts/sweep.py --rounds 3 --workload $wl ${EXTRA} > gpurun_out/wl_$wl.log 2>&1 || { echo "SWEEP FAILED"; tail -20 gpurun_out/wl_$wl.log; exit 1; }
    echo "$wl hybrid=$hy $(grep main gpurun_out/wl_$wl.log)"
  done
done
