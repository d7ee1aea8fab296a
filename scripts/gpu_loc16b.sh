#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for lds in 45056 81920 163840; do
  THRS_LOC16_LDS=$lds timeout -k 10 200 python -u scripts/sweep.py --rounds 4 --workload c2 > gpurun_out/l16b.log 2>&1 || { echo "SWEEP FAILED"; tail -20 gpurun_out/l16b.log; exit 1; }
  echo "c2 loc16 lds=$lds $(grep main gpurun_out/l16b.log)"
done
