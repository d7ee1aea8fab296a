#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for cfg in "THRS_RANK=atomic" "THRS_RANK=ballot" "THRS_HYBRID=0"; do
  env $cfg timeout -k 10 200 python -u scripts/sweep.py --rounds 3 > gpurun_out/hyb5.log 2>&1 || { echo "SWEEP FAILED $cfg"; tail -20 gpurun_out/hyb5.log; exit 1; }
  echo "$cfg $(tail -1 gpurun_out/hyb5.log)"
done
