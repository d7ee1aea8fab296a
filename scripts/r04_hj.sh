#!/bin/bash
# round-4: checked f32 histogram, 3 vs 2 loads in flight (sweep, interleaved)
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
for wl in f32k kf32v32 c4; do
  timeout -k 10 240 python -u scripts/sweep.py --workload $wl --rounds 4 hjun2 > gpurun_out/hj_$wl.log 2>&1 || { echo FAIL $wl; tail -20 gpurun_out/hj_$wl.log; exit 1; }
  echo $wl; grep variant gpurun_out/hj_$wl.log
done
