#!/bin/bash
# round-4: local sorts of pairs (C3) and 8-byte keys (C5 shape) against the round-3 build (sweep, interleaved)
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
for wl in c3 c5; do
  timeout -k 10 300 python -u scripts/sweep.py --workload $wl --rounds 4 r03 > gpurun_out/loc_$wl.log 2>&1 || { echo FAIL $wl; tail -20 gpurun_out/loc_$wl.log; exit 1; }
  echo $wl; grep variant gpurun_out/loc_$wl.log
done
