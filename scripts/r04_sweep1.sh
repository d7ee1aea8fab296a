#!/bin/bash
# round-4 A/B sweep (one process per workload, variants interleaved): main vs round-3 build and experiments
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
for wl in c2 c4 kf32v32; do
  echo "== $wl"
  timeout -k 10 400 python -u scripts/sweep.py --workload $wl --rounds 5 r03 noalign merge bo2 || exit 1
done
timeout -k 10 300 python -u scripts/seg_stamps.py > gpurun_out/seg_stamps.log 2>&1 && cat gpurun_out/seg_stamps.log
