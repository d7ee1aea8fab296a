#!/bin/bash
# Per-launch timeline of one sort (rocprofv3 kernel trace of a short bench run,
# scripts/gaps.py): each kernel's duration and the idle gap before it.
# usage: bash scripts/timeline.sh <tag> <workload>...  -> gpurun_out/tl_<tag>_<workload>.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=$1
shift
for wl in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl_${TAG}_$wl -o run -- \
    python3 bench.py --workload $wl --steps 3 --warmup 1 --cpu-baseline off --vendor off --ref-gpu off \
    > gpurun_out/tl_${TAG}_$wl.json 2> gpurun_out/tl_${TAG}_$wl.log || { echo "trace $wl failed"; tail -5 gpurun_out/tl_${TAG}_$wl.log; exit 1; }
  python3 scripts/gaps.py gpurun_out/tl_${TAG}_$wl --sort 2 > gpurun_out/tl_${TAG}_$wl.txt && tail -3 gpurun_out/tl_${TAG}_$wl.txt
done
