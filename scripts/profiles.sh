#!/bin/bash
# rocprofv3 evidence for profiles/: scripts/profile.sh (kernel trace + stats
# of the bench command, then one --pmc pass per counter group) per workload,
# and the LDS counter groups of scripts/sqprof.sh for a workload's kernels
# when "lds:<workload>" is named.  usage: bash scripts/profiles.sh <tag> c2 lds:c2 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1
shift
for wl in "$@"; do
  if [[ "$wl" == lds:* ]]; then
    SQ_GROUPS="2 3" bash scripts/sqprof.sh ${TAG}_lds_${wl#lds:} ${wl#lds:} || exit 1
  else
    bash scripts/profile.sh $TAG $wl > gpurun_out/prof_${TAG}_$wl.out 2>&1 || { tail -5 gpurun_out/prof_${TAG}_$wl.out; exit 1; }
    tail -3 gpurun_out/prof_${TAG}_$wl.out
  fi
done
