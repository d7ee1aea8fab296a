#!/bin/bash
# Round-5 rocprofv3 evidence: scripts/profile.sh (kernel trace + stats of the
# bench command, then one --pmc pass per counter group) per workload, and the
# LDS counter groups of scripts/sqprof.sh for C2's local sort when "lds" is named.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for wl in "$@"; do
  if [ "$wl" = lds ]; then
    SQ_GROUPS="2 3" bash scripts/sqprof.sh r05_lds c2 || exit 1
  else
    bash scripts/profile.sh r05 $wl > gpurun_out/prof_r05_$wl.out 2>&1 || { tail -5 gpurun_out/prof_r05_$wl.out; exit 1; }
    tail -3 gpurun_out/prof_r05_$wl.out
  fi
done
