#!/bin/bash
# Round-6 end-of-round evidence on one MI355X box (run through gpurun, two
# calls): "lines" = the GPU test suite, smoke and a bench line per workload
# (-> gpurun_out/bench_<workload>.json); "profiles" = rocprofv3 kernel trace +
# PMC per workload (scripts/profile.sh) and the world-1 RCCL lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
case $1 in
  lines)
    bash scripts/gpu.sh tests smoke bench=c2 bench=c3 bench=c4 bench=c5 bench=u64k bench=f32k bench=kf32v32 \
      bench=kf64v64 bench=k64v128 bench=ref160m bench=ref160m_pairs bench=u32large ;;
  profiles)
    bash scripts/profiles.sh r06 c2 c4 c5 u64k ref160m c3 && bash scripts/r06_dist.sh ;;
esac
