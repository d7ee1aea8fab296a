#!/bin/bash
# round evidence: full GPU tests + smoke, default bench lines (C2 with CPU baseline, C3, C4), rocprof profile of C2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash scripts/gpu_full2.sh || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { echo "BENCH C2 FAILED"; tail -20 gpurun_out/bench_c2.err; exit 1; }
cat gpurun_out/bench_c2.json
for wl in c3 c4; do
  timeout -k 10 400 python -u bench.py --workload $wl --cpu-baseline off > gpurun_out/bench_$wl.json 2> gpurun_out/bench_$wl.err || { echo "BENCH $wl FAILED"; tail -20 gpurun_out/bench_$wl.err; exit 1; }
  cat gpurun_out/bench_$wl.json
done
bash scripts/profile.sh ${TAG:-r01h2} c2 > gpurun_out/prof.log 2>&1 || { echo "PROFILE FAILED"; tail -20 gpurun_out/prof.log; exit 1; }
echo profile ok
