#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo "BENCH FAILED"; tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
bash scripts/profile.sh ${TAG:-r01h} c2 > gpurun_out/prof.log 2>&1 || { echo "PROFILE FAILED"; tail -20 gpurun_out/prof.log; exit 1; }
tail -5 gpurun_out/prof.log
