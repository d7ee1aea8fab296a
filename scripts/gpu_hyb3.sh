#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py \
  -k "hybrid_paths or matrix" > gpurun_out/hyb3_t.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/hyb3_t.log; exit 1; }
tail -1 gpurun_out/hyb3_t.log
timeout -k 10 300 python -u scripts/sweep.py --rounds 4 ${SWEEP_ARGS} ${VARS} > gpurun_out/hyb3_sweep.log 2>&1 || { echo "SWEEP FAILED"; tail -20 gpurun_out/hyb3_sweep.log; exit 1; }
cat gpurun_out/hyb3_sweep.log
