#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "hybrid or matrix or streams or special or cpp_port_of" > gpurun_out/hyb4_t.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/hyb4_t.log; exit 1; }
tail -1 gpurun_out/hyb4_t.log
timeout -k 10 300 python -u scripts/sweep.py --rounds 4 ${VARS} > gpurun_out/hyb4_sweep.log 2>&1 || { echo "SWEEP FAILED"; tail -20 gpurun_out/hyb4_sweep.log; exit 1; }
cat gpurun_out/hyb4_sweep.log
THRS_COUNT=0 timeout -k 10 300 python -u scripts/sweep.py --rounds 3 > gpurun_out/hyb4_sweep_rank.log 2>&1 || { echo "SWEEP2 FAILED"; tail -20 gpurun_out/hyb4_sweep_rank.log; exit 1; }
cat gpurun_out/hyb4_sweep_rank.log
timeout -k 10 300 python -u scripts/sweep.py --rounds 3 --workload c4 > gpurun_out/hyb4_sweep_c4.log 2>&1 || { echo "SWEEP3 FAILED"; tail -20 gpurun_out/hyb4_sweep_c4.log; exit 1; }
cat gpurun_out/hyb4_sweep_c4.log
