#!/bin/bash
# hybrid path: parity first (small/medium sizes), then one C2 bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_parity.py \
  -k "hybrid_paths or matrix or streams_bit_exact" > gpurun_out/hyb_t1.log 2>&1 || { echo "TESTS FAILED rc=$?"; tail -40 gpurun_out/hyb_t1.log; exit 1; }
tail -3 gpurun_out/hyb_t1.log
timeout -k 10 240 python -u bench.py --steps 10 --warmup 2 --cpu-baseline off > gpurun_out/hyb_b1.log 2>&1 || { echo "BENCH FAILED"; tail -30 gpurun_out/hyb_b1.log; exit 1; }
tail -2 gpurun_out/hyb_b1.log
THRS_HYBRID=0 timeout -k 10 240 python -u bench.py --steps 10 --warmup 2 --cpu-baseline off > gpurun_out/hyb_b0.log 2>&1 || { echo "BENCH0 FAILED"; tail -30 gpurun_out/hyb_b0.log; exit 1; }
tail -1 gpurun_out/hyb_b0.log
