#!/bin/bash
# round-4: the pass kernels' packed digit cache (main) vs recomputed digits (dc0), interleaved sweeps
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "hybrid or fallback or float or lowentropy or low_entropy or sorted or extreme" > gpurun_out/dc_tests.log 2>&1 || { echo FAIL tests; tail -30 gpurun_out/dc_tests.log; exit 1; }
tail -1 gpurun_out/dc_tests.log
for wl in kf32v32 c3 c2 c5; do
  timeout -k 10 300 python -u scripts/sweep.py --workload $wl --rounds 4 dc0 > gpurun_out/dc_$wl.log 2>&1 || { echo FAIL $wl; tail -20 gpurun_out/dc_$wl.log; exit 1; }
  echo $wl; grep variant gpurun_out/dc_$wl.log
done
