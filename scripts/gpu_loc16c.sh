#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "hybrid or cpp_port" > gpurun_out/l16c_t.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/l16c_t.log; exit 1; }
tail -1 gpurun_out/l16c_t.log
for wl in c2 c3 c4; do
  timeout -k 10 200 python -u scripts/sweep.py --rounds 5 --workload $wl base nohoist > gpurun_out/l16c_$wl.log 2>&1 || { echo "SWEEP FAILED"; tail -20 gpurun_out/l16c_$wl.log; exit 1; }
  echo "== $wl"; grep variant gpurun_out/l16c_$wl.log
done
THRS_LOC16=0 timeout -k 10 200 python -u scripts/sweep.py --rounds 5 --workload c2 base nohoist > gpurun_out/l16c_c2_32.log 2>&1 || { echo "SWEEP FAILED"; exit 1; }
echo "== c2 loc16=0"; grep variant gpurun_out/l16c_c2_32.log
