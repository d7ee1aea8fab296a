#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "hybrid" > gpurun_out/small_t.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/small_t.log; exit 1; }
tail -1 gpurun_out/small_t.log
WLS="c4" bash scripts/gpu_wl.sh
for n in 134217728 268435456 402653184 536870912; do WLS="c2" EXTRA="--n $n" bash scripts/gpu_wl.sh | sed "s/^/n=$n /"; done
