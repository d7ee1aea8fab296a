#!/bin/bash
# probe + sweep + stamps (no tests) in one GPU call
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/lds_order_probe > gpurun_out/lds_probe.log 2>&1; echo "probe rc=$?"; cat gpurun_out/lds_probe.log
timeout -k 10 400 python scripts/sweep.py --rounds 4 "$@" > gpurun_out/iter_sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; grep -v amdgpu.ids gpurun_out/iter_sweep.log | tail -20
[ $rc -eq 0 ] || exit $rc
THRS_TILE=${THRS_TILE:-16384} timeout -k 10 300 python scripts/stamps.py > gpurun_out/stamps.log 2>&1
rc=$?; echo "stamps rc=$rc"; grep -v amdgpu.ids gpurun_out/stamps.log | head -1
