#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash scripts/gpu_exp2.sh all1 --workload c3 --rounds 4 --vendor k44a k44b all1 > gpurun_out/cfg_c3.log 2>&1
rc=$?; cat gpurun_out/cfg_c3.log | grep -v amdgpu; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/sweep.py --workload c5 --rounds 4 --vendor k88a k88b all1 > gpurun_out/cfg_c5.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/cfg_c5.log | tail -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/sweep.py --workload k64 --rounds 4 --vendor k80a k80b all1 > gpurun_out/cfg_k64.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/cfg_k64.log | tail -5; exit $rc
