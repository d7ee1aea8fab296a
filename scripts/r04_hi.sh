#!/bin/bash
# round-4: pass B's u8 plane as dwords + lane permutes (THRS_HI_DWORD) vs byte loads (hi0); float workloads
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "f32_planes or float or squeeze or key_range or fallback or hybrid or plane" > gpurun_out/hi_tests.log 2>&1 || { echo FAIL tests; tail -30 gpurun_out/hi_tests.log; exit 1; }
tail -1 gpurun_out/hi_tests.log
timeout -k 10 300 python -u scripts/sweep.py --workload c2 --rounds 6 hi0 r03 > gpurun_out/hi_c2.log 2>&1 || { echo FAIL sweep; tail -20 gpurun_out/hi_c2.log; exit 1; }
grep variant gpurun_out/hi_c2.log
bash scripts/r04_f32b.sh 2>&1 | grep -v "^\.\|passed"
