#!/bin/bash
# round-4: per-kernel times of the f32 keys-only workload (2^30, the reference's float generator)
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/pr_f32k -o run -- python3 scripts/sweep.py --workload f32k --rounds 3 none > gpurun_out/pr_f32k.log 2>&1 || { echo FAIL; tail gpurun_out/pr_f32k.log; exit 1; }
python3 scripts/rpd_stats.py gpurun_out/pr_f32k
