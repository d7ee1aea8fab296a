#!/bin/bash
# round-4: per-kernel times of the main build against the round-3 build (c2), one library per rocprofv3 run
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pr_main -o run -- python3 scripts/sweep.py --workload c2 --rounds 4 none > gpurun_out/pr_main.log 2>&1 || { echo FAIL main; tail gpurun_out/pr_main.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pr_r03 -o run -- python3 scripts/sweep.py --workload c2 --rounds 4 --no-main r03 > gpurun_out/pr_r03.log 2>&1 || { echo FAIL r03; tail gpurun_out/pr_r03.log; exit 1; }
grep variant gpurun_out/pr_main.log gpurun_out/pr_r03.log
bash scripts/r04_batch2.sh
