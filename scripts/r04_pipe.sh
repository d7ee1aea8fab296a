#!/bin/bash
# round-4: the software-pipelined top-digit pass (THRS_SEG_PIPE) against the main build
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
timeout -k 10 240 python -u scripts/sweep.py --workload c2 --rounds 5 r03 pipe pipewo0 merge > gpurun_out/pipe_c2.log 2>&1 || { echo "FAIL c2"; tail -20 gpurun_out/pipe_c2.log; exit 1; }
cat gpurun_out/pipe_c2.log
timeout -k 10 240 python -u scripts/sweep.py --workload f32k --rounds 3 pipe > gpurun_out/pipe_f32k.log 2>&1 || { echo "FAIL f32k"; tail -20 gpurun_out/pipe_f32k.log; exit 1; }
cat gpurun_out/pipe_f32k.log
timeout -k 10 240 python -u scripts/sweep.py --workload ref160m --rounds 3 pipe > gpurun_out/pipe_160m.log 2>&1 || { echo "FAIL 160m"; tail -20 gpurun_out/pipe_160m.log; exit 1; }
cat gpurun_out/pipe_160m.log
