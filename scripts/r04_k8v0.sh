#!/bin/bash
# round-4: u64 keys-only passes with one stage round (k8v0r1) vs two (default)
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
for n in 1073741824 67108864; do
  timeout -k 10 300 python -u scripts/sweep.py --workload k64 --n $n --rounds 4 k8v0r1 > gpurun_out/k8v0_$n.log 2>&1 || { echo FAIL $n; tail -20 gpurun_out/k8v0_$n.log; exit 1; }
  echo $n; grep variant gpurun_out/k8v0_$n.log
done
