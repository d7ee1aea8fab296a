#!/bin/bash
# bucket path vs LSD passes at sizes below the bucket path's default window
# (ms per sort from bench.py lines), into gpurun_out/crossover.txt;
# WL=c3 for u32 pairs (default c2: u32 keys-only)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/crossover.txt
for n in "$@"; do
  for path in bucket lsd; do
    timeout -k 10 120 python -u bench.py --workload ${WL:-c2} --n $n --opt path=$path --vendor off --cpu-baseline off \
      --ref-gpu off --steps 10 --warmup 3 --quiet > gpurun_out/xo.json 2> gpurun_out/xo.err || { tail -3 gpurun_out/xo.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/xo.json')); print(sys.argv[3], sys.argv[1], sys.argv[2], d['ms_per_step'])" $n $path ${WL:-c2} >> gpurun_out/crossover.txt
  done
done
cat gpurun_out/crossover.txt
