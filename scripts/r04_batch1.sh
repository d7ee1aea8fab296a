#!/bin/bash
# round-4 batch: baseline + squeeze + size-window measurements (one gpurun call)
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
set -o pipefail
B="--cpu-baseline off --vendor off --ref-gpu off --steps 5 --warmup 1"
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python -u bench.py $B "$@" > gpurun_out/b1_$name.json 2> gpurun_out/b1_$name.err || { echo "FAIL $name"; tail -5 gpurun_out/b1_$name.err; return 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/b1_$name.json')); r=d['roofline']
print('$name', d['ms_per_step'], d['value'], r['kernel'], r['frac'], ' '.join(f\"{k}={v['ms_per_sort']}x{v['launches_per_sort']}\" for k,v in r['kernels'].items()))"
}
run c2 --workload c2 --steps 10 --warmup 2 &&
run kf32v32 --workload kf32v32 &&
run f32k --workload f32k &&
run kf64v64 --workload kf64v64 &&
run c4 --workload c4 &&
run c3 --workload c3 &&
run ref160m --workload ref160m &&
run ref160m_lsd --workload ref160m --opt path=lsd &&
run ref160m_bucket --workload ref160m --opt path=bucket &&
run ref160m_pairs --workload ref160m_pairs &&
run ref160m_pairs_bucket --workload ref160m_pairs --opt path=bucket &&
run n27_lsd --workload c2 --n 134217728 --opt path=lsd &&
run n27_bucket --workload c2 --n 134217728 --opt path=bucket &&
run n28_lsd --workload c2 --n 268435456 --opt path=lsd &&
run n28_bucket --workload c2 --n 268435456 --opt path=bucket &&
echo "batch1 done"
