#!/bin/bash
# round-4 batch 2: where the bucket path starts to pay (keys-only and pairs), and the float workloads after the sampled squeeze
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
B="--cpu-baseline off --vendor off --ref-gpu off --steps 5 --warmup 1"
run() {
  local name=$1; shift
  timeout -k 10 300 python -u bench.py $B "$@" > gpurun_out/b2_$name.json 2> gpurun_out/b2_$name.err || { echo "FAIL $name"; tail -5 gpurun_out/b2_$name.err; return 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/b2_$name.json')); r=d['roofline']
print('$name', d['ms_per_step'], d['value'], r['kernel'], r['frac'], ' '.join(f\"{k}={v['ms_per_sort']}x{v['launches_per_sort']}\" for k,v in r['kernels'].items()))"
}
for n in 140000000 150000000; do
  run k${n}_lsd --workload c2 --n $n --opt path=lsd && run k${n}_bucket --workload c2 --n $n --opt path=bucket || exit 1
done
for n in 100000000 134217728; do
  run p${n}_lsd --workload c3 --n $n --opt path=lsd && run p${n}_bucket --workload c3 --n $n --opt path=bucket || exit 1
done
run kf32v32 --workload kf32v32 && run f32k --workload f32k && run c4 --workload c4 && run c4_nosq --workload c4 --opt squeeze=off && run kf32v32_nosq --workload kf32v32 --opt squeeze=off &&
echo "batch2 done"
