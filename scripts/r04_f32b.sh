#!/bin/bash
# round-4: float workloads after the split-codec images, 3-load checked histogram, squeezed items shifted
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
true

B="--cpu-baseline off --vendor off --ref-gpu off --steps 5 --warmup 1"
run() {
  local name=$1; shift
  timeout -k 10 300 python -u bench.py $B "$@" > gpurun_out/b4_$name.json 2> gpurun_out/b4_$name.err || { echo "FAIL $name"; tail -5 gpurun_out/b4_$name.err; return 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/b4_$name.json')); r=d['roofline']
print('$name', d['ms_per_step'], d['value'], r['kernel'], r['frac'], ' '.join(f\"{k}={v['ms_per_sort']}x{v['launches_per_sort']}\" for k,v in r['kernels'].items()), r['kinds']['pass'].get('by_launch_ms'))"
}
run f32k --workload f32k && run c4 --workload c4 && run kf32v32 --workload kf32v32 && run c2 --workload c2 && run kf64v64 --workload kf64v64 && echo done
