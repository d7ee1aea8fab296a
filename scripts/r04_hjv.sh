#!/bin/bash
# round-4: the checked f32 histogram's cost (no check / 2 iterations per epoch) on f32 workloads
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
B="--cpu-baseline off --vendor off --ref-gpu off --steps 5 --warmup 1"
for lib in main hjnochk hjep; do
  L=""; [ $lib != main ] && L="--lib exp/variants/libthrs_$lib.so"
  for wl in f32k kf32v32; do
    timeout -k 10 300 python -u bench.py $B $L --workload $wl > gpurun_out/hv_${lib}_$wl.json 2> gpurun_out/hv_${lib}_$wl.err || { echo "FAIL $lib $wl"; tail -5 gpurun_out/hv_${lib}_$wl.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/hv_${lib}_$wl.json')); r=d['roofline']
print('$lib $wl', d['ms_per_step'], ' '.join(f\"{k}={v['ms_per_sort']}\" for k,v in r['kernels'].items()))"
  done
done
