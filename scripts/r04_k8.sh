#!/bin/bash
# round-4: 8-byte-key pass geometries with one stage round (k8r1) vs the default two rounds
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
for wl in c5 k64; do
  timeout -k 10 300 python -u scripts/sweep.py --workload $wl --rounds 4 k8r1 > gpurun_out/k8_$wl.log 2>&1 || { echo FAIL $wl; tail -20 gpurun_out/k8_$wl.log; exit 1; }
  echo $wl; grep variant gpurun_out/k8_$wl.log
done
B="--cpu-baseline off --vendor off --ref-gpu off --steps 4 --warmup 1"
for lib in main k8r1; do
  L=""; [ $lib != main ] && L="--lib exp/variants/libthrs_$lib.so"
  timeout -k 10 300 python -u bench.py $B $L --workload c5 > gpurun_out/k8b_$lib.json 2> gpurun_out/k8b_$lib.err || { echo "FAIL bench $lib"; tail -5 gpurun_out/k8b_$lib.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/k8b_$lib.json')); r=d['roofline']
print('$lib c5', d['ms_per_step'], ' '.join(f\"{k}={v['ms_per_sort']}\" for k,v in r['kernels'].items()))"
done
