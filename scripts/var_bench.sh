#!/bin/bash
# A/B of libthrs variant builds (make variants -> exp/variants/): for each
# "WORKLOAD:variant" argument (variant "base" = the in-tree libthrs.so), one
# short bench.py run; prints ms/step, avg pass, hist and local kernel ms.
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
for a in "$@"; do
  wl=${a%%:*}; v=${a#*:}
  lib=""; [ "$v" != base ] && lib="--lib exp/variants/libthrs_$v.so"
  timeout -k 10 200 python -u bench.py --workload $wl --steps 5 --warmup 1 --cpu-baseline off --vendor off --ref-gpu off $lib \
    > gpurun_out/var_${wl}_$v.json 2>gpurun_out/var_${wl}_$v.err || { echo "FAIL $a"; tail -3 gpurun_out/var_${wl}_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/var_${wl}_$v.json')); r=d['roofline']
print('$wl $v', d['ms_per_step'], r['avg_launch_ms'], r['hist_avg_ms'], (r.get('local') or {}).get('avg_launch_ms'))"
done
