#!/bin/bash
# A/B of libthrs variant builds (make variants -> exp/variants/): for each
# "WORKLOAD:variant" argument (variant "base" = the in-tree libthrs.so), one
# short bench.py run; prints ms/step and per-kind ms/sort / launches.
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
# (WORKLOAD:variant:OPTS -- OPTS passed as bench.py --opt, e.g. c2:base:planes=off)
for a in "$@"; do
  wl=${a%%:*}; v=${a#*:}; o=""
  [[ "$v" == *:* ]] && { o=${v#*:}; v=${v%%:*}; }
  lib=""; [ "$v" != base ] && lib="--lib exp/variants/libthrs_$v.so"
  tag=$v${o:+_$(echo $o | tr ',=' '__')}
  timeout -k 10 200 python -u bench.py --workload $wl --steps 5 --warmup 1 --cpu-baseline off --vendor off --ref-gpu off $lib \
    ${o:+--opt $o} ${VB_EXTRA:-} > gpurun_out/var_${wl}_$tag.json 2>gpurun_out/var_${wl}_$tag.err || { echo "FAIL $a"; tail -3 gpurun_out/var_${wl}_$tag.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/var_${wl}_$tag.json')); r=d['roofline']
k=r['kinds']
print('$wl $tag', d['ms_per_step'], ' '.join(f\"{n}={v['ms_per_sort']}/{v['launches_per_sort']}{v.get('by_launch_ms') or ''}\" for n,v in k.items()))"
done
