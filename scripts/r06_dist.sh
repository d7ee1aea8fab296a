#!/bin/bash
# round 6: the multi-GPU path at world 1 over RCCL (bench.py --force-dist): per-phase times for C2 and the C5 shape
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29613 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0
for wl in c2 c5; do
  timeout -k 10 300 python -u bench.py --force-dist --workload $wl --steps 5 --warmup 1 --cpu-baseline off --vendor off --ref-gpu off > gpurun_out/dist_$wl.json 2> gpurun_out/dist_$wl.err || { echo "FAIL $wl"; tail -10 gpurun_out/dist_$wl.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/dist_$wl.json'))
print('$wl', d['ms_per_step'], d['value'], d.get('phases_ms'), {k: v['avg_launch_ms'] for k, v in d['roofline']['kernels'].items()})"
done
