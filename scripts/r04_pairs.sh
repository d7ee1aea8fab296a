#!/bin/bash
# round-4: f32 pairs rebuild keys from images (no -0); tests + kf32v32 bench
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_ref.py -k "float or f32 or F32 or pairs or squeeze or key_range or fallback or hybrid" > gpurun_out/pairs_tests.log 2>&1 || { echo FAIL tests; tail -30 gpurun_out/pairs_tests.log; exit 1; }
tail -1 gpurun_out/pairs_tests.log
B="--cpu-baseline off --vendor off --ref-gpu off --steps 5 --warmup 1"
for wl in kf32v32 f32k c4 c2; do
  timeout -k 10 300 python -u bench.py $B --workload $wl > gpurun_out/b5_$wl.json 2> gpurun_out/b5_$wl.err || { echo "FAIL $wl"; tail -5 gpurun_out/b5_$wl.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/b5_$wl.json')); r=d['roofline']
print('$wl', d['ms_per_step'], ' '.join(f\"{k}={v['ms_per_sort']}\" for k,v in r['kernels'].items()))"
done
