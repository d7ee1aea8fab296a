#!/bin/bash
# occupancy of the local kernel + per-kernel times of the hybrid C2 sort
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/hyb2
timeout -k 10 120 python3 -c "
import tinyhipradixsort_amd as T, torch
torch.cuda.set_device(0)
print('local occupancy (WG/CU):', T.lib().thrs_debug_local_occupancy())
" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/hyb2/bench -o run -- python3 bench.py --steps 5 --warmup 1 --cpu-baseline off > gpurun_out/hyb2/bench.json 2> gpurun_out/hyb2/bench.log || { tail -5 gpurun_out/hyb2/bench.log; exit 1; }
cat gpurun_out/hyb2/bench.json
find gpurun_out/hyb2/bench -name "*kernel_stats.csv" | head -1 | xargs cat | cut -d, -f1-8 | head -20
