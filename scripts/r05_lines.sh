#!/bin/bash
# Round-5 bench lines for every headline workload (one GPU box): each
# workload once through bench.py (vendor leg on; CPU and reference legs only
# on c2, whose line carries them), into gpurun_out/r05_lines/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r05_lines
export TMPDIR=/tmp
for wl in "$@"; do
  extra="--cpu-baseline off --ref-gpu off"
  [ "$wl" = c2 ] && extra=""
  timeout -k 10 400 python -u bench.py --workload $wl $extra > gpurun_out/r05_lines/bench_$wl.json \
    2> gpurun_out/r05_lines/bench_$wl.err || { echo "BENCH $wl FAILED"; tail -5 gpurun_out/r05_lines/bench_$wl.err; exit 1; }
  python3 - "$wl" <<'PY'
import json, sys
wl = sys.argv[1]
d = json.load(open(f"gpurun_out/r05_lines/bench_{wl}.json"))
k = d["roofline"]["kinds"]
print(wl, d["ms_per_step"], d["value"], {n: v["avg_launch_ms"] for n, v in k.items()},
      "vendor", (d.get("vendor") or {}).get("ms_per_sort"))
PY
done
