#!/bin/bash
# rocprofv3 collection for profiles/: kernel trace + stats, then one --pmc pass
# per counter group (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950),
# never combined with sys/runtime traces.  usage: bash scripts/profile.sh <tag> [workload]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r01}; WL=${2:-c2}
OUT=gpurun_out/prof_${TAG}_${WL}
mkdir -p $OUT
# 1) the bench command itself (its thrs_pass average must agree with bench.py's roofline)
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bench -o run -- python3 bench.py --workload $WL --steps 5 --warmup 1 --cpu-baseline off --vendor off --ref-gpu off > $OUT/bench.json 2> $OUT/bench.log || { echo "bench trace failed"; tail -5 $OUT/bench.log; exit 1; }
cat $OUT/bench.json
# 2) calibration copies + sorts: trace, then one --pmc pass per counter group
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 scripts/profile_run.py --workload $WL > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -5 $OUT/trace.log; exit 1; }
for C in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  name=$(echo $C | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/pmc_$name -o run -- python3 scripts/profile_run.py --workload $WL > $OUT/pmc_$name.log 2>&1 || { echo "pmc $C failed"; tail -5 $OUT/pmc_$name.log; exit 1; }
done
python3 scripts/prof_summary.py $OUT > $OUT/summary.json && cat $OUT/summary.json
