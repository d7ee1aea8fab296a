#!/bin/bash
# LDS counters per kernel for one workload (one --pmc pass, SQ block only)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_lds_${1:-c2}${TAG:-}
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc ${PMC:-SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_LDS} --kernel-trace --output-format csv -d $OUT -o run -- python3 scripts/profile_run.py --workload ${1:-c2} --steps 2 > $OUT/log.txt 2>&1 || { tail -5 $OUT/log.txt; exit 1; }
python3 - $OUT <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"][:50]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[(k, r["Counter_Name"])] += 1
for k, d in agg.items():
    n = max(cnt[(k, c)] for c in d)
    print(k, {c: round(v / n) for c, v in d.items()})
PY
