#!/bin/bash
# round-4: instruction counts of the local sort, u32 (C2) vs f32 keys (one --pmc pass each)
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
export TMPDIR=/tmp
for wl in c2 f32k; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_INSTS_SALU SQ_INSTS_SMEM --kernel-trace --output-format csv -d gpurun_out/sq_$wl -o run -- python3 scripts/profile_run.py --workload $wl > gpurun_out/sq_$wl.log 2>&1 || { echo "pmc $wl failed"; tail -5 gpurun_out/sq_$wl.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for wl in ("c2", "f32k"):
    agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for p in glob.glob(f"gpurun_out/sq_{wl}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            name = r.get("Kernel_Name", "")
            if "local16" not in name and "pass_seg" not in name: continue
            key = ("local16" if "local16" in name else "pass_seg<" + name.split("thrs_pass_seg<")[1][:14])
            agg[(key, r.get("Dispatch_Id"))][r["Counter_Name"]] += float(r["Counter_Value"])
    tot = collections.defaultdict(lambda: collections.defaultdict(list))
    for (key, d), cs in agg.items():
        if cs.get("SQ_WAVES", 0) < 1000: continue
        for c, v in cs.items(): tot[key][c].append(v)
    for key, cs in tot.items():
        print(wl, key, {c: round(sum(v) / len(v) / 1e6, 2) for c, v in sorted(cs.items())})
PY
