cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; : > gpurun_out/ab_geom.txt
for spec in "kf32v32 80000000" "kf32v32 150000000" "c4 100000000" "c4 180000000"; do set -- $spec
  for g in auto tiny16; do
    timeout -k 10 120 python -u bench.py --workload $1 --n $2 --opt localGeometry=$g --vendor off --cpu-baseline off --ref-gpu off --steps 10 --warmup 3 --quiet > gpurun_out/x.json 2>gpurun_out/x.err || { tail -3 gpurun_out/x.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/x.json')); print(sys.argv[1], sys.argv[2], sys.argv[3], d['ms_per_step'], d['roofline']['path']['local_cap'])" $1 $2 $g >> gpurun_out/ab_geom.txt
  done
done
cat gpurun_out/ab_geom.txt
