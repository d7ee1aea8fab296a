set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for i in 1 2; do
for o in offsets=lookback offsets=reserve; do
  timeout -k 10 120 python -u bench.py --workload c2 --steps 10 --cpu-baseline off --vendor off --ref-gpu off --opt $o > gpurun_out/ab_$o.$i.json 2> gpurun_out/ab_$o.$i.err || exit 1
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_$o.$i.json')); print('$o', d['ms_per_step'], d['roofline']['kinds']['pass']['by_launch_ms'])"
done; done
for o in offsets=lookback offsets=reserve; do
  timeout -k 10 120 python -u bench.py --workload c4 --steps 10 --cpu-baseline off --vendor off --ref-gpu off --opt $o > gpurun_out/ab4_$o.json 2> gpurun_out/ab4_$o.err || exit 1
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab4_$o.json')); print('c4 $o', d['ms_per_step'], d['roofline']['kinds']['pass']['by_launch_ms'])"
done
