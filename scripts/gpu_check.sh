set -o pipefail
cd "$GRAFT_REPO_ROOT"
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 700 python -m pytest tests -m "gpu and not large" -x -q > gpurun_out/t1.log 2>&1; rc=$?
echo "pytest rc=$rc"
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 400 python bench.py --steps 5 --warmup 1 > gpurun_out/bench1.json 2> gpurun_out/bench1.err; echo "bench rc=$?"
fi
tail -5 gpurun_out/t1.log; cat gpurun_out/bench1.json
