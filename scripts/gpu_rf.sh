set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "hybrid or cpp_port" > gpurun_out/rf_t.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/rf_t.log; exit 1; }
tail -1 gpurun_out/rf_t.log
for wl in c2 c3 c4; do
  timeout -k 10 300 python -u scripts/sweep.py --rounds 8 --workload $wl old new > gpurun_out/rf_$wl.log 2>&1 || { echo "SWEEP FAILED"; tail -20 gpurun_out/rf_$wl.log; exit 1; }
  echo $wl; grep variant gpurun_out/rf_$wl.log
done
