#!/bin/bash
# full GPU regression: smoke + every -m gpu test (incl. large), one process each
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log | tail -1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/full_t.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/full_t.log; exit 1; }
tail -3 gpurun_out/full_t.log
