#!/bin/bash
# round-4: the whole GPU suite + smoke on one box
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.txt 2>&1
rc=$?
tail -15 gpurun_out/gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.txt 2>&1 && tail -2 gpurun_out/smoke.txt
