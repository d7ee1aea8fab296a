#!/bin/bash
# correctness of one VARIANT library (copied over the main one in a scratch copy) + sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
V=$1; shift
if [ -n "$V" ]; then
  cp tinyhipradixsort_amd/libthrs.so /tmp/libthrs_main.so
  cp build/variants/libthrs_$V.so tinyhipradixsort_amd/libthrs.so
  timeout -k 10 400 python -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -m "gpu and not large" -x -q > gpurun_out/exp_tests.log 2>&1
  rc=$?; echo "tests[$V] rc=$rc"; tail -3 gpurun_out/exp_tests.log
  cp /tmp/libthrs_main.so tinyhipradixsort_amd/libthrs.so
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 400 python scripts/sweep.py "$@" > gpurun_out/exp_sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; grep -v amdgpu.ids gpurun_out/exp_sweep.log | tail -20
exit $rc
