#!/bin/bash
# parity tests, then the bench without ESS / CPU legs, then phase stamps
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-ess > gpurun_out/bench_quick.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/bench_quick.log | tail -3
[ $rc -eq 0 ] || exit $rc
if [ -f adaptive-mcmc_amd/lib/diag/libamh_stamps.so ]; then
  timeout -k 10 120 python3 tools/stamps.py > gpurun_out/stamps.log 2>&1
  rc=$?; echo "stamps rc=$rc"; grep -v amdgpu.ids gpurun_out/stamps.log
fi
exit $rc
