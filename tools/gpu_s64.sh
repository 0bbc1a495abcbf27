#!/bin/bash
# d = 64 step kernel A/B: parity tests of the Gaussian paths, then the headline
# bench with the LDS-staged kernel and with the general kernel (AMH_STEP64=0)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s64
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_drivers.py tests/test_gpu_eval.py -x -v --timeout 120 --timeout-method thread > gpurun_out/s64/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error|error" gpurun_out/s64/pytest.log | tail -8
[ $rc -eq 0 ] || exit $rc
for v in 1 0 1; do
  AMH_STEP64=$v timeout -k 10 200 python3 bench.py --steps 400 --warmup 50 --no-extra > gpurun_out/s64/b$v.log 2>&1
  rc=$?; echo "AMH_STEP64=$v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep -o '"ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*\|"frac": [0-9.]*' gpurun_out/s64/b$v.log | tr '\n' ' '; echo
done
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-extra > gpurun_out/s64/drv.log 2>&1
rc=$?; echo "driver-shape rc=$rc"
grep -o '"ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*\|"frac": [0-9.]*' gpurun_out/s64/drv.log | tr '\n' ' '; echo
exit $rc
