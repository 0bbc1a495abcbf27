#!/bin/bash
# 16-wave d = 64 step kernel: parity of the Gaussian paths, then step-launch
# timing of the default build against the lib/var_* variants
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/w16
timeout -k 10 300 python -u tools/dbg_s64.py 3000 > gpurun_out/w16/dbg.log 2>&1
rc=$?; echo "dbg rc=$rc"; cat gpurun_out/w16/dbg.log | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_drivers.py -x -q --timeout 120 --timeout-method thread > gpurun_out/w16/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/w16/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_variants.sh 32768 65536 131072
