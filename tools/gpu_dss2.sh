#!/bin/bash
# sufficient-statistics diamonds across the kernels (per-chain, pooled, ASSS)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_pooled.py tests/test_gpu_asss.py -k "diamonds" > gpurun_out/pt_dss2.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/pt_dss2.log | tail -30; exit $rc
