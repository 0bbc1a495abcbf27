#!/bin/bash
# sufficient-statistics diamonds: parity tests, then the diamonds configs
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "diamonds" > gpurun_out/pt_dss.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/pt_dss.log | tail -30; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/bench_configs.py --only diamonds,diamonds_ss --steps 20 > gpurun_out/cfg_dss.log 2>&1
rc=$?; grep config gpurun_out/cfg_dss.log; exit $rc
