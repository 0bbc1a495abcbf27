#!/bin/bash
# sufficient-statistics diamonds: all diamonds parity cases, then its config bench
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_pooled.py tests/test_gpu_asss.py -k "diamonds" > gpurun_out/pt_dss3.log 2>&1
rc=$?; tail -3 gpurun_out/pt_dss3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/bench_configs.py --only diamonds_ss --steps 20 > gpurun_out/cfg_dss3.log 2>&1
rc=$?; grep config gpurun_out/cfg_dss3.log; exit $rc
