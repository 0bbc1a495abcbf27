#!/bin/bash
# large-d per-chain path: parity (incl. chained proposals), then the d = 256 regime-A config
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "big_dim or 96 or 256 or sharded" > gpurun_out/pt_big.log 2>&1
rc=$?; tail -5 gpurun_out/pt_big.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/bench_configs.py --only gauss256 --steps 20 > gpurun_out/cfg_big.log 2>&1
rc=$?; grep config gpurun_out/cfg_big.log; exit $rc
