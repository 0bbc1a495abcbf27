#!/bin/bash
# Whole GPU suite, headline bench and per-config bench (one gpurun call).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -3
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench_full.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/bench_full.log | tail -2
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --configs --steps 20 > gpurun_out/cfg.log 2>&1
rc=$?; echo "configs rc=$rc"; grep config gpurun_out/cfg.log
exit $rc
