#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_pooled.py -x -q -m gpu > gpurun_out/pytest_pooled.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -20 gpurun_out/pytest_pooled.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-ess > gpurun_out/bench_pooled.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/bench_pooled.log | tail -3
exit $rc
