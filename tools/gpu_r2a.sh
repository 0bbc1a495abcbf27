#!/bin/bash
# GPU suite, the clock/state ramp diagnostic, the driver's headline command and
# the 2-rank self-spawned bench on the box's one GPU
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2a
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r2a/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/r2a/pytest_gpu.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/ramp.py > gpurun_out/r2a/ramp.log 2>&1
rc=$?; echo "ramp rc=$rc"; cat gpurun_out/r2a/ramp.log | grep -v amdgpu.ids
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2a/bench1.log 2>&1
rc=$?; echo "bench1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/r2a/bench2.log 2>&1
rc=$?; echo "bench2 rc=$rc"; exit $rc
