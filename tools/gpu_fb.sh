#!/bin/bash
# fused large-d pooled stats: bit-exact tests, config-size regime B, timings + kernel trace
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/fb
timeout -k 10 600 python -u -m pytest tests/test_gpu_pooled.py tests/test_gpu_configs.py -x -v --timeout 200 --timeout-method thread -k "pooled or regime_b" > gpurun_out/fb/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error|assert" gpurun_out/fb/pytest.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/bench_configs.py --only gauss256_pooled,gauss256_pooled_k16 --steps 20 > gpurun_out/fb/cfg.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/fb/cfg.log | cut -c1-220; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fb/prof -o run --output-format csv -- python3 tools/bench_configs.py --only gauss256_pooled --steps 20 > gpurun_out/fb/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
