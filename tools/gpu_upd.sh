#!/bin/bash
# pooled large-d update: bit-exact tests, update phase stamps, config timings
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/upd
timeout -k 10 600 python -u -m pytest tests/test_gpu_pooled.py tests/test_gpu_configs.py -x -v --timeout 200 --timeout-method thread -k "pooled or regime_b" > gpurun_out/upd/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error" gpurun_out/upd/pytest.log | tail -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 tools/upd_stamps.py --dim 256 || exit 1
timeout -k 10 120 python3 tools/upd_stamps.py --dim 64 --chains 65536 || exit 1
timeout -k 10 300 python3 tools/bench_configs.py --only pooled64,gauss256_pooled --steps 20 > gpurun_out/upd/cfg.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/upd/cfg.log | cut -c1-220; exit $rc
