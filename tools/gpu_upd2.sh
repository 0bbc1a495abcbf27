#!/bin/bash
# pooled large-d update: bit-exact tests, phase stamps, config timings
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/upd
timeout -k 10 600 python -u -m pytest tests/test_gpu_pooled.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread -k "pooled or regime_b" > gpurun_out/upd/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error|assert" gpurun_out/upd/pytest.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 tools/upd_stamps.py --dim 256 || exit 1
timeout -k 10 300 python3 tools/bench_configs.py --only gauss256_pooled,gauss256_pooled_k16 --steps 20 > gpurun_out/upd/cfg.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/upd/cfg.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
for v in adaptive-mcmc_amd/lib/var_*/; do
  AMH_LIB_PATH=$PWD/${v}libamh.so timeout -k 10 300 python3 tools/bench_configs.py --only gauss256_pooled --steps 20 > gpurun_out/upd/cfg_$(basename $v).log 2>&1 || exit 1
  echo "$(basename $v): $(grep -v amdgpu.ids gpurun_out/upd/cfg_$(basename $v).log | cut -c1-160)"
done
