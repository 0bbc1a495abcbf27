#!/bin/bash
# diamonds potential on MFMA: parity (split/fused/oracle, config size), timing + kernel trace;
# also the 16-wave pooled update's bit-exact tests
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/dia
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_pooled.py tests/test_gpu_asss.py -x -q --timeout 200 --timeout-method thread -k "${DIA_K:-diamonds or pooled or regime_b}" > gpurun_out/dia/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error|assert" gpurun_out/dia/pytest.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/dia/prof -o run --output-format csv -- python3 tools/bench_configs.py --only ${DIA_CFG:-diamonds,gauss256_pooled} --steps 20 > gpurun_out/dia/cfg.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/dia/cfg.log | cut -c1-220; [ $rc -eq 0 ] || exit $rc
python3 tools/kstats.py gpurun_out/dia/prof/run_kernel_stats.csv diamonds propose step_kernel pooled
