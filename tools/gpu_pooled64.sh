#!/bin/bash
# pooled (regime B) GPU tests, then the pooled bench legs at d = 64
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/p64
timeout -k 10 600 python -u -m pytest tests/test_gpu_pooled.py -x -v --timeout 200 --timeout-method thread > gpurun_out/p64/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error|error" gpurun_out/p64/pytest.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/bench_configs.py --only pooled64,gauss256_pooled --steps 20 > gpurun_out/p64/cfg.log 2>&1
rc=$?; echo "configs rc=$rc"; grep -v amdgpu.ids gpurun_out/p64/cfg.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
rm -rf gpurun_out/p64prof; mkdir -p gpurun_out/p64prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p64prof -o run --output-format csv -- python3 tools/bench_configs.py --only pooled64 --steps 20 > gpurun_out/p64prof/log.txt 2>&1
rc=$?; f=$(find gpurun_out/p64prof -name "*kernel_stats.csv" | head -1); python3 tools/kstats.py $f amh; exit $rc
