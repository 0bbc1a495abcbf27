#!/bin/bash
# pooled large-d iteration: pooled GPU tests, the regime B configs, kernel stats
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-pb}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests/test_gpu_pooled.py tests/test_gpu_configs.py tests/test_gpu_drivers.py -x -v --timeout 150 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error" gpurun_out/$TAG/pytest.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/bench_configs.py --only gauss256_pooled,pooled64 --steps 50 > gpurun_out/$TAG/cfg.log 2>&1
rc=$?; echo "cfg rc=$rc"; grep config gpurun_out/$TAG/cfg.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof -o run --output-format csv -- \
  python3 tools/bench_configs.py --only gauss256_pooled,pooled64 --steps 50 > gpurun_out/$TAG/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
if [ -f adaptive-mcmc_amd/lib/diag/libamh_stamps.so ]; then timeout -k 10 120 python3 tools/upd_stamps.py --dim 256 || exit 1; fi
