#!/bin/bash
# regime A large-d iteration: large-d parity tests, the d=256 config, kernel stats
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-ra}
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_drivers.py -x -v --timeout 150 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error" gpurun_out/$TAG/pytest.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof -o run --output-format csv -- \
  python3 tools/bench_configs.py --only gauss256 --steps 20 > gpurun_out/$TAG/cfg.log 2>&1
rc=$?; echo "cfg rc=$rc"; grep config gpurun_out/$TAG/cfg.log; exit $rc
