#!/bin/bash
# regime B large-d: parity tests + kernel profile of the d=256 config
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_bp3
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pooled.py -k "256 or 128" > gpurun_out/pt_bp.log 2>&1
rc=$?; tail -2 gpurun_out/pt_bp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bp3 -o run --output-format csv -- python3 tools/bench_configs.py --only gauss256_pooled --steps 20 > gpurun_out/cfg.log 2>&1
rc=$?; grep config gpurun_out/cfg.log; [ $rc -eq 0 ] || exit $rc
python3 tools/kstats.py gpurun_out/prof_bp3/run_kernel_stats.csv pooled pot
