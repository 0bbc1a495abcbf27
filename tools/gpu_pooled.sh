#!/bin/bash
# Pooled-mode iteration in one gpurun call: the pooled parity tests, a
# rocprofv3 kernel trace of 200 d = 64 steps (65,536 chains), plain timing at
# d = 64 and d = 256, and the d = 64 phase stamps.
# Usage (on the box): bash tools/gpu_pooled.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-pooled}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_pooled.py tests/test_gpu_drivers.py} -v -m gpu --timeout 300 --timeout-method thread > $O/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED" $O/t.log | tail -12
[ $rc -eq 0 -o $rc -eq 1 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pool -o run --output-format csv -- python3 tools/pooled_run.py 65536 64 200 > $O/pool.log 2>&1
r=$?; echo "pool rc=$r"; grep pooled $O/pool.log; [ $r -eq 0 ] || exit $r
timeout -k 10 120 python3 tools/pooled_run.py 65536 64 400 > $O/pool_plain.log 2>&1 && grep pooled $O/pool_plain.log || exit 9
timeout -k 10 120 python3 tools/pooled_run.py 32768 256 100 > $O/pool256.log 2>&1 && grep pooled $O/pool256.log || exit 9
timeout -k 10 120 python3 tools/f64_stamps.py > $O/stamps.txt 2>&1; grep -v amdgpu.ids $O/stamps.txt
# A/B: no noise drawn ahead (the update launch's own path alone)
AMH_LIB_PATH=adaptive-mcmc_amd/lib/diag/libamh_stamps.so AMH_POOLED_NOISE_AHEAD=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pool_nonoise -o run --output-format csv -- python3 tools/pooled_run.py 65536 64 200 > $O/pool_nonoise.log 2>&1; grep pooled $O/pool_nonoise.log
exit $rc
