#!/bin/bash
# Pooled-kernel iteration on one box: the pooled GPU parity tests, then the
# per-kernel times of the release library (and variants), the d = 64 update
# timeline and the d = 256 regime-B step.
# Usage (on the box): bash tools/gpu_pooled_iter.sh TAG [VARIANT...]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${1:-pi}; shift
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pooled.py tests/test_gpu_configs.py > $O/pytest_pooled.log 2>&1
r=$?; tail -3 $O/pytest_pooled.log; [ $r -eq 0 ] || { grep -E "Error|FAIL" $O/pytest_pooled.log | head -20; exit $r; }
bash tools/gpu_pooled_kprof.sh $T "$@" || exit 7
timeout -k 10 120 python3 tools/u64_timeline.py --steps 8 > $O/u64_tl.txt 2>&1; r=$?
grep median $O/u64_tl.txt; [ $r -eq 0 ] || exit $r
timeout -k 10 120 python3 tools/f64_stamps.py > $O/f64_stamps.txt 2>&1; r=$?
grep -v amdgpu.ids $O/f64_stamps.txt; [ $r -eq 0 ] || exit $r
timeout -k 10 120 python3 tools/pooled_run.py 32768 256 100 > $O/p256.txt 2>&1; r=$?
grep pooled $O/p256.txt; exit $r
