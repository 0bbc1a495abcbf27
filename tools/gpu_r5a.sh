#!/bin/bash
# Round-5 baseline on the GPU: pooled / ASSS parity after the zero-tangent
# and check_device changes, kernel traces of the pooled d = 64 step at K = 1
# and K = 16 and of the multi-rank (1-rank nccl) step, and the stats phases.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r5a}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_pooled.py tests/test_gpu_asss.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/t.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/k1 -o run --output-format csv -- python3 tools/pooled_run.py 65536 64 200 1 > $O/k1.log 2>&1 || exit 11
grep pooled $O/k1.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/k16 -o run --output-format csv -- python3 tools/pooled_run.py 65536 64 320 16 > $O/k16.log 2>&1 || exit 12
grep pooled $O/k16.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/rccl -o run --output-format csv -- python3 tools/rccl_one_rank.py 65536 64 100 > $O/rccl.log 2>&1 || exit 13
grep -E "ms/step|bit-equal" $O/rccl.log
timeout -k 10 120 python3 tools/f64_stamps.py > $O/stamps.txt 2>&1 || exit 14
grep -v amdgpu.ids $O/stamps.txt
exit 0
