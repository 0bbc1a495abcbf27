#!/bin/bash
# ASSS d = 64 through the step64 kernel: parity (ASSS + steady), timing
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r5p}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_asss.py tests/test_gpu_steady.py tests/test_gpu_parity.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/t.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 tools/asss_run.py > $O/asss.log 2>&1 || exit 10
grep asss $O/asss.log
timeout -k 10 300 python3 bench.py --configs asss64 > $O/cfg.log 2>&1 || exit 11
grep -o '"metric"[^}]*asss[^}]*}' $O/cfg.log | head -3; tail -c 1500 $O/cfg.log
exit 0
