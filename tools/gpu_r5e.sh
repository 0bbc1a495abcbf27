#!/bin/bash
# Round 5: the whole GPU suite (large-d ASSS, K-template stats kernel) and
# the pooled timing.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r5e}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -x -v -m gpu --timeout 300 --timeout-method thread > $O/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/t.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/k1 -o run --output-format csv -- python3 tools/pooled_run.py 65536 64 200 1 > $O/k1.log 2>&1 || exit 11
grep pooled $O/k1.log
timeout -k 10 200 python3 tools/pooled_run.py 65536 64 320 16 > $O/k16.log 2>&1 || exit 12
grep pooled $O/k16.log
exit 0
