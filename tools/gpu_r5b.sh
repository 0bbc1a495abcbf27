#!/bin/bash
# Full GPU suite + pooled / RCCL timing + the headline bench (round 5).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r5b}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/t.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/k1 -o run --output-format csv -- python3 tools/pooled_run.py 65536 64 200 1 > $O/k1.log 2>&1 || exit 11
grep pooled $O/k1.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/k16 -o run --output-format csv -- python3 tools/pooled_run.py 65536 64 320 16 > $O/k16.log 2>&1 || exit 12
grep pooled $O/k16.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/rccl -o run --output-format csv -- python3 tools/rccl_one_rank.py 65536 64 100 > $O/rccl.log 2>&1 || exit 13
grep -E "ms/step|bit-equal" $O/rccl.log
timeout -k 10 200 python3 tools/rccl_one_rank.py 65536 64 320 16 > $O/rccl16.log 2>&1 || exit 14
grep -E "ms/step|bit-equal" $O/rccl16.log
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 15
tail -c 3000 $O/bench.json
exit 0
