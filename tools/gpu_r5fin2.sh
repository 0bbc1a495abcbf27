#!/bin/bash
# final build: GPU suite, smoke, bench.py --configs
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r5fin2}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 10
tail -2 $O/smoke.log
timeout -k 10 500 python3 bench.py --configs > $O/cfg.log 2>&1 || exit 11
grep -c "^{" $O/cfg.log
exit 0
