#!/bin/bash
# One gpurun call of evidence: whole GPU suite, smoke, headline bench, then a
# rocprofv3 kernel trace of the pooled d = 64 step (configs[4] per GPU).
# Usage (on the box): bash tools/gpu_evidence.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-r3}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/pytest_gpu.log | tail -12
[ $rc -eq 0 -o $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rs=$?; echo "smoke rc=$rs"; grep smoke $O/smoke.log
[ $rs -eq 0 ] || exit $rs
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1
rb=$?; echo "bench rc=$rb"; grep -v amdgpu.ids $O/bench.log | tail -c 600
[ $rb -eq 0 ] || exit $rb
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pool -o run --output-format csv -- python3 tools/pooled_run.py 65536 64 200 > $O/pool.log 2>&1
rp=$?; echo "pool rc=$rp"; grep pooled $O/pool.log
exit $rc
