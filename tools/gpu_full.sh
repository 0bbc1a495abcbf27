#!/bin/bash
# One gpurun call of round evidence, in order, each step under its own time
# limit and stopping at the first failure:
#   whole GPU suite -> smoke -> rocprofv3 kernel trace of the driver's default
#   bench command -> FETCH_SIZE / WRITE_SIZE passes of the headline leg ->
#   the plain default bench -> rocprofv3 of 200 pooled d = 64 steps.
# Usage (on the box): bash tools/gpu_full.sh TAG [pytest -k expression]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-r4}
O=gpurun_out/$TAG
mkdir -p $O
KX=()
[ -n "$2" ] && KX=(-k "$2")
# progress line every minute (the last finished test), so a long CPU-side
# oracle check inside one test is not taken for a hang; every step below
# still has its own time limit
( while sleep 60; do echo "[$(date +%T)] $(tail -n 1 $O/pytest_gpu.log 2>/dev/null | cut -c1-120)"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 900 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread --durations=20 "${KX[@]}" > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/pytest_gpu.log | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rs=$?; echo "smoke rc=$rs"; grep smoke $O/smoke.log
[ $rs -eq 0 ] || exit $rs
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python3 bench.py > $O/bench_trace.log 2>&1
rt=$?; echo "trace rc=$rt"; [ $rt -eq 0 ] || exit $rt
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C -d $O/pmc_$C -o pmc --output-format csv -- \
    python3 bench.py --steps 20 --warmup 2 --no-extra --no-fused > $O/bench_$C.log 2>&1
  rp=$?; echo "pmc $C rc=$rp"; [ $rp -eq 0 ] || exit $rp
done
timeout -k 10 300 python3 bench.py > $O/bench.log 2>&1
rb=$?; echo "bench rc=$rb"; grep -v amdgpu.ids $O/bench.log | tail -c 400
[ $rb -eq 0 ] || exit $rb
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pool -o run --output-format csv -- python3 tools/pooled_run.py 65536 64 200 > $O/pool.log 2>&1
rp=$?; echo "pool rc=$rp"; grep pooled $O/pool.log
exit $rp
