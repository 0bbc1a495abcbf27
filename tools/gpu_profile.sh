#!/bin/bash
# rocprofv3 kernel-trace/stats of the driver's default bench command
# (`python bench.py`), then separate PMC passes (FETCH_SIZE, WRITE_SIZE) of the
# headline leg alone for HBM traffic.  Output under gpurun_out/prof_<tag>/.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r2}
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG/trace -o run --output-format csv -- \
  python3 bench.py > gpurun_out/prof_$TAG/bench_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C -d gpurun_out/prof_$TAG/pmc_$C -o pmc --output-format csv -- \
    python3 bench.py --steps 20 --warmup 2 --no-extra --no-fused > gpurun_out/prof_$TAG/bench_$C.log 2>&1
  rc=$?; echo "pmc $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python3 bench.py > gpurun_out/prof_$TAG/bench_plain.log 2>&1
rc=$?; echo "plain bench rc=$rc"; tail -c 600 gpurun_out/prof_$TAG/bench_plain.log; exit $rc
