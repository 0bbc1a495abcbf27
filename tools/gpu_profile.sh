#!/bin/bash
# rocprofv3 kernel-trace/stats of the headline bench + separate PMC passes
# (FETCH_SIZE, WRITE_SIZE) for HBM traffic.  Output under gpurun_out/.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r1}
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG/trace -o run --output-format csv -- \
  python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-ess --no-pooled --no-fused > gpurun_out/prof_$TAG/bench_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C -d gpurun_out/prof_$TAG/pmc_$C -o pmc --output-format csv -- \
    python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-ess --no-pooled --no-fused > gpurun_out/prof_$TAG/bench_$C.log 2>&1
  rc=$?; echo "pmc $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
find gpurun_out/prof_$TAG -name '*.csv' | head -20
