#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the d = 256 regime-A kernels (one PMC pass each)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/bigpmc
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --pmc $C -d gpurun_out/bigpmc/$C -o pmc --output-format csv -- \
    python3 tools/bench_configs.py --only gauss256 --steps 10 > gpurun_out/bigpmc/$C.log 2>&1
  rc=$?; echo "$C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
