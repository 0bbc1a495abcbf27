#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the pooled d = 64 step (configs[4] per GPU),
# one pass each (rocprofv3 --pmc), 30 in-place steps of 65,536 chains.
# Usage (on the box): bash tools/gpu_pooled_pmc.sh TAG [K] (K = sync_every: 30 blocks)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-pool_pmc}
K=${2:-1}
mkdir -p $O
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C -d $O/pmc_$C -o pmc --output-format csv -- \
    python3 tools/pooled_run.py 65536 64 $((30 * K)) $K > $O/pool_$C.log 2>&1
  r=$?; echo "pooled pmc $C rc=$r"; [ $r -eq 0 ] || exit $r
done
