#!/bin/bash
# pooled d = 64, K = 1: noise drawn ahead (update launch) vs in the stats
# kernel, diagnostic library (AMH_POOLED_NOISE_AHEAD), kernel times + step time
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-nab}
mkdir -p $O
export AMH_LIB_PATH=adaptive-mcmc_amd/lib/diag/libamh_stamps.so
for rep in 1 2; do
  for v in 1 0; do
    AMH_POOLED_NOISE_AHEAD=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/n${v}_$rep -o run --output-format csv -- \
      python3 tools/pooled_run.py 65536 64 400 1 > $O/n${v}_$rep.log 2>&1 || exit 10
    echo "ahead=$v: $(grep pooled $O/n${v}_$rep.log)"
    f=$(find $O/n${v}_$rep -name "*kernel_stats.csv" | head -1)
    grep -E "pooled" $f | cut -d, -f1-4 | cut -c1-120
  done
done
exit 0
