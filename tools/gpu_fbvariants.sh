#!/bin/bash
# fused pooled kernel time per diagnostic variant (rocprofv3 kernel stats)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for d in default adaptive-mcmc_amd/lib/var_*/; do
  n=$(basename $d); rm -rf gpurun_out/fbv/$n; mkdir -p gpurun_out/fbv/$n
  if [ $n = default ]; then unset AMH_LIB_PATH; else export AMH_LIB_PATH=$PWD/${d}libamh.so; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/fbv/$n -o run --output-format csv -- python3 tools/bench_configs.py --only gauss256_pooled --steps 20 > gpurun_out/fbv/$n/log.txt 2>&1 || exit 1
  f=$(find gpurun_out/fbv/$n -name "*kernel_stats.csv" | head -1)
  echo "$n: $(python3 tools/kstats.py $f fused_big)"
done
