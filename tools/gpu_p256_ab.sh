#!/bin/bash
# d = 256 regime-B step: per-kernel times (rocprofv3) for the release library
# and each variant library.  Usage (on the box): bash tools/gpu_p256_ab.sh TAG VARIANT...
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-p256}; shift
mkdir -p $O
for v in release "$@"; do
  lib=adaptive-mcmc_amd/lib/libamh.so
  [ $v = release ] || lib=adaptive-mcmc_amd/lib/var_$v/libamh.so
  AMH_LIB_PATH=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/kp_$v -o run --output-format csv -- \
    python3 tools/pooled_run.py 32768 256 100 > $O/kp_$v.log 2>&1
  r=$?; [ $r -eq 0 ] || { echo "$v rc=$r"; exit $r; }
  f=$(find $O/kp_$v -name "*kernel_stats.csv" | head -1)
  echo "$v: $(grep pooled $O/kp_$v.log)"
  grep -E "amh::pooled" $f | cut -d, -f1-4 | cut -c1-150
done
