#!/bin/bash
# Pooled-step A/B on one box: release library vs each variant library that
# rebuilt amh_big_pooled.hip (lib/var_<name>/, tools/build_variants.sh), at
# d = 64 (65,536 chains, configs[4] per GPU) and d = 256 (32,768 chains).
# Usage (on the box): bash tools/gpu_ab_pooled.sh TAG VARIANT...
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-abp}; shift
mkdir -p $O
for rep in 1 2; do
  for v in release "$@"; do
    for cfg in "65536 64 400" "32768 256 100"; do
      if [ $v = release ]; then
        timeout -k 10 120 python3 tools/pooled_run.py $cfg > $O/p_${v}.txt 2>&1; r=$?
      else
        AMH_LIB_PATH=adaptive-mcmc_amd/lib/var_$v/libamh.so timeout -k 10 120 python3 tools/pooled_run.py $cfg > $O/p_${v}.txt 2>&1; r=$?
      fi
      echo "$v: $(grep pooled $O/p_${v}.txt)"
      [ $r -eq 0 ] || exit $r
    done
  done
done
