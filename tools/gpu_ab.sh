#!/bin/bash
# Generic A/B on one box: run one python command (a tools/ script and its
# arguments) with the release library and each named variant library
# (adaptive-mcmc_amd/lib/var_<name>/, tools/build_variants.sh), twice.
# Usage (on the box): bash tools/gpu_ab.sh TAG "script args" VARIANT...
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-ab}; CMD=$2; shift 2
mkdir -p $O
for rep in 1 2; do
  for v in release "$@"; do
    if [ $v = release ]; then
      timeout -k 10 180 python3 $CMD > $O/ab_${v}_$rep.txt 2>&1; r=$?
    else
      AMH_LIB_PATH=adaptive-mcmc_amd/lib/var_$v/libamh.so timeout -k 10 180 python3 $CMD > $O/ab_${v}_$rep.txt 2>&1; r=$?
    fi
    echo "$v: $(grep -v amdgpu.ids $O/ab_${v}_$rep.txt | tail -1)"
    [ $r -eq 0 ] || exit $r
  done
done
