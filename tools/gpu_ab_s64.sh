#!/bin/bash
# Headline-kernel A/B on one box: the drain stamps (diagnostic build), then
# the d = 64 step launch time for the release library and each variant
# library under adaptive-mcmc_amd/lib/var_*/ (tools/build_variants.sh).
# Usage (on the box): bash tools/gpu_ab_s64.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-ab}
mkdir -p $O
timeout -k 10 120 python3 tools/s64_tail.py > $O/tail.txt 2>&1
r=$?; grep -v amdgpu.ids $O/tail.txt; [ $r -eq 0 ] || exit $r
for rep in 1 2; do
  for lib in release adaptive-mcmc_amd/lib/var_*/libamh.so; do
    if [ $lib = release ]; then
      timeout -k 10 120 python3 tools/s64_sweep.py 65536 > $O/sweep_release_$rep.txt 2>&1; r=$?
      echo "release: $(grep C= $O/sweep_release_$rep.txt)"
    else
      n=$(basename $(dirname $lib))
      AMH_LIB_PATH=$lib timeout -k 10 120 python3 tools/s64_sweep.py 65536 > $O/sweep_${n}_$rep.txt 2>&1; r=$?
      echo "$n: $(grep C= $O/sweep_${n}_$rep.txt)"
    fi
    [ $r -eq 0 ] || exit $r
  done
done
