#!/bin/bash
cd "$GRAFT_REPO_ROOT"
for V in NONE RNG POT SWEEP1 SWEEP2; do
  AMH_LIB_PATH=$PWD/adaptive-mcmc_amd/lib/libamh_abl_$V.so timeout -k 10 120 python3 tools/ablate.py 2>&1 | grep -v amdgpu.ids
  rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || exit $rc
done
