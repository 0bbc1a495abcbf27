#!/bin/bash
# d = 64 pooled update timeline (diagnostic build): default, without the
# noise drawn ahead, and with the relaxed-ticket variant's source built into
# the diagnostic library when lib/diag_relaxed exists.
# Usage (on the box): bash tools/gpu_u64_tl.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-tl}
mkdir -p $O
timeout -k 10 120 python3 tools/u64_timeline.py --steps 8 > $O/tl_default.txt 2>&1 || exit 1
echo "default:  $(grep median $O/tl_default.txt)"
AMH_POOLED_NOISE_AHEAD=0 timeout -k 10 120 python3 tools/u64_timeline.py --steps 8 > $O/tl_nonoise.txt 2>&1 || exit 1
echo "no noise: $(grep median $O/tl_nonoise.txt)"
if [ -f adaptive-mcmc_amd/lib/diag_relaxed/libamh_stamps.so ]; then
  AMH_LIB_PATH=adaptive-mcmc_amd/lib/diag_relaxed/libamh_stamps.so timeout -k 10 120 python3 tools/u64_timeline.py --steps 8 > $O/tl_relaxed.txt 2>&1 || exit 1
  echo "relaxed:  $(grep median $O/tl_relaxed.txt)"
fi
