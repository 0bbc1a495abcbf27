#!/bin/bash
# Round-end evidence in one call: GPU suite, smoke, headline bench, per-config
# bench with kernel stats (gpu_final.sh), then the headline's rocprofv3 trace
# and FETCH/WRITE passes (gpu_profile.sh).  Usage: tools/gpu_evidence.sh TAG
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r2c}
bash tools/gpu_final.sh $TAG || exit $?
bash tools/gpu_profile.sh $TAG
