#!/bin/bash
# Headline kernel trace + FETCH/WRITE PMC passes (tools/gpu_profile.sh), then
# the kernel stats of the per-config bench.  Output under gpurun_out/.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r1}
bash tools/gpu_profile.sh $TAG || exit $?
mkdir -p gpurun_out/prof_$TAG/cfg
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG/cfg -o run --output-format csv -- \
  python3 tools/bench_configs.py --steps 20 > gpurun_out/prof_$TAG/cfg.log 2>&1
rc=$?; echo "cfg trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
find gpurun_out/prof_$TAG -name '*kernel_stats.csv'
