#!/bin/bash
# round-end evidence in one call: GPU suite + smoke + headline bench + per-config
# bench, then rocprofv3 kernel stats of the per-config bench
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r1c}
mkdir -p gpurun_out/prof_$TAG/cfg
bash tools/gpu_round.sh || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; grep smoke gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG/cfg -o run --output-format csv -- \
  python3 bench.py --configs --steps 20 > gpurun_out/prof_$TAG/cfg.log 2>&1
rc=$?; echo "cfg trace rc=$rc"; exit $rc
