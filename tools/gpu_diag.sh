#!/bin/bash
# Diagnostics in one gpurun call: pooled d = 64 phase stamps, the headline's
# memory ceiling (tools/membound.py) and the per-config bench lines.
# Usage (on the box): bash tools/gpu_diag.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-diag}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 120 python3 tools/f64_stamps.py > $O/stamps.txt 2>&1
r=$?; echo "stamps rc=$r"; grep -v amdgpu.ids $O/stamps.txt
[ $r -eq 0 ] || exit $r
timeout -k 10 300 python3 tools/membound.py > $O/membound.txt 2>&1
r=$?; echo "membound rc=$r"; grep -v amdgpu.ids $O/membound.txt
[ $r -eq 0 ] || exit $r
timeout -k 10 700 python3 -u bench.py --configs > $O/configs.jsonl 2> $O/configs.err
r=$?; echo "configs rc=$r"; tail -c 1500 $O/configs.err | grep -v amdgpu.ids
exit $r
