#!/bin/bash
# Pooled d = 64 evidence on the current build: FETCH/WRITE passes at K = 1 and
# K = 16, and a kernel trace of the multi-rank step (RCCL on the compute stream)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r5s}
mkdir -p $O
bash tools/gpu_pooled_pmc.sh ${1:-r5s}/k1 1 || exit 10
bash tools/gpu_pooled_pmc.sh ${1:-r5s}/k16 16 || exit 11
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rccl -o run --output-format csv -- \
  python3 tools/rccl_one_rank.py 65536 64 40 1 > $O/rccl.log 2>&1 || exit 12
grep -E "ms/step|bit-equal" $O/rccl.log
exit 0
