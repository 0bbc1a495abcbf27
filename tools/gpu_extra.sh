#!/bin/bash
# Round-4 extra evidence, one gpurun call: per-config bench lines, the pooled
# d = 64 FETCH/WRITE passes, the RCCL one-rank check with the multi-rank path
# timed beside the fused one, and cell 101 over four keys.
# Usage (on the box): bash tools/gpu_extra.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-extra}
mkdir -p $O
( while sleep 60; do echo "[$(date +%T)] $(ls $O | tr '\n' ' ')"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 900 python3 -u bench.py --configs > $O/configs.jsonl 2> $O/configs.err
r=$?; echo "configs rc=$r"; cut -c1-300 $O/configs.jsonl; [ $r -eq 0 ] || exit $r
bash tools/gpu_pooled_pmc.sh ${1:-extra} || exit 9
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/p256 -o run --output-format csv -- \
  python3 tools/pooled_run.py 32768 256 100 > $O/p256.log 2>&1
r=$?; echo "p256 rc=$r"; grep pooled $O/p256.log; [ $r -eq 0 ] || exit $r
timeout -k 10 240 python3 -u tools/rccl_one_rank.py 65536 64 200 > $O/rccl.txt 2>&1
r=$?; echo "rccl rc=$r"; grep -v amdgpu.ids $O/rccl.txt | tail -4; [ $r -eq 0 ] || exit $r
timeout -k 10 600 python3 -u tools/cell101.py 8 > $O/cell101.txt 2>&1
r=$?; echo "cell101 rc=$r"; grep -v amdgpu.ids $O/cell101.txt; exit $r
