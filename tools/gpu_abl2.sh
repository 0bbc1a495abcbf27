#!/bin/bash
# fused large-d stats kernel per ablation variant + update kernel phase stamps
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/upd_stamps.py --dim 256 || exit 1
bash tools/gpu_fbvariants.sh
