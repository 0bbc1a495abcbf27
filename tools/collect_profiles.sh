#!/bin/bash
# Copy one tools/gpu_full.sh run (gpurun_out/<run>) into profiles/<tag>_*:
# the step-kernel summary with FETCH/WRITE traffic (prof_summary.py), the
# rocprofv3 kernel stats of the default bench command and of 200 pooled
# d = 64 steps, the bench line, the smoke line and the pytest tail.
# Usage (here): bash tools/collect_profiles.sh RUN TAG
set -e
cd "$(dirname "$0")/.."
R=gpurun_out/$1; T=$2
python3 tools/prof_summary.py $T --src $R > /dev/null
grep -v amdgpu.ids $R/bench.log | tail -1 > profiles/${T}_bench.json
f=$(ls $R/pool/*/run_kernel_stats.csv 2>/dev/null | head -1 || true)
[ -z "$f" ] && f=$(find $R/pool -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cp $f profiles/${T}_pooled64_kernel_stats.csv
grep -E "passed|failed" $R/pytest_gpu.log | tail -3 > profiles/${T}_pytest_gpu_tail.txt
grep -A25 "slowest" $R/pytest_gpu.log >> profiles/${T}_pytest_gpu_tail.txt || true
grep smoke $R/smoke.log >> profiles/${T}_pytest_gpu_tail.txt || true
ls -la profiles/${T}_*
