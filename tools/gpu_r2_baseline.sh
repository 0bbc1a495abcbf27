#!/bin/bash
# round-2 baseline: the driver's headline command three times back to back,
# then a long run, to see the spread of the step-kernel time
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2base
for k in 1 2 3; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ess --no-pooled > gpurun_out/r2base/drv_$k.log 2>&1
  rc=$?; echo "drv $k rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep -o '"ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*\|"frac": [0-9.]*' gpurun_out/r2base/drv_$k.log | tr '\n' ' '; echo
done
timeout -k 10 200 python3 bench.py --steps 400 --warmup 50 --no-cpu-baseline --no-ess --no-pooled > gpurun_out/r2base/long.log 2>&1
rc=$?; echo "long rc=$rc"; [ $rc -eq 0 ] || exit $rc
grep -o '"ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*\|"frac": [0-9.]*' gpurun_out/r2base/long.log | tr '\n' ' '; echo
rocm-smi --showclocks > gpurun_out/r2base/clocks.txt 2>&1 || true
exit 0
