#!/bin/bash
cd "$GRAFT_REPO_ROOT"
for W in 3 4 5; do
  AMH_LIB_PATH=$PWD/adaptive-mcmc_amd/lib/libamh_w$W.so timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-ess > gpurun_out/occ_w$W.log 2>&1
  rc=$?; echo "w$W rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json;d=json.loads(open('gpurun_out/occ_w$W.log').read().strip().splitlines()[-1]);print('w$W', d['value'], d['roofline']['kernel_ms'], d['fused_chain_steps_per_s'])"
done
