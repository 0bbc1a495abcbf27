#!/bin/bash
# headline step kernel: default build vs lib/var_prio (built with a -D switch of
# amh_kernels.hip by tools/build_variants.sh; the s_setprio A/B used -DAMH_S64_PRIO
# before the priority became the default)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prio
for rep in 1 2; do
  timeout -k 10 200 python3 bench.py --no-extra --no-fused --steps 200 > gpurun_out/prio/base_$rep.log 2>&1 || exit 1
  AMH_LIB_PATH=$PWD/adaptive-mcmc_amd/lib/var_prio/libamh.so timeout -k 10 200 python3 bench.py --no-extra --no-fused --steps 200 > gpurun_out/prio/prio_$rep.log 2>&1 || exit 1
  python3 -c "
import json
for n in ('base','prio'):
    j=json.loads(open('gpurun_out/prio/%s_$rep.log'%n).read().strip().splitlines()[-1]); print(n, j['value'], j['roofline']['kernel_ms'], j['roofline']['frac'])"
done
