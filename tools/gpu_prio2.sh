#!/bin/bash
# generic step kernel (non-headline configs): default build vs lib/var_prio
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prio2
for rep in 1 2; do
  timeout -k 10 200 python3 tools/bench_configs.py --only diamonds_ss,asss_es,diamonds --steps 40 > gpurun_out/prio2/base_$rep.log 2>&1 || exit 1
  AMH_LIB_PATH=$PWD/adaptive-mcmc_amd/lib/var_prio/libamh.so timeout -k 10 200 python3 tools/bench_configs.py --only diamonds_ss,asss_es,diamonds --steps 40 > gpurun_out/prio2/prio_$rep.log 2>&1 || exit 1
  for n in base prio; do echo "$n $rep"; grep config gpurun_out/prio2/${n}_$rep.log | cut -c1-170; done
done
