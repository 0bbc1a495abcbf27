#!/bin/bash
# pooled large-d: default build vs every lib/var_* (regime B configs, 2 reps)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/bpvar
for rep in 1 2; do
  for v in default adaptive-mcmc_amd/lib/var_*/; do
    n=$(basename $v)
    if [ $n = default ]; then unset AMH_LIB_PATH; else export AMH_LIB_PATH=$PWD/${v}libamh.so; fi
    timeout -k 10 200 python3 tools/bench_configs.py --only gauss256_pooled --steps 50 > gpurun_out/bpvar/${n}_$rep.log 2>&1 || exit 1
    echo "$n $rep $(grep config gpurun_out/bpvar/${n}_$rep.log | python3 -c 'import sys,json; [print(round(json.loads(l)["ms_per_step"]*1e3,1), end=" ") for l in sys.stdin]')"
  done
done
