#!/bin/bash
# headline step kernel: default build vs every lib/var_* (bench.py headline leg, HIP-event kernel time)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s64var
for rep in 1 2; do
  for v in default adaptive-mcmc_amd/lib/var_*/; do
    n=$(basename $v)
    if [ $n = default ]; then unset AMH_LIB_PATH; else export AMH_LIB_PATH=$PWD/${v}libamh.so; fi
    timeout -k 10 200 python3 bench.py --no-extra --no-fused --steps 200 > gpurun_out/s64var/${n}_$rep.log 2>&1 || exit 1
    python3 -c "
import json
j=json.loads(open('gpurun_out/s64var/${n}_$rep.log').read().strip().splitlines()[-1]); print('$n', $rep, round(j['value']/1e6,1), round(j['roofline']['kernel_ms']*1e3,1))"
  done
done
