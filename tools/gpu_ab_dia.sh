#!/bin/bash
# A/B of library variants on the diamonds literal transition (tools/dia_run.py,
# 262,144 chains): release vs adaptive-mcmc_amd/lib/ab/libamh_<v>.so, twice
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-abd}; shift
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 120 python3 tools/dia_run.py 262144 40 > $O/rel_$rep.log 2>&1 || exit 10
  echo "release: $(grep diamonds $O/rel_$rep.log)"
  for v in "$@"; do
    AMH_LIB_PATH=adaptive-mcmc_amd/lib/ab/libamh_$v.so timeout -k 10 120 python3 tools/dia_run.py 262144 40 > $O/${v}_$rep.log 2>&1 || exit 11
    echo "$v: $(grep diamonds $O/${v}_$rep.log)"
  done
done
exit 0
