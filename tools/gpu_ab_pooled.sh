#!/bin/bash
# A/B of library variants on the pooled d = 64 step (K = 1): release vs
# adaptive-mcmc_amd/lib/ab/libamh_<v>.so, alternated twice
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-ab}; shift
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 120 python3 tools/pooled_run.py 65536 64 400 1 > $O/rel_$rep.log 2>&1 || exit 10
  echo "release: $(grep pooled $O/rel_$rep.log)"
  for v in "$@"; do
    AMH_LIB_PATH=adaptive-mcmc_amd/lib/ab/libamh_$v.so timeout -k 10 120 python3 tools/pooled_run.py 65536 64 400 1 > $O/${v}_$rep.log 2>&1 || exit 11
    echo "$v: $(grep pooled $O/${v}_$rep.log)"
  done
done
exit 0
