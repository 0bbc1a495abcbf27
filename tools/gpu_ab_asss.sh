#!/bin/bash
# A/B of library variants on ASSS d = 64 sample() (tools/asss_run.py):
# release vs adaptive-mcmc_amd/lib/ab/libamh_<v>.so, alternated twice
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-abs}; shift
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 120 python3 tools/asss_run.py > $O/rel_$rep.log 2>&1 || exit 10
  echo "release: $(grep asss $O/rel_$rep.log)"
  for v in "$@"; do
    AMH_LIB_PATH=adaptive-mcmc_amd/lib/ab/libamh_$v.so timeout -k 10 120 python3 tools/asss_run.py > $O/${v}_$rep.log 2>&1 || exit 11
    echo "$v: $(grep asss $O/${v}_$rep.log)"
  done
done
exit 0
