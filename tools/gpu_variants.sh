#!/bin/bash
# time the step kernel of every lib/var_*/libamh.so variant plus the default build
cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 python3 tools/s64_sweep.py "$@" || exit 1
for d in adaptive-mcmc_amd/lib/var_*/; do
  AMH_LIB_PATH=$PWD/${d}libamh.so timeout -k 10 120 python3 tools/s64_sweep.py "$@" || exit 1
done
