cd "$GRAFT_REPO_ROOT"
for v in default nop sw1 bcrl all; do
  if [ $v = default ]; then unset AMH_LIB_PATH; else export AMH_LIB_PATH=$PWD/adaptive-mcmc_amd/lib/var_$v/libamh.so; fi
  echo "== $v"; timeout -k 10 120 python3 tools/dbg_s64.py 1000 2>&1 | grep "step 2" || exit 1
done
