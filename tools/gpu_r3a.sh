cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r3a
timeout -k 10 900 python -u -m pytest tests/test_gpu_steady.py tests/test_gpu_drivers.py tests/test_gpu_pooled.py -v --timeout 400 --timeout-method thread > gpurun_out/r3a/new.log 2>&1
rc=$?; echo "new rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/r3a/new.log | tail -15
[ $rc -eq 0 -o $rc -eq 1 ] || exit $rc
timeout -k 10 1200 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread --ignore=tests/test_gpu_steady.py --ignore=tests/test_gpu_drivers.py --ignore=tests/test_gpu_pooled.py > gpurun_out/r3a/rest.log 2>&1
rc2=$?; echo "rest rc=$rc2"; grep -E "passed|failed|FAILED" gpurun_out/r3a/rest.log | tail -8
[ $rc2 -eq 0 -o $rc2 -eq 1 ] || exit $rc2
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3a/pool -o run --output-format csv -- python3 tools/pooled_run.py 65536 64 200 > gpurun_out/r3a/pool.log 2>&1
echo "pool rc=$?"; cat gpurun_out/r3a/pool.log | grep pooled
for v in norng noprop nopot nosdd; do
  AMH_LIB_PATH=$PWD/adaptive-mcmc_amd/lib/var_$v/libamh.so timeout -k 10 120 python3 tools/pooled_run.py 65536 64 200 > gpurun_out/r3a/var_$v.log 2>&1 || exit 9
  echo "$v: $(grep pooled gpurun_out/r3a/var_$v.log)"
done
timeout -k 10 400 python3 bench.py > gpurun_out/r3a/bench.log 2>&1
echo "bench rc=$?"; tail -c 400 gpurun_out/r3a/bench.log
exit $rc2
