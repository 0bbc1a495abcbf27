# pooled d = 64 rework: parity first, then timing + kernel stats
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r3e
timeout -k 10 600 python -u -m pytest tests/test_gpu_pooled.py tests/test_gpu_drivers.py -v --timeout 300 --timeout-method thread -k "64 or config5 or overlap or noise or keep" > gpurun_out/r3e/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/r3e/t.log | tail -12
[ $rc -eq 0 -o $rc -eq 1 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3e/pool -o run --output-format csv -- python3 tools/pooled_run.py 65536 64 200 > gpurun_out/r3e/pool.log 2>&1
echo "pool rc=$?"; grep pooled gpurun_out/r3e/pool.log
timeout -k 10 120 python3 tools/pooled_run.py 65536 64 400 > gpurun_out/r3e/pool_plain.log 2>&1; grep pooled gpurun_out/r3e/pool_plain.log
exit $rc
timeout -k 10 120 python3 tools/f64_stamps.py > gpurun_out/r3e/stamps.txt 2>&1; cat gpurun_out/r3e/stamps.txt | grep -v amdgpu.ids
