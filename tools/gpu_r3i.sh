# pooled: one-launch reduction, update launch 1 block/CU: parity (all pooled + configs), timing, stamps
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r3i
timeout -k 10 900 python -u -m pytest tests/test_gpu_pooled.py tests/test_gpu_drivers.py -v --timeout 300 --timeout-method thread > gpurun_out/r3i/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/r3i/t.log | tail -12
[ $rc -eq 0 -o $rc -eq 1 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3i/pool -o run --output-format csv -- python3 tools/pooled_run.py 65536 64 200 > gpurun_out/r3i/pool.log 2>&1
echo "pool rc=$?"; grep pooled gpurun_out/r3i/pool.log
timeout -k 10 120 python3 tools/pooled_run.py 65536 64 400 > gpurun_out/r3i/pool_plain.log 2>&1; grep pooled gpurun_out/r3i/pool_plain.log
timeout -k 10 120 python3 tools/pooled_run.py 32768 256 100 > gpurun_out/r3i/pool256.log 2>&1; grep pooled gpurun_out/r3i/pool256.log
timeout -k 10 120 python3 tools/f64_stamps.py > gpurun_out/r3i/stamps.txt 2>&1; grep -v amdgpu.ids gpurun_out/r3i/stamps.txt
exit $rc
