#!/bin/bash
# Headline kernel iteration in one gpurun call: d = 64 parity (steady state
# at config sizes + the single/fused/in-place cases), then the default
# headline leg three times (bench.py --no-extra) and a kernel trace.
# Usage (on the box): bash tools/gpu_headline.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-head}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_steady.py tests/test_gpu_parity.py -v -m gpu --timeout 300 --timeout-method thread -k "64 or step64 or headline or sharded" > $O/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED" $O/t.log | tail -8
[ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --no-extra > $O/bench_$r.log 2>&1 || exit 9
  grep -v amdgpu.ids $O/bench_$r.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('bench', j['value'], j['roofline']['kernel_ms'], round(j['roofline']['frac'],4))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --no-extra > $O/trace.log 2>&1
echo "trace rc=$?"; grep step64 $O/trace/run_kernel_stats.csv | cut -d, -f1-5
