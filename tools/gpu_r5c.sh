#!/bin/bash
# Round 5: pooled / parity suites after the fused K-step stats kernel and the
# noise spec change, pooled + RCCL timing, headline bench with a kernel trace.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r5c}
mkdir -p $O
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_pooled.py tests/test_gpu_parity.py tests/test_gpu_steady.py} -x -v -m gpu --timeout 300 --timeout-method thread > $O/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/t.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/k1 -o run --output-format csv -- python3 tools/pooled_run.py 65536 64 200 1 > $O/k1.log 2>&1 || exit 11
grep pooled $O/k1.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/k16 -o run --output-format csv -- python3 tools/pooled_run.py 65536 64 320 16 > $O/k16.log 2>&1 || exit 12
grep pooled $O/k16.log
timeout -k 10 200 python3 tools/rccl_one_rank.py 65536 64 100 > $O/rccl.log 2>&1 || exit 13
grep -E "ms/step|bit-equal" $O/rccl.log
timeout -k 10 200 python3 tools/rccl_one_rank.py 65536 64 320 16 > $O/rccl16.log 2>&1 || exit 14
grep -E "ms/step|bit-equal" $O/rccl16.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/bench -o run --output-format csv -- python3 bench.py --no-ess --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 15
python3 - <<PY
import json,csv,glob
l=json.loads(open("$O/bench.json").read().strip().splitlines()[-1])
print("bench", l["value"], l["ms_per_step"], l["roofline"]["kernel_ms"], l["roofline"]["frac"], {k: l[k]["ms_per_step"] for k in ("pooled","pooled_sync_every_16","pooled_overlap")})
for r in csv.DictReader(open(glob.glob("$O/bench/**/*kernel_stats.csv",recursive=True)[0])):
    if float(r["Percentage"])>1: print(" ", r["Name"][:70], r["Calls"], round(float(r["AverageNs"])/1e3,1))
PY
exit 0
