#!/bin/bash
# pooled d = 64: parity (pooled GPU tests), phase stamps, K = 1 / K = 16 timing
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r5m}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_pooled.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/t.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/f64_stamps.py 65536 > $O/f64.txt 2>&1 || exit 10
grep -v "^W2026\|amdgpu.ids" $O/f64.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/k1 -o run --output-format csv -- python3 tools/pooled_run.py 65536 64 200 1 > $O/k1.log 2>&1 || exit 11
grep pooled $O/k1.log
python3 - $O/k1 <<'PY'
import csv,glob,sys
f=glob.glob(sys.argv[1]+'/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if float(r['Percentage'])>1: print('  %-70s %6s %9.1f'%(r['Name'][:70],r['Calls'],float(r['AverageNs'])/1e3))
PY
timeout -k 10 200 python3 tools/pooled_run.py 65536 64 320 16 > $O/k16.log 2>&1 || exit 12
grep pooled $O/k16.log
exit 0
