#!/bin/bash
# split-path (diamonds) parity and timing after reading z' from the split buffer
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r5g}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_steady.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/t.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/dia -o run --output-format csv -- python3 tools/dia_run.py 262144 20 > $O/dia.log 2>&1 || exit 11
tail -1 $O/dia.log
python3 - $O/dia <<'PY'
import csv,glob,sys
f=glob.glob(sys.argv[1]+'/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if float(r['Percentage'])>0.5: print('  %-70s %6s %9.1f'%(r['Name'][:70],r['Calls'],float(r['AverageNs'])/1e3))
PY
exit 0
