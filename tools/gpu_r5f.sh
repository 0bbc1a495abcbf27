#!/bin/bash
# Round 5 profiling: diamonds literal (kernel trace), ASSS d = 64 (kernel
# trace), d = 256 regime B (kernel trace), pooled d = 64 stats phases.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r5f}
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/dia -o run --output-format csv -- python3 tools/dia_run.py 262144 20 > $O/dia.log 2>&1 || exit 11
tail -2 $O/dia.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/asss -o run --output-format csv -- python3 tools/asss_run.py > $O/asss.log 2>&1 || exit 12
tail -2 $O/asss.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/p256 -o run --output-format csv -- python3 tools/pooled_run.py 32768 256 100 1 > $O/p256.log 2>&1 || exit 13
grep pooled $O/p256.log
timeout -k 10 120 python3 tools/f64_stamps.py > $O/stamps.txt 2>&1 || exit 14
grep -v amdgpu.ids $O/stamps.txt
for t in dia asss p256; do python3 - $O/$t <<'PY'
import csv,glob,sys
f=glob.glob(sys.argv[1]+'/**/*kernel_stats.csv',recursive=True)[0]
print(sys.argv[1])
for r in csv.DictReader(open(f)):
    if float(r['Percentage'])>0.5: print('  %-70s %6s %9.1f'%(r['Name'][:70],r['Calls'],float(r['AverageNs'])/1e3))
PY
done
exit 0
