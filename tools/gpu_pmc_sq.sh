#!/bin/bash
# SQ instruction / cycle counters of the headline step kernel, one pass per
# counter group (each pass its own run), plus the list of available counters
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r2}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
timeout -s KILL 90 rocprofv3 -L > $OUT/avail.txt 2>&1 || echo "list-avail rc=$?"
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $OUT/p$i -o pmc --output-format csv -- \
    python3 bench.py --steps 20 --warmup 2 --no-extra ${BENCH_ARGS} > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_summary.py $OUT/p1 $OUT/p2 ${PMC_ARGS} 2>&1 | tail -40
exit 0
