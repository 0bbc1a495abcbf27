#!/bin/bash
# SQ / LDS counters for the step kernel (single-step bench and fused steps).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-pmc}
mkdir -p gpurun_out/$TAG
i=0
for SET in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
           "SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAVES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $SET -d gpurun_out/$TAG/p$i -o pmc --output-format csv -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-ess > gpurun_out/$TAG/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
