#!/bin/bash
# Round 5: every per-config line after the noise-spec change, and a kernel
# trace of the multi-rank (1-rank nccl) pooled step with RCCL on the compute stream.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r5d}
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/rccl -o run --output-format csv -- python3 tools/rccl_one_rank.py 65536 64 100 > $O/rccl.log 2>&1 || exit 13
grep -E "ms/step|bit-equal" $O/rccl.log
timeout -k 10 900 python3 -u bench.py --configs > $O/configs.jsonl 2> $O/configs.err || { tail -5 $O/configs.err; exit 15; }
python3 - <<PY
import json
for l in open("$O/configs.jsonl"):
    j=json.loads(l); r=j.get("roofline",{})
    print(j["config"][:60], "%.4g"%j["value"], "kms", j.get("kernel_ms", j.get("ms_per_step")), "frac", r.get("frac"))
PY
exit 0
