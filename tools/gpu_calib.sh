#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration (tools/calib_fetch.hip), one PMC pass each.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/calib
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 60 rocprofv3 --pmc $C -d gpurun_out/calib/$C -o pmc --output-format csv -- ./tools/calib_fetch > gpurun_out/calib/$C.log 2>&1
  rc=$?; echo "$C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 - <<'PY'
import csv, glob
for C in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(f"gpurun_out/calib/{C}/**/pmc_counter_collection.csv", recursive=True)[0]
    for r in csv.DictReader(open(f)):
        kib = float(r["Counter_Value"])
        print(f'{C:10s} {r["Kernel_Name"][:40]:40s} {kib:14.1f} KiB  ratio {kib / (1 << 20):.3f}')
PY
