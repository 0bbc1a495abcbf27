"""Average rocprofv3 --pmc counters per dispatch of one kernel.

  python3 tools/pmc_summary.py DIR [DIR...] [--kernel SUBSTR] [--skip N] [--take M]

Every DIR is searched for *counter_collection.csv.  Rows of dispatches whose
kernel name contains SUBSTR are grouped by dispatch; the first N such
dispatches (warm-up launches) are skipped and the next M averaged.  Derived
per-wave figures are printed when SQ_WAVES is present.
"""
import argparse
import collections
import csv
import glob
import os


def load(d, kernel):
    per = collections.OrderedDict()
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel not in r["Kernel_Name"]:
                continue
            key = int(r["Dispatch_Id"])
            per.setdefault(key, {})
            per[key][r["Counter_Name"]] = per[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [per[k] for k in sorted(per)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", default="arwmh_step_kernel<64")
    ap.add_argument("--skip", type=int, default=2)
    ap.add_argument("--take", type=int, default=20)
    a = ap.parse_args()
    tot = {}
    for d in a.dirs:
        rows = load(d, a.kernel)[a.skip:a.skip + a.take]
        if not rows:
            print(f"{d}: no dispatches of {a.kernel}")
            continue
        for name in rows[0]:
            tot[name] = sum(r.get(name, 0.0) for r in rows) / len(rows)
        print(f"{d}: {len(rows)} dispatches")
    w = tot.get("SQ_WAVES")
    for k in sorted(tot):
        extra = f"   per wave {tot[k] / w:12.1f}" if w and k != "SQ_WAVES" else ""
        print(f"{k:28s} {tot[k]:18.1f}{extra}")


if __name__ == "__main__":
    main()
