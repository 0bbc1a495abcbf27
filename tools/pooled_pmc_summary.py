"""HBM traffic of the pooled d = 64 step (configs[4] per GPU) from the two
rocprofv3 --pmc passes (tools/gpu.sh pmcpy:NAME:tools/pooled_run.py+...): FETCH_SIZE (KiB; doubled,
the gfx950 correction for 16-B/lane streaming reads -- the factor and noise
rows are read that way, MI355X_MICROARCH.md) and WRITE_SIZE (KiB) per launch
of each pooled kernel, averaged over the last N launches, and the step's
total against the algorithmic B_B(64) = 2 * 4 * (64 + 3) = 536 B per
chain-step.
  python3 tools/pooled_pmc_summary.py gpurun_out/<tag>/<name> [--chains 65536] [--last 20] [--k K]"""
import argparse
import collections
import csv
import glob
import json
import os


def per_kernel(d, counter):
    rows = collections.defaultdict(dict)
    for f in glob.glob(os.path.join(d, f"pmc_{counter}", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = r["Kernel_Name"].split("(")[0].replace("amh::", "")
            disp = int(r["Dispatch_Id"])
            rows[k][disp] = rows[k].get(disp, 0.0) + float(r["Counter_Value"])
    return {k: [v[i] for i in sorted(v)] for k, v in rows.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--chains", type=int, default=65536)
    ap.add_argument("--last", type=int, default=20)
    ap.add_argument("--k", type=int, default=1, help="sync_every of the run: one stats + one update launch per K steps")
    a = ap.parse_args()
    out = {"chains": a.chains, "dim": 64, "sync_every": a.k, "B_B_bytes_per_step": a.chains * 536, "kernels": {}}
    fetch, write = per_kernel(a.dir, "FETCH_SIZE"), per_kernel(a.dir, "WRITE_SIZE")
    total = 0.0
    for k in sorted(set(fetch) | set(write)):
        if "pooled" not in k:
            continue
        f = fetch.get(k, [])[-a.last:]
        w = write.get(k, [])[-a.last:]
        fb = 2 * 1024 * sum(f) / max(len(f), 1)
        wb = 1024 * sum(w) / max(len(w), 1)
        out["kernels"][k] = {"read_bytes_corrected": fb, "write_bytes": wb, "launches": len(f)}
        total += fb + wb
    out["traffic_bytes_per_step"] = total / a.k  # (per launch pair) / K
    out["traffic_over_B_B"] = out["traffic_bytes_per_step"] / out["B_B_bytes_per_step"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
