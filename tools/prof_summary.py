"""Summarise a `tools/gpu.sh TAG trace pmc` run into profiles/<tag>_*.

Inputs (gpurun_out/prof_<tag>/): rocprofv3 --kernel-trace --stats of
`bench.py --steps S --warmup W` and two --pmc passes (FETCH_SIZE,
WRITE_SIZE) of `bench.py --steps S2 --warmup W2`.  The step-kernel launches
of bench.py come in order: W warmup, the clock-warm launches (a fixed wall
time, so a variable count), S timed single-step launches, then (default
command) one fused 50-step launch and the ESS leg's launches; the S launches
before the first long (fused) launch are summarised.

HBM traffic per launch (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts half the bytes of wide
(16 B/lane) streaming reads -- the factor, 94 % of the bytes read here, is
moved by 16 B/lane buffer_load...lds -- so it is doubled.

  python tools/prof_summary.py r2 [--steps 200 --pmc-steps 20]
"""
import argparse
import datetime
import csv
import json
import os
import shutil
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "arwmh_step64_kernel"  # the d = 64 specialisation (amh_kernels.hip)


def step_rows(path):
    return [r for r in csv.DictReader(open(path)) if KERNEL in r["Kernel_Name"]]


def lib_sha256():
    import hashlib
    p = os.path.join(ROOT, "adaptive-mcmc_amd", "lib", "libamh.so")
    try:
        with open(p, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()
    except OSError:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--pmc-steps", type=int, default=20)
    ap.add_argument("--pmc-warmup", type=int, default=2)
    ap.add_argument("--chains", type=int, default=65536)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--src", default=None, help="run directory (default gpurun_out/prof_<tag>; tools/gpu.sh "
                                                "writes gpurun_out/<tag>)")
    a = ap.parse_args()
    src = a.src or os.path.join(ROOT, "gpurun_out", f"prof_{a.tag}")
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)

    tr = step_rows(os.path.join(src, "trace", "run_kernel_trace.csv"))
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3 for r in tr]  # us
    # the timed launches end where the fused 50-step launch (if any) begins
    med = statistics.median(dur)
    long_ = [i for i, x in enumerate(dur) if x > 10 * med]
    end = long_[0] if long_ else len(dur)
    timed = dur[end - a.steps:end]

    def pmc(name):
        rows = step_rows(os.path.join(src, f"pmc_{name}", "pmc_counter_collection.csv"))
        v = [float(r["Counter_Value"]) for r in rows][-a.pmc_steps:]
        return statistics.mean(v)

    fetch_kib, write_kib = pmc("FETCH_SIZE"), pmc("WRITE_SIZE")
    d, C = a.dim, a.chains
    alg_read = C * 4 * (d * (d + 1) // 2 + 2 * d + 6)
    traffic = 2 * fetch_kib * 1024 + write_kib * 1024
    out = {
        "tag": a.tag,
        "kernel": next(iter(r["Kernel_Name"] for r in tr)),
        "workload": f"bench.py single-step launches, {C} chains, d={d} (timed region, after the clock warm)",
        "launches_timed": len(timed),
        "avg_us": statistics.mean(timed),
        "median_us": statistics.median(timed),
        "min_us": min(timed),
        "max_us": max(timed),
        "algorithmic_bytes_per_launch": 2 * alg_read,
        "achieved_GBps_at_avg": 2 * alg_read / (statistics.mean(timed) * 1e-6) / 1e9,
        "FETCH_SIZE_KiB_per_launch": fetch_kib,
        "WRITE_SIZE_KiB_per_launch": write_kib,
        "hbm_read_bytes_corrected": 2 * fetch_kib * 1024,
        "hbm_write_bytes": write_kib * 1024,
        "traffic_bytes_per_launch": traffic,
        "traffic_over_algorithmic": traffic / (2 * alg_read),
        "chains": C,
        "dim": d,
        # which build this is (bench.py measured_traffic matches it against
        # the library it loads) and when it was summarised
        "libamh_sha256": lib_sha256(),
        "created_utc": datetime.datetime.now(datetime.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ"),
    }
    with open(os.path.join(dst, f"{a.tag}_step_kernel.json"), "w") as f:
        json.dump(out, f, indent=1)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, f"{a.tag}_kernel_stats.csv"))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
