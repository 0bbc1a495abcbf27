"""Headline benchmark: chain-steps/s of ARWMH.sample on the 64-d correlated
Gaussian (BASELINE.json configs[1]: 65,536 chains per MI355X), plus ESS/s,
roofline of the step kernel and the CPU baseline (C oracle, OpenMP).

A "step" is one ARWMH.sample transition of every chain: one launch of the
step kernel that reads and writes the whole chain state in HBM (the
sample() API contract).  Weak scaling: each rank owns 65,536 chains (global
ids rank*C ...); chains are independent, so there is no collective in the
timed region.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--chains C] [--dim D]
  N > 1: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(ROOT, "adaptive-mcmc_amd"), ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def bytes_per_chain_step(d: int) -> int:
    """SURVEY.md §8(d) B_A(d): state round trip, packed factor."""
    return 2 * 4 * (d * (d + 1) // 2 + 2 * d + 6)


def ess_of(x: np.ndarray) -> float:
    """Multi-chain ESS of x [chains, draws] (numpyro's estimator, the n_eff
    of print_summary: adaptive-mcmc_amd/infer_amd/diagnostics.py)."""
    from infer_amd.diagnostics import effective_sample_size
    return float(effective_sample_size(x))


def measured_traffic(C: int, d: int):
    """HBM bytes per launch of the step kernel from the newest committed PMC
    summary for this workload (profiles/<round>_step_kernel.json, written by
    tools/prof_summary.py from FETCH_SIZE/WRITE_SIZE passes of this bench)."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_step_kernel.json"))):
        try:
            j = json.load(open(f))
        except (OSError, ValueError):
            continue
        if j.get("chains") == C and j.get("dim") == d:
            best = (j["traffic_bytes_per_launch"], os.path.relpath(f, ROOT))
    return best


def bench_pooled(g, C: int, dev, rank: int, world: int, steps: int, warmup: int, sync_every: int = 1):
    """Regime B (pooled covariance, BASELINE.json configs[4] at N = 8): every
    step = per-chain transition + local sums, all-reduce(sum) of the sums over
    RCCL (world > 1), shared refactorisation on every rank.  sync_every = K:
    one all-reduce and refactorisation per K transitions."""
    import torch
    import torch.distributed as dist
    from kernels_amd import PooledARWMH, PRNGKey
    K = sync_every
    steps, warmup = -(-steps // K) * K, -(-warmup // K) * K
    k = PooledARWMH(potential_fn=g, num_chains=C, device=dev, chain_offset=rank * C, sync_every=K)
    gen = torch.Generator(device=dev)
    gen.manual_seed(99 + rank)
    z0 = (torch.rand(C, g.dim, device=dev, generator=gen) * 4.0 - 2.0).contiguous()
    st = k.init(PRNGKey(0), 0, z0, (), {})
    k.sample_(st, warmup)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    k.sample_(st, steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([wall], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())
    return {"value": world * C * steps / wall, "unit": "chain-steps/s", "ms_per_step": wall / steps * 1e3,
            "steps": steps, "chains_per_gpu": C, "allreduce_doubles": g.dim + g.dim * (g.dim + 1) // 2 + 2,
            "mean_accept_prob": float(st.mean_accept_prob[0]), "sync_every": K,
            "collective": (f"all_reduce(sum) per {K} step(s)" if world > 1 else "none (1 rank)")}


def cpu_baseline(g, d: int, budget_s: float = 12.0):
    """C oracle (test infrastructure) timed on this host: same step, same
    layout, OpenMP over chains.  Bounded sample: 65,536 chains, as many whole
    steps as fit the time budget (at least one)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import orc
    from kernels_amd import PRNGKey
    data, _ = g.pack("cpu")
    om = orc.Model(orc.GAUSSIAN, d, data.numpy())
    C = 65536
    z0 = np.random.default_rng(0).uniform(-2, 2, size=(C, d)).astype(np.float32)
    st = orc.init(om, PRNGKey(0), C, init_z=z0)
    orc.step(om, st, 1)  # warm
    steps, t0 = 0, time.perf_counter()
    while True:
        orc.step(om, st, 1)
        steps += 1
        el = time.perf_counter() - t0
        if el >= budget_s or el / steps * (steps + 1) > 2.5 * budget_s:
            break
    return {"value": C * steps / el, "unit": "chain-steps/s", "cores": orc.num_threads(), "kind": "port",
            "sample": f"C oracle (oracle/amh_oracle.c), {C} chains x {steps} steps, d={d}, {el:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--chains", type=int, default=65536, help="chains per GPU (weak scaling)")
    ap.add_argument("--total-chains", type=int, default=0,
                    help="strong scaling: this many chains split over the ranks (SURVEY.md §8(d) config 5: 524288)")
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ess", action="store_true")
    ap.add_argument("--no-pooled", action="store_true")
    ap.add_argument("--no-fused", action="store_true", help="skip the fused 50-step launch (profiling runs)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    import posteriors as P
    from kernels_amd import ARWMH, PRNGKey

    from kernels_amd.distributed import shard_range
    d, C = args.dim, args.chains
    off = rank * C
    strong = args.total_chains > 0
    if strong:
        off, C = shard_range(args.total_chains, rank, world)
    g = P.correlated_gaussian(d)
    k = ARWMH(potential_fn=g, num_chains=C, device=dev, chain_offset=off)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1234 + rank)
    z0 = (torch.rand(C, d, device=dev, generator=gen) * 4.0 - 2.0).contiguous()
    st = k.init(PRNGKey(0), 0, z0, (), {})

    # untimed warmup (also burns in the adaptation)
    for _ in range(args.warmup):
        k.sample_(st, 1)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()

    stream = torch.cuda.current_stream(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        k.sample_(st, 1)  # one full-state round trip per step (sample() semantics)
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps  # events bracket only step launches on this stream
    t = torch.tensor([wall], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall = float(t.item())

    total = args.total_chains if strong else world * C
    value = total * args.steps / wall
    per_launch_bytes = C * bytes_per_chain_step(d)
    achieved_gbs = per_launch_bytes / (kern_ms * 1e-3) / 1e9

    # fused multi-step launch (numpyro fori_collect semantics, state on chip)
    fused_rate = None
    if not args.no_fused:
        fused_steps = 50
        torch.cuda.synchronize()
        f0 = time.perf_counter()
        k.sample_(st, fused_steps)
        torch.cuda.synchronize()
        fused_rate = C * fused_steps / (time.perf_counter() - f0)

    ess = None
    if not args.no_ess and rank == 0:
        # ESS/s: 1,000 recorded post-warmup steps of 4,096 chains (4 coordinates + U)
        T, Cs = 1000, 4096
        ks = ARWMH(potential_fn=g, num_chains=Cs, device=dev)
        zs = (torch.rand(Cs, d, device=dev, generator=gen) * 4.0 - 2.0).contiguous()
        ss = ks.init(PRNGKey(1), 0, zs, (), {})
        ks.sample_(ss, 2000)  # adaptation burn-in
        torch.cuda.synchronize()
        e0 = time.perf_counter()
        ss, cz, cp = ks.run(ss, T, collect_z=True, collect_pe=True)
        torch.cuda.synchronize()
        el = time.perf_counter() - e0
        zc = cz.cpu().numpy()
        pc = cp.cpu().numpy()
        vals = [ess_of(zc[:, :, j].T.astype(np.float64)) for j in (0, 1, d // 2, d - 1)]
        vals.append(ess_of(pc.T.astype(np.float64)))
        ess = {"ess_min": min(vals), "ess_per_s": min(vals) / el, "chains": Cs, "draws": T,
               "seconds": el, "coords": [0, 1, d // 2, d - 1, "U"]}

    pooled = None
    if not args.no_pooled:
        pooled = bench_pooled(g, C, dev, rank, world, steps=max(args.steps, 20), warmup=5)
        pooled["sync_every_16"] = bench_pooled(g, C, dev, rank, world, steps=max(args.steps, 32), warmup=16,
                                               sync_every=16)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(g, d)

    traffic = measured_traffic(C, d)
    if rank == 0:
        line = {
            "metric": "chain-steps/sec (whole node) + ESS/sec, 64-dim Gaussian",
            "value": value,
            "unit": "chain-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": wall / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (64-d correlated Gaussian, kappa=1e2, default_rng(64) rotation)",
            "config": {"workload": f"ARWMH.sample, d={d} correlated Gaussian, "
                                   + (f"{total} chains in total" if strong else f"{C} chains per GPU")
                                   + ", per-chain adaptation (BASELINE.json configs[1])",
                       "chains_per_gpu": C, "dim": d, "parallelism": f"chains sharded x{world}, no collective"},
            "roofline": {"bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved_gbs / HBM_PEAK_GBS,
                         "traffic": traffic[0] if traffic else None,
                         "traffic_source": traffic[1] if traffic else None,
                         "kernel_ms": kern_ms, "algorithmic_bytes_per_launch": per_launch_bytes},
            "cpu_baseline": cpu,
            "ess": ess,
            "fused_chain_steps_per_s": fused_rate * total / C if fused_rate else None,
            "pooled": pooled,
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
