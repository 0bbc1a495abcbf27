"""Headline benchmark (BASELINE.json): chain-steps/s of the whole node + ESS/s
on the 64-d correlated Gaussian.

A "step" is one transition of every chain.

N = 1 (BASELINE configs[1]): ARWMH.sample, per-chain adaptation (the
  reference's semantics, arwmh.py:140-207), 65,536 chains: one launch of the
  step kernel per step, reading and writing the whole chain state in HBM (the
  sample() API contract).  Roofline: HBM, B_A(64) = 17,712 B per chain-step.
N > 1 (BASELINE configs[4]): pooled-covariance ARWMH, 65,536 chains per GPU
  (weak scaling), all-reduce(sum) of the pooled sums over RCCL every step and
  a shared refactorisation on every rank (kernels_amd/pooled.py).  Sub-fields:
  the same with pooling every 16 steps, with the all-reduce overlapped
  (lag-one pooling), the strong-scaling forms (524,288 chains in total), and
  regime A (no collective).

  python bench.py [--gpus N] [--steps K] [--warmup W]

With --gpus N > 1 and no launcher environment (WORLD_SIZE unset) the script
starts its N ranks itself, as child processes, before anything touches a
GPU; under torch.distributed.run it is one of the launched ranks.  Every rank
asserts WORLD_SIZE == --gpus.  When fewer GPUs are visible than ranks (the
1-GPU test box), the ranks share the devices and exchange over gloo; the line
then says so in config.parallelism.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(ROOT, "adaptive-mcmc_amd"), ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 vector = FP32 matrix (dense)
CONFIG5_TOTAL = 524288  # BASELINE configs[4]: 8 x 65,536 chains


def bytes_per_chain_step(d: int) -> int:
    """SURVEY.md §8(d) B_A(d): state round trip, packed factor."""
    return 2 * 4 * (d * (d + 1) // 2 + 2 * d + 6)


def pooled_flops_per_chain_step(d: int) -> int:
    """SURVEY.md §8(d) regime B: proposal L xi (d(d+1)/2 FMA), the quadratic
    form of the potential (d^2 FMA), the outer-product sum (d(d+1)/2 FMA)."""
    return 2 * (d * (d + 1) // 2 + d * d + d * (d + 1) // 2)


def ess_of(x):
    """Multi-chain ESS of x [chains, draws, ...] (numpyro's estimator, the n_eff
    of print_summary: adaptive-mcmc_amd/infer_amd/diagnostics.py; a device
    tensor is reduced on the device)."""
    from infer_amd.diagnostics import effective_sample_size
    return np.atleast_1d(effective_sample_size(x))


def cpu_model() -> str:
    """`lscpu` model name of this host (BASELINE.md §2 asks for it)."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def lib_sha256() -> str | None:
    """sha256 of the libamh.so this process loads (the build a profile came from)."""
    import hashlib
    from kernels_amd import _lib
    try:
        with open(_lib.LIB_PATH, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()
    except OSError:
        return None


def measured_traffic(C: int, d: int):
    """HBM bytes per launch of the step kernel from a committed PMC summary for
    this workload (profiles/<tag>_step_kernel.json, written by
    tools/prof_summary.py from FETCH_SIZE/WRITE_SIZE passes of this bench).
    The summary of the library being measured (its `libamh_sha256`) is taken
    when one exists; otherwise the newest by its own `created_utc` stamp (files
    without one rank oldest, by tag).  Returns (bytes, path, same_build)."""
    import glob
    me = lib_sha256()
    cands = []
    for f in glob.glob(os.path.join(ROOT, "profiles", "*_step_kernel.json")):
        try:
            j = json.load(open(f))
        except (OSError, ValueError):
            continue
        if j.get("chains") == C and j.get("dim") == d:
            same = me is not None and j.get("libamh_sha256") == me
            cands.append(((same, j.get("created_utc", ""), j.get("tag", "")), j["traffic_bytes_per_launch"],
                          os.path.relpath(f, ROOT), same))
    if not cands:
        return None
    best = max(cands, key=lambda c: c[0])
    return best[1], best[2], best[3]


def step_kernel_name(d: int) -> str:
    """The kernel the headline leg launches (amh_kernels.hip run_step dispatch)."""
    if d == 64:
        return "arwmh_step64_kernel<16> (d = 64 specialisation, 16 waves/CU)"
    return f"arwmh_step_kernel<{d}, GaussianM>"


# ----------------------------------------------------------------- ranks --
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(n: int) -> int:
    """Start n ranks of this script (no GPU call in this process) and return
    the first non-zero exit code; if one rank fails the others are stopped."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    while procs:
        for p in list(procs):
            code = p.poll()
            if code is None:
                continue
            procs.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in procs:
                    q.terminate()
        time.sleep(0.05)
    return rc


class Ctx:
    def __init__(self, args):
        import torch
        import torch.distributed as dist
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        if self.world != args.gpus:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={self.world}")
        self.rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        ndev = torch.cuda.device_count()  # does not initialise the GPU
        if ndev < 1:
            raise SystemExit("bench.py: no GPU visible")
        self.ndev = ndev
        self.shared = ndev < self.world
        self.dev_index = local % ndev
        self.backend = None
        if self.world > 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            self.backend = "gloo" if self.shared else "nccl"
            torch.cuda.set_device(self.dev_index)
            if self.backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", self.dev_index))
            else:
                dist.init_process_group("gloo")
        torch.cuda.set_device(self.dev_index)
        self.dev = torch.device("cuda", self.dev_index)

    def barrier(self):
        import torch.distributed as dist
        if self.world > 1:
            dist.barrier()

    def max_over_ranks(self, x: float) -> float:
        import torch
        import torch.distributed as dist
        if self.world == 1:
            return float(x)
        t = torch.tensor([float(x)], dtype=torch.float64)
        if self.backend == "nccl":
            t = t.to(self.dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def parallelism(self, what: str) -> str:
        if self.world == 1:
            return what
        if self.shared:
            return f"{what}; {self.world} ranks sharing {self.ndev} GPU(s), gloo exchange (test box)"
        return f"{what}; {self.world} ranks, one per GPU, RCCL"


def timed_region(ctx, fn):
    """barrier + synchronize on both sides of `fn()`, max wall over ranks."""
    import torch
    torch.cuda.synchronize()
    ctx.barrier()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    ctx.barrier()
    return ctx.max_over_ranks(time.perf_counter() - t0)


# ------------------------------------------------------------------- legs --
CLOCK_WARM_S = 0.3


def clock_warm(step, ctx, seconds: float = CLOCK_WARM_S):
    """Untimed launches for a fixed wall time before the timed region.  After
    an idle gap the GPU needs ~30 ms (~100 launches) of back-to-back step
    launches to reach its steady clocks (tools/ramp.py: 0.30-0.34 ms per
    launch at first, 0.258 ms after), so a 5-step warmup times
    the ramp, not the kernel.  These are real transitions: the chains just
    advance further before the timed steps.  Reported as `clock_warm`."""
    import torch
    t0 = time.perf_counter()
    n = 0
    while True:  # every rank takes the same decision (pooled legs run collectives per step)
        for _ in range(25):
            step()
        n += 25
        torch.cuda.synchronize()
        if ctx.max_over_ranks(time.perf_counter() - t0) >= seconds:
            break
    ctx.barrier()
    return {"seconds": round(time.perf_counter() - t0, 3), "launches": n}


def leg_regime_a(ctx, g, C, off, steps, warmup):
    """ARWMH.sample per step (per-chain adaptation); HIP events on the launch
    stream bracket the step launches only."""
    import torch
    from kernels_amd import ARWMH, PRNGKey
    d = g.dim
    k = ARWMH(potential_fn=g, num_chains=C, device=ctx.dev, chain_offset=off)
    gen = torch.Generator(device=ctx.dev)
    gen.manual_seed(1234 + ctx.rank)
    z0 = (torch.rand(C, d, device=ctx.dev, generator=gen) * 4.0 - 2.0).contiguous()
    st = k.init(PRNGKey(0), 0, z0, (), {})
    for _ in range(warmup):
        k.sample_(st, 1)
    warm = clock_warm(lambda: k.sample_(st, 1), ctx)
    stream = torch.cuda.current_stream(ctx.dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def run():
        ev0.record(stream)
        for _ in range(steps):
            k.sample_(st, 1)  # one full-state round trip per step (sample() semantics)
        ev1.record(stream)

    wall = timed_region(ctx, run)
    kern_ms = ev0.elapsed_time(ev1) / steps
    return dict(wall=wall, kern_ms=kern_ms, kernel=k, state=st, clock_warm=warm)


def leg_pooled(ctx, g, C, off, steps, warmup, K=1, overlap=False, burn_in=0):
    """Regime B (pooled covariance): per-chain transitions with the shared
    state, all-reduce(sum) of the sums over the ranks, shared update.  The
    adaptation burns in for `burn_in` untimed steps before the warmup."""
    import torch
    from kernels_amd import PooledARWMH, PRNGKey
    steps, warmup, burn_in = (-(-x // K) * K for x in (steps, warmup, burn_in))
    k = PooledARWMH(potential_fn=g, num_chains=C, device=ctx.dev, chain_offset=off, sync_every=K,
                    overlap=overlap)
    gen = torch.Generator(device=ctx.dev)
    gen.manual_seed(99 + ctx.rank)
    z0 = (torch.rand(C, g.dim, device=ctx.dev, generator=gen) * 4.0 - 2.0).contiguous()
    st = k.init(PRNGKey(0), 0, z0, (), {})
    k.sample_(st, burn_in + warmup)
    warm = clock_warm(lambda: k.sample_(st, K), ctx)
    wall = timed_region(ctx, lambda: k.sample_(st, steps))
    return dict(wall=wall, steps=steps, kernel=k, state=st, burn_in=burn_in, warmup=warmup, clock_warm=warm)


def pooled_stats_ms(k, st, C, reps=20):
    """HIP-event time of the dominant pooled kernel (per-chain transitions +
    chunk sums, amh_pooled_stats_k) alone, on the launch stream."""
    import ctypes
    import torch
    from kernels_amd import _lib
    L = _lib.lib()
    dev = st.z.device.index
    c = k._c(st)
    zt, pt = torch.empty_like(st.z), torch.empty_like(st.potential_energy)
    sums = torch.empty_like(k._bufs[0])
    stream = torch.cuda.current_stream(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(reps + 2):
        if r == 2:
            ev0.record(stream)
        _lib.check(L.amh_pooled_stats_k(k._handle.h, C, ctypes.byref(c), k.sync_every, _lib.ptr(zt), _lib.ptr(pt),
                                        _lib.ptr(sums), _lib.stream_ptr(dev)), k._handle.h)
    ev1.record(stream)
    torch.cuda.synchronize()
    return ev0.elapsed_time(ev1) / reps


def pooled_line(ctx, r, total, d, C):
    k = r["kernel"]
    K = k.sync_every
    st = r["state"]
    coll = "none (1 rank)"
    if ctx.world > 1:
        coll = f"all_reduce(sum) per {K} step(s)" + (", lag-one overlap" if k.overlap else "")
    return {"value": total * r["steps"] / r["wall"], "unit": "chain-steps/s",
            "ms_per_step": r["wall"] / r["steps"] * 1e3, "steps": r["steps"], "chains_per_gpu": C,
            "chains_total": total, "sync_every": K, "overlap": bool(k.overlap), "burn_in": r["burn_in"],
            "mean_accept_prob": float(st.mean_accept_prob[0]), "allreduce_doubles": d + d * (d + 1) // 2 + 2,
            "collective": coll, "clock_warm": r["clock_warm"]}


def ess_leg(k, st, burn_in=20000, T=1000, headline_s_per_step=None):
    """ESS/s of the headline's own chains (all of them): after the timed region
    they adapt for `burn_in` more steps (fused launches), then T recorded
    transitions in one fused launch that collects z and U on the device; ESS
    (numpyro's multi-chain estimator, reduced on the device) over 4
    coordinates + U, the minimum reported; ESS/s = that / the recorded
    launch's wall time."""
    import torch
    d = st.z.shape[1]
    C = st.z.shape[0]
    i0 = int(st.i[0])
    for _ in range(burn_in // 1000):
        k.sample_(st, 1000)
    torch.cuda.synchronize()
    acc_burn = float(st.mean_accept_prob.mean())
    e0 = time.perf_counter()
    st2, cz, cp = k.run(st, T, collect_z=True, collect_pe=True)
    torch.cuda.synchronize()
    el = time.perf_counter() - e0
    coords = [0, 1, d // 2, d - 1]
    x = cz[:, :, coords].permute(1, 0, 2)  # [C, T, 4]
    vals = [float(v) for v in ess_of(x)]
    del x, cz
    vals.append(float(ess_of(cp.t())[0]))
    return {"ess_min": min(vals), "ess_per_s": min(vals) / el, "chains": C, "draws": T, "seconds": el,
            "ess_per_s_timing": ("ess_min / the wall time of the one FUSED run() launch that recorded the T "
                                 "draws (state in registers between steps)"),
            "ess_per_s_at_headline_rate": (min(vals) / (T * headline_s_per_step)
                                           if headline_s_per_step else None),
            "chains_source": "the headline run's own chains, continued after its timed region",
            "burn_in": burn_in, "steps_before_burn_in": i0, "mean_accept_prob_after_burn_in": acc_burn,
            "mean_accept_prob_window": float(st2.mean_accept_prob.mean()), "coords": coords + ["U"],
            "ess_per_coord": vals}


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
            "cpu_model": cpu_model(),
            "sample": f"C oracle (oracle/amh_oracle.c), {C} chains x {steps} steps, d={d}, {el:.1f} s"}


# ------------------------------------------------------- per-config lines --
# `bench.py --configs [names]`: one JSON line per BASELINE.json single-GPU
# configuration that is not the headline (BASELINE.md §2 asks, per config, for
# GPU and CPU chain-steps/s, the speed-up, ESS/s and the roofline).  Synthetic
# data of the reference shapes.
CONFIG_NAMES = ("diamonds", "diamonds_ss", "gauss256", "gauss256_pooled", "gauss256_pooled_k16", "pooled64",
                "pooled64_k16", "asss64", "asss256", "asss_es", "pnx")
DIAMONDS_FLOPS = 2 * 5000 * 24 + 20000  # contraction + residual terms per chain-step


def cpu_bounded(make_step, C_full: int, budget_s: float = 6.0, label: str = ""):
    """CPU baseline of one config: the C oracle (test infrastructure, OpenMP
    over chains) on a bounded sample -- a chain subset sized so that a step
    takes about a third of the budget, as many whole steps as fit."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import orc
    n = min(C_full, 512)
    step = make_step(n)
    step()
    t0 = time.perf_counter()
    step()
    el = max(time.perf_counter() - t0, 1e-6)
    n = int(min(C_full, max(n, n * (budget_s / 3.0) / el)))
    step = make_step(n)
    steps, t0 = 0, time.perf_counter()
    while True:
        step()
        steps += 1
        el = time.perf_counter() - t0
        if el >= budget_s or el / steps * (steps + 1) > 2.0 * budget_s:
            break
    return {"value": n * steps / el, "unit": "chain-steps/s", "cores": orc.num_threads(), "kind": "port",
            "cpu_model": cpu_model(),
            "sample": f"C oracle{label}: {n} of the config's {C_full} chains x {steps} steps, {el:.1f} s"}


def _orc_model(kind, obj, data=None):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import orc
    import posteriors as P
    if kind == "gaussian":
        arr, _ = obj.pack("cpu")
        return orc.Model(orc.GAUSSIAN, obj.dim, arr.numpy())
    arr, ip = obj.pack_fn(data)
    if obj is P.eight_schools:
        return orc.Model(orc.EIGHT_SCHOOLS, ip[0] + 2, arr)
    mid = orc.DIAMONDS if obj is P.diamonds else orc.DIAMONDS_SS
    return orc.Model(mid, ip[1] + 1, arr, n_data=ip[0], k_data=ip[1])


def cpu_regime_a(om, C_full, asss=False):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import orc
    from kernels_amd import PRNGKey

    def make(n):
        z0 = np.random.default_rng(0).uniform(-2, 2, size=(n, om.d)).astype(np.float32)
        st = orc.init(om, PRNGKey(0), n, init_z=z0)
        return (lambda: orc.asss_step(om, st, 1)) if asss else (lambda: orc.step(om, st, 1))
    return cpu_bounded(make, C_full, label=" (ASSS)" if asss else "")


def cpu_pooled(om, C_full, K=1):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import orc
    from kernels_amd import PRNGKey

    def make(n):
        z = np.random.default_rng(0).uniform(-2, 2, size=(n, om.d)).astype(np.float32)
        box = {"z": z, "pe": orc.potential(om, z), "sh": orc.pooled_init_shared(om.d)}
        keys = orc.chain_keys(PRNGKey(0), 0, n)

        def step():
            sh = box["sh"]
            box["z"], box["pe"], sums = orc.pooled_stats(om, int(sh["i"][0]), box["z"], box["pe"], keys, sh["mu"],
                                                         sh["L"], float(sh["lam"][0]), k_steps=K)
            orc.pooled_update(om, sums, sh, k_steps=K)
        return step
    r = cpu_bounded(make, C_full, label=" (pooled stats + update)")
    if K > 1:
        r["value"] *= K  # one call = K transitions of every chain
    return r


def ess_window(kernel, st, T, coords, every=1):
    """ESS over `coords` + U of T recorded draws (one fused run() launch with
    on-device collection), reduced on the device; ESS/s over that launch."""
    import torch
    torch.cuda.synchronize()
    e0 = time.perf_counter()
    st2, cz, cp = kernel.run(st, T * every, thinning=every, collect_z=True, collect_pe=True)
    torch.cuda.synchronize()
    el = time.perf_counter() - e0
    vals = [float(ess_of(cz[:, :, j].t())[0]) for j in coords]
    vals.append(float(ess_of(cp.t())[0]))
    del cz, cp
    return {"ess_min": min(vals), "ess_per_s": min(vals) / el, "chains": st.z.shape[0], "draws": T,
            "thinning": every, "seconds": el, "coords": list(coords) + ["U"], "ess_per_coord": vals}


def _timed_events(fn, steps, stream):
    import torch
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(steps):
        fn()
    ev1.record(stream)
    torch.cuda.synchronize()
    return time.perf_counter() - t0, ev0.elapsed_time(ev1) / steps


def config_regime_a(name, kernel, C, d, kwargs, steps, dev, om, roof, ess_burn=0, asss=False, cpu=True):
    """sample() per launch (one transition of every chain, state round trip
    through HBM), after a 0.3 s clock warm-up; then the fused rate, the CPU
    baseline and (ess_burn > 0) ESS/s after ess_burn fused adaptation steps."""
    import torch
    from kernels_amd import PRNGKey
    gen = torch.Generator(device=dev)
    gen.manual_seed(7)
    z0 = (torch.rand(C, d, device=dev, generator=gen) * 4.0 - 2.0).contiguous()
    st = kernel.init(PRNGKey(0), 0, z0, (), kwargs)
    warm = clock_warm(lambda: kernel.sample_(st, 1), _SoloCtx())
    wall, kms = _timed_events(lambda: kernel.sample_(st, 1), steps, torch.cuda.current_stream(dev))
    torch.cuda.synchronize()
    f0 = time.perf_counter()
    kernel.sample_(st, 10)
    torch.cuda.synchronize()
    fused = C * 10 / (time.perf_counter() - f0)
    rate = C * steps / wall
    line = {"config": name, "chains": C, "dim": d, "steps": steps, "value": rate, "unit": "chain-steps/s",
            "kernel_ms": kms, "fused_chain_steps_per_s": fused, "clock_warm": warm,
            "mean_accept_prob": float(st.mean_accept_prob.mean()) if hasattr(st, "mean_accept_prob") else None}
    if roof == "hbm":
        b = C * bytes_per_chain_step(d)
        line["roofline"] = {"bound": "hbm", "achieved": b / (kms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": b / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS, "algorithmic_bytes_per_step": b}
    elif roof == "fp32":
        fl = C * DIAMONDS_FLOPS
        line["roofline"] = {"bound": "mfma", "achieved": fl / (kms * 1e-3) / 1e12, "peak": FP32_PEAK_TFLOPS,
                            "unit": "TFLOP/s", "frac": fl / (kms * 1e-3) / 1e12 / FP32_PEAK_TFLOPS,
                            "algorithmic_flops_per_step": fl, "over": "the whole transition (all its launches)"}
    if ess_burn:
        for _ in range(ess_burn // 1000):
            kernel.sample_(st, 1000)
        torch.cuda.synchronize()
        line["ess"] = ess_window(kernel, st, 1000, [0, 1, d // 2, d - 1])
        line["ess"]["burn_in"] = ess_burn
        line["ess"]["mean_accept_prob_after_burn_in"] = line["mean_accept_prob"] = (
            float(st.mean_accept_prob.mean()) if hasattr(st, "mean_accept_prob") else None)
    if cpu and CONFIG_CPU:
        line["cpu_baseline"] = cpu_regime_a(om, C, asss=asss)
        line["speedup_vs_cpu"] = rate / line["cpu_baseline"]["value"]
    return line


class _SoloCtx:
    """Ctx stand-in for the single-process per-config runs."""
    world = 1

    def barrier(self):
        pass

    def max_over_ranks(self, x):
        return float(x)


def config_pooled(key, d, C, kappa, K, steps, dev, burn_in, ess=True, cpu=True):
    import torch
    import posteriors as P
    from kernels_amd import PooledARWMH, PRNGKey
    g = P.correlated_gaussian(d, log10_kappa=kappa)
    k = PooledARWMH(potential_fn=g, num_chains=C, device=dev, sync_every=K)
    gen = torch.Generator(device=dev)
    gen.manual_seed(9)
    z0 = (torch.rand(C, d, device=dev, generator=gen) * 4.0 - 2.0).contiguous()
    st = k.init(PRNGKey(0), 0, z0, (), {})
    burn_in = -(-burn_in // K) * K
    k.sample_(st, burn_in)
    torch.cuda.synchronize()
    macc_burn = float(st.mean_accept_prob[0])
    warm = clock_warm(lambda: k.sample_(st, K), _SoloCtx())
    nb = -(-steps // K)
    wall, kms = _timed_events(lambda: k.sample_(st, K), nb, torch.cuda.current_stream(dev))
    fl = pooled_flops_per_chain_step(d)
    rate = C * nb * K / wall
    sms = pooled_stats_ms(k, st, C) / K
    line = {"config": f"{key} regime B" + (f", sync_every={K}" if K > 1 else ""), "chains": C, "dim": d,
            "steps": nb * K, "value": rate, "unit": "chain-steps/s", "ms_per_step": kms / K, "burn_in": burn_in,
            "mean_accept_prob_after_burn_in": macc_burn, "mean_accept_prob": float(st.mean_accept_prob[0]),
            "clock_warm": warm,
            "roofline": {"bound": "mfma", "achieved": rate * fl / 1e12, "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": rate * fl / 1e12 / FP32_PEAK_TFLOPS, "over": "the whole step",
                         "flops_per_chain_step": fl, "stats_kernel_ms": sms,
                         "stats_kernel_frac": C * fl / (sms * 1e-3) / 1e12 / FP32_PEAK_TFLOPS}}
    if ess and K == 1:
        line["ess"] = ess_window(k, st, 1000, [0, 1, d // 2, d - 1])
    if cpu and CONFIG_CPU:
        line["cpu_baseline"] = cpu_pooled(_orc_model("gaussian", g), C, K)
        line["speedup_vs_cpu"] = rate / line["cpu_baseline"]["value"]
    return line


CONFIG_CPU = True  # --configs --no-cpu-baseline: GPU lines only (A/B runs)


def configs_main(names, steps):
    import torch
    import posteriors as P
    from kernels_amd import ARWMH, ASSS, PRNGKey
    want = set(names)
    bad = want - set(CONFIG_NAMES)
    if bad:
        raise SystemExit(f"bench.py --configs: unknown {sorted(bad)}; known {CONFIG_NAMES}")
    if not torch.cuda.is_available():
        raise SystemExit("bench.py: no GPU visible")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)

    def emit(line):
        print(json.dumps(line), flush=True)
    if "diamonds" in want:
        data = P.synthetic_diamonds()
        k = ARWMH(model=P.diamonds, num_chains=262144, device=dev)
        emit(config_regime_a("diamonds, literal per-row likelihood (BASELINE configs[2])", k, 262144,
                             P.diamonds.dim(data), data, steps, dev, _orc_model("m", P.diamonds, data), "fp32"))
    if "diamonds_ss" in want:
        data = P.synthetic_diamonds()
        k = ARWMH(model=P.diamonds_suffstat, num_chains=262144, device=dev)
        emit(config_regime_a("diamonds, sufficient-statistics likelihood (BASELINE configs[2])", k, 262144,
                             P.diamonds_suffstat.dim(data), data, steps, dev,
                             _orc_model("m", P.diamonds_suffstat, data), "hbm", ess_burn=20000))
    if "gauss256" in want:
        g = P.correlated_gaussian(256, log10_kappa=4.0)
        k = ARWMH(potential_fn=g, num_chains=32768, device=dev)
        emit(config_regime_a("gauss256 regime A, kappa=1e4 (BASELINE configs[3])", k, 32768, 256, {}, steps, dev,
                             _orc_model("gaussian", g), "hbm"))
    if "asss64" in want:
        g = P.correlated_gaussian(64)
        k = ASSS(potential_fn=g, num_chains=65536, device=dev)
        emit(config_regime_a("ASSS d=64 correlated Gaussian", k, 65536, 64, {}, steps, dev, _orc_model("gaussian", g),
                             "hbm", asss=True))
    if "asss256" in want:
        # not a BASELINE config: ASSS past d = 64 (the large-d kernel, DESIGN.md
        # §3.6) on configs[3]'s target and chain count
        g = P.correlated_gaussian(256, log10_kappa=4.0)
        k = ASSS(potential_fn=g, num_chains=32768, device=dev)
        emit(config_regime_a("ASSS d=256 correlated Gaussian, kappa=1e4 (large-d kernel)", k, 32768, 256, {}, steps,
                             dev, _orc_model("gaussian", g), "hbm", asss=True))
    if "asss_es" in want:
        data = dict(P.EIGHT_SCHOOLS_DATA)
        k = ASSS(model=P.eight_schools, num_chains=262144, device=dev)
        emit(config_regime_a("ASSS eight schools", k, 262144, 10, data, steps, dev,
                             _orc_model("m", P.eight_schools, data), None, asss=True))
    for key, d, C, kappa, K, burn in (("gauss256_pooled", 256, 32768, 4.0, 1, 4096),
                                      ("gauss256_pooled_k16", 256, 32768, 4.0, 16, 4096),
                                      ("pooled64", 64, 65536, 2.0, 1, 256), ("pooled64_k16", 64, 65536, 2.0, 16, 4096)):
        if key in want:
            emit(config_pooled(key.replace("_k16", ""), d, C, kappa, K, max(steps, 32), dev, burn))
    if "pnx" in want:
        # many-chain frozen kernel (sample_Pnx, the Lipschitz sweeps' sampler):
        # 5e4 start points x 1e3 chains each x 1 step, eight schools
        data = dict(P.EIGHT_SCHOOLS_DATA)
        for Kc in (ARWMH, ASSS):
            k = Kc(model=P.eight_schools, num_chains=64, device=dev)
            st = k.init(PRNGKey(0), 0, None, (), data)
            k.sample_(st, 2000)
            x = st.z[:50].repeat(1000, 1).contiguous()  # 5e4 points
            adapt = st.adapt_state
            shared = (adapt.loc[0], adapt.scale[0]) + ((adapt.log_step_size[0],) if Kc is ARWMH else ())
            k.sample_Pnx(PRNGKey(1), x, shared, n=1, n_samples=1000)  # warm
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            reps = 5
            for r in range(reps):
                k.sample_Pnx(PRNGKey(2 + r), x, shared, n=1, n_samples=1000)
            torch.cuda.synchronize()
            wall = time.perf_counter() - t0
            emit({"config": f"{Kc.__name__}.sample_Pnx eight schools", "chains": 50000 * 1000, "dim": 10, "steps": 1,
                  "value": reps * 5e7 / wall, "unit": "chain-steps/s", "ms_per_call": wall / reps * 1e3})


# ------------------------------------------------------------------- main --
def refuse_overrides(environ=os.environ):
    """The bench measures the release libamh.so as the driver runs it: any
    AMH_* variable (a library path, or the diagnostic build's A/B switches,
    which the release library ignores anyway) is refused, not silently
    measured."""
    bad = sorted(k for k in environ if k.startswith("AMH_"))
    if bad:
        raise SystemExit(f"bench.py: unset {', '.join(bad)} (the bench times the release libamh.so only)")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--chains", type=int, default=65536, help="chains per GPU (weak scaling)")
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ess", action="store_true")
    ap.add_argument("--no-pooled", action="store_true", help="N = 1: skip the pooled sub-fields")
    ap.add_argument("--no-extra", action="store_true", help="headline leg only (profiling runs)")
    ap.add_argument("--no-fused", action="store_true", help="skip the fused 50-step launch (profiling runs)")
    ap.add_argument("--configs", nargs="?", const=",".join(CONFIG_NAMES), default=None,
                    help="per-config lines instead of the headline (comma list; default all): " + ",".join(CONFIG_NAMES))
    args = ap.parse_args()
    refuse_overrides()
    if args.configs is not None:
        if args.gpus != 1:
            raise SystemExit("--configs runs on one GPU")
        global CONFIG_CPU
        CONFIG_CPU = not args.no_cpu_baseline
        return configs_main(args.configs.split(","), args.steps if args.steps != 200 else 20)
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))

    import torch
    import torch.distributed as dist

    ctx = Ctx(args)
    import posteriors as P
    from kernels_amd.distributed import shard_range
    d, C = args.dim, args.chains
    world, rank = ctx.world, ctx.rank
    g = P.correlated_gaussian(d)
    extra = not args.no_extra
    data = "synthetic (64-d correlated Gaussian, kappa=1e2, default_rng(64) rotation)"
    metric = "chain-steps/sec (whole node) + ESS/sec, 64-dim Gaussian"

    if world == 1:
        # ---- headline: configs[1], regime A
        r = leg_regime_a(ctx, g, C, 0, args.steps, args.warmup)
        value = C * args.steps / r["wall"]
        per_launch_bytes = C * bytes_per_chain_step(d)
        achieved = per_launch_bytes / (r["kern_ms"] * 1e-3) / 1e9
        traffic = measured_traffic(C, d)
        roofline = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": achieved / HBM_PEAK_GBS, "traffic": traffic[0] if traffic else None,
                    "traffic_source": traffic[1] if traffic else None,
                    "traffic_same_build": traffic[2] if traffic else None, "kernel_ms": r["kern_ms"],
                    "kernel": step_kernel_name(d),
                    "algorithmic_bytes_per_launch": per_launch_bytes}
        fused = None
        if extra and not args.no_fused:
            k, st = r["kernel"], r["state"]
            torch.cuda.synchronize()
            f0 = time.perf_counter()
            k.sample_(st, 50)
            torch.cuda.synchronize()
            fused = C * 50 / (time.perf_counter() - f0)
        sub = {}
        if extra and not args.no_pooled:
            for name, K, ov in (("pooled", 1, False), ("pooled_sync_every_16", 16, False),
                                ("pooled_overlap", 1, True)):
                pr = leg_pooled(ctx, g, C, 0, max(args.steps, 32), 16, K=K, overlap=ov, burn_in=256 * K)
                sub[name] = pooled_line(ctx, pr, C, d, C)
        ess = (ess_leg(r["kernel"], r["state"], headline_s_per_step=r["wall"] / args.steps)
               if extra and not args.no_ess else None)
        cpu = cpu_baseline(g, d) if extra and not args.no_cpu_baseline else None
        line = {"metric": metric, "value": value, "unit": "chain-steps/s", "n_gpus": 1, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": r["wall"] / args.steps * 1e3, "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": data,
                "config": {"workload": (f"ARWMH.sample, d={d} correlated Gaussian, {C} chains, per-chain "
                                        f"adaptation (BASELINE.json configs[1])"),
                           "chains_per_gpu": C, "dim": d, "parallelism": "1 GPU"},
                "roofline": roofline, "cpu_baseline": cpu, "clock_warm": r["clock_warm"], "ess": ess,
                "fused_chain_steps_per_s": fused, **sub}
        print(json.dumps(line), flush=True)
        return

    # ---- N > 1 headline: configs[4], pooled all-reduce every step, weak
    r = leg_pooled(ctx, g, C, rank * C, args.steps, args.warmup, K=1, burn_in=256)
    total = world * C
    head = pooled_line(ctx, r, total, d, C)
    stats_ms = pooled_stats_ms(r["kernel"], r["state"], C)
    flops = C * pooled_flops_per_chain_step(d)
    achieved = flops / (stats_ms * 1e-3) / 1e12
    roofline = {"bound": "mfma", "achieved": achieved, "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": achieved / FP32_PEAK_TFLOPS, "traffic": None, "kernel_ms": stats_ms,
                "kernel": ("pooled_fused64_kernel (amh_pooled_stats_k: transitions + 128-chain chunk sums on MFMA)"
                           if d == 64 else "pooled stats (amh_pooled_stats_k: transitions + chunk sums)"),
                "algorithmic_flops_per_launch": flops}
    sub = {}
    if extra:
        for name, K, ov, strong in (("pooled_sync_every_16", 16, False, False), ("pooled_overlap", 1, True, False),
                                    ("strong_pooled", 1, False, True), ("strong_pooled_sync_every_16", 16, False, True)):
            if strong:
                off, cnt = shard_range(CONFIG5_TOTAL, rank, world)
                pr = leg_pooled(ctx, g, cnt, off, max(args.steps, 32), 16, K=K, overlap=ov, burn_in=256 * K)
                sub[name] = pooled_line(ctx, pr, CONFIG5_TOTAL, d, cnt)
                sub[name]["scaling"] = "strong"
            else:
                pr = leg_pooled(ctx, g, C, rank * C, max(args.steps, 32), 16, K=K, overlap=ov, burn_in=256 * K)
                sub[name] = pooled_line(ctx, pr, total, d, C)
        ra = leg_regime_a(ctx, g, C, rank * C, args.steps, args.warmup)
        sub["regime_a"] = {"value": total * args.steps / ra["wall"], "unit": "chain-steps/s", "clock_warm": ra["clock_warm"],
                           "ms_per_step": ra["wall"] / args.steps * 1e3, "kernel_ms": ra["kern_ms"],
                           "collective": "none (chains independent, BASELINE configs[1] per GPU)"}
    cpu = None
    if rank == 0 and extra and not args.no_cpu_baseline:
        # the same pooled transition + update on the host (C oracle, bounded
        # sample of one rank's chains), after every rank has finished timing
        cpu = cpu_pooled(_orc_model("gaussian", g), C)
        cpu["sample"] += " (one rank's share of config 5; no all-reduce on the host)"
    if rank == 0:
        line = {"metric": metric, "value": head["value"], "unit": "chain-steps/s", "n_gpus": world,
                "steps": head["steps"], "warmup": args.warmup, "ms_per_step": head["ms_per_step"],
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": data,
                "config": {"workload": (f"pooled-covariance ARWMH, d={d} correlated Gaussian, {C} chains per GPU "
                                        f"({total} in total), all_reduce(sum) of the pooled sums every step "
                                        f"(BASELINE.json configs[4])"),
                           "chains_per_gpu": C, "dim": d, "parallelism": ctx.parallelism(f"chains sharded x{world}")},
                "roofline": roofline, "cpu_baseline": cpu, "clock_warm": head["clock_warm"], "pooled": head, **sub}
        print(json.dumps(line), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
