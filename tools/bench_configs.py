"""Per-config throughput of the BASELINE.json single-GPU configurations that
are not the headline (bench.py measures configs[1]).

  python tools/bench_configs.py [--only diamonds,gauss256,...] [--steps K]

One JSON line per config: chain-steps/s of ARWMH.sample (one launch = one
transition of every chain, state round trip through HBM), plus the fused
multi-step rate.  Synthetic data of the reference shapes.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (os.path.join(ROOT, "adaptive-mcmc_amd"), ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)


def timed(fn, steps, stream):
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


def run_regime_a(name, kernel, C, d, kwargs, steps, warmup, dev):
    import torch
    from kernels_amd import PRNGKey
    gen = torch.Generator(device=dev)
    gen.manual_seed(7)
    z0 = (torch.rand(C, d, device=dev, generator=gen) * 4.0 - 2.0).contiguous()
    st = kernel.init(PRNGKey(0), 0, z0, (), kwargs)
    for _ in range(warmup):
        kernel.sample_(st, 1)
    wall, kms = timed(lambda: kernel.sample_(st, 1), steps, torch.cuda.current_stream(dev))
    torch.cuda.synchronize()
    f0 = time.perf_counter()
    kernel.sample_(st, 10)
    torch.cuda.synchronize()
    fused = C * 10 / (time.perf_counter() - f0)
    return {"config": name, "chains": C, "dim": d, "steps": steps, "value": C * steps / wall,
            "unit": "chain-steps/s", "kernel_ms": kms, "fused_chain_steps_per_s": fused,
            "mean_accept_prob": float(st.mean_accept_prob.mean()) if hasattr(st, "mean_accept_prob") else None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="diamonds,diamonds_ss,gauss256,gauss256_pooled,pooled64,asss64,asss_es,pnx")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    args = ap.parse_args()
    import torch
    import posteriors as P
    from kernels_amd import ARWMH, ASSS, PooledARWMH, PRNGKey
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    want = set(args.only.split(","))
    if "diamonds" in want:
        data = P.synthetic_diamonds()
        C = 262144
        k = ARWMH(model=P.diamonds, num_chains=C, device=dev)
        print(json.dumps(run_regime_a("diamonds (BASELINE configs[2])", k, C, P.diamonds.dim(data), data,
                                      args.steps, args.warmup, dev)), flush=True)
    if "diamonds_ss" in want:
        data = P.synthetic_diamonds()
        C = 262144
        k = ARWMH(model=P.diamonds_suffstat, num_chains=C, device=dev)
        print(json.dumps(run_regime_a("diamonds, sufficient-statistics likelihood (BASELINE configs[2])", k, C,
                                      P.diamonds_suffstat.dim(data), data, args.steps, args.warmup, dev)), flush=True)
    if "gauss256" in want:
        g = P.correlated_gaussian(256, log10_kappa=4.0)
        C = 32768
        k = ARWMH(potential_fn=g, num_chains=C, device=dev)
        print(json.dumps(run_regime_a("gauss256 regime A (BASELINE configs[3])", k, C, 256, {},
                                      args.steps, args.warmup, dev)), flush=True)
    if "asss64" in want:
        g = P.correlated_gaussian(64)
        C = 65536
        k = ASSS(potential_fn=g, num_chains=C, device=dev)
        print(json.dumps(run_regime_a("ASSS d=64 correlated Gaussian", k, C, 64, {}, args.steps, args.warmup, dev)),
              flush=True)
    if "asss_es" in want:
        C = 262144
        k = ASSS(model=P.eight_schools, num_chains=C, device=dev)
        print(json.dumps(run_regime_a("ASSS eight schools", k, C, 10, dict(P.EIGHT_SCHOOLS_DATA), args.steps,
                                      args.warmup, dev)), flush=True)
    if "pnx" in want:
        # many-chain frozen kernel (sample_Pnx, the Lipschitz sweeps' sampler):
        # 5e4 start points x 1e3 chains each x 1 step, eight schools
        data = dict(P.EIGHT_SCHOOLS_DATA)
        for K in (ARWMH, ASSS):
            k = K(model=P.eight_schools, num_chains=64, device=dev)
            st = k.init(PRNGKey(0), 0, None, (), data)
            k.sample_(st, 2000)
            x = st.z[:50].repeat(1000, 1).contiguous()  # 5e4 points
            adapt = st.adapt_state
            shared = (adapt.loc[0], adapt.scale[0]) + ((adapt.log_step_size[0],) if K is ARWMH else ())
            k.sample_Pnx(PRNGKey(1), x, shared, n=1, n_samples=1000)  # warm
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            reps = 5
            for r in range(reps):
                k.sample_Pnx(PRNGKey(2 + r), x, shared, n=1, n_samples=1000)
            torch.cuda.synchronize()
            wall = time.perf_counter() - t0
            print(json.dumps({"config": f"{K.__name__}.sample_Pnx eight schools", "chains": 50000 * 1000, "dim": 10,
                              "steps": 1, "value": reps * 5e7 / wall, "unit": "chain-steps/s",
                              "ms_per_call": wall / reps * 1e3}), flush=True)
    for key, d, C, kappa, K in (("gauss256_pooled", 256, 32768, 4.0, 1), ("pooled64", 64, 65536, 2.0, 1),
                                ("gauss256_pooled_k16", 256, 32768, 4.0, 16), ("pooled64_k16", 64, 65536, 2.0, 16)):
        if key.replace("_k16", "") not in want:
            continue
        g = P.correlated_gaussian(d, log10_kappa=kappa)
        k = PooledARWMH(potential_fn=g, num_chains=C, device=dev, sync_every=K)
        gen = torch.Generator(device=dev)
        gen.manual_seed(9)
        z0 = (torch.rand(C, d, device=dev, generator=gen) * 4.0 - 2.0).contiguous()
        st = k.init(PRNGKey(0), 0, z0, (), {})
        k.sample_(st, -(-args.warmup // K) * K)
        nb = -(-args.steps // K)  # timed blocks of K transitions
        wall, kms = timed(lambda: k.sample_(st, K), nb, torch.cuda.current_stream(dev))
        import bench  # the flop count and the stats-kernel timer of the N > 1 headline
        fl = bench.pooled_flops_per_chain_step(d)
        rate = C * nb * K / wall
        sms = bench.pooled_stats_ms(k, st, C) / K  # transitions + chunk sums alone, per transition
        print(json.dumps({"config": f"{key} regime B" + (f", sync_every={K}" if K > 1 else ""), "chains": C,
                          "dim": d, "steps": nb * K, "value": rate, "unit": "chain-steps/s",
                          "ms_per_step": kms / K, "mean_accept_prob": float(st.mean_accept_prob[0]),
                          "fp32": {"flops_per_chain_step": fl, "step_tflops": rate * fl / 1e12,
                                   "step_frac": rate * fl / 1e12 / bench.FP32_PEAK_TFLOPS, "stats_ms": sms,
                                   "stats_tflops": C * fl / (sms * 1e-3) / 1e12,
                                   "stats_frac": C * fl / (sms * 1e-3) / 1e12 / bench.FP32_PEAK_TFLOPS,
                                   "peak_tflops": bench.FP32_PEAK_TFLOPS}}), flush=True)


if __name__ == "__main__":
    main()
