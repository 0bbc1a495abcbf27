"""Why is the headline step slower in a short run?  Times every launch of the
d = 64 step kernel (65,536 chains) with HIP events in three phases:
  A  fresh state, 400 launches right after init (the driver's situation)
  B  the same (adapted) state after 2 s of idle GPU
  C  a fresh init right after a hot phase
Per-launch ms in blocks of 10 are printed; if B is slow and C is fast the
ramp is the clock, if B is fast and C is slow it is the chain state."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "adaptive-mcmc_amd"))

import posteriors as P  # noqa: E402
from kernels_amd import ARWMH, PRNGKey  # noqa: E402


def timed(k, st, n):
    s = torch.cuda.current_stream()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
    evs[0].record(s)
    for j in range(n):
        k.sample_(st, 1)
        evs[j + 1].record(s)
    torch.cuda.synchronize()
    return [evs[j].elapsed_time(evs[j + 1]) for j in range(n)]


def blocks(ms, w=10):
    return " ".join(f"{sum(ms[i:i + w]) / len(ms[i:i + w]):.3f}" for i in range(0, len(ms), w))


def fresh(g, C, seed):
    k = ARWMH(potential_fn=g, num_chains=C)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(seed)
    z0 = (torch.rand(C, 64, device="cuda", generator=gen) * 4.0 - 2.0).contiguous()
    return k, k.init(PRNGKey(seed), 0, z0, (), {})


def main():
    g = P.correlated_gaussian(64)
    C = 65536
    k, st = fresh(g, C, 0)
    torch.cuda.synchronize()
    print("A fresh      :", blocks(timed(k, st, 400)), flush=True)
    time.sleep(2.0)
    print("B idle 2s    :", blocks(timed(k, st, 100)), flush=True)
    k2, st2 = fresh(g, C, 1)
    torch.cuda.synchronize()
    print("C fresh, hot :", blocks(timed(k2, st2, 100)), flush=True)
    # D: hot, adapted state, same as the bench's timed window
    print("D hot adapted:", blocks(timed(k, st, 100)), flush=True)


if __name__ == "__main__":
    main()
