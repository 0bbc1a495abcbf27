"""Time the d = 64 step launch (HIP events, 100 launches after 300 warm ones)
for several chain counts; run once per library variant (AMH_LIB_PATH)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "adaptive-mcmc_amd"))
import posteriors as P  # noqa: E402
from kernels_amd import ARWMH, PRNGKey  # noqa: E402

g = P.correlated_gaussian(64)
out = []
for C in [int(c) for c in (sys.argv[1:] or ["32768", "65536", "131072"])]:
    k = ARWMH(potential_fn=g, num_chains=C)
    z0 = (torch.rand(C, 64, device="cuda") * 4 - 2).contiguous()
    st = k.init(PRNGKey(0), 0, z0, (), {})
    for _ in range(300):
        k.sample_(st, 1)
    s = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(100):
        k.sample_(st, 1)
    b.record(s)
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 100
    out.append(f"C={C}: {ms:.4f} ms, {C * 17712 / ms / 1e9:.2f} TB/s")
    del k, st
print(os.path.basename(os.path.dirname(os.environ.get("AMH_LIB_PATH", "default/x"))), " | ".join(out), flush=True)
