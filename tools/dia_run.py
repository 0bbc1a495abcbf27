"""Diamonds literal transition (BASELINE configs[2]), sample() per step at
262,144 chains: ms per transition over 20 steps after a 0.3 s warm-up.
For library A/B (AMH_LIB_PATH; bench.py refuses overrides).
Usage (GPU box): python3 tools/dia_run.py [C] [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "adaptive-mcmc_amd"))
import torch  # noqa: E402

import posteriors as P  # noqa: E402
from kernels_amd import ARWMH, PRNGKey  # noqa: E402

C = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
dev = torch.device("cuda", 0)
data = P.synthetic_diamonds()
k = ARWMH(model=P.diamonds, num_chains=C, device=dev)
d = P.diamonds.dim(data)
g = torch.Generator(device=dev)
g.manual_seed(7)
st = k.init(PRNGKey(0), 0, (torch.rand(C, d, device=dev, generator=g) * 4 - 2).contiguous(), (), data)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.3:
    k.sample_(st, 1)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(steps):
    k.sample_(st, 1)
torch.cuda.synchronize()
el = time.perf_counter() - t
print(f"diamonds C={C}: {el / steps * 1e3:.4f} ms per transition, {C * steps / el:.4g} chain-steps/s")
