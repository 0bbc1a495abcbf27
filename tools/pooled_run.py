"""Pooled-mode steps for profiling: python3 tools/pooled_run.py [C] [d] [steps] [sync_every]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "adaptive-mcmc_amd"))
import torch  # noqa: E402

import posteriors as P  # noqa: E402
from kernels_amd import PooledARWMH, PRNGKey  # noqa: E402

C = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
d = int(sys.argv[2]) if len(sys.argv) > 2 else 64
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 50
K = int(sys.argv[4]) if len(sys.argv) > 4 else 1
steps = -(-steps // K) * K
k = PooledARWMH(potential_fn=P.correlated_gaussian(d), num_chains=C, sync_every=K)
st = k.init(PRNGKey(0), 0, (torch.rand(C, d, device="cuda") * 4 - 2).contiguous(), (), {})
k.sample_(st, 5 * K)
torch.cuda.synchronize()
t = time.perf_counter()
k.sample_(st, steps)
torch.cuda.synchronize()
el = time.perf_counter() - t
print(f"pooled C={C} d={d} K={K}: {el / steps * 1e3:.4f} ms/step, {C * steps / el:.4g} chain-steps/s, "
      f"macc {float(st.mean_accept_prob[0]):.3f}")
