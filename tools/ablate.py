"""Time the step kernel (single-step launches and one fused launch) for the
library given in AMH_LIB_PATH; used to compare ablation builds."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "adaptive-mcmc_amd"))
import torch
import posteriors as P
from kernels_amd import ARWMH, PRNGKey
dev = torch.device("cuda", 0)
C, d = 65536, 64
k = ARWMH(potential_fn=P.correlated_gaussian(d), num_chains=C, device=dev)
st = k.init(PRNGKey(0), 0, (torch.rand(C, d, device=dev) * 4 - 2).contiguous(), (), {})
for _ in range(5):
    k.sample_(st, 1)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(50):
    k.sample_(st, 1)
torch.cuda.synchronize()
single = C * 50 / (time.perf_counter() - t)
t = time.perf_counter()
k.sample_(st, 50)
torch.cuda.synchronize()
fused = C * 50 / (time.perf_counter() - t)
print(f"{os.path.basename(os.environ.get('AMH_LIB_PATH', 'libamh.so'))}: single {single:.4g} fused {fused:.4g}")
