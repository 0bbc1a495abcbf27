"""Phase breakdown of the pooled d = 64 kernels (diagnostic build, make -C
adaptive-mcmc_amd/csrc stamps): s_memtime ticks of thread 0 of block 0 per
phase of pooled_fused64_kernel (work / barrier after it) and of
pooled_update64_kernel.  Usage (GPU box): python3 tools/f64_stamps.py [C]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("AMH_LIB_PATH", os.path.join(ROOT, "adaptive-mcmc_amd", "lib", "diag", "libamh_stamps.so"))
sys.path.insert(0, os.path.join(ROOT, "adaptive-mcmc_amd"))

import torch  # noqa: E402

import posteriors as P  # noqa: E402
from kernels_amd import PooledARWMH, PRNGKey, _lib  # noqa: E402

C = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
k = PooledARWMH(potential_fn=P.correlated_gaussian(64), num_chains=C)
st = k.init(PRNGKey(0), 0, (torch.rand(C, 64, device="cuda") * 4 - 2).contiguous(), (), {})
k.sample_(st, 200)
torch.cuda.synchronize()
L = _lib.lib()
f = np.zeros(16, np.uint64)
u = np.zeros(8, np.uint64)
L.amh_diag_f64_stamps.argtypes = [ctypes.c_void_p]
L.amh_diag_upd_stamps.argtypes = [ctypes.c_void_p]
assert L.amh_diag_f64_stamps(f.ctypes.data) == 0 and L.amh_diag_upd_stamps(u.ctypes.data) == 0
names = ["(1) noise", "bar", "(2) proposal", "bar", "(3) potential", "bar", "(4) accept", "bar", "(5) delta", "bar",
         "(6) sums", "bar", "", "", "prologue", ""]
print("pooled_fused64_kernel, block 0 thread 0 (ticks):")
for n, v in zip(names, f):
    if n:
        print(f"  {n:15s} {int(v):9d}")
print(f"  total {int(f.sum())}")
print("pooled_update64_kernel (ticks):")
for n, v in zip(["loads + Sigma'", "barrier", "factor (wave 0)", "barrier", "write-out + as_change"], u[:5]):
    print(f"  {n:22s} {int(v):9d}")
print(f"  total {int(u[:5].sum())}")
