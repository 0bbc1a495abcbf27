"""Phase breakdown of the pooled large-d update kernel (diagnostic build,
make -C adaptive-mcmc_amd/csrc stamps): s_memtime totals of thread 0 for
init / panel columns / panel loads / the barrier behind the look-ahead
trailing update / write-out / the next column block's update / panel
write-back.  Usage (GPU box):
  python3 tools/upd_stamps.py [--dim 256] [--chains 32768]
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("AMH_LIB_PATH", os.path.join(ROOT, "adaptive-mcmc_amd", "lib", "diag", "libamh_stamps.so"))
sys.path.insert(0, os.path.join(ROOT, "adaptive-mcmc_amd"))

import torch  # noqa: E402

import posteriors as P  # noqa: E402
from kernels_amd import PooledARWMH, PRNGKey  # noqa: E402
from kernels_amd import _lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--chains", type=int, default=32768)
ap.add_argument("--dim", type=int, default=256)
a = ap.parse_args()
dev = torch.device("cuda", 0)
k = PooledARWMH(potential_fn=P.correlated_gaussian(a.dim, log10_kappa=4.0), num_chains=a.chains, device=dev)
st = k.init(PRNGKey(0), 0, (torch.rand(a.chains, a.dim, device=dev) * 4 - 2).contiguous(), (), {})
k.sample_(st, 5)
torch.cuda.synchronize()
buf = np.zeros(8, np.uint64)
L = _lib.lib()
L.amh_diag_upd_stamps.argtypes = [ctypes.c_void_p]
assert L.amh_diag_upd_stamps(buf.ctypes.data) == 0
names = ["init", "panel columns", "panel loads", "look-ahead barrier", "write-out", "next column block",
         "(unused)", "panel write-back"]
tot = buf[:8].sum()
for n, v in zip(names, buf[:8]):
    print(f"{n:15s} {int(v):9d} ticks  {100.0 * v / tot:5.1f} %")
print(f"total {int(tot)} ticks (s_memtime = shader clock; ~{tot / 2400.0:.1f} us at 2.4 GHz)")
