"""Timeline of the pooled d = 64 update launch (diagnostic build,
make -C adaptive-mcmc_amd/csrc stamps): per step, on the 100 MHz constant
clock relative to the first block's entry -- the last reduce slice done, the
ticket won, Sigma' formed, the factorisation done, the update's end, and the
noise workers' first start / last end.  Usage (GPU box):
  python3 tools/u64_timeline.py [--chains 65536] [--steps 8]
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
ap.add_argument("--chains", type=int, default=65536)
ap.add_argument("--steps", type=int, default=8)
a = ap.parse_args()
dev = torch.device("cuda", 0)
k = PooledARWMH(potential_fn=P.correlated_gaussian(64), num_chains=a.chains, device=dev)
st = k.init(PRNGKey(0), 0, (torch.rand(a.chains, 64, device=dev) * 4 - 2).contiguous(), (), {})
L = _lib.lib()
L.amh_diag_u64_timeline.argtypes = [ctypes.c_void_p]
buf = np.zeros(16, np.uint64)
k.sample_(st, 20)
torch.cuda.synchronize()
assert L.amh_diag_u64_timeline(buf.ctypes.data) == 0
rows = []
for s in range(a.steps):
    k.sample_(st, 1)
    torch.cuda.synchronize()
    assert L.amh_diag_u64_timeline(buf.ctypes.data) == 0
    t0 = int(~buf[0] & np.uint64(0xFFFFFFFFFFFFFFFF))
    rel = lambda v: (int(v) - t0) / 100.0  # noqa: E731  (10 ns ticks -> us)
    nz0 = int(~buf[7] & np.uint64(0xFFFFFFFFFFFFFFFF)) if buf[7] else None
    rows.append([rel(buf[1]), rel(buf[2]), rel(buf[3]), rel(buf[4]), rel(buf[5]), rel(buf[6]),
                 (nz0 - t0) / 100.0 if nz0 is not None else float("nan"), rel(buf[8]), rel(buf[9])])
    print("step %d: group sums %.2f  stored %.2f  reduce done %.2f  ticket %.2f  sigma' %.2f  factor %.2f  "
          "update end %.2f  noise %.2f..%.2f us" % (s, rows[-1][7], rows[-1][8], *rows[-1][:5], rows[-1][6], rows[-1][5]))
m = np.median(np.array(rows), axis=0)
print("median: group sums %.2f  stored %.2f  reduce done %.2f  ticket %.2f  sigma' %.2f  factor %.2f  "
      "update end %.2f  noise %.2f..%.2f us" % (m[7], m[8], m[0], m[1], m[2], m[3], m[4], m[6], m[5]))
