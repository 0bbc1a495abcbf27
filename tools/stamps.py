"""Phase breakdown of the step kernel from the diagnostic build
(make -C adaptive-mcmc_amd/csrc stamps): per-wave s_memtime totals of
wait-for-DMA / store previous / LDS->registers / prefetch issue / compute /
tail, averaged over waves, per item.  Usage (GPU box):
  python3 tools/stamps.py [--chains C] [--steps N]
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
from kernels_amd import ARWMH, PRNGKey  # noqa: E402
from kernels_amd import _lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--chains", type=int, default=65536)
ap.add_argument("--dim", type=int, default=64)
ap.add_argument("--steps", type=int, default=1)
ap.add_argument("--model", default="gaussian", help="gaussian | diamonds (split path: the ExtPotM step kernel)")
a = ap.parse_args()
dev = torch.device("cuda", 0)
C, d = a.chains, a.dim
if a.model == "diamonds":
    mk = P.synthetic_diamonds()
    k = ARWMH(model=P.diamonds, num_chains=C, device=dev)
    st = k.init(PRNGKey(0), 0, None, (), mk)
else:
    k = ARWMH(potential_fn=P.correlated_gaussian(d), num_chains=C, device=dev)
    st = k.init(PRNGKey(0), 0, (torch.rand(C, d, device=dev) * 4 - 2).contiguous(), (), {})
for _ in range(20):
    k.sample_(st, a.steps)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
k.sample_(st, a.steps)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1)

W, S = 1 << 16, 8
buf = np.zeros(W * S, np.uint64)
L = _lib.lib()
L.amh_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int64]
assert L.amh_diag_stamps(buf.ctypes.data, buf.nbytes) == 0
s = buf.reshape(W, S).astype(np.float64)
s = s[s[:, 7] > 0]
nb = len(s) // 16
blk = s[: nb * 16, 7].reshape(nb, 16)
it = s[: nb * 16, 6].reshape(nb, 16)
names = ["wait_dma", "store_prev", "lds_to_reg", "prefetch", "compute", "tail"]
items = s[:, 6]
print(f"waves {len(s)}  items/wave {items.mean():.2f}  kernel {ms:.4f} ms  wave cycles {s[:, 7].mean():.0f} "
      f"(max {s[:, 7].max():.0f})  -> clock {s[:, 7].max() / (ms * 1e-3) / 1e9:.2f} GHz (s_memtime)")
tot = s[:, :6].sum(axis=1).mean()
for i, n in enumerate(names):
    per_item = (s[:, i] / np.maximum(items, 1)).mean()
    print(f"  {n:11s} {s[:, i].mean():10.0f} cyc/wave  {100 * s[:, i].mean() / tot:5.1f}%  {per_item:8.0f} cyc/item")
print(f"  block wall (max over its waves): mean {blk.max(1).mean():.0f} min {blk.max(1).min():.0f} "
      f"max {blk.max(1).max():.0f};  in-block wave spread max/mean {np.mean(blk.max(1) / blk.mean(1)):.3f};  "
      f"items per wave min {it.min():.0f} max {it.max():.0f}")
