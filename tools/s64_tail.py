"""How the headline launch (arwmh_step64_kernel, d = 64, 65,536 chains)
drains: per-wave start / end stamps on the constant 100 MHz clock from the
diagnostic build (make -C adaptive-mcmc_amd/csrc stamps).  Prints the launch
span, the spread of block end times, and the fraction of CU-time spent after a
CU's last wave finished while other CUs were still running (the tail a
grid-wide work queue could recover).  Usage (GPU box): python3 tools/s64_tail.py"""
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

dev = torch.device("cuda", 0)
C, d = 65536, 64
k = ARWMH(potential_fn=P.correlated_gaussian(d), num_chains=C, device=dev)
st = k.init(PRNGKey(0), 0, (torch.rand(C, d, device=dev) * 4 - 2).contiguous(), (), {})
for _ in range(300):
    st = k.sample(st, (), {})
torch.cuda.synchronize()
W, S = 1 << 16, 8
L = _lib.lib()
L.amh_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int64]
for rep in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    st = k.sample(st, (), {})
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    buf = np.zeros(W * S, np.uint64)
    assert L.amh_diag_stamps(buf.ctypes.data, buf.nbytes) == 0
    s = buf.reshape(W, S)
    s = s[s[:, 7] == 1]
    t0 = s[:, 0].min()
    start = (s[:, 0] - t0) * 10e-3  # us
    end = (s[:, 1] - t0) * 10e-3
    blk = s[:, 3].astype(np.int64)
    nb = blk.max() + 1
    bend = np.zeros(nb)
    bstart = np.full(nb, 1e9)
    np.maximum.at(bend, blk, end)
    np.minimum.at(bstart, blk, start)
    span = end.max()
    idle = (span - bend).sum() / (nb * span)
    q = np.quantile(bend, [0.0, 0.1, 0.5, 0.9, 1.0])
    per_xcd = [bend[np.arange(nb) % 8 == x].mean() for x in range(8)]
    print(f"launch {ms * 1e3:.1f} us (events); stamped span {span:.1f} us; waves {len(s)}, blocks {nb}; "
          f"items/wave {s[:, 2].mean():.2f} (min {s[:, 2].min()} max {s[:, 2].max()})")
    print(f"  block start: max {bstart.max():.1f} us; block end quantiles 0/10/50/90/100%: "
          + " ".join(f"{v:.1f}" for v in q))
    print(f"  CU-time idle after a block's end while others run: {100 * idle:.1f} %; "
          f"mean block end per blockIdx % 8: " + " ".join(f"{v:.1f}" for v in per_xcd))
