"""Compare one pooled step's sums (GPU vs oracle) component by component."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "adaptive-mcmc_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import orc  # noqa: E402
from helpers import make_case  # noqa: E402
from kernels_amd import PooledARWMH, PRNGKey  # noqa: E402

d, C = 64, int(sys.argv[1]) if len(sys.argv) > 1 else 3000
kw, mk, om = make_case("gaussian", d)
k = PooledARWMH(num_chains=C, **kw)
z0 = np.random.default_rng(0).uniform(-2, 2, size=(C, d)).astype(np.float32)
st = k.init(PRNGKey(0), 0, torch.as_tensor(z0), (), mk)
ost = orc.init(om, PRNGKey(0), C, init_z=z0)
sh = orc.pooled_init_shared(d)
st1 = k.sample(st)
z, pe, sums = orc.pooled_stats(om, 0, ost.z, ost.potential_energy, ost.rng_key, sh["mu"], sh["L"], 0.0)
torch.cuda.synchronize()
g = k._sums.cpu().numpy()
P = d * (d + 1) // 2
for name, sl in (("sd", slice(0, d)), ("sdd", slice(d, d + P)), ("sa", slice(d + P, d + P + 1)),
                 ("N", slice(d + P + 1, d + P + 2))):
    a, b = g[sl], sums[sl]
    bad = np.flatnonzero(a.view(np.uint64) != b.view(np.uint64))
    print(name, "differs at", bad[:8], len(bad), "max rel", np.max(np.abs(a - b) / (np.abs(b) + 1e-30)) if len(bad) else 0)
zz = st1.z.cpu().numpy()
print("z equal:", np.array_equal(zz.view(np.uint32), z.view(np.uint32)),
      "pe equal:", np.array_equal(st1.potential_energy.cpu().numpy().view(np.uint32), pe.view(np.uint32)))
