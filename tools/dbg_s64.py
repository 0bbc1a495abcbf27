"""Debug the d = 64 step kernel against the oracle: run 2 steps, then take step
3 twice from the same input (determinism) and compare every field with the
oracle; print the chains and fields that differ."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "adaptive-mcmc_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import orc  # noqa: E402
from helpers import FIELDS, make_case, state_to_orc  # noqa: E402
from kernels_amd import ARWMH, PRNGKey  # noqa: E402


def diff(tag, g, o):
    bad = False
    for f in FIELDS:
        a, b = np.asarray(getattr(g, f)), np.asarray(getattr(o, f))
        av = a.view(np.uint32) if a.dtype != np.int64 else a
        bv = b.view(np.uint32) if b.dtype != np.int64 else b
        ne = (av != bv).reshape(a.shape[0], -1).any(axis=1)
        if ne.any():
            bad = True
            idx = np.flatnonzero(ne)
            print(f"{tag}: {f} differs in chains {idx[:12]} ({ne.sum()} total)")
    if not bad:
        print(f"{tag}: all fields equal")


def main():
    C = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    kw, mk, om = make_case("gaussian", 64)
    k = ARWMH(num_chains=C, **kw)
    z0 = np.random.default_rng(0).uniform(-2, 2, size=(C, 64)).astype(np.float32)
    st = k.init(PRNGKey(0), 10, torch.as_tensor(z0), (), mk)
    ost = orc.init(om, PRNGKey(0), C, init_z=z0)
    for t in range(2):
        st = k.sample(st, (), {})
        orc.step(om, ost, 1, num_warmup=10)
        torch.cuda.synchronize()
        diff(f"step {t}", state_to_orc(st), ost)
    a = k.sample(st, (), {})
    b = k.sample(st, (), {})
    orc.step(om, ost, 1, num_warmup=10)
    torch.cuda.synchronize()
    diff("step 2 run a vs run b", state_to_orc(a), state_to_orc(b))
    diff("step 2 run a vs oracle", state_to_orc(a), ost)


if __name__ == "__main__":
    main()
