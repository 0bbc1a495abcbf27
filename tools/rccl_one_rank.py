"""The RCCL branch of the pooled mode on one GPU (round-4 VERDICT item 3): a
1-rank `nccl` process group, PooledARWMH.force_collective = True so the step
runs the multi-rank path (stats launch, all_reduce(sum) of the sums on the
side stream, event wait, update launch) -- against the fused one-rank path
(amh_pooled_step_k) on the same inputs.  Asserts bit equality of every state
leaf and prints the per-step times of both paths.
Usage (GPU box): python3 tools/rccl_one_rank.py [C] [d] [steps]"""
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "adaptive-mcmc_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import posteriors as P  # noqa: E402
from kernels_amd import PooledARWMH, PRNGKey  # noqa: E402


def main():
    C = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    d = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 50
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    g = P.correlated_gaussian(d)
    z0 = (torch.rand(C, d, device="cuda", generator=torch.Generator("cuda").manual_seed(0)) * 4 - 2).contiguous()
    res = {}
    for name, force in (("fused", False), ("rccl", True)):
        k = PooledARWMH(potential_fn=g, num_chains=C)
        k.force_collective = force
        st = k.init(PRNGKey(0), 0, z0, (), {})
        for _ in range(3):  # out of place (sample) then in place (sample_)
            st = k.sample(st)
        k.sample_(st, 3)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        k.sample_(st, steps)
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / steps
        res[name] = (st, el, k)
        print(f"{name}: {el * 1e3:.4f} ms/step ({C / el:.4g} chain-steps/s), force_collective={force}", flush=True)
    a, b = res["fused"][0], res["rccl"][0]
    for f in ("i", "z", "potential_energy", "mean_accept_prob", "as_change", "cov"):
        assert torch.equal(getattr(a, f), getattr(b, f)), f
    for x, y in zip(a.adapt_state, b.adapt_state):
        assert torch.equal(x, y)
    assert res["rccl"][2]._comm is not None, "the RCCL side stream was not used"
    print(f"rccl one-rank: bit-equal to the fused path after {steps + 6} steps (C={C}, d={d})")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
