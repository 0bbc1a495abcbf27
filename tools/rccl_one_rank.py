"""The RCCL branch of the pooled mode on one GPU (round-4 VERDICT item 3): a
1-rank `nccl` process group, PooledARWMH.force_collective = True so the step
runs the multi-rank path (stats launch, all_reduce(sum) of the sums on the
side stream, event wait, update launch) -- against the fused one-rank path
(amh_pooled_step_k) on the same inputs.  Asserts bit equality of every state
leaf and prints the per-step times of both paths.
Usage (GPU box): python3 tools/rccl_one_rank.py [C] [d] [steps] [sync_every]"""
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
    K = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    steps = -(-steps // K) * K
    g = P.correlated_gaussian(d)
    z0 = (torch.rand(C, d, device="cuda", generator=torch.Generator("cuda").manual_seed(0)) * 4 - 2).contiguous()
    res = {}
    # fused: amh_pooled_step_k (one rank, no exchange); rccl: the multi-rank
    # step with RCCL on the compute stream; rccl_torch: the same through
    # torch.distributed on its side stream (the round-4 path); overlap:
    # lag-one pooling (a different recurrence, timed only)
    for name, force, torch_stream, overlap in (("fused", False, False, False), ("rccl", True, False, False),
                                               ("rccl_torch", True, True, False), ("overlap", True, False, True)):
        k = PooledARWMH(potential_fn=g, num_chains=C, sync_every=K, overlap=overlap)
        k.force_collective = force
        k.torch_stream_collective = torch_stream
        st = k.init(PRNGKey(0), 0, z0, (), {})
        for _ in range(3):  # out of place (sample) then in place (sample_)
            st = k.sample(st)
        k.sample_(st, 3 * K)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        k.sample_(st, steps)
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / steps
        res[name] = (st, el, k)
        print(f"{name}: {el * 1e3:.4f} ms/step ({C / el:.4g} chain-steps/s), K={K}, force_collective={force}, "
              f"torch_stream={torch_stream}, overlap={overlap}", flush=True)
    a = res["fused"][0]
    for other in ("rccl", "rccl_torch"):
        b = res[other][0]
        for f in ("i", "z", "potential_energy", "mean_accept_prob", "as_change", "cov"):
            assert torch.equal(getattr(a, f), getattr(b, f)), (other, f)
        for x, y in zip(a.adapt_state, b.adapt_state):
            assert torch.equal(x, y), other
    assert res["rccl"][2]._rccl_comm is not None and res["rccl"][2]._comm is None, "RCCL not on the compute stream"
    assert res["rccl_torch"][2]._comm is not None, "the torch side stream was not used"
    print(f"rccl one-rank: bit-equal to the fused path after {steps + 3 * K + 3 * K} steps (C={C}, d={d}, K={K})")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
