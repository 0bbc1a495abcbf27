"""Memory ceiling of the headline workload on this GPU: a plain device copy of
the same bytes (torch), the d = 64 step kernel with its arithmetic removed
(AMH_S64_MOVE_ONLY=1: load, swap, write-back only; the state is left as it
was, i.e. no transition -- diagnostic only) and the real step kernel.
Prints ms per launch (HIP events, 50 launches after 100 warm ones)."""
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "adaptive-mcmc_amd"))
# the move-only switch exists in the diagnostic build only (make stamps)
os.environ.setdefault("AMH_LIB_PATH", os.path.join(ROOT, "adaptive-mcmc_amd", "lib", "diag", "libamh_stamps.so"))


def timeit(fn, n=50, warm=100):
    for _ in range(warm):
        fn()
    s = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(n):
        fn()
    b.record(s)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "step":
        import posteriors as P
        from kernels_amd import ARWMH, PRNGKey
        g = P.correlated_gaussian(64)
        C = 65536
        k = ARWMH(potential_fn=g, num_chains=C)
        z0 = (torch.rand(C, 64, device="cuda") * 4 - 2).contiguous()
        st = k.init(PRNGKey(0), 0, z0, (), {})
        k.sample_(st, 3)
        ms = timeit(lambda: k.sample_(st, 1))
        print(f"{os.environ.get('AMH_S64_MOVE_ONLY', '0') == '1' and 'move-only' or 'step'}: {ms:.4f} ms "
              f"-> {65536 * 17712 / ms / 1e9:.2f} TB/s algorithmic", flush=True)
        return
    nbytes = 65536 * 17712 // 2
    src = torch.empty(nbytes // 4, dtype=torch.float32, device="cuda").uniform_()
    dst = torch.empty_like(src)
    ms = timeit(lambda: dst.copy_(src))
    print(f"torch copy {nbytes / 1e6:.0f} MB: {ms:.4f} ms -> {2 * nbytes / ms / 1e9:.2f} TB/s (read + write)", flush=True)
    del src, dst
    for mo in ("1", "0"):
        r = subprocess.run([sys.executable, __file__, "step"], env=dict(os.environ, AMH_S64_MOVE_ONLY=mo),
                           capture_output=True, text=True, timeout=300)
        print(r.stdout.strip() or r.stderr[-2000:], flush=True)


if __name__ == "__main__":
    main()
