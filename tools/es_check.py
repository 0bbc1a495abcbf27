"""Eight-schools posterior under infer.MCMC at several run lengths (GPU)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "adaptive-mcmc_amd"))
import torch
import posteriors as P
from infer_amd import MCMC
from kernels_amd import ARWMH, PRNGKey
dev = torch.device("cuda", 0)
for C, W, N, th in [(64, 5000, 50000, 50), (64, 50000, 500000, 50), (1024, 50000, 500000, 50)]:
    k = ARWMH(model=P.eight_schools, num_chains=C, device=dev)
    m = MCMC(k, num_warmup=W, num_samples=N, thinning=th)
    t0 = time.time()
    m.run(PRNGKey(0), extra_fields=("potential_energy",), **P.EIGHT_SCHOOLS_DATA)
    torch.cuda.synchronize()
    s = m.get_samples()
    print(C, W, N, f"{time.time()-t0:.2f}s", "mu %.3f sd %.3f tau %.3f sd %.3f tb0 %.3f" % (
        s["mu"].mean(), s["mu"].std(), s["tau"].mean(), s["tau"].std(), s["theta_base"][:, 0].mean()),
        "accept %.3f" % float(m.last_state.mean_accept_prob.mean()), flush=True)
m.print_summary()
