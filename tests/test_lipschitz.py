"""utils.lipschitz (lipschitz.py): the spectral normalisation and the
1-Lipschitz network on the CPU; the contraction estimate on the GPU with the
device sample_Pnx as the sampler (the notebook's 1-D example)."""
import numpy as np
import pytest
import torch

from utils_amd import lipschitz as Lz


def test_spectral_norm_caps_sigma():
    g = torch.Generator().manual_seed(0)
    W = torch.randn(20, 7, generator=g) * 3.0
    Wn = Lz.spectral_norm(W)
    assert float(torch.linalg.matrix_norm(Wn, 2)) == pytest.approx(1.0, rel=1e-3)
    small = torch.randn(5, 4, generator=g) * 0.01  # sigma < 1: unchanged
    assert torch.allclose(Lz.spectral_norm(small), small)


def test_network_is_1_lipschitz():
    net = Lz.LipschitzNN(3)
    g = torch.Generator().manual_seed(1)
    x = torch.randn(2000, 3, generator=g)
    y = x + 0.1 * torch.randn(2000, 3, generator=g)
    with torch.no_grad():
        r = (net(x) - net(y)).abs() / torch.linalg.norm(x - y, dim=1)
    assert float(r.max()) <= 1.0 + 1e-4
    assert net(x).shape == (2000,)


@pytest.mark.gpu
def test_contraction_and_kernel_distance_on_device(gpu):
    """1-D N(0, 1) target with the frozen kernel L = 1, lambda = 0 (the
    notebook's asumptions_check.ipynb cell 38 setting): tau(P^0), the
    identity, is close to 1 and no estimate exceeds 1 beyond Monte Carlo noise
    (f is 1-Lipschitz; Pf from 2e4 draws per point, pairs 0.2 apart); the
    kernel distance of P to itself (independent draws) is small."""
    import posteriors as P
    from kernels_amd import ARWMH, PRNGKey
    g = P.gaussian(np.zeros(1), cov=np.eye(1))
    k = ARWMH(potential_fn=g, num_chains=1)
    adapt = k.get_init_adapt_state(PRNGKey(0), torch.zeros(1, 1))
    X = torch.linspace(-5, 5, 100).reshape(-1, 1)
    for n in (0, 1, 5):
        fn = lambda key, x, n_samples, n=n: k.sample_Pnx(key, x, adapt, n, n_samples)
        # P^0 = I: the exact tau is 1 (sup over 1-Lipschitz f of a pair's
        # |f(x) - f(y)| / |x - y|); the estimate is the trained f's own largest
        # pair ratio, so it is trained until it gets there (10 Adam steps stop
        # at 0.78 with the reference's fixed power-iteration start)
        tau, model, params = Lz.compute_wasserstein_contraction(fn, PRNGKey(0), X, n_train_batches=5,
                                                                n_eval_batches=20, max_steps=200 if n == 0 else 10)
        assert 0.0 < tau <= 1.15
        if n == 0:
            print(f"tau(P^0) = {tau:.4f} (exact 1)")
            assert 0.8 < tau <= 1.0 + 1e-4  # no noise at n = 0 (Pf = f); float32 ratio rounding
    fn = lambda key, x, n_samples: k.sample_Pnx(key, x, adapt, 1, n_samples)
    rho, _, _ = Lz.compute_kernel_distance_1d(fn, fn, PRNGKey(1), torch.linspace(-3, 3, 31), max_steps=10,
                                              n_eval_batches=10)
    assert 0.0 <= rho < 0.2


@pytest.mark.gpu
def test_kernel_distance_multid_on_device(gpu):
    """compute_kernel_distance (lipschitz.py:221-344) with the device
    sample_Pnx on a 2-D N(0, I) target: rho(P, P) (same keys per batch, so
    the two estimates cancel exactly) is 0; rho(P, Q) for Q = the same kernel
    at a 10x smaller proposal scale is clearly positive and at most ~1 (a
    1-Lipschitz f moves by at most the mean displacement gap)."""
    import posteriors as P
    from kernels_amd import ARWMH, PRNGKey
    g = P.gaussian(np.zeros(2), cov=np.eye(2))
    k = ARWMH(potential_fn=g, num_chains=1)
    k.get_init_adapt_state(PRNGKey(0), torch.zeros(1, 2))
    s_p = (torch.zeros(2), torch.eye(2), torch.zeros(()))
    s_q = (torch.zeros(2), 0.1 * torch.eye(2), torch.zeros(()))
    g1 = torch.linspace(-2, 2, 8)
    X = torch.stack(torch.meshgrid(g1, g1, indexing="ij"), -1).reshape(-1, 2)
    fp = lambda key, x, n_samples: k.sample_Pnx(key, x, s_p, 1, n_samples)
    fq = lambda key, x, n_samples: k.sample_Pnx(key, x, s_q, 1, n_samples)
    rho_pp, _, _ = Lz.compute_kernel_distance(fp, fp, PRNGKey(2), X, n_train_batches=2, n_eval_batches=10,
                                              max_steps=5)
    assert rho_pp == 0.0
    rho_pq, model, params = Lz.compute_kernel_distance(fp, fq, PRNGKey(2), X, n_train_batches=2, n_eval_batches=20,
                                                       max_steps=50)
    assert 0.05 < rho_pq < 1.2
    assert set(params) == set(model.state_dict())


@pytest.mark.gpu
def test_kernel_distance_1d_notebook_cell101(gpu):
    """asumptions_check.ipynb cell 101: rho(P, Q) between the frozen 1-D
    N(0, 1) kernels with scale 1 and 0.1 (+ eps 1e-6), n = 1, x =
    linspace(-5, 5, 100) and the notebook's rho_conf (1000 training steps,
    1000 x 1000-sample evaluation batches, ratio_rad 5).  The notebook prints
    0.544187 from one key.

    Pinned to exact answers (oracle/metropolis_1d.py, the kernel's CDF in
    closed form; profiles/r5_cell101_*.txt, tools/cell101_exact.py):
      * the value the estimator approaches with no noise is a property of
        the TRAINED f: for each key the build's estimate must equal the exact
        quadrature value of its own network's ratios, max_i |(P - Q) f(x_i+1)
        - (P - Q) f(x_i)| / h, within the evaluation's Monte Carlo spread
        (the max over 99 noisy ratios sits at most a few sd above it);
      * no pair exceeds its Kantorovich-Rubinstein supremum over ALL
        1-Lipschitz f (int |F_mu|; the largest is 0.9591 at x = 1.263), so
        the notebook's 0.544 is reachable -- it is not bounded away;
      * the keys land where the reference's own procedure lands: the float64
        CPU restatement of lipschitz.py:396-491 (Monte Carlo training as the
        notebook trains) gives exact rho 0.28..0.54 over 20 keys (mean 0.447,
        sd 0.069; the notebook-style estimate 0.29..0.54), and 0.46..0.55
        when trained on the exact objective.  The notebook's 0.544 is +1.4 sd
        from that mean: a favourable key, not Monte Carlo evaluation bias
        (<= 0.007 for every trained f) and not a short-fall of the build's
        sampler or evaluation, which the first check pins."""
    from oracle import metropolis_1d as M
    import posteriors as P
    from kernels_amd import ARWMH, PRNGKey
    g = P.gaussian(np.zeros(1), cov=np.eye(1))
    k = ARWMH(potential_fn=g, num_chains=1)
    s_p = (torch.zeros(1), torch.ones(1, 1), torch.zeros(()))
    s_q = (torch.zeros(1), 0.1 * torch.ones(1, 1), torch.zeros(()))
    fp = lambda key, x, n_samples: k.sample_Pnx(key, x, s_p, 1, n_samples)
    fq = lambda key, x, n_samples: k.sample_Pnx(key, x, s_q, 1, n_samples)
    x = torch.linspace(-5, 5, 100)
    x64 = x.double().numpy()
    SP, SQ = 1.0 + 1e-6, 0.1 + 1e-6  # arwmh.py:166: L e^lam + eps
    kr = M.kr_bound(x64, SP, SQ)
    grid = torch.linspace(-8, 8, 16001, device=gpu).reshape(-1, 1)
    rows = []
    for seed in range(4):
        rho, model, _ = Lz.compute_kernel_distance_1d(fp, fq, PRNGKey(seed), x, sample_batch_size=1000,
                                                      n_train_batches=1, n_eval_batches=1000, max_steps=1000,
                                                      lr=0.1, ratio_rad=5)

        def f(t, model=model):
            with torch.no_grad():
                tt = torch.as_tensor(np.asarray(t), dtype=torch.float32, device=gpu).reshape(-1, 1)
                return model(tt).double().cpu().numpy()

        with torch.no_grad():
            fg = model(grid)
            lip = float((fg[1:] - fg[:-1]).abs().max() / (grid[1, 0] - grid[0, 0]))
        assert lip <= 1.01, (seed, lip)  # the spectral normalisation holds
        r, vP, vQ = M.exact_ratios(f, x64, SP, SQ)
        sd = M.mc_sd(vP, vQ, x64, 1000 * 1000)
        i = int(r.argmax())
        assert np.all(r <= max(lip, 1.0) * kr + 1e-6), seed
        rows.append((rho, float(r[i]), float(sd[i])))
        print(f"cell 101 key {seed}: estimate {rho:.4f}, exact rho of the trained f {r[i]:.4f} at x = {x64[i]:.3f} "
              f"(ratio sd {sd[i]:.4f}), Lipschitz {lip:.4f}")
        assert -4 * sd[i] - 1e-3 <= rho - r[i] <= 0.02, (seed, rho, r[i], sd[i])
        assert 0.25 <= rho <= 0.56, (seed, rho)  # the restated procedure's range
    m = float(np.mean([a for a, _, _ in rows]))
    print(f"cell 101: mean over keys 0..3 {m:.4f}; KR supremum {kr.max():.4f}; notebook 0.544187 "
          f"(restated procedure over 20 keys: 0.28..0.54, mean 0.447, sd 0.069)")
    assert 0.544187 < kr.max()


def test_power_iteration_start_is_fixed_like_fold_in():
    """lipschitz.py:27 folds jnp.uint32(W[0, 0]) into PRNGKey(0): XLA's
    float-to-uint32 conversion truncates and saturates, so every weight below
    1 -- negative ones included -- starts the power iteration from the same
    vector (the same at every training step), a different integer part from
    another, and 2^32 or more from the last seed."""
    g = torch.Generator().manual_seed(3)
    W = torch.randn(32, 32, generator=g) * 0.2
    starts = []
    for w00 in (0.3, -0.7, 0.0, 0.999, -1.5, -3.0, float("nan"), 1.5, 2.2, 5e9, 2.0 ** 32 - 1):
        W[0, 0] = w00
        starts.append(Lz._start_vector(W))
    for u in starts[1:7]:
        assert torch.equal(u, starts[0])
    assert not torch.equal(starts[7], starts[0]) and not torch.equal(starts[8], starts[7])
    assert torch.equal(starts[9], starts[10]) and not torch.equal(starts[9], starts[8])
    assert float(torch.linalg.norm(starts[0])) == pytest.approx(1.0, rel=1e-6)
