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
        tau, model, params = Lz.compute_wasserstein_contraction(fn, PRNGKey(0), X, n_train_batches=5,
                                                                n_eval_batches=20, max_steps=10)
        assert 0.0 < tau <= 1.15
        if n == 0:
            assert tau > 0.8
    fn = lambda key, x, n_samples: k.sample_Pnx(key, x, adapt, 1, n_samples)
    rho, _, _ = Lz.compute_kernel_distance_1d(fn, fn, PRNGKey(1), torch.linspace(-3, 3, 31), max_steps=10,
                                              n_eval_batches=10)
    assert 0.0 <= rho < 0.2
