"""utils.evaluation on the GPU (HIP Gaussian-kernel sums and pairwise
distances, amh_eval.hip) against float64 numpy restatements of the
reference's python/utils/evaluation.py on the same inputs.  Tolerances:
kernel sums / MMD^2 rel 1e-5 (float32 distances, double accumulation);
distances rel 1e-6; sliced Wasserstein rel 1e-5 with the same directions."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _np_kernel(x, y, gamma):
    d2 = ((x[:, None, :] - y[None, :, :]) ** 2).sum(-1)
    return np.exp(-gamma * d2)


def _np_mmd2_unbiased(x, y, gamma):
    n, m = len(x), len(y)
    kxx, kyy, kxy = _np_kernel(x, x, gamma), _np_kernel(y, y, gamma), _np_kernel(x, y, gamma)
    np.fill_diagonal(kxx, 0)
    np.fill_diagonal(kyy, 0)
    return kxx.sum() / (n * (n - 1)) + kyy.sum() / (m * (m - 1)) - 2 * kxy.sum() / (n * m)


@pytest.mark.parametrize("n,m,d", [(300, 257, 26), (129, 128, 1), (64, 500, 70)])
def test_mmd2_unbiased_and_kernel(n, m, d, gpu):
    from utils_amd import evaluation as E
    rng = np.random.default_rng(n + m + d)
    x = rng.normal(size=(n, d)).astype(np.float32)
    y = (rng.normal(size=(m, d)) * 1.2 + 0.3).astype(np.float32)
    gamma = 1.0 / d
    got = E.mmd2_unbiased(x, y, gamma)
    ref = _np_mmd2_unbiased(x.astype(np.float64), y.astype(np.float64), gamma)
    assert got == pytest.approx(ref, rel=1e-4, abs=1e-7)
    K = E.gaussian_kernel(x, y, gamma).cpu().numpy()
    np.testing.assert_allclose(K, _np_kernel(x.astype(np.float64), y.astype(np.float64), gamma), rtol=1e-5,
                               atol=1e-7)
    assert E.mmd2_unbiased(x, y, gamma) == got  # deterministic reduction order


def test_mmd_heuristic(gpu):
    from utils_amd import evaluation as E
    rng = np.random.default_rng(5)
    x = rng.normal(size=(400, 10)).astype(np.float32)
    y = rng.normal(size=(301, 10)).astype(np.float32)
    yy = y.astype(np.float64)
    d2 = ((yy[:, None, :] - yy[None, :, :]) ** 2).sum(-1)
    gamma = 4.0 / np.median(d2)
    xx = x.astype(np.float64)
    mmd2 = (_np_kernel(xx, xx, gamma).sum() / 400 ** 2 + _np_kernel(yy, yy, gamma).sum() / 301 ** 2
            - 2 * _np_kernel(xx, yy, gamma).sum() / (400 * 301))
    assert E.mmd_heuristic(x, y) == pytest.approx(np.sqrt(mmd2), rel=1e-4)


def test_sliced_and_moments(gpu):
    from kernels_amd import PRNGKey
    from utils_amd import evaluation as E
    rng = np.random.default_rng(6)
    mu = rng.normal(size=(1000, 8)).astype(np.float32)
    nu = (rng.normal(size=(1000, 8)) + 0.5).astype(np.float32)
    dirs = E._directions(PRNGKey(3), 50, 8, torch.device("cuda", 0)).cpu().numpy().astype(np.float64)
    assert np.allclose(np.linalg.norm(dirs, axis=1), 1.0, atol=1e-6)
    pm, pn = mu.astype(np.float64) @ dirs.T, nu.astype(np.float64) @ dirs.T
    ref = np.max(np.mean(np.abs(np.sort(pm, 0) - np.sort(pn, 0)), axis=0))
    got = E.max_sliced_wasserstein(mu, nu, PRNGKey(3), p=1.0, n_directions=50)
    assert got == pytest.approx(ref, rel=1e-4)
    # shift by 0.5 in every coordinate: the best direction sees ~0.5 * sqrt(8)
    assert 1.0 < E.max_sliced_wasserstein(mu, nu, PRNGKey(4), n_directions=2000) < 1.5
    assert E.pth_moment_rmse(mu, nu, 1.0) == pytest.approx(
        np.linalg.norm(mu.mean(0) - nu.mean(0)), rel=1e-4)
    w = E.wasserstein_1d(mu[:, 0], nu[:, 0], p=2.0)
    assert float(w) == pytest.approx(np.sqrt(np.mean((np.sort(mu[:, 0]) - np.sort(nu[:, 0])) ** 2)), rel=1e-5)


def test_mmd_of_asss_draws_vs_reference_sample(gpu):
    """MMD between ARWMH and ASSS draws of the same 4-d Gaussian is tiny
    compared with a shifted sample (a use of the metrics as in the
    reference's evaluation scripts)."""
    import posteriors as P
    from kernels_amd import ARWMH, ASSS, PRNGKey
    from utils_amd import evaluation as E
    g = P.gaussian(np.zeros(4), cov=np.diag([1.0, 2.0, 0.5, 1.0]))
    draws = []
    for K in (ARWMH, ASSS):
        k = K(potential_fn=g, num_chains=2000)
        st = k.init(PRNGKey(1), 0, torch.zeros(2000, 4), (), {})
        k.sample_(st, 1500)
        draws.append(st.z.clone())
    a, b = draws
    same = E.mmd2_unbiased(a, b, 0.25)
    shifted = E.mmd2_unbiased(a, b + 0.5, 0.25)
    assert abs(same) < 0.003 and shifted > 10 * abs(same)


@pytest.mark.parametrize("n,m,d,cost_fn", [(300, 257, 26, "euclidean"), (128, 500, 3, "sqeuclidean"),
                                           (1000, 1000, 10, "euclidean")])
def test_sinkhorn_against_float64(n, m, d, cost_fn, gpu):
    """wasserstein_sinkhorn (evaluation.py:69-101) on the HIP log-sum-exp
    half-iterations vs the float64 restatement (oracle/sinkhorn_np.py), same
    iteration order: potentials after a fixed 40 iterations within 1e-4 eps,
    the converged cost within 1e-4 relative.  Parity against ott-jax itself is
    unpinned (not importable)."""
    import sinkhorn_np as S
    from utils_amd import evaluation as E
    rng = np.random.default_rng(n + d)
    x = rng.normal(size=(n, d)).astype(np.float32)
    y = (rng.normal(size=(m, d)) * 0.8 + 0.5).astype(np.float32)
    got = E.sinkhorn(x, y, cost_fn=cost_fn, threshold=0.0, max_iterations=40)
    ref = S.sinkhorn(x, y, cost_fn=cost_fn, threshold=0.0, max_iterations=40)
    assert got["epsilon"] == pytest.approx(ref["epsilon"], rel=1e-5)
    eps = ref["epsilon"]
    np.testing.assert_allclose(got["f"].cpu().numpy(), ref["f"], rtol=0, atol=1e-4 * max(eps, 1.0))
    np.testing.assert_allclose(got["g"].cpu().numpy(), ref["g"], rtol=0, atol=1e-4 * max(eps, 1.0))
    a = E.sinkhorn(x, y, cost_fn=cost_fn)
    b = S.sinkhorn(x, y, cost_fn=cost_fn)
    assert a["converged"] and b["converged"] and a["error"] < 1e-3
    assert a["cost"] == pytest.approx(b["cost"], rel=1e-4)
    assert E.wasserstein_sinkhorn(x, y, cost_fn=cost_fn) == pytest.approx(b["cost"], rel=1e-4)


def test_sinkhorn_unbiased_and_exact_limit(gpu):
    """The unbiased divergence of a set with itself is 0, it is symmetric, and
    with a small epsilon the regularised cost approaches the exact optimal
    1-1 coupling cost (scipy's Hungarian, wasserstein_dist11_p)."""
    from utils_amd import evaluation as E
    rng = np.random.default_rng(11)
    x = rng.normal(size=(200, 4)).astype(np.float32)
    y = (rng.normal(size=(200, 4)) + 0.7).astype(np.float32)
    assert abs(E.wasserstein_sinkhorn_unbiased(x, x)) < 1e-5
    uv, vu = E.wasserstein_sinkhorn_unbiased(x, y), E.wasserstein_sinkhorn_unbiased(y, x)
    assert uv == pytest.approx(vu, rel=1e-4) and uv > 0
    exact = E.wasserstein_dist11_p(x, y, ord=2.0)
    r = E.sinkhorn(x, y, epsilon=0.01, threshold=1e-4, max_iterations=20000)
    assert r["converged"]
    # dual cost = <P, C> + eps KL(P | a b^T) with 0 <= KL <= log n
    assert exact - 1e-4 <= r["cost"] <= exact + 0.01 * np.log(200) + 1e-4


# ---- the reference's stored diamonds draws (tests/golden/diamonds_example.npz) --
def _diamonds_fixture():
    import os
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "diamonds_example.npz"))
    return z["references"], z["samples"]


def test_pth_moment_rmse_pins_notebook_cell12(gpu):
    """wasserstein-computation.ipynb cell 12 printed 3.4000627994537354 for
    pth_moment_rmse(references, samples).  The stored references are that
    input; the samples side enters through cell 10's printed second moments
    (two rows +-sqrt(m_j) per column have exactly those).  The notebook's
    value is the mean-square form, i.e. the vector norm of evaluation.py:37
    divided by sqrt(d) (tests/test_diamonds_fixture.py)."""
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import extract_diamonds_pkl as X
    from utils_amd import evaluation as E
    ref, _ = _diamonds_fixture()
    m = np.array([X.CELL10[c][1] for c in X.COLUMNS])
    y = np.stack([np.sqrt(m), -np.sqrt(m)]).astype(np.float32)
    got = E.pth_moment_rmse(torch.as_tensor(ref, device=gpu), y)
    assert got / np.sqrt(26) == pytest.approx(3.4000627994537354, rel=2e-6)


def test_mmd2_on_reference_draws_full_size(gpu):
    """mmd2_unbiased on the full 10,000 x 26 stored references and samples
    (3 x 10^8 kernel pairs on amh_kernel_sum) against a float64 torch
    restatement of evaluation.py:224-259.  The notebook's 0.32471025 (cell 38)
    was computed on a samples file the reference no longer holds, so the value
    here is pinned to the restatement (rel 1e-5), not to cell 38."""
    from utils_amd import evaluation as E
    ref, smp = _diamonds_fixture()
    x = torch.as_tensor(smp, device=gpu)
    y = torch.as_tensor(ref, device=gpu)

    def ksum(a, b, skip):
        a64, b64 = a.double(), b.double()
        s = 0.0
        for i in range(0, a64.shape[0], 1000):
            blk = torch.exp(-torch.cdist(a64[i:i + 1000], b64, compute_mode="donot_use_mm_for_euclid_dist") ** 2)
            if skip:
                idx = torch.arange(blk.shape[0], device=gpu)
                blk[idx, idx + i] = 0.0
            s += float(blk.sum())
        return s

    n = m = 10000
    want = ksum(x, x, True) / (n * (n - 1)) + ksum(y, y, True) / (m * (m - 1)) - 2 * ksum(x, y, False) / (n * m)
    got = E.mmd2_unbiased(x, y)
    assert got == pytest.approx(want, rel=1e-5)
