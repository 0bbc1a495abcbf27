"""infer.diagnostics: known answers for the numpyro estimators restated in
adaptive-mcmc_amd/infer_amd/diagnostics.py (numpyro itself is not importable
here, so the definitions are pinned by closed forms and by a direct O(N^2)
restatement of the same formulas)."""
import numpy as np
import pytest

from infer_amd import diagnostics as D


def _ar1(rng, C, N, phi):
    x = np.empty((C, N))
    x[:, 0] = rng.standard_normal(C) / np.sqrt(1 - phi * phi)
    e = rng.standard_normal((C, N))
    for t in range(1, N):
        x[:, t] = phi * x[:, t - 1] + e[:, t]
    return x


def _ess_direct(x):
    """The same estimator with the autocovariance summed directly."""
    C, N = x.shape
    xc = x - x.mean(axis=1, keepdims=True)
    acov = np.stack([np.array([(xc[c, : N - k] * xc[c, k:]).sum() / N for k in range(N)]) for c in range(C)])
    W = x.var(axis=1, ddof=1).mean()
    var_plus = W * (N - 1) / N + (x.mean(axis=1).var(ddof=1) if C > 1 else 0.0)
    if C == 1:
        W = var_plus
    rho = 1.0 - (W - acov.mean(axis=0)) / var_plus
    rho[0] = 1.0
    R = rho[:-1:2] + rho[1::2]
    out = [R[0]]
    m = np.inf
    for v in R[1:]:
        m = min(m, max(v, 0.0))
        out.append(m)
    tau = -1.0 + 2.0 * np.sum(out)
    return C * N / tau


@pytest.mark.parametrize("C,N", [(1, 200), (4, 101), (3, 64)])
def test_ess_matches_direct_sum(C, N):
    x = _ar1(np.random.default_rng(C * N), C, N, 0.6)
    assert np.allclose(D.effective_sample_size(x), _ess_direct(x), rtol=1e-9)


@pytest.mark.parametrize("shape", [(1, 200), (4, 101), (3, 64), (6, 150, 3)])
def test_ess_torch_path_matches_numpy(shape):
    # bench.py hands device tensors (65,536 chains x 1,000 draws) to the torch
    # restatement; on CPU tensors it must agree with the numpy path
    import torch
    rng = np.random.default_rng(sum(shape))
    x = _ar1(rng, shape[0] * (shape[2] if len(shape) > 2 else 1), shape[1], 0.5)
    if len(shape) > 2:
        x = x.reshape(shape[0], shape[2], shape[1]).transpose(0, 2, 1).copy()
    got = D.effective_sample_size(torch.as_tensor(x))
    assert np.allclose(got, D.effective_sample_size(x), rtol=1e-10)
    with pytest.raises(ValueError):
        D.effective_sample_size(torch.zeros(3, 1))


def test_ess_ar1_closed_form():
    # tau = (1 + phi) / (1 - phi) for an AR(1) chain
    phi = 0.8
    x = _ar1(np.random.default_rng(0), 64, 4000, phi)
    ess = D.effective_sample_size(x)
    assert abs(ess / (x.size * (1 - phi) / (1 + phi)) - 1) < 0.08


def test_ess_iid_and_rhat():
    rng = np.random.default_rng(1)
    x = rng.standard_normal((8, 2000, 3))
    ess = D.effective_sample_size(x)
    assert ess.shape == (3,)
    assert np.all(np.abs(ess / x[..., 0].size - 1) < 0.1)
    assert np.all(np.abs(D.split_gelman_rubin(x) - 1) < 0.01)
    shifted = x + np.arange(8)[:, None, None]
    assert np.all(D.split_gelman_rubin(shifted) > 2)
    # single chain drifting in its second half: split R-hat sees it
    drift = rng.standard_normal((1, 1000))
    drift[:, 500:] += 3
    assert D.split_gelman_rubin(drift) > 1.5


def test_hpdi_exact():
    x = np.arange(100.0)
    assert np.array_equal(D.hpdi(x, 0.9), [0.0, 90.0])
    # skewed: the narrowest 50 % window lies in the dense part
    y = np.concatenate([np.linspace(0, 1, 80), np.linspace(1, 10, 20)])
    lo, hi = D.hpdi(y, 0.5)
    assert hi <= 1.0 and hi - lo <= 50 / 79 + 1e-12


def test_summary_table_layout():
    rng = np.random.default_rng(2)
    s = {"mu": rng.standard_normal((1, 500)), "theta_base": rng.standard_normal((1, 500, 8))}
    txt = D.format_summary(s)
    lines = txt.split("\n")
    # numpyro's header for a 13-character widest row label (posteriordb_eight-schools.ipynb cell 28)
    assert lines[1] == "                   mean       std    median      5.0%     95.0%     n_eff     r_hat"
    assert lines[2].startswith("           mu ")
    assert lines[3].startswith("theta_base[0] ")
    assert len(lines) == 2 + 1 + 8 + 1
    st = D.summary(s)
    assert set(st["mu"]) == {"mean", "std", "median", "5.0%", "95.0%", "n_eff", "r_hat"}


def test_autocorrelation_lag0_and_bias():
    x = np.random.default_rng(3).standard_normal(257)
    ac = D.autocorrelation(x)
    assert ac[0] == pytest.approx(1.0)
    acu = D.autocorrelation(x, bias=False)
    xc = x - x.mean()
    k = 5
    assert acu[k] == pytest.approx((xc[:-k] * xc[k:]).sum() / (257 - k) / ((xc * xc).sum() / 257), rel=1e-9)
    assert D.autocovariance(x)[0] == pytest.approx(x.var())
