"""Host-side API of the drop-in (reference python/kernels/arwmh.py) that runs
without a GPU: constructor / init ValueErrors, state layout helpers, the
model registry (sorted-site ravel order, transforms, packed data)."""
import math

import numpy as np
import pytest
import torch

import posteriors as P
from kernels_amd import ARWMH, PRNGKey, pack_scale, packed_size, split, unpack_scale


def test_model_xor_potential_fn():
    with pytest.raises(ValueError):
        ARWMH()
    with pytest.raises(ValueError):
        ARWMH(model=P.eight_schools, potential_fn=P.correlated_gaussian(4))


def test_potential_fn_needs_init_params():
    k = ARWMH(potential_fn=P.correlated_gaussian(4))
    with pytest.raises(ValueError):
        k.init(PRNGKey(0), 0, None, (), {})


def test_reference_defaults():
    k = ARWMH(model=P.eight_schools)
    assert k._lr_decay == pytest.approx(2 / 3) and k._target_accept_prob == 0.234 and k._eps == 1e-6
    assert k.sample_field == "z" and k.model is P.eight_schools


def test_pack_unpack_roundtrip():
    d = 7
    L = torch.tril(torch.randn(3, d, d))
    Lp = pack_scale(L)
    assert Lp.shape == (3, packed_size(d))
    assert torch.equal(unpack_scale(Lp, d), L)
    # column-major: column j starts at j*d - j(j-1)/2
    j = 3
    off = j * d - j * (j - 1) // 2
    assert torch.equal(Lp[0, off:off + d - j], L[0, j:, j])


def test_eight_schools_layout():
    data = P.EIGHT_SCHOOLS_DATA
    sites = P.eight_schools.sites(data)
    assert [s.name for s in sites] == sorted(s.name for s in sites) == ["mu", "tau", "theta_base"]
    assert P.eight_schools.dim(data) == 10
    z = torch.arange(10, dtype=torch.float32)[None]
    out = P.eight_schools.postprocess(z, data)
    assert out["mu"].item() == 0 and out["tau"].item() == pytest.approx(math.e)
    assert torch.allclose(out["theta"], out["mu"][..., None] + out["tau"][..., None] * out["theta_base"])
    arr, ip = P.eight_schools.pack_fn(data)
    assert ip == (8,) and arr.shape == (24,) and np.allclose(arr[16:], np.log(data["sigma"]))


def test_diamonds_layout():
    data = P.synthetic_diamonds(N=200)
    assert [s.name for s in P.diamonds.sites(data)] == ["Intercept", "b", "sigma"]
    assert P.diamonds.dim(data) == 26
    arr, (N, K) = P.diamonds.pack_fn(data)
    assert (N, K) == (200, 25) and arr.size == N * (K - 1) + N
    Xc = arr[:N * (K - 1)].reshape(N, K - 1)
    assert np.abs(Xc.mean(axis=0)).max() < 1e-4
    c = np.corrcoef(data["X"][:, 1:].T)[np.triu_indices(K - 1, 1)]
    assert c.min() > 0.85


def test_correlated_gaussian_target():
    g = P.correlated_gaussian(64)
    ev = np.linalg.eigvalsh(np.linalg.inv(g.precision))
    assert ev.min() == pytest.approx(0.1, rel=1e-6) and ev.max() == pytest.approx(10.0, rel=1e-6)
    data, ip = g.pack("cpu")
    assert data.numel() == 64 + 64 * 64 + 1 and ip == ()
    x = np.zeros(64)
    assert float(data[-1]) == pytest.approx(g(x), rel=1e-6)


def test_keys():
    k = PRNGKey(5)
    a, b = split(k)
    assert not np.array_equal(np.asarray(a), np.asarray(b))
    assert np.array_equal(np.asarray(split(k)[0]), np.asarray(a))
