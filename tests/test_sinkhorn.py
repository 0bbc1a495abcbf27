"""The float64 Sinkhorn restatement (oracle/sinkhorn_np.py, the checker of
utils_amd.evaluation.sinkhorn) against known answers: the converged plan's
marginals, the small-epsilon limit (exact optimal coupling by scipy's
Hungarian algorithm, as the reference's wasserstein_dist11_p), symmetry and
the zero self-divergence of the unbiased form (evaluation.py:104-130)."""
import numpy as np
import pytest
from scipy.optimize import linear_sum_assignment

import sinkhorn_np as S


def test_marginals_and_limit():
    rng = np.random.default_rng(0)
    x = rng.normal(size=(60, 3))
    y = rng.normal(size=(60, 3)) + 0.5
    r = S.sinkhorn(x, y, epsilon=0.02, threshold=1e-5, max_iterations=20000)
    assert r["converged"]
    C = S.cost_matrix(x, y)
    P = S.transport_plan(C, r["f"], r["g"], r["epsilon"])
    np.testing.assert_allclose(P.sum(0), 1 / 60, rtol=1e-5)
    np.testing.assert_allclose(P.sum(1), 1 / 60, rtol=1e-3)
    ri, ci = linear_sum_assignment(C)
    exact = C[ri, ci].mean()
    # dual cost = <P, C> + eps KL(P | a b^T), with 0 <= KL <= log n; <P, C> -> exact as eps -> 0
    assert exact - 1e-6 <= (P * C).sum() <= r["cost"] + 1e-9
    assert r["cost"] <= exact + r["epsilon"] * np.log(60) + 1e-6
    assert (P * C).sum() == pytest.approx(exact, rel=2e-2)


def test_default_epsilon_and_unbiased():
    rng = np.random.default_rng(1)
    x, y = rng.normal(size=(80, 2)), rng.normal(size=(60, 2)) * 2
    r = S.sinkhorn(x, y)
    assert r["epsilon"] == pytest.approx(0.05 * S.cost_matrix(x, y).std())
    assert r["converged"] and r["error"] < 1e-3
    self_div = S.sinkhorn(x, x)["cost"] - (S.sinkhorn(x, x)["cost"] + S.sinkhorn(x, x)["cost"]) / 2
    assert abs(self_div) < 1e-12
    a = S.sinkhorn(x, y)["cost"]
    b = S.sinkhorn(y, x)["cost"]
    assert a == pytest.approx(b, rel=1e-3)


def test_cost_fn_objects():
    """ott cost objects map by class name (the reference passes
    costs.Euclidean(), evaluation.py:69); anything else is refused."""
    from utils_amd.evaluation import _cost_mode

    class Euclidean:
        pass

    class SqEuclidean:
        pass

    class Cosine:
        pass

    assert _cost_mode(Euclidean()) == "euclidean" and _cost_mode("euclidean") == "euclidean"
    assert _cost_mode(SqEuclidean()) == "sqeuclidean" and _cost_mode("SqEuclidean") == "sqeuclidean"
    with pytest.raises(ValueError):
        _cost_mode(Cosine())
