"""The reference's stored diamonds draws (tests/golden/diamonds_example.npz,
extracted byte-wise by tests/golden/extract_diamonds_pkl.py) against the
outputs python/jupyter/wasserstein-computation.ipynb prints for them.

  cell 10   E[X^2] per column: the references file reproduces all 26 printed
            values of the "reference" column (6 decimals)
  cell 12   pth_moment_rmse(references, samples) = 3.4000627994537354 equals
            sqrt(mean_j (E_ref[X_j^2] - E_smp[X_j^2])^2) with the first term
            from the stored references and the second from cell 10's printed
            "samples" column (rel 1e-7: only the table's 6-decimal rounding
            enters).  That is the mean-square form; evaluation.py:37 now
            returns the vector norm, sqrt(26) times larger, which is what
            utils_amd.evaluation follows (the API a caller binds).
  samples   the stored samples file is not the notebook's draw set (26/26
            columns differ from cell 10), so cells 19, 21-24, 31 and 38 have
            no reachable inputs; this test keeps that statement true.
"""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

import extract_diamonds_pkl as X  # noqa: E402

CELL12 = 3.4000627994537354


@pytest.fixture(scope="module")
def fx():
    z = np.load(os.path.join(HERE, "golden", "diamonds_example.npz"))
    return z["references"], z["samples"], [str(c) for c in z["columns"]]


def test_columns_and_shapes(fx):
    ref, smp, cols = fx
    assert ref.shape == smp.shape == (10000, 26) and ref.dtype == np.float32
    assert cols == X.COLUMNS


def test_references_reproduce_cell10(fx):
    ref, _, _ = fx
    assert X.cell10_mismatch(ref, 0) == []


def test_cell12_from_references_and_printed_samples_column(fx):
    ref, _, _ = fx
    m_ref = np.mean(ref.astype(np.float64) ** 2, axis=0)
    t_smp = np.array([X.CELL10[c][1] for c in X.COLUMNS])
    rmse = np.sqrt(np.mean((m_ref - t_smp) ** 2))
    assert rmse == pytest.approx(CELL12, rel=1e-7)
    # the vector-norm form of evaluation.py:37 is sqrt(d) times that
    assert np.linalg.norm(m_ref - t_smp) == pytest.approx(CELL12 * np.sqrt(26), rel=1e-7)


def test_stored_samples_are_not_the_notebooks(fx):
    _, smp, _ = fx
    assert len(X.cell10_mismatch(smp, 1)) == 26


def test_synthetic_diamonds_centre_is_the_reference_draw_mean(fx):
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "adaptive-mcmc_amd"))
    import posteriors as P
    ref, _, _ = fx
    np.testing.assert_allclose(P._DIAMONDS_B_HEAD, ref[:, :4].astype(np.float64).mean(0), atol=5e-4)


@pytest.mark.skipif(not os.path.exists(X.SRC.format("references")), reason="reference files absent (GPU box)")
def test_extraction_reproduces_fixture(fx):
    ref, smp, _ = fx
    np.testing.assert_array_equal(X.matrix(X.load("references")), ref)
    np.testing.assert_array_equal(X.matrix(X.load("samples")), smp)
