"""Shared test helpers: the same model in product form (posteriors) and in
oracle form (oracle/orc.py), built from the same packed float32 data."""
from __future__ import annotations

import numpy as np


def make_case(kind: str, d: int = None):
    """-> (product kwargs for ARWMH, model_kwargs, orc.Model)"""
    import orc
    import posteriors as P
    if kind == "gaussian":
        g = P.correlated_gaussian(d or 64)
        data, _ = g.pack("cpu")
        return dict(potential_fn=g), {}, orc.Model(orc.GAUSSIAN, g.dim, data.numpy())
    if kind == "eight_schools":
        mk = dict(P.EIGHT_SCHOOLS_DATA)
        arr, ip = P.eight_schools.pack_fn(mk)
        return dict(model=P.eight_schools), mk, orc.Model(orc.EIGHT_SCHOOLS, ip[0] + 2, arr)
    if kind == "kidiq":
        mk = P.synthetic_kidiq()
        arr, ip = P.kidiq.pack_fn(mk)
        return dict(model=P.kidiq), mk, orc.Model(orc.KIDIQ, 4, arr, n_data=ip[0])
    if kind == "diamonds":
        mk = P.synthetic_diamonds(N=500)
        arr, ip = P.diamonds.pack_fn(mk)
        N, K = ip
        return dict(model=P.diamonds), mk, orc.Model(orc.DIAMONDS, K + 1, arr, n_data=N, k_data=K)
    if kind == "diamonds_ss":
        mk = P.synthetic_diamonds(N=500)
        arr, ip = P.diamonds_suffstat.pack_fn(mk)
        N, K = ip
        return dict(model=P.diamonds_suffstat), mk, orc.Model(orc.DIAMONDS_SS, K + 1, arr, n_data=N, k_data=K)
    if kind == "mixture":  # asumptions_check.ipynb cell 61, on every coordinate
        mx = P.notebook_mixture() if (d or 1) == 1 else P.mixture([0.5, 0.5], [-1.0, 1.0], [0.1, 0.1], dim=d)
        data, ip = mx.pack("cpu")
        return dict(potential_fn=mx), {}, orc.Model(orc.MIXTURE, mx.dim, data.numpy(), n_data=ip[0])
    raise ValueError(kind)


def state_to_orc(state):
    import orc
    s = state
    return orc.State(s.i.cpu().numpy().copy(), s.z.cpu().numpy().copy(), s.potential_energy.cpu().numpy().copy(),
                     s.mean_accept_prob.cpu().numpy().copy(), s.adapt_state.loc.cpu().numpy().copy(),
                     s.adapt_state.scale.cpu().numpy().copy(), s.adapt_state.log_step_size.cpu().numpy().copy(),
                     s.as_change.cpu().numpy().copy(), s.rng_key.cpu().numpy().view(np.uint32).copy())


FIELDS = ("i", "z", "potential_energy", "mean_accept_prob", "loc", "scale", "log_step_size", "as_change", "rng_key")


def assert_state_bitequal(gpu_state, orc_state, what=""):
    g = state_to_orc(gpu_state)
    for f in FIELDS:
        a = np.asarray(getattr(g, f))
        b = np.asarray(getattr(orc_state, f))
        assert a.shape == b.shape, (what, f, a.shape, b.shape)
        av = a.view(np.uint32) if a.dtype in (np.float32, np.int32, np.uint32) else a
        bv = b.view(np.uint32) if b.dtype in (np.float32, np.int32, np.uint32) else b
        bad = np.flatnonzero((av != bv).reshape(-1))
        assert bad.size == 0, (f"{what}: field {f} differs in {bad.size} of {av.size} entries; "
                               f"first at {bad[:5]}: gpu {a.reshape(-1)[bad[:5]]} oracle {b.reshape(-1)[bad[:5]]}")
