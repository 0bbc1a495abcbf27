"""Keys for the counter-based (Philox4x32-10) noise streams.

The reference threads a JAX threefry key through ARWMHState and splits it
every step (arwmh.py:162).  Here a key is two uint32 words, exactly like a
JAX key; each chain's key is derived once from the run key and the global
chain id, and the position inside the chain's stream is the state's
iteration counter `i`, so the step kernel never has to split.
"""
from __future__ import annotations

import numpy as np


def PRNGKey(seed: int) -> np.ndarray:
    """jax.random.PRNGKey layout: [seed >> 32, seed & 0xffffffff] as uint32."""
    seed = int(seed)
    return np.array([(seed >> 32) & 0xFFFFFFFF, seed & 0xFFFFFFFF], dtype=np.uint32)


def as_key(key) -> np.ndarray:
    if isinstance(key, (int, np.integer)):
        return PRNGKey(int(key))
    k = np.asarray(key.cpu() if hasattr(key, "cpu") else key).astype(np.uint32).reshape(-1)
    if k.size != 2:
        raise ValueError("an rng key is two uint32 words")
    return k


_M0, _M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_W0, _W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
TAG_SPLIT = 0x54494C50


def _philox(c0, c1, c2, c3, k0, k1):
    mask = np.uint64(0xFFFFFFFF)
    c0, c1, c2, c3 = np.broadcast_arrays(*(np.asarray(c, np.uint32) for c in (c0, c1, c2, c3)))
    k0, k1 = np.uint32(k0), np.uint32(k1)
    with np.errstate(over="ignore"):
        for _ in range(10):
            p0 = _M0 * c0.astype(np.uint64)
            p1 = _M1 * c2.astype(np.uint64)
            c0, c1, c2, c3 = ((p1 >> np.uint64(32)).astype(np.uint32) ^ c1 ^ k0, (p1 & mask).astype(np.uint32),
                              (p0 >> np.uint64(32)).astype(np.uint32) ^ c3 ^ k1, (p0 & mask).astype(np.uint32))
            k0 = np.uint32(k0 + _W0)
            k1 = np.uint32(k1 + _W1)
    return c0, c1


def split(key, num=2) -> np.ndarray:
    """Host-side key split (e.g. one key per seed / per run); shape [*num, 2]."""
    k = as_key(key)
    shape = (num,) if isinstance(num, int) else tuple(num)
    n = int(np.prod(shape))
    idx = np.arange(n, dtype=np.uint64)
    a, b = _philox((idx & np.uint64(0xFFFFFFFF)).astype(np.uint32), (idx >> np.uint64(32)).astype(np.uint32),
                   0, TAG_SPLIT, k[0], k[1])
    return np.stack([a, b], axis=-1).reshape(shape + (2,))
