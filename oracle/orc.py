"""ctypes binding for the C oracle (oracle/amh_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the product package.

Arrays are numpy, chain-major, matching the device layout of the product:
z/loc [C, d], scale [C, d(d+1)/2] packed lower triangle column-major,
scalars [C], rng keys [C, 2] uint32.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# AMH_ORACLE_LIB selects another build of the same source (the sanitizer build,
# `make -C oracle asan`, run by tests/test_oracle_asan.py)
_LIB_PATH = os.environ.get("AMH_ORACLE_LIB") or os.path.join(_HERE, "build", "libamh_oracle.so")

GAUSSIAN, EIGHT_SCHOOLS, KIDIQ, DIAMONDS, DIAMONDS_SS, MIXTURE = 1, 2, 3, 4, 5, 6

_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I32 = ctypes.c_int32
_F = ctypes.c_float


class OrcCfg(ctypes.Structure):
    _fields_ = [
        ("model_id", ctypes.c_int32),
        ("d", ctypes.c_int32),
        ("num_warmup", ctypes.c_int32),
        ("lr_decay", ctypes.c_float),
        ("target_accept_prob", ctypes.c_float),
        ("eps", ctypes.c_float),
        ("data", ctypes.c_void_p),
        ("n_data", ctypes.c_int64),
        ("k_data", ctypes.c_int64),
    ]


_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.orc_group_width.argtypes = [ctypes.c_int]
        L.orc_group_width.restype = ctypes.c_int
        L.orc_potential.argtypes = [_P, _P, _P, _I64]
        L.orc_potential1.argtypes = [_P, _P]
        L.orc_potential1.restype = ctypes.c_float
        L.orc_chain_keys.argtypes = [_P, _I64, _I64, _P]
        L.orc_split_keys.argtypes = [_P, _I64, _P]
        L.orc_init.argtypes = [_P, _P, _I64, _I64, _P] + [_P] * 9
        L.orc_step.argtypes = [_P, _I64, _I32] + [_P] * 11
        L.orc_sample_pnx.argtypes = [_P, _P, _P, _I64, _I64, _P, _P, _F, _I32, _P]
        L.orc_philox.argtypes = [_P, _P, _P, _I64]
        for name in ("orc_logf", "orc_expf", "orc_log1pf", "orc_erfinvf"):
            getattr(L, name).argtypes = [_P, _P, _I64]
        L.orc_normal_bits.argtypes = [_P, _P, _I64]
        L.orc_lr_gamma.argtypes = [_P, _F, _P, _I64]
        L.orc_num_threads.restype = ctypes.c_int
        L.orc_asss_step.argtypes = [_P, _I64, _I32] + [_P] * 9
        L.orc_asss_step.restype = None
        L.orc_asss_sample_pnx.argtypes = [_P, _P, _P, _I64, _I64, _P, _P, _I32, _P]
        L.orc_asss_sample_pnx.restype = None
        L.orc_pooled_cpw.argtypes = [_I64]
        L.orc_pooled_cpw.restype = ctypes.c_int
        L.orc_pooled_stats.argtypes = [_P, _I64, _I32, _P, _P, _P, _P, _P, _F, _P, _P, _P]
        L.orc_pooled_update.argtypes = [_P, _P] + [_P] * 7
        L.orc_pooled_update.restype = ctypes.c_int
        L.orc_pooled_stats_k.argtypes = [_P, _I64, _I32, _I32, _P, _P, _P, _P, _P, _F, _P, _P, _P]
        L.orc_pooled_update_k.argtypes = [_P, _P, _I32] + [_P] * 7
        L.orc_pooled_update_k.restype = ctypes.c_int
        _lib = L
    return _lib


def _ptr(a):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


def _c(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


# ------------------------------------------------------------ elementwise --
def elementwise(name: str, x: np.ndarray) -> np.ndarray:
    x = _c(x, np.float32)
    y = np.empty_like(x)
    getattr(lib(), "orc_" + name)(_ptr(x), _ptr(y), x.size)
    return y


def philox(ctr: np.ndarray, key: np.ndarray) -> np.ndarray:
    ctr = _c(ctr, np.uint32).reshape(-1, 4)
    key = _c(key, np.uint32).reshape(-1, 2)
    out = np.empty_like(ctr)
    lib().orc_philox(_ptr(ctr), _ptr(key), _ptr(out), ctr.shape[0])
    return out


def normal_from_bits(bits: np.ndarray) -> np.ndarray:
    bits = _c(bits, np.uint32)
    y = np.empty(bits.shape, np.float32)
    lib().orc_normal_bits(_ptr(bits), _ptr(y), bits.size)
    return y


def lr_gamma(n: np.ndarray, a: float) -> np.ndarray:
    n = _c(n, np.int32)
    y = np.empty(n.shape, np.float32)
    lib().orc_lr_gamma(_ptr(n), a, _ptr(y), n.size)
    return y


def group_width(d: int) -> int:
    return lib().orc_group_width(d)


def num_threads() -> int:
    return lib().orc_num_threads()


# ------------------------------------------------------------------ model --
@dataclass
class Model:
    model_id: int
    d: int
    data: np.ndarray
    n_data: int = 0
    k_data: int = 0

    def cfg(self, num_warmup=0, lr_decay=2 / 3, target_accept_prob=0.234, eps=1e-6) -> OrcCfg:
        self.data = _c(self.data, np.float32)
        return OrcCfg(self.model_id, self.d, num_warmup, lr_decay, target_accept_prob, eps,
                      self.data.ctypes.data, self.n_data, self.k_data)


def potential(model: Model, z: np.ndarray) -> np.ndarray:
    z = _c(z, np.float32).reshape(-1, model.d)
    pe = np.empty(z.shape[0], np.float32)
    cfg = model.cfg()
    lib().orc_potential(ctypes.byref(cfg), _ptr(z), _ptr(pe), z.shape[0])
    return pe


@dataclass
class State:
    i: np.ndarray
    z: np.ndarray
    potential_energy: np.ndarray
    mean_accept_prob: np.ndarray
    loc: np.ndarray
    scale: np.ndarray
    log_step_size: np.ndarray
    as_change: np.ndarray
    rng_key: np.ndarray

    def copy(self) -> "State":
        return State(*[np.array(getattr(self, f)) for f in self.__dataclass_fields__])


def chain_keys(key, chain_offset: int, n: int) -> np.ndarray:
    key = _c(key, np.uint32)
    out = np.empty((n, 2), np.uint32)
    lib().orc_chain_keys(_ptr(key), chain_offset, n, _ptr(out))
    return out


def split_keys(key, n: int) -> np.ndarray:
    key = _c(key, np.uint32)
    out = np.empty((n, 2), np.uint32)
    lib().orc_split_keys(_ptr(key), n, _ptr(out))
    return out


def init(model: Model, key, num_chains: int, chain_offset: int = 0, init_z=None) -> State:
    d, C = model.d, num_chains
    P = d * (d + 1) // 2
    s = State(np.zeros(C, np.int32), np.zeros((C, d), np.float32), np.zeros(C, np.float32),
              np.zeros(C, np.float32), np.zeros((C, d), np.float32), np.zeros((C, P), np.float32),
              np.zeros(C, np.float32), np.zeros(C, np.float32), np.zeros((C, 2), np.uint32))
    key = _c(key, np.uint32)
    iz = None if init_z is None else _c(init_z, np.float32).reshape(C, d)
    cfg = model.cfg()
    lib().orc_init(ctypes.byref(cfg), _ptr(key), chain_offset, C, _ptr(iz), _ptr(s.i), _ptr(s.z),
                   _ptr(s.potential_energy), _ptr(s.mean_accept_prob), _ptr(s.loc), _ptr(s.scale),
                   _ptr(s.log_step_size), _ptr(s.as_change), _ptr(s.rng_key))
    return s


def step(model: Model, state: State, n_steps: int = 1, num_warmup: int = 0, lr_decay: float = 2 / 3,
         target_accept_prob: float = 0.234, eps: float = 1e-6, accept_count=None, collect_z=False):
    """Advance `state` in place by n_steps; returns collected z [n_steps, C, d] if asked."""
    C = state.z.shape[0]
    cfg = model.cfg(num_warmup, lr_decay, target_accept_prob, eps)
    cz = np.empty((n_steps, C, model.d), np.float32) if collect_z else None
    lib().orc_step(ctypes.byref(cfg), C, n_steps, _ptr(state.i), _ptr(state.z), _ptr(state.potential_energy),
                   _ptr(state.mean_accept_prob), _ptr(state.loc), _ptr(state.scale), _ptr(state.log_step_size),
                   _ptr(state.as_change), _ptr(state.rng_key), _ptr(accept_count), _ptr(cz))
    return cz


def asss_step(model: Model, state: State, n_steps: int = 1, num_warmup: int = 0, lr_decay: float = 2 / 3,
              eps: float = 1e-6, collect_z=False, collect_pe=False):
    """ASSS transitions (asss.py:197-251) in place, one launch; the state's
    mean_accept_prob / log_step_size are not touched.  Returns (cz, cp)."""
    C = state.z.shape[0]
    cfg = model.cfg(num_warmup, lr_decay, 0.234, eps)
    cz = np.empty((n_steps, C, model.d), np.float32) if collect_z else None
    cp = np.empty((n_steps, C), np.float32) if collect_pe else None
    lib().orc_asss_step(ctypes.byref(cfg), C, n_steps, _ptr(state.i), _ptr(state.z), _ptr(state.potential_energy),
                        _ptr(state.loc), _ptr(state.scale), _ptr(state.as_change), _ptr(state.rng_key), _ptr(cz),
                        _ptr(cp))
    return cz, cp


def asss_sample_pnx(model: Model, key, x: np.ndarray, loc, scale_packed, n: int, n_samples: int,
                    eps: float = 1e-6) -> np.ndarray:
    x = _c(x, np.float32).reshape(-1, model.d)
    out = np.empty((x.shape[0], n_samples, model.d), np.float32)
    cfg = model.cfg(0, 2 / 3, 0.234, eps)
    lib().orc_asss_sample_pnx(ctypes.byref(cfg), _ptr(_c(key, np.uint32)), _ptr(x), x.shape[0], n_samples,
                              _ptr(_c(loc, np.float32)), _ptr(_c(scale_packed, np.float32)), n, _ptr(out))
    return out


def sample_pnx(model: Model, key, x: np.ndarray, loc, scale_packed, log_step_size: float, n: int,
               n_samples: int, eps: float = 1e-6) -> np.ndarray:
    x = _c(x, np.float32).reshape(-1, model.d)
    npts = x.shape[0]
    out = np.empty((npts, n_samples, model.d), np.float32)
    cfg = model.cfg(0, 2 / 3, 0.234, eps)
    key = _c(key, np.uint32)
    loc = _c(loc, np.float32)
    sp = _c(scale_packed, np.float32)
    lib().orc_sample_pnx(ctypes.byref(cfg), _ptr(key), _ptr(x), npts, n_samples, _ptr(loc), _ptr(sp),
                         log_step_size, n, _ptr(out))
    return out


# ------------------------------------------------------------- pooled mode --
def pooled_cpw(C: int) -> int:
    return lib().orc_pooled_cpw(C)


def pooled_stats(model: Model, i: int, z, pe, keys, mu, Lpacked, lam: float, eps: float = 1e-6, k_steps: int = 1):
    """-> (z_out, pe_out, sums[V]) for one pooled step, or a block of k_steps
    transitions with the frozen shared state (orc_pooled_stats_k)."""
    d = model.d
    z = _c(z, np.float32).reshape(-1, d)
    C = z.shape[0]
    pe = _c(pe, np.float32)
    keys = _c(keys, np.uint32)
    mu = _c(mu, np.float32)
    Lp = _c(Lpacked, np.float32)
    zo = np.empty_like(z)
    po = np.empty_like(pe)
    sums = np.empty(d + d * (d + 1) // 2 + 2, np.float64)
    cfg = model.cfg(0, 2 / 3, 0.234, eps)
    lib().orc_pooled_stats_k(ctypes.byref(cfg), C, int(i), int(k_steps), _ptr(z), _ptr(pe), _ptr(keys), _ptr(mu),
                             _ptr(Lp), ctypes.c_float(lam), _ptr(zo), _ptr(po), _ptr(sums))
    return zo, po, sums


def pooled_update(model: Model, sums, shared: dict, num_warmup: int = 0, lr_decay: float = 2 / 3,
                  target_accept_prob: float = 0.234, k_steps: int = 1) -> int:
    """In-place update of shared = {i, macc, mu, L, lam, asc, cov} (numpy
    arrays: i int32[1], macc/lam/asc float32[1], mu float32[d], L float32[P],
    cov float64[P]).  Returns 1 if refactorised."""
    cfg = model.cfg(num_warmup, lr_decay, target_accept_prob, 1e-6)
    sums = _c(sums, np.float64)
    return lib().orc_pooled_update_k(ctypes.byref(cfg), _ptr(sums), int(k_steps), _ptr(shared["i"]),
                                     _ptr(shared["macc"]), _ptr(shared["mu"]), _ptr(shared["L"]), _ptr(shared["lam"]),
                                     _ptr(shared["asc"]), _ptr(shared["cov"]))


def pooled_init_shared(d: int) -> dict:
    P = d * (d + 1) // 2
    L = np.zeros(P, np.float32)
    cov = np.zeros(P, np.float64)
    k = 0
    for j in range(d):
        L[k] = 1.0
        cov[k] = 1.0
        k += d - j
    return dict(i=np.zeros(1, np.int32), macc=np.zeros(1, np.float32), mu=np.zeros(d, np.float32), L=L,
                lam=np.zeros(1, np.float32), asc=np.zeros(1, np.float32), cov=cov)
