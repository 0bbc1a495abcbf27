"""ctypes binding of libamh.so (include/amh.h).

The product path has exactly one implementation of the transition: the HIP
kernels in libamh.so.  If the library is missing, or no GPU is visible, every
compute entry point raises -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import torch  # noqa: F401  (loads the HIP runtime libamh.so binds against)

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("AMH_LIB_PATH") or os.path.join(_PKG, "lib", "libamh.so")
CSRC = os.path.join(_PKG, "csrc")

AMH_MODEL_GAUSSIAN = 1
AMH_MODEL_EIGHT_SCHOOLS = 2
AMH_MODEL_KIDIQ = 3
AMH_MODEL_DIAMONDS = 4
AMH_MODEL_DIAMONDS_SS = 5
AMH_MODEL_MIXTURE = 6
AMH_MODEL_EXTERNAL = 7  # the caller's potential (amh_propose / amh_step_external)
AMH_STEP_PROPOSAL_READY = 1
AMH_STEP_KEEP_PROPOSAL = 2

# every symbol include/amh.h declares
EXPORTS = ("amh_version", "amh_last_error", "amh_create", "amh_destroy", "amh_bind_model", "amh_init",
           "amh_step", "amh_step_chained", "amh_potential", "amh_sample_pnx", "amh_chain_keys", "amh_pooled_sums_size",
           "amh_pooled_stats", "amh_pooled_update", "amh_pooled_step", "amh_pooled_stats_k", "amh_pooled_update_k",
           "amh_pooled_step_k", "amh_asss_step",
           "amh_asss_sample_pnx", "amh_kernel_sum_scratch", "amh_kernel_sum", "amh_pairwise_dist2",
           "amh_normals", "amh_sinkhorn_lse", "amh_check_device", "amh_pooled_allreduce", "amh_propose",
           "amh_step_external", "amh_pnx_propose", "amh_pnx_accept")


class AmhConfig(ctypes.Structure):
    _fields_ = [("dim", ctypes.c_int32), ("num_warmup", ctypes.c_int32), ("lr_decay", ctypes.c_float),
                ("target_accept_prob", ctypes.c_float), ("eps", ctypes.c_float),
                ("reserved", ctypes.c_int32 * 3)]


class AmhState(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("i", "z", "potential_energy", "mean_accept_prob", "loc", "scale",
                                               "log_step_size", "as_change", "rng_key")]


class AmhCollect(ctypes.Structure):
    _fields_ = [("z", ctypes.c_void_p), ("potential_energy", ctypes.c_void_p), ("accept_count", ctypes.c_void_p),
                ("thinning", ctypes.c_int32)]


class AmhPooledState(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("i", "z", "potential_energy", "rng_key", "mean_accept_prob", "loc",
                                               "scale", "log_step_size", "as_change", "cov")]


class AmhError(RuntimeError):
    pass


_lib = None


def build(arch: str = "gfx950") -> str:
    """Compile libamh.so in-tree (hipcc, gfx950)."""
    subprocess.run(["make", "-s", "-C", CSRC, f"ARCH={arch}"], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise AmhError(f"libamh.so not built ({LIB_PATH}); run `make -C {CSRC}` or __graft_entry__.build()")
    L = ctypes.CDLL(LIB_PATH)
    P, I32, I64, F = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_float
    L.amh_version.restype = ctypes.c_int
    L.amh_last_error.argtypes = [P]
    L.amh_last_error.restype = ctypes.c_char_p
    L.amh_create.argtypes = [ctypes.POINTER(AmhConfig), ctypes.c_int, ctypes.POINTER(P)]
    L.amh_destroy.argtypes = [P]
    L.amh_check_device.argtypes = [P]
    L.amh_check_device.restype = ctypes.c_int
    L.amh_bind_model.argtypes = [P, I32, P, I64, ctypes.POINTER(I64), I32]
    L.amh_init.argtypes = [P, ctypes.POINTER(ctypes.c_uint32), I64, I64, P, ctypes.POINTER(AmhState), P]
    L.amh_step.argtypes = [P, I64, ctypes.POINTER(AmhState), ctypes.POINTER(AmhState), I32,
                           ctypes.POINTER(AmhCollect), P]
    L.amh_step_chained.argtypes = [P, I64, ctypes.POINTER(AmhState), ctypes.POINTER(AmhState), I32,
                                   ctypes.POINTER(AmhCollect), I32, P]
    L.amh_step_chained.restype = ctypes.c_int
    L.amh_potential.argtypes = [P, P, P, I64, P]
    L.amh_sample_pnx.argtypes = [P, ctypes.POINTER(ctypes.c_uint32), P, I64, I64, P, P, F, I32, P, P]
    L.amh_chain_keys.argtypes = [ctypes.POINTER(ctypes.c_uint32), I64, I64, P, P]
    L.amh_asss_step.argtypes = [P, I64, ctypes.POINTER(AmhState), ctypes.POINTER(AmhState), I32,
                                ctypes.POINTER(AmhCollect), P]
    L.amh_asss_step.restype = ctypes.c_int
    L.amh_asss_sample_pnx.argtypes = [P, ctypes.POINTER(ctypes.c_uint32), P, I64, I64, P, P, I32, P, P]
    L.amh_propose.argtypes = [P, I64, ctypes.POINTER(AmhState), P, P]
    L.amh_propose.restype = ctypes.c_int
    L.amh_step_external.argtypes = [P, I64, ctypes.POINTER(AmhState), ctypes.POINTER(AmhState), P, P, P,
                                    ctypes.POINTER(AmhCollect), P]
    L.amh_step_external.restype = ctypes.c_int
    L.amh_pnx_propose.argtypes = [P, ctypes.POINTER(ctypes.c_uint32), P, I64, P, F, I32, P, P]
    L.amh_pnx_propose.restype = ctypes.c_int
    L.amh_pnx_accept.argtypes = [P, ctypes.POINTER(ctypes.c_uint32), P, P, I64, P, P, I32, P]
    L.amh_pnx_accept.restype = ctypes.c_int
    L.amh_asss_sample_pnx.restype = ctypes.c_int
    L.amh_kernel_sum_scratch.argtypes = [I64, I64]
    L.amh_kernel_sum_scratch.restype = I64
    L.amh_kernel_sum.argtypes = [P, I64, P, I64, I32, F, I32, P, P, P]
    L.amh_kernel_sum.restype = ctypes.c_int
    L.amh_pairwise_dist2.argtypes = [P, I64, P, I64, I32, P, P]
    L.amh_pairwise_dist2.restype = ctypes.c_int
    L.amh_normals.argtypes = [ctypes.POINTER(ctypes.c_uint32), I64, P, P]
    L.amh_normals.restype = ctypes.c_int
    L.amh_sinkhorn_lse.argtypes = [P, I64, I64, P, F, F, P, P]
    L.amh_sinkhorn_lse.restype = ctypes.c_int
    PS = ctypes.POINTER(AmhPooledState)
    L.amh_pooled_sums_size.argtypes = [I32, ctypes.POINTER(I64)]
    L.amh_pooled_stats.argtypes = [P, I64, PS, P, P, P, P]
    L.amh_pooled_update.argtypes = [P, P, PS, PS, P]
    L.amh_pooled_step.argtypes = [P, I64, PS, PS, I32, P, P]
    L.amh_pooled_stats_k.argtypes = [P, I64, PS, I32, P, P, P, P]
    L.amh_pooled_update_k.argtypes = [P, P, PS, PS, I32, P]
    L.amh_pooled_allreduce.argtypes = [P, P, I64, P, P]
    L.amh_pooled_step_k.argtypes = [P, I64, PS, PS, I32, I32, P, P]
    for name in ("amh_pooled_sums_size", "amh_pooled_stats", "amh_pooled_update", "amh_pooled_step",
                 "amh_pooled_stats_k", "amh_pooled_update_k", "amh_pooled_step_k", "amh_pooled_allreduce"):
        getattr(L, name).restype = ctypes.c_int
    L.amh_version.argtypes = []
    for name in EXPORTS[:10]:
        getattr(L, name).restype = ctypes.c_int if name != "amh_last_error" else ctypes.c_char_p
    _lib = L
    return L


def check(rc: int, handle=None):
    if rc != 0:
        msg = lib().amh_last_error(handle)
        raise AmhError(f"libamh error {rc}: {msg.decode() if msg else ''}")


def require_gpu(t: torch.Tensor):
    if not t.is_cuda:
        raise AmhError("libamh operates on device tensors; no CPU fallback exists (is a GPU visible?)")


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_ptr(device) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def key_arr(key) -> "ctypes.Array":
    k = [int(v) & 0xFFFFFFFF for v in key]
    return (ctypes.c_uint32 * 2)(*k)


class Handle:
    """Owns one amh_handle (one device, one model binding)."""

    def __init__(self, dim: int, num_warmup: int, lr_decay: float, target_accept_prob: float, eps: float,
                 device: int):
        self._lib = lib()
        cfg = AmhConfig(dim, num_warmup, lr_decay, target_accept_prob, eps, (ctypes.c_int32 * 3)(0, 0, 0))
        h = ctypes.c_void_p()
        with torch.cuda.device(device):
            check(self._lib.amh_create(ctypes.byref(cfg), device, ctypes.byref(h)))
        self.h = h
        self.device = device
        self.dim = dim
        self._data = None

    def bind_model(self, model_id: int, data: torch.Tensor, iparams=()):
        require_gpu(data)
        ip = (ctypes.c_int64 * max(1, len(iparams)))(*iparams)
        with torch.cuda.device(self.device):
            # the library may copy `data` on the null stream: let the stream
            # that produced it finish first
            torch.cuda.current_stream(data.device).synchronize()
            check(self._lib.amh_bind_model(self.h, model_id, ptr(data), data.numel(), ip, len(iparams)), self.h)
        self._data = data  # keep alive

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            rc = self._lib.amh_destroy(self.h)
            self.h = None
            if rc != 0:  # a device-side failure nobody had collected (amh_check_device)
                import warnings
                msg = self._lib.amh_last_error(None)
                warnings.warn(f"libamh: {msg.decode() if msg else rc}", RuntimeWarning)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
