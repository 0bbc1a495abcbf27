"""The C-ABI library (include/amh.h) without a GPU: it loads, exports every
symbol the header declares, the ctypes binding covers exactly those symbols,
and calls that need a device fail with a status code and a message (no
crash, no CPU fallback)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "amh.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int64_t|int|const char\s*\*)\s*(amh_\w+)\s*\(", src, flags=re.M)))


@pytest.fixture(scope="module")
def lib():
    from kernels_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        _lib.build()
    return _lib


def test_header_declares_the_boundary():
    syms = header_symbols()
    for s in ("amh_create", "amh_init", "amh_step", "amh_sample_pnx", "amh_potential", "amh_last_error"):
        assert s in syms


def test_library_exports_every_declared_symbol(lib):
    L = ctypes.CDLL(lib.LIB_PATH)
    for s in header_symbols():
        assert hasattr(L, s), s
    assert sorted(lib.EXPORTS) == header_symbols()


def header_arity():
    """{symbol: parameter count} from the prototypes in include/amh.h."""
    src = open(os.path.join(ROOT, "include", "amh.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    out = {}
    for m in re.finditer(r"^\s*(?:int64_t|int|const char\s*\*)\s*(amh_\w+)\s*\(([^;]*?)\)\s*;", src, flags=re.M | re.S):
        params = " ".join(m.group(2).split())
        out[m.group(1)] = 0 if params in ("", "void") else params.count(",") + 1
    return out


def test_binding_arity_matches_header(lib):
    """Every ctypes binding declares exactly as many argtypes as the header's
    prototype has parameters (amh_pooled_stats_k was bound with
    7 of its 8)."""
    ar = header_arity()
    assert sorted(ar) == header_symbols()
    L = lib.lib()
    for s, n in ar.items():
        at = getattr(L, s).argtypes
        assert at is not None, f"{s}: no argtypes bound"
        assert len(at) == n, f"{s}: binding has {len(at)} argtypes, amh.h declares {n} parameters"


def test_version(lib):
    assert lib.lib().amh_version() == 1


def test_calls_fail_cleanly_without_device(lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    L = lib.lib()
    h = ctypes.c_void_p()
    cfg = lib.AmhConfig(4, 0, 2 / 3, 0.234, 1e-6, (ctypes.c_int32 * 3)(0, 0, 0))
    assert L.amh_create(ctypes.byref(cfg), 0, ctypes.byref(h)) == -3  # AMH_EHIP
    assert L.amh_last_error(None)
    assert L.amh_step(None, 1, None, None, 1, None, None) == -1  # AMH_EINVAL: null handle
    bad = lib.AmhConfig(257, 0, 2 / 3, 0.234, 1e-6, (ctypes.c_int32 * 3)(0, 0, 0))
    assert L.amh_create(ctypes.byref(bad), 0, ctypes.byref(h)) == -1
    assert b"dim" in L.amh_last_error(None)
    # the pooled exchange's entry refuses a null handle / communicator before touching RCCL
    assert L.amh_pooled_allreduce(None, None, 17, None, None) == -1
    assert b"amh_pooled_allreduce" in L.amh_last_error(None)


def test_product_refuses_cpu_tensors(lib):
    import torch
    with pytest.raises(lib.AmhError):
        lib.require_gpu(torch.zeros(3))
