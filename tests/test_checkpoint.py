"""Checkpoint helpers on the host (kernels_amd.checkpoint): state_dict /
load_state_dict / save_state / load_state round trips for every state kind,
with no pickles in the file (np.load(allow_pickle=False))."""
import numpy as np
import pytest
import torch


@pytest.mark.parametrize("kind", ["ARWMHState", "ASSSState", "PooledState"])
def test_roundtrip(kind, tmp_path):
    import kernels_amd as K
    cls, acls = {"ARWMHState": (K.ARWMHState, K.ARWMHAdaptState), "ASSSState": (K.ASSSState, K.ASSSAdaptState),
                 "PooledState": (K.PooledState, K.PooledAdaptState)}[kind]
    g = torch.Generator().manual_seed(1)
    leaves = [torch.randn(5, 3, generator=g) for _ in cls._fields if _ != "adapt_state"]
    ad = acls(*[torch.randint(-9, 9, (5, 2), dtype=torch.int32, generator=g) for _ in acls._fields])
    it = iter(leaves)
    st = cls(*[ad if f == "adapt_state" else next(it) for f in cls._fields])
    sd = K.state_dict(st)
    assert str(sd["__kind__"]) == kind
    back = K.load_state_dict(sd, "cpu")
    assert type(back) is cls
    for a, b in zip(torch.utils._pytree.tree_leaves(st), torch.utils._pytree.tree_leaves(back)):
        assert a.dtype == b.dtype and torch.equal(a, b)
    p = str(tmp_path / "s.npz")
    K.save_state(p, st, accept_count=torch.arange(5))
    with np.load(p, allow_pickle=False) as f:
        assert "accept_count" in f.files and str(f["__kind__"]) == kind
    back = K.load_state(p, "cpu")
    for a, b in zip(torch.utils._pytree.tree_leaves(st), torch.utils._pytree.tree_leaves(back)):
        assert torch.equal(a, b)


def test_path_suffix_and_extras(tmp_path):
    """save_state appends ".npz" as np.savez does and load_state finds it;
    extra arrays come back with with_extras=True."""
    import kernels_amd as K
    st = K.ARWMHState(torch.zeros(3, dtype=torch.int32), torch.ones(3, 2), torch.zeros(3), torch.zeros(3),
                      K.ARWMHAdaptState(torch.zeros(3, 2), torch.ones(3, 3), torch.zeros(3)), torch.zeros(3),
                      torch.zeros(3, 2, dtype=torch.int32))
    p = K.save_state(str(tmp_path / "run"), st, accept_count=torch.arange(3, dtype=torch.int32))
    assert p.endswith("run.npz")
    back, extra = K.load_state(str(tmp_path / "run"), "cpu", with_extras=True)
    assert torch.equal(back.z, st.z) and list(extra) == ["accept_count"]
    assert np.array_equal(extra["accept_count"], np.arange(3))
    with pytest.raises(ValueError):
        K.save_state(str(tmp_path / "x"), st, z=torch.zeros(1))
    sd = K.state_dict(st)
    sd["__pooled_pending_sums__"] = np.zeros(4)
    with pytest.raises(ValueError):
        K.load_state_dict(sd, "cpu")  # pending pooled sums need the continuing kernel


def test_rejects_unknown():
    import kernels_amd as K
    with pytest.raises(TypeError):
        K.state_dict((torch.zeros(1),))
    with pytest.raises(ValueError):
        K.load_state_dict({"__kind__": np.array("Nope")}, "cpu")
