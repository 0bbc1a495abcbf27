"""Extract the raw float32 buffers of the reference's stored diamonds runs
into a data-only fixture, WITHOUT unpickling anything.

Sources (reference data files, read as bytes):
  /root/reference/python/mcmc_runs/diamonds-example-references.pkl
  /root/reference/python/mcmc_runs/diamonds-example-samples.pkl

They are the inputs of python/jupyter/wasserstein-computation.ipynb (cells
7-38), whose printed outputs are the only reference outputs that exist for
inputs available here.  Each file is a protocol-4 pickle of a dict
{name: jax Array}; every array is a numpy `_reconstruct` whose BUILD state is
(version, shape, dtype, fortran_order, raw bytes).

This script walks the opcode stream with `pickletools.genops` and evaluates
it on a tiny inert stack machine: GLOBAL / STACK_GLOBAL become plain
("global", module, name) tuples, REDUCE and BUILD become plain tuples, and no
callable is ever looked up or invoked.  Only the opcodes these files use are
accepted; anything else raises.  The arrays are then read back from the raw
bytes with numpy.frombuffer('<f4').

Finding: the references file reproduces cell 10's "reference" column (all 26
second moments to the printed 6 decimals).  The samples file does not
reproduce the "samples" column (26 of 26 columns differ; b[2]: 122.7 vs 29.6),
and its Hungarian distance at n = 30, d = 5 is 2.933 against the 0.596 of the
cell-31 table: the notebook evaluated an earlier samples file that the
reference no longer holds.

Column order: the notebook builds `references` / `samples` from the combined
frame's columns b[1..24], Intercept, sigma (cell 10 prints the E[X^2] table in
that order), so the fixture stores (10000, 26) matrices in that order.  The
cell-10 table is checked here before anything is written.

  python tests/golden/extract_diamonds_pkl.py   ->  tests/golden/diamonds_example.npz
"""
import os
import pickletools
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = "/root/reference/python/mcmc_runs/diamonds-example-{}.pkl"
OUT = os.path.join(HERE, "diamonds_example.npz")

# wasserstein-computation.ipynb cell 10: E[|X|^2] per column (reference, samples)
CELL10 = {
    "b[1]": (44.417422, 44.700661), "b[2]": (40.598356, 29.606578), "b[3]": (22.040444, 13.948840),
    "b[4]": (2.113180, 1.985428), "b[5]": (0.018108, 0.018292), "b[6]": (0.001659, 0.001652),
    "b[7]": (0.000552, 0.000467), "b[8]": (0.000024, 0.000020), "b[9]": (0.197932, 0.198012),
    "b[10]": (0.008616, 0.008529), "b[11]": (0.000186, 0.000184), "b[12]": (0.000138, 0.000142),
    "b[13]": (0.000022, 0.000023), "b[14]": (0.000018, 0.000019), "b[15]": (0.812011, 0.810522),
    "b[16]": (0.048908, 0.049238), "b[17]": (0.017276, 0.017382), "b[18]": (0.003388, 0.003382),
    "b[19]": (0.000363, 0.000363), "b[20]": (0.000030, 0.000032), "b[21]": (0.001026, 0.001040),
    "b[22]": (37.391151, 29.081815), "b[23]": (21.490083, 14.777230), "b[24]": (2.099530, 1.827760),
    "Intercept": (60.652883, 60.653602), "sigma": (0.015101, 0.015247),
}
COLUMNS = [f"b[{i}]" for i in range(1, 25)] + ["Intercept", "sigma"]

_MARK = object()


def _inert_eval(data: bytes):
    """Evaluate the opcode stream into inert tuples/dicts/bytes (no imports,
    no calls)."""
    stack, memo = [], {}

    def pop_mark():
        i = len(stack) - 1
        while stack[i] is not _MARK:
            i -= 1
        items = stack[i + 1:]
        del stack[i:]
        return items

    for op, arg, _pos in pickletools.genops(data):
        n = op.name
        if n in ("PROTO", "FRAME"):
            continue
        if n == "STOP":
            break
        if n == "EMPTY_DICT":
            stack.append({})
        elif n == "MEMOIZE":
            memo[len(memo)] = stack[-1]
        elif n in ("BINGET", "LONG_BINGET"):
            stack.append(memo[arg])
        elif n == "MARK":
            stack.append(_MARK)
        elif n in ("SHORT_BINUNICODE", "BINUNICODE", "SHORT_BINBYTES", "BINBYTES", "BININT1", "BININT2", "BININT"):
            stack.append(arg)
        elif n == "NONE":
            stack.append(None)
        elif n == "NEWTRUE":
            stack.append(True)
        elif n == "NEWFALSE":
            stack.append(False)
        elif n == "STACK_GLOBAL":
            name = stack.pop()
            mod = stack.pop()
            stack.append(("global", mod, name))
        elif n == "TUPLE":
            stack.append(tuple(pop_mark()))
        elif n in ("TUPLE1", "TUPLE2", "TUPLE3"):
            k = int(n[-1])
            items = tuple(stack[-k:])
            del stack[-k:]
            stack.append(items)
        elif n == "EMPTY_TUPLE":
            stack.append(())
        elif n == "REDUCE":
            args = stack.pop()
            fn = stack.pop()
            stack.append(("reduce", fn, args))
        elif n == "BUILD":
            state = stack.pop()
            obj = stack.pop()
            stack.append(("build", obj, state))
        elif n == "SETITEM":
            v = stack.pop()
            k = stack.pop()
            stack[-1][k] = v
        elif n == "SETITEMS":
            items = pop_mark()
            d = stack[-1]
            for k, v in zip(items[0::2], items[1::2]):
                d[k] = v
        else:
            raise ValueError(f"opcode {n} not expected in these files")
    assert len(stack) == 1 and isinstance(stack[0], dict)
    return stack[0]


def _array(node) -> np.ndarray:
    """jax _reconstruct_array(np._reconstruct, (ndarray, (0,), b), state, aux):
    state = (version, shape, dtype, fortran_order, raw bytes)."""
    assert node[0] == "reduce" and node[1] == ("global", "jax._src.array", "_reconstruct_array"), node[:2]
    fn, base_args, state, _aux = node[2]
    assert fn == ("global", "numpy._core.multiarray", "_reconstruct")
    assert base_args[0] == ("global", "numpy", "ndarray")
    _version, shape, dtype, fortran, raw = state
    if dtype[0] == "build":  # first use is BUILT with the byte-order state; later uses come from the memo
        assert dtype[2][1] == "<", dtype
        dtype = dtype[1]
    assert dtype[0] == "reduce" and dtype[1] == ("global", "numpy", "dtype") and dtype[2][0] == "f4", dtype
    assert fortran is False and isinstance(raw, (bytes, bytearray))
    shape = tuple(shape) if isinstance(shape, tuple) else (shape,)
    return np.frombuffer(bytes(raw), dtype="<f4").reshape(shape).astype(np.float32)


def load(which: str) -> dict:
    with open(SRC.format(which), "rb") as f:
        data = f.read()
    return {k: _array(v) for k, v in _inert_eval(data).items()}


def matrix(d: dict) -> np.ndarray:
    cols = []
    for name in COLUMNS:
        if name.startswith("b["):
            cols.append(d["b"][:, int(name[2:-1]) - 1])
        else:
            cols.append(d[name])
    return np.stack(cols, axis=1).astype(np.float32)


def cell10_mismatch(x: np.ndarray, side: int):
    """Columns whose E[X^2] differs from cell 10's printed value (6 decimals)."""
    m = np.mean(x.astype(np.float64) ** 2, axis=0)
    bad = []
    for j, name in enumerate(COLUMNS):
        want = CELL10[name][side]
        if abs(m[j] - want) > 6e-7 + 1e-6 * abs(want):
            bad.append((name, float(m[j]), want))
    return bad


def main():
    ref = matrix(load("references"))
    smp = matrix(load("samples"))
    assert ref.shape == smp.shape == (10000, 26)
    bad = cell10_mismatch(ref, 0)
    if bad:
        sys.exit(f"references do not reproduce cell 10: {bad[:3]}")
    # The stored samples file is NOT the draw set the notebook evaluated (its
    # b[2] second moment is 122.7 against cell 10's 29.6), so every
    # samples-dependent printed value (cells 12, 19, 21-24, 38, 31) is
    # unreachable from the files the reference holds.  Recorded, not fatal.
    bad_s = cell10_mismatch(smp, 1)
    np.savez_compressed(OUT, references=ref, samples=smp, columns=np.array(COLUMNS))
    print(f"wrote {OUT}: references {ref.shape} reproduce cell 10 (26/26 columns); "
          f"stored samples differ from the notebook's in {len(bad_s)}/26 columns")


if __name__ == "__main__":
    main()
