"""The drop-in swap of INTEGRATION.md §1, performed verbatim on a stand-in of
the reference's package layout (python/kernels/__init__.py:1-3,
python/scripts/run_diamonds_lr_decay.py:13-14).

The reference itself cannot be imported here (JAX / NumPyro are absent,
SURVEY.md §8c), so the test writes the reference's `kernels` package as a
maintainer would leave it after the swap: lines 1-2 replaced by the
`kernels_amd` imports, line 3 (`from .numpyro_kernels import NUTS, ...`)
untouched, with a stand-in `numpyro_kernels` module because numpyro is
absent.  What is checked is the import resolution: the script's
`from kernels import ARWMH, ASSS, NUTS` must find the device ARWMH / ASSS
and the reference's own NUTS, i.e. nothing in adaptive-mcmc_amd/ shadows the
reference's `kernels` or `utils` packages."""
import os
import subprocess
import sys
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "adaptive-mcmc_amd")

# INTEGRATION.md §1, the two swapped lines (kept in sync by test_doc_snippet_matches)
SWAP = ("from kernels_amd import ARWMH, ARWMHState, ARWMHAdaptState\n"
        "from kernels_amd import ASSS, ASSSState, ASSSAdaptState\n")


def _make_reference_tree(tmp):
    py = os.path.join(tmp, "python")
    os.makedirs(os.path.join(py, "kernels"))
    os.makedirs(os.path.join(py, "utils"))
    with open(os.path.join(py, "kernels", "__init__.py"), "w") as f:
        f.write(SWAP + "from .numpyro_kernels import NUTS, HMCState, SA, SAState\n")
    with open(os.path.join(py, "kernels", "numpyro_kernels.py"), "w") as f:
        f.write("class NUTS: pass\nclass HMCState: pass\nclass SA: pass\nclass SAState: pass\n")
    with open(os.path.join(py, "utils", "__init__.py"), "w") as f:
        f.write("")
    with open(os.path.join(py, "utils", "evaluation.py"), "w") as f:
        f.write("REFERENCE_UTILS = True\n")
    return py


def test_no_top_level_shadowing():
    names = set(os.listdir(PKG))
    for ref_pkg in ("kernels", "utils"):  # the reference's top-level packages
        assert ref_pkg not in names and f"{ref_pkg}.py" not in names


def test_doc_snippet_matches():
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    for line in SWAP.splitlines():
        assert line in doc, line


def test_import_swap_verbatim(tmp_path):
    py = _make_reference_tree(str(tmp_path))
    # the scripts' order: MCMC_WORKDIR/python appended, the build ahead of it
    script = textwrap.dedent(f"""
        import sys
        sys.path.insert(0, {PKG!r})
        sys.path.append({py!r})
        from kernels import ARWMH, ASSS, NUTS                       # run_diamonds_lr_decay.py:13
        from kernels import ARWMHState, ARWMHAdaptState, SA
        from utils.evaluation import REFERENCE_UTILS                # the reference's utils stay reachable
        from utils_amd.kernel_utils import ns_logscale, collect_states_logscale
        import kernels, kernels_amd
        assert kernels.__file__.startswith({py!r}), kernels.__file__
        assert ARWMH is kernels_amd.ARWMH and ASSS is kernels_amd.ASSS
        assert NUTS.__module__ == "kernels.numpyro_kernels"
        assert list(ns_logscale(2)[:3]) == [1, 2, 3]
        import posteriors as P
        k = ARWMH(model=P.eight_schools, num_chains=4)              # constructor surface, no GPU call
        print("swap ok")
    """)
    r = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=300,
                       env={**os.environ, "PYTHONPATH": ""})
    assert r.returncode == 0, r.stderr[-3000:]
    assert "swap ok" in r.stdout
