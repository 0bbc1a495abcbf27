"""Host sanitizer run of the C oracle (race detection /
sanitizers): `make -C oracle asan` builds amh_oracle.c with AddressSanitizer
and UBSan (-fno-sanitize-recover, so undefined behaviour aborts), and the
oracle's own CPU tests run against that build in a child python with libasan
preloaded.  Every oracle entry point those tests reach (init, single / fused
/ large-d steps, pooled stats and updates per step and per K, ASSS, the
float64 restatement comparisons, the golden trajectories) runs instrumented;
the slowest statistical cases are left out to keep the CPU suite short."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _asan_runtime():
    try:
        p = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True, check=True)
    except (OSError, subprocess.CalledProcessError):
        return None
    path = p.stdout.strip()
    return path if os.path.isabs(path) and os.path.exists(path) else None


def test_oracle_under_asan_ubsan():
    rt = _asan_runtime()
    if rt is None:
        pytest.skip("gcc's libasan is not available")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"], check=True)
    env = dict(os.environ)
    env.update(LD_PRELOAD=rt, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1",
               AMH_ORACLE_LIB=os.path.join(ROOT, "oracle", "build", "libamh_oracle_asan.so"))
    slow = ("diamonds_suffstat_same_chain_statistics or eight_schools_posterior or two_ranks "
            "or eight_schools-2-10 or pooled_adaptation_converges")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", "-p", "no:xdist",
                        "tests/test_oracle.py", "tests/test_pooled.py", "tests/test_asss.py", "tests/test_golden.py",
                        "-k", f"not ({slow})"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    tail = (r.stdout + r.stderr)[-4000:]
    assert r.returncode == 0, tail
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, tail
