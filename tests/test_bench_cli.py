"""bench.py's rank handling (CPU): a rank whose launcher world size does not
match --gpus refuses to run, and the self-spawn path hands every child the
launcher environment (the children fail cleanly here, with no GPU)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=300, env=env)


def test_world_mismatch_refused():
    r = _run(["--gpus", "3"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "--gpus 3 but WORLD_SIZE=2" in (r.stderr + r.stdout)


def test_self_spawn_starts_n_ranks():
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0", "--no-extra"], {})
    assert r.returncode != 0  # no GPU in this container: the ranks stop at the device check
    # (the parent stops the other rank once one has failed, so it may not get to print)
    assert 1 <= (r.stderr + r.stdout).count("no GPU visible") <= 2
    assert "WORLD_SIZE" not in (r.stderr + r.stdout)  # the children got the launcher environment


def test_configs_names_checked_before_any_gpu_call():
    r = _run(["--configs", "diamonds,bogus"], {})
    assert r.returncode != 0
    assert "unknown ['bogus']" in (r.stderr + r.stdout)
    r = _run(["--configs", "diamonds", "--gpus", "2"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0


def test_library_overrides_refused():
    """Any AMH_* variable (a library path, the diagnostic build's A/B
    switches) stops the bench before it touches a GPU: the line always
    describes the release libamh.so."""
    for var, val in (("AMH_S64_MOVE_ONLY", "1"), ("AMH_LIB_PATH", "/tmp/x.so"), ("AMH_STEP64", "0")):
        r = _run(["--steps", "1", "--warmup", "0"], {var: val})
        assert r.returncode != 0
        assert f"unset {var}" in (r.stderr + r.stdout)
    # the release library ignores the switches whatever the environment says
    src = open(os.path.join(ROOT, "adaptive-mcmc_amd", "csrc", "amh_kernels.hip")).read()
    i = src.index('getenv("AMH_S64_MOVE_ONLY")')
    assert src.rfind("#ifdef AMH_DIAG", 0, i) > src.rfind("#endif", 0, i)
