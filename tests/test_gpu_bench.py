"""bench.py on the GPU box: the driver's single-GPU command shape, and
`--gpus 2` on the box's one GPU (the script starts its two ranks itself; they
share the device and exchange over gloo) prints n_gpus 2 with the config-5
pooled workload (BASELINE configs[4], at reduced chain count)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, timeout=110):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       timeout=timeout, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_two_ranks_one_gpu(gpu):
    j = _bench(["--gpus", "2", "--steps", "8", "--warmup", "2", "--chains", "8192", "--no-extra"])
    assert j["n_gpus"] == 2 and j["steps"] == 8
    assert "configs[4]" in j["config"]["workload"] and "gloo" in j["config"]["parallelism"]
    assert j["pooled"]["chains_total"] == 2 * 8192 and j["pooled"]["sync_every"] == 1
    assert j["value"] > 0 and j["roofline"]["unit"] == "TFLOP/s"


@pytest.mark.timeout(600)
def test_bench_eight_ranks_config5_shape(gpu):
    """`bench.py --gpus 8` at config 5's own shape (8 x 65,536 chains) on the
    box's one GPU, every sub-leg included: the weak pooled headline, K = 16,
    lag-one overlap, the strong-scaling forms over 524,288 chains in total
    and regime A.  The ranks share the device over
    gloo, so the numbers are not a scaling measurement."""
    j = _bench(["--gpus", "8", "--steps", "8", "--warmup", "2"], timeout=540)
    assert j["n_gpus"] == 8 and "gloo" in j["config"]["parallelism"]
    assert j["pooled"]["chains_total"] == 8 * 65536 and j["pooled"]["chains_per_gpu"] == 65536
    for leg in ("pooled_sync_every_16", "pooled_overlap", "strong_pooled", "strong_pooled_sync_every_16", "regime_a"):
        assert leg in j and j[leg]["value"] > 0, leg
    assert j["strong_pooled"]["chains_total"] == 524288 and j["strong_pooled"]["chains_per_gpu"] == 65536
    assert j["strong_pooled_sync_every_16"]["sync_every"] == 16


def test_bench_one_gpu_headline(gpu):
    j = _bench(["--steps", "5", "--warmup", "2", "--chains", "4096", "--no-extra"])
    assert j["n_gpus"] == 1 and "configs[1]" in j["config"]["workload"]
    assert j["roofline"]["bound"] == "hbm" and 0 < j["roofline"]["frac"] < 1.2
