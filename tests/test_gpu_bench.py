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


def _bench(args):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       timeout=110, env=env)
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


def test_bench_one_gpu_headline(gpu):
    j = _bench(["--steps", "5", "--warmup", "2", "--chains", "4096", "--no-extra"])
    assert j["n_gpus"] == 1 and "configs[1]" in j["config"]["workload"]
    assert j["roofline"]["bound"] == "hbm" and 0 < j["roofline"]["frac"] < 1.2
