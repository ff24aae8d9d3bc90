"""bench.py --gpus N without a launcher starts N ranks itself (RANK = LOCAL_RANK = device,
WORLD_SIZE = N, 127.0.0.1 rendezvous) and rank 0 prints one line; a --gpus that disagrees with a
launcher's WORLD_SIZE fails loudly.  CPU (gloo) rehearsal of the plumbing the driver's 1/2/4/8-GPU
runs use; the GPU work itself is the same code as N = 1."""
import json
import os
import subprocess
import sys

from conftest import REPO

BENCH = os.path.join(REPO, "bench.py")


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def test_bench_self_launches_ranks():
    out = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--selftest-ranks"], env=_env(), capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout          # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["ranks_local"] == [0]
    assert abs(d["max_t"] - 0.02) < 1e-12       # the slowest rank's time


def test_bench_rejects_gpus_world_size_mismatch():
    env = _env()
    env.update(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, BENCH, "--gpus", "1"], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode != 0 and "WORLD_SIZE=2" in out.stderr


def test_cpu_baseline_fields_on_cpu():
    """The cpu_baseline leg (the oracle timed on the host, rank 0 at N = 1) on a small image: a
    positive median rate over three repeats, their spread, the process's CPU use per repeat and
    the cgroup throttling field (None where cpu.stat is not readable)."""
    import numpy as np
    sys.path[:0] = [REPO, os.path.join(REPO, "pnp-pds_amd")]
    import bench
    from oracle import pnp_oracle as O
    from pnppds.operators import load_blur_kernel
    cfg = dict(bench.CONFIGS["cfg2"])
    h = load_blur_kernel("blur_1")
    xt = np.random.default_rng(0).random((3, 32, 32)).astype(np.float32)
    obs, x0 = O.make_observation(xt, "blur", h, 0.8, 0.01, 0.0, False, 300.0)
    rate, sample, psnr, info = bench.cpu_baseline(cfg, xt, obs.astype(np.float32), x0.astype(np.float32), h, 1.0, 8)
    assert rate > 0 and len(info["repeat_rates"]) == 3 and info["spread"] >= 0
    assert len(info["cpu_use_of_threads"]) == 3 and all(u > 0 for u in info["cpu_use_of_threads"])
    assert "cgroup_throttled_s" in info and "3 repeats" in sample
