"""bench.py --gpus N without a launcher starts N ranks itself (RANK = LOCAL_RANK = device,
WORLD_SIZE = N, 127.0.0.1 rendezvous) and rank 0 prints one line; a --gpus that disagrees with a
launcher's WORLD_SIZE fails loudly.  CPU (gloo) rehearsal of the plumbing the driver's 1/2/4/8-GPU
runs use; the GPU work itself is the same code as N = 1."""
import json
import os
import subprocess
import sys
import time

import pytest

from conftest import REPO

sys.path[:0] = [REPO]

BENCH = os.path.join(REPO, "bench.py")


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


@pytest.mark.parametrize("n", [2, 4, 8])
def test_bench_self_launches_ranks(n):
    """The driver's 1/2/4/8-GPU shapes: one line from rank 0 carrying n_gpus = N, the weak-scaling
    label, global_batch = 256 N and value = 256 N K / the slowest rank's time."""
    K = 5
    out = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--steps", str(K), "--warmup", "1",
                          "--selftest-ranks"], env=_env(), capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout          # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["ranks_local"] == [0]
    t = 0.01 * n * K                            # the slowest rank's time
    assert abs(d["max_t"] - t) < 1e-12
    assert d["scaling"] == "weak" and d["config"]["global_batch"] == 256 * n
    import bench
    assert d["metric"] == bench.METRIC          # the BASELINE.json metric string at 256 RGB 256^2 per GPU
    assert abs(d["value"] - 256 * n * K / t) < 0.01 and d["steps"] == K and d["warmup"] == 1
    assert d["config"]["parallelism"].startswith(f"dp{n} ")


def test_bench_failing_rank_stops_the_others():
    """One rank fails before the first barrier: the launcher stops the ranks waiting there and
    exits with the failing rank's status, without a line."""
    t0 = time.time()
    out = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--selftest-ranks", "--selftest-fail-rank", "2"],
                         env=_env(), capture_output=True, text=True, timeout=300)
    assert out.returncode == 3, (out.returncode, out.stderr[-2000:])
    assert not [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert "stopping the others" in out.stderr
    assert time.time() - t0 < 120


def test_bench_rejects_gpus_world_size_mismatch():
    env = _env()
    env.update(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, BENCH, "--gpus", "1"], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode != 0 and "WORLD_SIZE=2" in out.stderr


def test_cpu_baseline_fields_on_cpu():
    """The cpu_baseline leg (the oracle timed on the host, rank 0 at N = 1) on a small image: a
    thread sweep with two runs per thread count, each with its rate, CPU use and cgroup
    throttling (None where cpu.stat is not readable); the value is the best run, the median and
    the thread count at the best run are reported."""
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
    sweep = bench.thread_sweep(info["threads_used"])
    assert len(info["sweep"]) == 3 * len(sweep) and [r["threads"] for r in info["sweep"]] == 3 * sweep
    assert rate == max(r["rate"] for r in info["sweep"]) and rate > 0
    assert info["best_threads"] in sweep and 0 < info["median"] <= rate and info["spread"] >= 0
    assert all(r["cpu_use_of_threads"] > 0 for r in info["sweep"])
    assert "cgroup_throttled_s" in info and "3 interleaved rounds" in sample
    assert psnr is not None and len(psnr) == info["sweep"][-1]["iters"]


def test_thread_sweep():
    import bench
    assert bench.thread_sweep(16) == [4, 8, 12, 16]
    assert bench.thread_sweep(10) == [4, 8, 10]
    assert bench.thread_sweep(2) == [2]


def test_cpu_baseline_cfg5_crop_scaled():
    """comparisonB-2 at more than 256^2: one outer iteration timed on the 256^2 crop at the config's
    m1 / m2 and scaled by pixels (here a 320^2 image, m1 = 2, m2 = 1 to keep the CPU test short)."""
    import numpy as np
    sys.path[:0] = [REPO, os.path.join(REPO, "pnp-pds_amd")]
    import bench
    from oracle import pnp_oracle as O
    from pnppds.operators import load_blur_kernel
    cfg = dict(bench.CONFIGS["cfg5"], m1=2, m2=1)
    h = load_blur_kernel("blur_1")
    xt = np.random.default_rng(1).random((3, 320, 320)).astype(np.float32)
    obs, x0 = O.make_observation(xt, "blur", h, 0.8, 0.01, 0.1, False, 300.0)
    rate, sample, psnr, info = bench.cpu_baseline(cfg, xt, obs.astype(np.float32), x0.astype(np.float32), h, 0.5, 2)
    assert rate > 0 and psnr is None
    assert "256x256 crop" in sample and "x1.5625" in sample
