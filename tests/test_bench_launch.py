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


def _selftest(n, K, *extra):
    out = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--steps", str(K), "--warmup", "1",
                          "--selftest-ranks", *extra], env=_env(), capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout          # rank 0 only
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 4, 8])
def test_bench_self_launches_ranks(n):
    """The driver's 1/2/4/8-GPU shapes: one line from rank 0 carrying n_gpus = N and, by default,
    strong scaling (the metric's global batch of 256 split as 256 / N contiguous
    images per rank), value = 256 K / the slowest rank's time; beside it the weak leg (256 per
    rank, 256 N in all) timed in the same run."""
    K = 5
    d = _selftest(n, K)
    assert d["n_gpus"] == n and d["ranks_local"] == [0]
    t = 0.01 * n * K                            # the slowest rank's time
    assert abs(d["max_t"] - t) < 1e-12
    assert d["scaling"] == "strong" and d["config"]["global_batch"] == 256
    assert d["config"]["images_per_gpu"] == [256 // n] * n
    import bench
    assert d["metric"] == bench.METRIC          # the BASELINE.json metric string: batch = 256 RGB 256^2
    assert abs(d["value"] - 256 * K / t) < 0.01 and d["steps"] == K and d["warmup"] == 1
    assert d["config"]["parallelism"].startswith(f"dp{n} ")
    w = d["weak_scaling"]
    tw = 0.02 * n * K
    assert w["scaling"] == "weak" and w["global_batch"] == 256 * n and w["images_per_gpu"] == 256
    assert abs(w["value"] - 256 * n * K / tw) < 0.01


@pytest.mark.parametrize("n", [2, 8])
def test_bench_weak_scaling_mode(n):
    """--scaling weak: every rank solves the config's 256 images, global_batch 256 N."""
    K = 3
    d = _selftest(n, K, "--scaling", "weak")
    t = 0.01 * n * K
    assert d["scaling"] == "weak" and d["config"]["global_batch"] == 256 * n
    assert d["config"]["images_per_gpu"] == [256] * n and "weak_scaling" not in d
    assert abs(d["value"] - 256 * n * K / t) < 0.01


def test_rank_shards_partition_the_global_batch():
    """Strong: contiguous shards covering the global batch once (256 over 1/2/4/8 ranks: 256 / N
    each); weak: rank r owns images [256 r, 256 (r + 1)); image i is the same array whichever rank
    generates it."""
    import numpy as np
    import bench
    for n in (1, 2, 4, 8, 3):
        spans = [bench.rank_shard(256, n, r, "strong") for r in range(n)]
        assert all(g == 256 for g, _, _ in spans)
        assert spans[0][1] == 0 and spans[-1][2] == 256
        assert all(a[2] == b[1] for a, b in zip(spans, spans[1:]))
        if 256 % n == 0:
            assert all(hi - lo == 256 // n for _, lo, hi in spans)
        assert [bench.rank_shard(256, n, r, "weak")[1:] for r in range(n)] == [(256 * r, 256 * (r + 1)) for r in range(n)]
    a = bench.synthetic_images(0, 4, 3, 64, 64)
    b = bench.synthetic_images(2, 3, 3, 64, 64)
    np.testing.assert_array_equal(a[2], b[0])
    with pytest.raises(SystemExit):
        bench.rank_shard(4, 8, 0, "strong")


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
    thread sweep in three rounds, each leg pinned to as many CPUs as it has threads, each run
    with its rate, CPU use, cgroup throttling (None where cpu.stat is not readable) and load;
    the value is the median at the thread count with the best median.  The process's affinity
    is restored afterwards."""
    before = os.sched_getaffinity(0)
    import numpy as np
    sys.path[:0] = [REPO, os.path.join(REPO, "pnp-pds_amd")]
    import bench
    from oracle import pnp_oracle as O
    from pnppds.operators import load_blur_kernel
    cfg = dict(bench.CONFIGS["cfg2"])
    h = load_blur_kernel("blur_1")
    xt = np.random.default_rng(0).random((3, 32, 32)).astype(np.float32)
    obs, x0 = O.make_observation(xt, "blur", h, 0.8, 0.01, 0.0, False, 300.0)
    rate, sample, psnr, info = bench.cpu_baseline(cfg, xt, obs.astype(np.float32), x0.astype(np.float32), h, 2.0, 8)
    sweep = bench.thread_sweep(info["threads_used"])
    if len(info["sweep"]) == 2:    # a loaded host: one iteration per run exceeds the budget -> all threads, 2 runs
        sweep, rounds = [sweep[-1]], 2
    else:
        rounds = 3
    assert len(info["sweep"]) == rounds * len(sweep) and [r["threads"] for r in info["sweep"]] == rounds * sweep
    at_best = [r["rate"] for r in info["sweep"] if r["threads"] == info["best_threads"]]
    assert rate == float(np.median(at_best)) and rate > 0 and len(at_best) == rounds
    assert rate == max(info["median_by_threads"].values()) and info["best_run"] >= rate
    assert info["best_threads"] in sweep and info["spread"] >= 0 and info["spread_at_best_threads"] >= 0
    assert all(r["cpu_use_of_threads"] > 0 and "loadavg_1m" in r and "throttle_cause" in r for r in info["sweep"])
    assert all(len(r["cpus"]) > 0 for r in info["sweep"])
    assert "cgroup_throttled_s" in info and f"{rounds} interleaved rounds" in sample and "pinned" in sample
    assert psnr is not None and len(psnr) == info["sweep"][-1]["iters"]
    assert os.sched_getaffinity(0) == before


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
