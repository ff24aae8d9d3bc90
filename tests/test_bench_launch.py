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
