"""bench.py --gpus N starts its own ranks: without a
launcher in the environment it runs torch.distributed.run with N processes on
127.0.0.1 and relays rank 0's JSON line.  The stub worker (--stub) forms the
process group over gloo and checks the world size; no GPU is touched."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    return env


@pytest.mark.parametrize("n", [2, 3])
def test_bench_self_launches_n_ranks(n):
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--stub"],
                       capture_output=True, text=True, timeout=300, env=_env(), cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout        # rank 0 only
    res = json.loads(lines[0])
    assert res["world_size"] == n and res["backend"] == "gloo"
    assert res["rank_sum"] == n * (n + 1) / 2


def test_bench_rejects_world_size_mismatch():
    env = _env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--stub"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert p.returncode == 2, (p.returncode, p.stderr[-1000:])
    assert "WORLD_SIZE=1" in p.stderr
