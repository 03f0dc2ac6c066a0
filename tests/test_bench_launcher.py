"""bench.py --gpus N starts its own ranks:
without a launcher in the environment it counts the visible GPUs WITHOUT any
HIP call (KFD topology, else amdsmi; VISIBLE_DEVICES masks), runs
torch.distributed.run with N processes on 127.0.0.1 and relays rank 0's JSON
line.  The topology is a fake one here (BIH_KFD_TOPOLOGY): this container has
no GPU.  The stub worker (--stub) forms the process group over gloo and checks
the world size; without --stub the ranks run bench.py's real main() and, with
no device on this machine, stop at their own device check."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _topology(tmp_path, gpus, cpus=1):
    """A KFD topology directory with `cpus` CPU nodes and `gpus` GPU nodes."""
    root = tmp_path / "nodes"
    for k in range(cpus + gpus):
        d = root / str(k)
        d.mkdir(parents=True)
        simd = 0 if k < cpus else 1024
        (d / "properties").write_text(f"cpu_cores_count {64 if k < cpus else 0}\nsimd_count {simd}\n"
                                      f"gfx_target_version {0 if k < cpus else 90500}\n")
    return str(root)


def _env(topo=None):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "ROCR_VISIBLE_DEVICES",
                        "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "BIH_BENCH_SHARE_GPU")}
    env["OMP_NUM_THREADS"] = "1"
    if topo:
        env["BIH_KFD_TOPOLOGY"] = topo
    return env


def test_visible_gpu_count_reads_topology_and_masks(tmp_path, monkeypatch):
    import bench
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    monkeypatch.setenv("BIH_KFD_TOPOLOGY", _topology(tmp_path, 8, cpus=2))
    assert bench.visible_gpu_count() == 8          # CPU nodes (simd_count 0) do not count
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,3")
    assert bench.visible_gpu_count() == 2
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "")
    assert bench.visible_gpu_count() == 0
    monkeypatch.delenv("ROCR_VISIBLE_DEVICES")
    monkeypatch.delenv("HIP_VISIBLE_DEVICES")
    monkeypatch.setenv("BIH_KFD_TOPOLOGY", str(tmp_path / "missing"))
    n = bench.visible_gpu_count()                   # amdsmi, when importable, else None
    assert n is None or n >= 0


@pytest.mark.parametrize("n", [2, 3])
def test_bench_self_launches_n_ranks(n, tmp_path):
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--stub"],
                       capture_output=True, text=True, timeout=300, env=_env(_topology(tmp_path, n)), cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout        # rank 0 only
    res = json.loads(lines[0])
    assert res["world_size"] == n and res["backend"] == "gloo"
    assert res["rank_sum"] == n * (n + 1) / 2


def test_launcher_refuses_fewer_devices_than_ranks(tmp_path):
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--stub"],
                       capture_output=True, text=True, timeout=120, env=_env(_topology(tmp_path, 2)), cwd=ROOT)
    assert p.returncode == 2, (p.returncode, p.stderr[-1000:])
    assert "--gpus 4 but 2 devices are visible" in p.stderr


def test_launcher_real_ranks_without_stub(tmp_path):
    """The N > 1 branch with the real rank code (no --stub): the launcher's
    count passes (2 GPUs in the fake topology), torch.distributed.run starts
    both ranks, each runs main() up to its device check, which fails on this
    GPU-less machine; the launcher reports the failed run."""
    env = _env(_topology(tmp_path, 2))
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1",
                        "--warmup", "0"], capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert p.returncode != 0
    assert "bench.py: 2-rank run failed" in p.stderr, p.stderr[-2000:]
    for r in (0, 1):
        assert f"bench.py: rank {r}: LOCAL_RANK {r} but 0 devices are visible" in p.stderr, p.stderr[-2000:]


def test_bench_rejects_world_size_mismatch():
    env = _env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--stub"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert p.returncode == 2, (p.returncode, p.stderr[-1000:])
    assert "WORLD_SIZE=1" in p.stderr
