"""bench.py launcher plumbing (CPU only): `--gpus N` without a launcher starts N ranks itself,
and a launcher whose WORLD_SIZE disagrees with --gpus is refused.  --dry-run stops every rank
right after the world-size check, before any GPU or model work."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(kw)
    return env


def test_gpus_n_spawns_n_ranks():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--dry-run"], env=_env(), capture_output=True,
                       text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [json.loads(s) for s in p.stdout.splitlines() if s.startswith("{")]
    assert sorted(d["rank"] for d in lines) == [0, 1, 2]
    assert all(d["world"] == 3 for d in lines)


def test_world_size_mismatch_is_refused():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run"],
                       env=_env(WORLD_SIZE="3", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True,
                       timeout=120)
    assert p.returncode == 2
    assert "WORLD_SIZE=3" in p.stderr


def test_single_gpu_runs_in_process():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--dry-run"], env=_env(), capture_output=True,
                       text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    assert json.loads(p.stdout.strip()) == {"rank": 0, "world": 1}
