"""bench.py's one-command multi-GPU launch (CPU): `python bench.py --gpus N` without
torchrun starts N rank processes through torchrun on 127.0.0.1 before anything touches a
GPU, and exits with their status.  `--probe-launch` makes each rank report its rank and
world size and stop before importing torch, so the relaunch path runs here end to end."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def test_gpus_n_without_torchrun_spawns_ranks():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--probe-launch",
                        "--steps", "2"], capture_output=True, text=True, env=_env(), timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert sorted(x["rank"] for x in lines) == [0, 1, 2]
    assert all(x["world"] == 3 and x["gpus"] == 3 for x in lines)
    assert sorted(x["local_rank"] for x in lines) == [0, 1, 2]
    assert "launching 3 ranks" in r.stderr


def test_single_gpu_probe_runs_in_process():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--probe-launch"], capture_output=True,
                       text=True, env=_env(), timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stdout.strip()) == {"rank": 0, "world": 1, "local_rank": 0, "gpus": 1}
    assert "launching" not in r.stderr


def test_world_size_mismatch_is_an_error():
    env = _env()
    env.update(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], capture_output=True,
                       text=True, env=env, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE 2" in r.stderr

