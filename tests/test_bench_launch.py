"""bench.py --gpus N outside a launcher starts N ranks itself (one process per
GPU, torch.distributed.run as a child process) instead of silently running
one rank.  SFM_BENCH_LAUNCH_CHECK makes every rank report
its rendezvous and exit before any GPU work, so this runs on CPU."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, extra_env=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["SFM_BENCH_LAUNCH_CHECK"] = "1"
    env.update(extra_env or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env, capture_output=True,
                       text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    return [json.loads(line) for line in r.stdout.splitlines() if line.startswith("{")]


def test_self_launch_spawns_n_ranks():
    rows = _run(["--gpus", "2", "--steps", "1"])
    assert sorted(r["rank"] for r in rows) == [0, 1]
    assert all(r["world"] == 2 and r["gpus"] == 2 for r in rows)
    assert sorted(r["local_rank"] for r in rows) == [0, 1]


def test_single_gpu_runs_in_process():
    rows = _run(["--gpus", "1"])
    assert rows == [{"rank": 0, "world": 1, "local_rank": 0, "gpus": 1}]
