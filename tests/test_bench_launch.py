"""bench.py --gpus N outside a launcher starts N ranks itself (one process per
GPU, torch.distributed.run as a child process) instead of silently running
one rank.  SFM_BENCH_LAUNCH_CHECK makes every rank report
its rendezvous and exit before any GPU work, so this runs on CPU."""
import json
import os
import subprocess
import sys

import pytest

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


def _bench_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)   # module level: argument helpers and the ABI binding only (no GPU work)
    return m


def test_loop_replica_line():
    """C5 at N > 1 is N independent sequences: the
    aggregate is named as such, over the slowest replica, with every
    replica's own rate beside it."""
    b = _bench_module()
    r = {"metric": "C5 incremental loop images/sec, fixed write-back", "value": 30.0, "seconds": 10.0,
         "unit": "images/s", "ba_calls": 299}
    out = b.loop_replica_line(r, [10.0, 12.0, 11.0, 10.5], 300)
    assert out["replicas"] == 4 and out["seconds"] == 12.0
    assert abs(out["value"] - 4 * 300 / 12.0) < 1e-9
    assert out["per_replica_images_per_sec"] == [30.0, 25.0, 300 / 11.0, 300 / 10.5]
    assert out["slowest_replica_images_per_sec"] == 25.0
    assert "aggregate of 4 independent replicas" in out["metric"] and out["scaling"].startswith("weak")
    assert out["ba_calls"] == 299 and r["value"] == 30.0   # the rank's own line is not modified


@pytest.mark.gpu
def test_loop_replicas_two_ranks_one_gpu():
    """bench.py's N > 1 loop branch end to end on one GPU: two ranks (the
    RCCL communicator cannot span one device twice, so the BA exchange falls
    back to the gloo hook, which the line names), each running its own short
    sequence; rank 0 prints one line whose loop entry is the replica
    aggregate."""
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["SFM_BENCH_SAME_DEVICE"] = "1"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "1", "--warmup", "0", "--n-cam", "40", "--n-pt", "4000",
           "--loop-images", "12", "--allow-host-allreduce", "--no-match", "--no-snavely", "--no-radial3",
           "--no-filter", "--no-dense", "--no-pmc", "--no-cpu-baseline"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = lines[0]
    assert line["n_gpus"] == 2 and "gloo" in line["config"]["transport"]
    lp = line["loop_fixed_writeback"]
    assert lp["replicas"] == 2 and len(lp["per_replica_images_per_sec"]) == 2
    assert abs(lp["value"] - 2 * 12 / lp["seconds"]) < 1e-6
    assert lp["kept_images"] >= 10 and lp["ba_calls"] == 11
