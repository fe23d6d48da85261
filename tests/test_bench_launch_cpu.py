"""bench.py's world-size contract (CPU, gloo): `--gpus N` without a launcher
starts N ranks itself (torch.distributed.run as a child process) and prints
rank 0's line once; under a launcher WORLD_SIZE must equal --gpus."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["CUDA_VISIBLE_DEVICES"] = ""  # gloo even where a GPU exists
    env["HIP_VISIBLE_DEVICES"] = ""
    return env


def test_bench_gpus2_self_launches_two_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check"], env=_env(),
                       capture_output=True, text=True, timeout=180, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    d = json.loads(lines[0])
    assert d["launch_check"] and d["n_gpus"] == 2 and d["max_rank"] == 1
    assert d["backend"] == "gloo"


def test_bench_world_size_mismatch_fails():
    env = _env()
    env.update(WORLD_SIZE="3", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="1")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check"], env=env,
                       capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert r.returncode == 2
    assert "WORLD_SIZE=3" in r.stderr


def test_bench_gpus1_runs_in_process():
    """--gpus 1 keeps the single-process path (no launcher, no process group)."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--launch-check"], env=_env(),
                       capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert d["n_gpus"] == 1 and d["backend"] is None
