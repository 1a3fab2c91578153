"""bench.py's multi-rank launch on CPU (gloo): `python bench.py --gpus N`
with no launcher starts N worker processes itself (spawn_ranks) and prints
one JSON line with N per-GPU rows; the same script under torchrun does the
same. --dry-run runs the launch and bookkeeping collectives only (no GPU)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(cmd, timeout=180):
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "CFWS_BENCH_LAUNCHER"):
        env.pop(k, None)
    return subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)


def _one_line(out: str) -> dict:
    lines = [ln for ln in out.splitlines() if ln.strip()]
    assert len(lines) == 1, out          # stdout holds the JSON line and nothing else
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 8])
def test_spawn_without_launcher(n):
    p = _run([sys.executable, BENCH, "--gpus", str(n), "--dry-run", "--steps", "2", "--warmup", "1",
              "--frames", "256"])
    assert p.returncode == 0, p.stderr[-2000:]
    line = _one_line(p.stdout)
    assert line["n_gpus"] == n and line["launcher"] == "spawn" and line["verified"]
    assert [r["rank"] for r in line["per_gpu"]] == list(range(n))
    assert all(r["payload_bytes"] == 256 * 65536 for r in line["per_gpu"])


def test_same_script_under_torchrun():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    p = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
              "--master-addr", "127.0.0.1", "--master-port", str(port), BENCH, "--gpus", "2",
              "--dry-run", "--steps", "2", "--warmup", "1", "--frames", "256"])
    assert p.returncode == 0, p.stderr[-2000:]
    line = _one_line(p.stdout)
    assert line["n_gpus"] == 2 and line["launcher"] == "torchrun"
    assert len(line["per_gpu"]) == 2


def test_spawned_ranks_fail_loudly_without_gpus():
    """A real workload on a box with no GPU: every rank exits non-zero, so
    the launching process does too, and prints no line."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("has a GPU")
    p = _run([sys.executable, BENCH, "--gpus", "2", "--steps", "1", "--warmup", "0"])
    assert p.returncode != 0
    assert p.stdout.strip() == ""
    assert "has no GPU" in p.stderr


def test_signalled_launcher_ends_its_ranks():
    """A time limit that signals the launching process (SIGTERM) ends the
    ranks it started as well: none is left running."""
    import signal
    import time

    import psutil
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "CFWS_BENCH_LAUNCHER"):
        env.pop(k, None)
    p = subprocess.Popen([sys.executable, BENCH, "--gpus", "2", "--dry-run", "--steps", "100000", "--warmup", "0",
                          "--frames", "65536"], cwd=ROOT, env=env, stdout=subprocess.DEVNULL,
                         stderr=subprocess.DEVNULL)
    try:
        kids = []
        for _ in range(300):
            kids = psutil.Process(p.pid).children()
            if len(kids) == 2:
                break
            time.sleep(0.1)
        assert len(kids) == 2
        time.sleep(1.0)
        p.send_signal(signal.SIGTERM)
        assert p.wait(timeout=60) == 128 + signal.SIGTERM
        gone, alive = psutil.wait_procs(kids, timeout=30)
        assert not alive
    finally:
        if p.poll() is None:
            p.kill()
