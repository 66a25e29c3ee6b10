"""bench.py's multi-GPU launcher on CPU (no GPU call): `--gpus N` without
torch.distributed.run spawns N rank processes with RANK / LOCAL_RANK / WORLD_SIZE set, and
they meet over gloo (the barrier and max-reduce of the timed region; no RCCL on the path)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_spawns_n_ranks(n):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n),
                          "--dry-run", "--no-cpu"], capture_output=True, text=True, timeout=240,
                         env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout  # one JSON line, from rank 0
    res = json.loads(lines[0])
    assert res["world"] == n
    assert [r["rank"] for r in res["ranks"]] == list(range(n))
    assert [r["local_rank"] for r in res["ranks"]] == list(range(n))
    assert len({r["pid"] for r in res["ranks"]}) == n
    # each rank's plan on its own GPU: rank r -> cuda:r on one node (no two ranks share a card)
    assert [r["plan_device"] for r in res["ranks"]] == list(range(n))


def test_torchrun_environment_is_honoured():
    """Under torch.distributed.run (the driver's N>1 launch) bench.py does not spawn again."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                          "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port", str(port),
                          os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run", "--no-cpu"],
                         capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    res = json.loads(lines[0])
    assert res["world"] == 2 and sorted(r["local_rank"] for r in res["ranks"]) == [0, 1]
    assert all(r["plan_device"] == r["local_rank"] for r in res["ranks"])


def test_failed_rank_ends_the_others():
    """A rank that dies before the barrier must not leave the others waiting in it: the
    launcher ends them and returns the failure."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env["BENCH_DRY_RUN_FAIL_RANK"] = "1"
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3",
                          "--dry-run", "--no-cpu"], capture_output=True, text=True, timeout=240,
                         env=env, cwd=ROOT)
    assert out.returncode != 0
    assert not [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
