"""bench.py's multi-GPU launch plumbing on the CPU (no GPU call): `--gpus N` run directly starts N
rank processes itself, under a torch.distributed launcher it takes the launcher's ranks, and a
launcher world that differs from --gpus is refused. `--dry-run` stops before any GPU call after
a gloo rendezvous of the ranks and prints what every rank saw."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR",
                                                              "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env.update(kw)
    return env


def _line(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [1, 2, 4])
def test_gpus_n_launches_n_ranks(n):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--dry-run"], capture_output=True, text=True,
                       timeout=180, env=_env())
    assert r.returncode == 0, r.stderr[-3000:]
    d = _line(r.stdout)
    assert d["dry_run"] and d["n_gpus"] == n and d["gpus_requested"] == n
    assert [x["rank"] for x in d["ranks"]] == list(range(n))
    assert [x["local_rank"] for x in d["ranks"]] == list(range(n))      # one GPU per rank
    assert all(x["world_size"] == n for x in d["ranks"])
    if n > 1:
        assert len({x["master"] for x in d["ranks"]}) == 1 and d["ranks"][0]["master"].startswith("127.0.0.1:")
    # configs[3]'s PER phase times the loop learn_and_update runs at this rank count
    assert d["per_loop"] == ("update_rows_n_per_dp" if n > 1 else "update_rows_n_per")


def test_torchrun_world_is_taken_as_is():
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29731", BENCH, "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=180, env=_env())
    assert r.returncode == 0, r.stderr[-3000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 2 and [x["rank"] for x in d["ranks"]] == [0, 1]


def test_world_mismatch_is_refused():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--dry-run"], capture_output=True, text=True,
                       timeout=120, env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"))
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_failing_rank_fails_the_launch():
    """A rank that exits non-zero ends the launch with its code; the ranks left waiting in the
    rendezvous are killed, not waited for."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--dry-run"], capture_output=True, text=True,
                       timeout=180, env=_env(CACTO_DRYRUN_FAIL_RANK="1"))
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert "rank 1 exited with 3" in r.stderr


def test_hanging_rank_is_killed_at_the_timeout():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run", "--launch-timeout", "8"],
                       capture_output=True, text=True, timeout=180, env=_env(CACTO_DRYRUN_HANG_RANK="0"))
    assert r.returncode == 124
    assert "killing them" in r.stderr
