"""bench.py --gpus N without a launcher starts its N rank processes itself
(one per GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, never exec),
relays rank 0's JSON line and fails when a rank fails.  CPU dry run over
gloo: the launch and timing contract without a device."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*extra, timeout=180):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", "--steps", "2",
                           "--warmup", "1", *extra], capture_output=True, text=True, timeout=timeout, env=env)


def test_launcher_starts_n_ranks():
    p = _run("--gpus", "2")
    assert p.returncode == 0, p.stderr[-2000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2
    assert line["ranks_seen"] == 2
    assert line["ranks"] == [0, 1]
    assert line["steps"] == 2 and line["ms_per_step"] > 0


def test_launcher_single_rank_runs_inline():
    p = _run("--gpus", "1")
    assert p.returncode == 0, p.stderr[-2000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 1 and line["ranks"] == [0]


def test_launcher_fails_when_a_rank_fails():
    p = _run("--gpus", "2", "--dry-fail-rank", "1")
    assert p.returncode != 0
