"""bench.py's own N-rank launcher (`python bench.py --gpus N` without WORLD_SIZE): the parent
starts N child ranks with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, the ranks agree on
the world size, and any rank's failure makes the launcher exit non-zero.  CPU only: the
children join a gloo group in --dry-launch mode (no model, no GPU)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*extra, timeout=240):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.pop("LOCAL_RANK", None)
    env.pop("MASTER_PORT", None)
    env["TVQ_BENCH_BACKEND"] = "gloo"
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *extra],
                          env=env, capture_output=True, text=True, timeout=timeout, cwd=ROOT)


def test_launcher_two_ranks_agree():
    p = _run("--gpus", "2", "--dry-launch")
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 alone prints
    out = json.loads(lines[0])
    assert out["dry_launch"] and out["world_size"] == 2 and out["backend"] == "gloo"
    assert out["ranks"] == [0, 1]


def test_launcher_three_ranks_agree():
    p = _run("--gpus", "3", "--dry-launch")
    assert p.returncode == 0, p.stderr[-2000:]
    out = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert out["world_size"] == 3 and out["ranks"] == [0, 1, 2]


def test_launcher_rank_failure_is_nonzero():
    p = _run("--gpus", "2", "--dry-launch", "--dry-fail-rank", "1", timeout=120)
    assert p.returncode != 0
    assert "rank 1 exited" in p.stderr, p.stderr[-2000:]
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def test_world_size_mismatch_is_refused():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert p.returncode != 0 and "WORLD_SIZE=1" in p.stderr
