"""bench.py --gpus N: the parent spawns N ranks (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*) before any
GPU work, relays rank 0's JSON line and fails when any rank fails.  Exercised on CPU with the
gloo 'dp_stub' workload (same bootstrap, barrier + max-over-ranks timing, JSON contract)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=240):
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=timeout)


def test_launcher_spawns_ranks_and_reports_world():
    p = _run(["--gpus", "3", "--workload", "dp_stub", "--steps", "4", "--warmup", "1"])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 3 and out["config"]["parallelism"] == "dp3"
    assert abs(out["mean"] - 2.0) < 1e-6          # mean of 1, 2, 3 over the three ranks
    assert out["steps"] == 4 and out["value"] > 0


def test_launcher_fails_when_a_rank_fails():
    p = _run(["--gpus", "2", "--workload", "dp_stub", "--steps", "2"], {"PCV_BENCH_FAIL_RANK": "1"})
    assert p.returncode != 0
    assert "injected failure" in p.stderr


def test_world_size_must_match_gpus():
    p = _run(["--gpus", "2", "--workload", "dp_stub"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0 and "WORLD_SIZE=1" in p.stderr
