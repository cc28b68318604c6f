"""bench.py's multi-rank launcher on the CPU (gloo): `--gpus N` without torch.distributed.run spawns N rank
processes, every rank checks the process group size, a failing rank fails the run, and a launcher/--gpus
mismatch is an error."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=120):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=timeout)


@pytest.mark.parametrize("n", [2, 3])
def test_launcher_spawns_n_ranks(n):
    r = _run(["--gpus", str(n), "--dry-run", "--backend", "gloo"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1            # rank 0 alone prints the line
    line = json.loads(lines[0])
    assert line["n_gpus"] == n and line["dry_run"]


def test_failing_rank_fails_the_run():
    r = _run(["--gpus", "2", "--dry-run", "--backend", "gloo"], {"HISEG_BENCH_FAIL_RANK": "1"})
    assert r.returncode != 0
    assert "a rank failed" in r.stderr


def test_gpus_must_match_the_launcher_world():
    r = _run(["--gpus", "2", "--dry-run"], {"WORLD_SIZE": "1"})
    assert r.returncode == 2
    assert "WORLD_SIZE=1" in r.stderr
