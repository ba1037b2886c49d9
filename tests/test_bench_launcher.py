"""bench.py's multi-GPU plumbing on the CPU (no GPU work): `bench.py --gpus N`
started without a launcher spawns N rank processes itself, the ranks meet over
the gloo control plane, exchange the RCCL unique id through the store and take
the max over ranks; a rank that dies stops the whole run with its exit code."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None, timeout=120):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=timeout, env=e, cwd=ROOT)


@pytest.mark.parametrize("n", [2, 4])
def test_launcher_spawns_n_ranks(n):
    r = _run(["--gpus", str(n), "--dry-run", "--steps", "3", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # ONE line, from rank 0
    assert r.stdout.strip() == lines[0], r.stdout  # and nothing else (gloo's banner goes to stderr)
    d = json.loads(lines[0])
    assert d["dry_run"] and d["n_gpus"] == n and d["max_over_ranks"] == float(n)
    assert d["steps"] == 3 and d["warmup"] == 1


def test_launcher_stops_the_run_when_a_rank_dies():
    r = _run(["--gpus", "3", "--dry-run"], env={"MEV_DRYRUN_FAIL_RANK": "1"}, timeout=90)
    assert r.returncode == 3
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_single_rank_dry_run():
    r = _run(["--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stdout.strip().splitlines()[-1])["n_gpus"] == 1


def test_config5_dry_run_over_8_ranks():
    """BASELINE config 5's plumbing: 8 ranks (one per GPU on the node) over the gloo control plane,
    128 beams, the gathered steps as the value."""
    r = _run(["--gpus", "8", "--config", "5", "--dry-run", "--steps", "3", "--warmup", "1"], timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["n_gpus"] == 8 and d["max_over_ranks"] == 8.0
    assert d["config"] == 5 and d["rays"] == 128 and d["value_includes_gather"]


def test_config5_refuses_no_gather():
    r = _run(["--config", "5", "--no-gather", "--dry-run"])
    assert r.returncode != 0 and "no-gather" in r.stderr
