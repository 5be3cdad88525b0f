"""bench.py's multi-GPU contract without a GPU (--dry-run: launcher, process group,
barrier + max-over-ranks timing, rank-0 JSON line; no engine): `--gpus N` starts N
rank processes itself, and a world size that disagrees with --gpus is refused."""
import json
import os
import subprocess
import sys

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env=None):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=240, env=e)


def _json(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_bench_spawns_two_ranks():
    r = _run(["--gpus", "2", "--dry-run", "--steps", "3", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    d = _json(r.stdout)
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["dry_run"] is True and d["value"] > 0


def test_bench_single_rank_default():
    r = _run(["--dry-run", "--steps", "2", "--warmup", "0"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert _json(r.stdout)["n_gpus"] == 1


def test_bench_rejects_world_size_mismatch():
    r = _run(["--gpus", "4", "--dry-run"], env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=2 but --gpus 4" in (r.stderr + r.stdout)
