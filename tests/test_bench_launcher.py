"""bench.py's own rank launcher, on the CPU: `python bench.py --gpus N` outside a
torch.distributed launcher starts N ranks itself (torch.distributed.run as a child process, before any
GPU call), forwards rank 0's single JSON line and propagates a failing rank's exit status. `--dry` stops
each rank after the gloo process group agreed on the world size (no device needed)."""
import json
import os
import subprocess
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def _run(args, **env):
    e = dict(os.environ, MGN_DIST_BACKEND="gloo", **env)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          env=e, timeout=240, cwd=ROOT)


def test_bench_spawns_n_ranks_and_reports_them():
    for n in (2, 3):
        r = _run(["--gpus", str(n), "--dry", "--no-secondary", "--cpu-steps", "0"])
        assert r.returncode == 0, r.stderr[-2000:]
        lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
        assert len(lines) == 1, r.stdout  # exactly one JSON line on stdout (rank 0's)
        out = json.loads(lines[0])
        assert out["n_gpus"] == n and out["ranks"] == list(range(n))
        assert out["config"]["parallelism"] == "dp%d" % n and out["launched_by"] == "bench.py"
        assert "starting %d ranks" % n in r.stderr


def test_bench_single_gpu_does_not_spawn():
    r = _run(["--gpus", "1", "--dry"])
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip())
    assert out["n_gpus"] == 1 and out["launched_by"] == "external" and "starting" not in r.stderr


def test_bench_failing_rank_fails_the_launch():
    # without --dry every rank selects its GPU first: on this GPU-less host each rank fails, and so must
    # the parent (never a JSON line, never exit status 0)
    r = _run(["--gpus", "2", "--no-secondary", "--cpu-steps", "0", "--steps", "1", "--warmup", "1"])
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
