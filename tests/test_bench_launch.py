"""bench.py's multi-rank launch on CPU: ``--gpus 2`` without a torch.distributed.run wrapper
starts two ranks itself (gloo here), each rank checks the process group really has two
ranks, and the fixed models of the strong-scaling lines are split into contiguous,
256-B-aligned parameter buckets that cover every element once.  The GPU
work of those lines runs on the MI355X (bench.py without --dry-run)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*extra, env=None):
    e = dict(os.environ, **(env or {}))
    e.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *extra], capture_output=True, text=True,
                       timeout=240, env=e, cwd=ROOT)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p, (json.loads(lines[-1]) if lines else None)


def test_gpus_2_self_spawns_two_ranks():
    p, res = _run("--gpus", "2", "--dist-backend", "gloo", "--dry-run")
    assert p.returncode == 0, p.stderr[-2000:]
    assert res["n_gpus"] == 2
    assert res["launch"]["world_size"] == 2 and res["launch"]["backend"] == "gloo"
    assert "self-spawned" in res["launch"]["started_by"]
    for name, buckets in res["buckets"].items():
        assert len(buckets) == 2
        assert buckets[0][0] == 0 and buckets[0][1] == buckets[1][0]
        es = 2 if "bf16" in name else 4
        assert buckets[1][0] * es % 256 == 0
    assert res["buckets"]["north star, 8 peers x 25 M f32"][1][1] == 25_000_000


def test_single_process_default_is_one_rank():
    p, res = _run("--dry-run")
    assert p.returncode == 0, p.stderr[-2000:]
    assert res["n_gpus"] == 1 and res["launch"]["world_size"] == 1


def test_rank_count_mismatch_fails_loudly():
    """A process group whose size differs from --gpus stops the run (no silent 1-rank line)."""
    env = {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"}
    e = dict(os.environ, **env)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--dry-run"],
                       capture_output=True, text=True, timeout=240, env=e, cwd=ROOT)
    assert p.returncode != 0
    assert "process group has 1 rank" in p.stderr
