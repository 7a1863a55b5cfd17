"""bench.py's multi-rank launch on CPU: ``--gpus 2`` without a torch.distributed.run wrapper
starts two ranks itself (gloo here), each rank checks the process group really has two
ranks, and the fixed models of the strong-scaling lines are split into contiguous,
256-B-aligned parameter buckets that cover every element once.  The GPU
work of those lines runs on the MI355X (bench.py without --dry-run)."""
import json
import os
import subprocess
import sys
import time

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


def test_dry_run_legs_agree_and_check_parity():
    """Every leg of the dry run goes through the Legs runner: agreed start, a parity flag agreed by
    both ranks (the gloo all-gather's payload rebuilt and compared on every rank)."""
    p, res = _run("--gpus", "2", "--dist-backend", "gloo", "--dry-run")
    assert p.returncode == 0, p.stderr[-2000:]
    assert res["legs"]["rendezvous"]["parity_ok"] is True
    assert res["legs"]["gloo_allgather"]["parity_ok"] is True
    assert res["legs_failed"] == []


def test_failure_before_collectives_skips_the_leg_on_every_rank():
    """A leg that fails on rank 1 before its collectives is skipped by BOTH ranks together (the
    gloo agreement in go()); the run goes on to the next leg and prints its line."""
    p, res = _run("--gpus", "2", "--dist-backend", "gloo", "--dry-run",
                  env={"BENCH_INJECT_FAIL": "rendezvous:1:raise_prepare"})
    assert p.returncode == 0, p.stderr[-2000:]
    assert "skipped" in res["legs"]["rendezvous"]
    assert res["legs"]["gloo_allgather"]["parity_ok"] is True
    assert res["legs_failed"] == ["rendezvous"]


def test_failure_inside_collectives_ends_the_run_nonzero_quickly():
    """A rank failing after every rank agreed to enter the collectives cannot resynchronise: it
    ends the run at once with a non-zero exit (no 10-minute collective timeout)."""
    t0 = time.monotonic()
    p, _ = _run("--gpus", "2", "--dist-backend", "gloo", "--dry-run", "--leg-timeout", "60",
                env={"BENCH_INJECT_FAIL": "gloo_allgather:1:raise_run"})
    assert p.returncode != 0
    assert time.monotonic() - t0 < 90, "the failing run took too long to end"
    assert "FATAL in leg gloo_allgather" in p.stderr


def test_hung_rank_hits_the_leg_deadline():
    """A rank that hangs inside a leg: the watchdog ends the run with a non-zero exit shortly after
    --leg-timeout; rank 0 prints the line measured so far, naming the leg."""
    t0 = time.monotonic()
    p, res = _run("--gpus", "2", "--dist-backend", "gloo", "--dry-run", "--leg-timeout", "8",
                  env={"BENCH_INJECT_FAIL": "gloo_allgather:1:hang"})
    elapsed = time.monotonic() - t0
    assert p.returncode != 0
    assert elapsed < 75, elapsed
    assert "gloo_allgather" in p.stderr
    if res is not None:  # rank 0 got to print before the launcher stopped it
        assert res["aborted_leg"]["leg"] == "gloo_allgather"


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


def test_four_ranks_report_the_fixed_model_strong_lines():
    """at N > 1 the line carries BASELINE's fixed-model multi-GPU configs as
    top-level ``strong_headline`` rows (north star, configs[3'] ResNet-8 x 64, configs[4] ResNet-34 x 128
    bf16), each with its own parity flag agreed by every rank.  Without a GPU the dry run splits each
    model (scaled) into 4 buckets and checks the gloo all-gather that reassembles it; the GPU run fills
    value / speedup_vs_one_gpu / efficiency / allgather_ms on the same keys."""
    p, res = _run("--gpus", "4", "--dist-backend", "gloo", "--dry-run")
    assert p.returncode == 0, p.stderr[-2000:]
    sh = res["strong_headline"]
    assert sh["n_gpus"] == 4 and sh["scaling"] == "strong"
    for key in ("north_star", "configs3_resnet8", "configs4_resnet34_bf16"):
        row = sh[key]
        assert row["parity_ok"] is True and row["buckets"] == 4, (key, row)
        assert {"value", "speedup_vs_one_gpu", "efficiency"} <= set(row)
    assert res["legs_failed"] == []
