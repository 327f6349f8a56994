"""bench.py's N-rank launch on CPU: `python bench.py --gpus N` with no launcher starts N ranks
itself (the driver's command form), they rendezvous over 127.0.0.1 and rank 0 reports the
world it saw; a WORLD_SIZE that disagrees with --gpus is an error.  --dry-run does no GPU work
(the GPU runs use RCCL; this checks the launcher, the rendezvous, the barrier and the
max-over-ranks plumbing with gloo)."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, drop=("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")):
    env = {k: v for k, v in os.environ.items() if k not in drop}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=240, cwd=REPO)


def test_gpus2_self_launches_two_ranks():
    r = _run(["--gpus", "2", "--config", "c1", "--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    out = lines[0]
    assert out["n_gpus"] == 2 and out["world_size_seen"] == 2 and out["dry_run"] is True
    assert out["max_elapsed_s"] >= 0.02  # the max over ranks (rank 1 sleeps longer)


def test_gpus4_self_launch():
    r = _run(["--gpus", "4", "--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][0])
    assert out["n_gpus"] == 4 and out["world_size_seen"] == 4


def test_world_size_mismatch_is_an_error():
    r = _run(["--gpus", "2", "--dry-run"], env_extra={"WORLD_SIZE": "3", "RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE=3" in r.stderr


def test_single_rank_dry_run():
    r = _run(["--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["n_gpus"] == 1 and out["world_size_seen"] == 1


def test_dist_report_keeps_rccl_world_size_key():
    """The one-GPU JSON keeps `rccl_world_size` (round-3 advice: a gloo-style rename broke the
    schema of the default run)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    r = bench.dist_report(None, 1)
    assert r["rccl_world_size"] == 1 and r["world_size_seen"] == 1

    class G:
        def __init__(self, be):
            self.be = be

        def get_backend(self):
            return self.be

        def get_world_size(self):
            return 4
    assert bench.dist_report(G("nccl"), 4)["rccl_world_size"] == 4
    r = bench.dist_report(G("gloo"), 4)
    assert r["rccl_world_size"] is None and r["world_size_seen"] == 4
