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


def _bench_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    return bench


def test_rank_plans_for_eight_gpus():
    """The 8-GPU configs' placement (BASELINE configs[3], [4]) without an 8-GPU node: rank r gets
    device r, C4 filter r built from keys [r*125M, (r+1)*125M) (disjoint, covering 1B), and C5 in
    the key-partitioned layout all 8 filters with a disjoint 1/8 of the 100M-key batch."""
    bench = _bench_module()
    world = 8
    c4 = [bench.rank_plan("c4", world, r, r) for r in range(world)]
    assert [p["device"] for p in c4] == list(range(8))
    assert [p["filters"] for p in c4] == [[r] for r in range(8)]
    spans = sorted(rng for p in c4 for rng in p["key_ranges"].values())
    assert spans[0][0] == 0 and spans[-1][1] == 1_000_000_000
    assert all(a[1] == b[0] for a, b in zip(spans, spans[1:])) and all(b - a == 125_000_000 for a, b in spans)
    c5 = [bench.rank_plan("c5", world, r, r) for r in range(world)]
    assert all(p["filters"] == list(range(8)) and p["layout"] == "keys" for p in c5)
    # each filter is built once, by one rank (the others receive it by replication)
    assert sorted(g for p in c5 for g in p["builds"]) == list(range(8))
    assert [p["builds"] for p in c5] == [[r] for r in range(world)]
    ks = [p["probe_keys"] for p in c5]
    assert ks[0][0] == 0 and ks[-1][1] == 100_000_000
    assert all(a[1] == b[0] for a, b in zip(ks, ks[1:]))
    assert all(a % 64 == 0 for a, _ in ks)  # whole 64-key hit-mask words per rank
    assert max(b - a for a, b in ks) - min(b - a for a, b in ks) <= 64
    c5f = [bench.rank_plan("c5", world, r, r, c5_layout="filters") for r in range(world)]
    assert [p["filters"] for p in c5f] == [[r] for r in range(8)]
    assert all(p["probe_keys"] == (0, 100_000_000) for p in c5f)
    for w in (1, 2, 3, 4):
        ks = [bench.rank_plan("c5", w, r, r, c5_probes=1_000_037)["probe_keys"] for r in range(w)]
        assert ks[0][0] == 0 and ks[-1][1] == 1_000_037 and all(a[1] == b[0] for a, b in zip(ks, ks[1:]))


def test_c5_probe_key_spans_tile_the_batch():
    """Every rank generates exactly its slice of the one global C5 batch: the spans of the ranks'
    slices, shifted to global positions, are the whole batch's spans cut at the slice edges."""
    bench = _bench_module()
    nq, n_f = 1_000_003, 10_000
    whole = {}
    for dst, start, cnt in bench.c5_probe_key_spans(nq, n_f, 0, nq):
        for i in range(cnt):
            whole[dst + i] = start + i
    assert sorted(whole) == list(range(nq))
    for w in (2, 3, 8):
        got = {}
        for r in range(w):
            a, b = bench.rank_plan("c5", w, r, r, c5_probes=nq)["probe_keys"]
            for dst, start, cnt in bench.c5_probe_key_spans(nq, n_f, a, b):
                for i in range(cnt):
                    got[a + dst + i] = start + i
        assert got == whole


def test_gpus8_dry_run_places_each_rank_on_its_device():
    """`bench.py --gpus 8` (the driver's N=8 command) run as a dry run: the 8 self-launched ranks
    report, over gloo, the plan each computed from its own LOCAL_RANK / RANK / WORLD_SIZE."""
    for config in ("c4", "c5"):
        r = _run(["--gpus", "8", "--config", config, "--dry-run"])
        assert r.returncode == 0, r.stderr[-2000:]
        out = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][0])
        assert out["n_gpus"] == 8 and out["world_size_seen"] == 8
        plans = out["plans"]
        assert [p["rank"] for p in plans] == list(range(8)) and [p["device"] for p in plans] == list(range(8))
        if config == "c4":
            assert [p["filters"] for p in plans] == [[r] for r in range(8)]
        else:
            ks = [tuple(p["probe_keys"]) for p in plans]
            assert ks[0][0] == 0 and ks[-1][1] == 100_000_000 and all(a[1] == b[0] for a, b in zip(ks, ks[1:]))


def test_rccl_init_failure_exits_3(capsys):
    """A process group that cannot come up over RCCL ends the rank with exit code 3 (never a
    silent fall-back to another backend)."""
    import pytest
    bench = _bench_module()

    class FailingDist:
        def init_process_group(self, **kw):
            raise RuntimeError("no RCCL here")

    class FakeTorch:
        @staticmethod
        def device(kind, idx):
            return (kind, idx)

    with pytest.raises(SystemExit) as e:
        bench.init_process_group_or_exit(FailingDist(), FakeTorch, "nccl", 5, 5)
    assert e.value.code == 3
    assert "RCCL process group failed" in capsys.readouterr().err
    seen = {}

    class GlooDist:
        def init_process_group(self, **kw):
            seen.update(kw)

    bench.init_process_group_or_exit(GlooDist(), FakeTorch, "gloo", 0, 0)
    assert seen["backend"] == "gloo"
