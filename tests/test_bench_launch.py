"""bench.py's multi-rank launcher on CPU (no device): `bench.py --gpus 2` outside torchrun starts two
ranks under torch.distributed.run itself and relays rank 0's JSON line.  `--dry-run`
runs the launcher, the shard split, the environment broadcast and the max-time / Σ-iteration reduction
without touching a GPU; tests/test_gpu_widen.py runs the same launcher with the kernels on the GPU box."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*argv):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *argv], stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, text=True, env=env, timeout=300, cwd=REPO)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def test_gpus_flag_launches_ranks():
    r = _bench("--gpus", "2", "--dry-run", "--max-inner", "200")
    assert r["n_gpus"] == 2
    assert r["config"]["global_batch"] == 2048 and r["config"]["batch_per_gpu"] == 1024
    assert r["iterations_all"] == 2 * 1024 * 200  # Σ over ranks
    assert r["elapsed_max"] == 2.0  # max over ranks (rank r reports 1 + r)
    assert r["obstacles_equal_rank0"]  # rank 1 started with shifted obstacles and received rank 0's
    c0, c1 = r["shard_checksums"]
    assert c0 != c1  # disjoint shards of the global batch


def test_single_rank_default():
    r = _bench("--dry-run", "--config", "c5")
    assert r["n_gpus"] == 1 and r["config"]["global_batch"] == 512
    # bench-mode deviations from main.py's defaults are recorded in the config
    ov = r["config"]["overrides_vs_reference_defaults"]
    assert ov["gd_lr"] == [1e-3] and ov["max_outer_iteration"] == 1
    assert r["config"]["gd_lr_first"] == 1e-3


def test_batched_bls_config():
    """c3bls: C3's 1024 problems with the reference's default optimiser (BLS); the line reports BLS
    inner iterations and records the bench-mode overrides like the GD configs."""
    r = _bench("--dry-run", "--config", "c3bls")
    assert r["metric"] == "BLS iterations/sec (batch of trajectories)"
    assert r["config"]["optimizer"] == "bls" and r["config"]["global_batch"] == 1024
    assert r["config"]["mode"].startswith("bench (200 fixed BLS inner iterations")
    assert r["iterations_all"] == 1024 * 200
    r = _bench("--dry-run", "--config", "c3bls", "--faithful")
    assert r["config"]["mode"] == "faithful" and r["config"]["overrides_vs_reference_defaults"] == {}


def test_bls_flop_model_counts_trials():
    """BLS lines: one direction round per inner iteration plus one evaluation per line-search trial."""
    import importlib
    sys.path.insert(0, REPO)
    bench = importlib.import_module("bench")
    d, t, ref = bench.flops_per_iteration(128, 3, 11, 32, split=True)
    e, ref2 = bench.flops_per_iteration(128, 3, 11, 32)
    assert e == d + t and ref == ref2
    assert t == 4 * 128 * 3 + 14 * 128 * 11 + 24 * 128 * 3  # update + obstacle pairs + FK / penalties
    # k_lean's BLS: every trial also forms its iterate, projects its residual and runs the F tiles
    db, tb, _ = bench.flops_per_iteration(128, 3, 11, 32, split=True, bls=True)
    assert db == (2 * 32 + 2 * 24) * 128 * 3 + 4 * 128 * 9
    assert tb == t + (14 + 2 * 16 + 4 * 16) * 128 * 3 + 4 * 128 * 9


def test_cpu_baseline_runs_before_process_group_init(monkeypatch):
    """At world > 1 rank 0 times the CPU baselines before init_process_group: with the nccl backend and
    a device_id the communicator forms eagerly (HIP initialised on the device), and the batched
    baseline forks worker processes, which must not happen after that."""
    import torch.distributed as dist

    sys.path.insert(0, REPO)
    import bench
    order = []

    class Stop(Exception):
        pass

    def fake_init(*a, **k):
        order.append("init_process_group")
        raise Stop

    monkeypatch.setattr(bench, "cpu_baseline", lambda *a, **k: order.append("cpu_baseline"))
    monkeypatch.setattr(dist, "init_process_group", fake_init)
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("LOCAL_RANK", "0")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--config", "c3"])
    try:
        bench.main()
    except Stop:
        pass
    assert order == ["cpu_baseline", "init_process_group"], order


import pytest  # noqa: E402


@pytest.mark.parametrize("cfg,global_batch", [("c4", 8192), ("c5", 4096)])
def test_eight_rank_dry_run_shards_cover_the_global_batch(cfg, global_batch):
    """BASELINE configs[3] / [4] as the driver's 8-GPU run launches them (--gpus 8, one rank per GPU):
    eight disjoint shards, in rank order, covering the global batch exactly; the collectives ran over
    eight ranks; the rendezvous timeout is explicit and covers rank 0's capped CPU-baseline budget
    (VERDICT r04 #6)."""
    sys.path.insert(0, REPO)
    import bench
    r = _bench("--gpus", "8", "--dry-run", "--config", cfg)
    assert r["n_gpus"] == 8 and r["world_size"] == 8
    assert r["config"]["global_batch"] == global_batch
    B = r["config"]["batch_per_gpu"]
    assert B * 8 == global_batch
    ranges = r["shard_ranges"]
    assert ranges == [[k * B, (k + 1) * B] for k in range(8)]  # disjoint, contiguous, in rank order
    assert len(set(r["shard_checksums"])) == 8
    assert r["obstacles_equal_rank0"]
    assert r["elapsed_max"] == 8.0 and r["iterations_all"] == global_batch * 200
    assert bench.cpu_budgets(8) < bench.cpu_budgets(1)
    assert r["rendezvous_timeout_s"] >= 10 * sum(bench.cpu_budgets(8))
