"""The N>1 path on CPU: world_size 2 over gloo.

Problems are independent, so the batch is sharded across ranks with no
data-path collective; the only collectives are the environment broadcast and
the timing/iteration reduction of bench.py.  Checked here: every rank gets
rank 0's environment, the shards tile the global batch, the reductions give
max-time / summed iterations, and a sharded solve equals the single-process
solve problem by problem (the oracle stands in for the device solver, which
is exercised per-problem by the gpu tests).
"""
import os
import socket
import sys

import numpy as np
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist

    import bench
    from irm_motion_planning_amd.params import params_from_args
    from oracle.oracle import Oracle

    dist.init_process_group("gloo", rank=rank, world_size=world)
    start, goal, obstacles = bench.make_problem("c3", world, rank)
    # a rank that starts with a different environment must end with rank 0's
    obs = torch.from_numpy(obstacles + (0.0 if rank == 0 else 1.0))
    bench.share_environment(obs, world)
    args = bench.make_args("c3", False, 6)
    orc = Oracle(params_from_args(args))
    n = 3  # a small slice of this rank's shard
    alpha, st = orc.optimize_batch(None, start[:n], goal[:n], obs.numpy(), n_threads=1)
    iters = float(sum(s["grad_evals"] for s in st))
    t_max, it_sum = bench.aggregate(1.0 + rank, iters, world, "cpu")
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), obs=obs.numpy(), start=start[:n], alpha=alpha,
             t_max=t_max, it_sum=it_sum)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_sharding(tmp_path):
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    import bench
    from irm_motion_planning_amd.params import params_from_args
    from oracle.oracle import Oracle

    r = [dict(np.load(tmp_path / f"r{i}.npz")) for i in range(world)]
    _, _, obstacles = bench.make_problem("c3", 1, 0)
    for x in r:
        np.testing.assert_array_equal(x["obs"], obstacles)  # broadcast from rank 0
        assert float(x["t_max"]) == 2.0  # max over ranks
        assert float(x["it_sum"]) == 2 * 3 * 6  # summed executed iterations
    # shards tile the global batch in rank order
    gs, _, _ = bench.make_problem("c3", 1, 0)
    B = bench.CONFIGS["c3"][1]
    full_start, full_goal, _ = bench.make_problem("c3", world, 0)
    np.testing.assert_array_equal(r[0]["start"], gs[:3])
    s1, g1, _ = bench.make_problem("c3", world, 1)
    np.testing.assert_array_equal(r[1]["start"], s1[:3])
    # sharded solve == single-process solve, problem by problem (bit-exact: same code, same inputs)
    orc = Oracle(params_from_args(bench.make_args("c3", False, 6)))
    for rank, (s, g) in enumerate([(full_start[:3], full_goal[:3]), (s1[:3], g1[:3])]):
        alpha, _ = orc.optimize_batch(None, s, g, obstacles, n_threads=1)
        np.testing.assert_array_equal(alpha, r[rank]["alpha"])
    assert len(full_start) == B


def _gather_worker(rank, world, port, out_dir):
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist

    from irm_motion_planning_amd import distributed as D
    dist.init_process_group("gloo", rank=rank, world_size=world)
    B = 7  # uneven shards: 4 + 3
    rng = np.random.default_rng(rank)  # every rank starts from different values ...
    obs = rng.uniform(-3, 3, (11, 2)).astype(np.float32)
    s = rng.uniform(-0.5, 0.5, (B, 3)).astype(np.float32)
    g = rng.uniform(0.2, 1.6, (B, 3)).astype(np.float32)
    obs, s, g = D.broadcast_environment(obs, s, g)  # ... and ends with rank 0's
    lo, hi = D.shard(B, world, rank)
    traj = np.repeat(s[lo:hi, None, :], 5, axis=1) * np.float32(2)  # a per-problem result
    iters = np.arange(lo, hi, dtype=np.int64) * 10
    ok = (np.arange(lo, hi) % 2).astype(np.uint8)
    full = D.gather_batch({"traj": traj, "iters": iters, "ok": ok}, B)
    t_max, it_sum = D.reduce_timing(0.5 * (rank + 1), hi - lo)
    assert (full is None) == (rank != 0)  # gathered to rank 0 only
    np.savez(os.path.join(out_dir, f"g{rank}.npz"), obs=obs, s=s, lo=lo, hi=hi, t_max=t_max, it_sum=it_sum,
             **(full or {}))
    dist.barrier()
    dist.destroy_process_group()


def test_distributed_helpers_two_ranks(tmp_path):
    """irm_motion_planning_amd.distributed over gloo, world 2: broadcast of rank 0's environment,
    contiguous uneven shards, gather of float/int/uint8 per-problem results to rank 0 in rank order,
    max/sum timing reduction (the nccl path of main.py --batch-size under torchrun)."""
    world = 2
    mp.start_processes(_gather_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    r = [dict(np.load(tmp_path / f"g{i}.npz")) for i in range(world)]
    rng0 = np.random.default_rng(0)
    obs0 = rng0.uniform(-3, 3, (11, 2)).astype(np.float32)
    s0 = rng0.uniform(-0.5, 0.5, (7, 3)).astype(np.float32)
    assert [(int(x["lo"]), int(x["hi"])) for x in r] == [(0, 4), (4, 7)]
    for x in r:
        np.testing.assert_array_equal(x["obs"], obs0)
        np.testing.assert_array_equal(x["s"], s0)
        assert float(x["t_max"]) == 1.0 and float(x["it_sum"]) == 7
    x = r[0]  # the gathered batch, on rank 0
    np.testing.assert_array_equal(x["traj"], np.repeat(s0[:, None, :], 5, axis=1) * np.float32(2))
    np.testing.assert_array_equal(x["iters"], np.arange(7) * 10)
    assert x["iters"].dtype == np.int64 and x["ok"].dtype == np.uint8
    np.testing.assert_array_equal(x["ok"], np.arange(7) % 2)
    assert "traj" not in r[1]


def test_shard_tiles_batch():
    from irm_motion_planning_amd.distributed import shard
    for B in (1, 7, 8, 1024, 8193):
        for world in (1, 2, 3, 8):
            rs = [shard(B, world, r) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == B
            assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
            assert max(h - l for l, h in rs) - min(h - l for l, h in rs) <= 1
