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
