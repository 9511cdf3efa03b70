"""Drop-in CLI: the reference's main.py (main.py:13-153) on the HIP backend.

Keeps every flag of the reference argparser with its default and meaning,
the stdout lines ("setup object, jit-compile took", "took X ms",
"runtimes in ms: mean M stddev S", the constraint report and
"result cost: ( avg A , max M ). constraint fulfiled F") and the output
files trajectory_result.txt / trajectory_series.txt (np.savetxt defaults).

Additive flags (no reference counterpart): --batch-size, --seed,
--operator-rank, --device, --whole-robot-cost.
"""
import argparse
import os
import time

import numpy as np

from . import batch_io, distributed
from .optimizer_BLS import BacktrackingLineSearchOptimizer
from .optimizer_GD import GradientDescentOptimizer


def _bool(x):
    return str(x).lower() == "true"


def build_parser():
    parser = argparse.ArgumentParser()
    # Profiling (main.py:16-23)
    parser.add_argument('--profiling', type=_bool, default=False,
                        help="Print per-call HIP timing breakdown (default: False)")
    parser.add_argument('--extended-vis', type=_bool, default=False,
                        help="Record the per-iteration trajectory series (default: False)")
    parser.add_argument('--n-measurements', type=int, default=1,
                        help="Number of measurements to be taken during one time measurement (default: 1)")
    parser.add_argument('--n-times', type=int, default=1,
                        help="Number of times the process is repeated to generate mean and stddev(default: 1)")
    # Optimizer (main.py:26-29)
    parser.add_argument('--optimizer-name', choices=['gd', 'bls'], default='bls',
                        help="Choose the optimizer: 'gd' for Gradient Descent, 'bls' for Backtracking Line Search")
    parser.add_argument('--jit-loop', type=_bool, default=True,
                        help="Run the whole loop as one persistent kernel (default: True)")
    # Trajectory (main.py:32-37)
    parser.add_argument('--n-timesteps', type=float, default=50,
                        help="Number of timesteps in the trajectory (default: 50)")
    parser.add_argument('--rbf-variance', type=float, default=0.1,
                        help="Variance parameter for Radial Basis Function (RBF) kernel (default: 0.1)")
    parser.add_argument('--jac-gaussian-mean', type=float, default=0.15,
                        help="Mean value for the Gaussian noise of the matrix J (default: 0.15)")
    # Minimization (main.py:40-43)
    parser.add_argument('--max-inner-iteration', type=int, default=200,
                        help="Maximum number of iterations for the inner optimization loop (default: 200)")
    parser.add_argument('--loop-loss-reduction', type=float, default=1e-3,
                        help="Minimum loss reduction threshold for each loop iteration (default: 1e-3)")
    # Constraint dual optimization (main.py:46-59)
    parser.add_argument('--max-outer-iteration', type=int, default=10,
                        help="Maximum number of iterations for the outer optimization loop (default: 10)")
    parser.add_argument('--lambda-constraint-increase', type=int, default=10,
                        help="Increase factor for lambda-sg-constraint and lambda-jl-constraint (default: 10)")
    parser.add_argument('--lambda-sg-constraint', type=float, default=0.5,
                        help="Initial weight for the SG (Start Goal) constraint (default: 0.5)")
    parser.add_argument('--lambda-jl-constraint', type=float, default=0.1,
                        help="Initial weight for the JL (Joint Limit) constraint (default: 0.1)")
    parser.add_argument('--eps-position', type=float, default=0.01,
                        help="Tolerance for start goal position constraints (default: 0.01)")
    parser.add_argument('--eps-velocity', type=float, default=0.01,
                        help="Tolerance for start goal velocity constraints (default: 0.01)")
    # Loss (main.py:62-69)
    parser.add_argument('--lambda-max-cost', type=float, default=0.5,
                        help="Maximum cost weight in the obstacle loss function (default: 0.5)")
    parser.add_argument('--lambda-reg', type=float, default=1e-4,
                        help="Regularization weight in the gradient update (default: 1e-4)")
    parser.add_argument('--constraint-violating-dependant-loss', type=_bool, default=True,
                        help="Enable or disable the loss dependency on constraint violations (default: True)")
    parser.add_argument('--joint-safety-limit', type=float, default=0.98,
                        help="Safety limit for the joint positions (default: 0.98)")
    # BLS (main.py:72-81)
    parser.add_argument('--max-bls-iteration', type=int, default=20,
                        help="Maximum number of iterations for the Backtracking Line Search (default: 20)")
    parser.add_argument('--bls-lr-start', type=float, default=0.2, help="Initial learning rate for BLS (default: 0.2)")
    parser.add_argument('--bls-alpha', type=float, default=0.01,
                        help="Alpha parameter for BLS, sufficient decrease condition (default: 0.01)")
    parser.add_argument('--bls-beta_plus', type=float, default=1.2,
                        help="Multiplicative factor to increase the learning rate in BLS (default: 1.2)")
    parser.add_argument('--bls-beta_minus', type=float, default=0.5,
                        help="Multiplicative factor to decrease the learning rate in BLS (default: 0.5)")
    # GD (main.py:84-85)
    parser.add_argument('--gd-lr', type=float, nargs='+',
                        default=[2e-3, 1e-4, 1e-5, 1e-6, 1e-7, 1e-8, 1e-8, 1e-8, 1e-8, 1e-8],
                        help="Learning rates for the dual optimization in Gradient Descent")
    # Robot (main.py:88-97)
    parser.add_argument('--n-joints', type=int, default=3, help="Number of joints in the robot (default: 3)")
    parser.add_argument('--link-length', type=float, nargs='+', default=[1.5, 1.0, 0.5],
                        help="Lengths of the robot's links, provided as a list (default: [1.5, 1.0, 0.5])")
    parser.add_argument('--max-joint-velocity', type=float, default=7,
                        help="Maximum velocity for the robot's joints (default: 7)")
    parser.add_argument('--max-joint-position', type=float, default=2,
                        help="Maximum allowable position for the robot's joints (default: 2)")
    parser.add_argument('--min-joint-position', type=float, default=-1,
                        help="Minimum allowable position for the robot's joints (default: -1)")
    # Additive (this build)
    parser.add_argument('--batch-size', type=int, default=1,
                        help="Optimise this many problems in one launch (>1: problem 0 is the reference "
                             "environment, the rest random start/goal; writes the batch files of batch_io.py)")
    parser.add_argument('--seed', type=int, default=1, help="Seed of the random batch problems (default: 1)")
    parser.add_argument('--operator-rank', type=int, default=0,
                        help="Kernel-operator rank inside the loop: 0 auto, -1 dense exact (default: 0)")
    parser.add_argument('--device', type=int, default=0, help="HIP device ordinal (default: 0)")
    parser.add_argument('--whole-robot-cost', type=_bool, default=False,
                        help="Obstacle cost summed over every joint position instead of the end effector only "
                             "(blog 'Complete Robot Obstacle Avoidance'; default: False)")
    return parser


def parse_args(argv=None):
    return build_parser().parse_args(argv)


def run_batch(optimizer, args):
    """--batch-size B > 1: B problems in one launch per optimize().

    Timing lines as main.py:118-128 (one "took" per measurement, for the whole batch); the
    reference's report and files for problem 0 (the reference environment); batch files
    and a one-line batch summary (batch_io.py).

    Under torchrun (WORLD_SIZE > 1, one process per GPU) the batch is sharded:
    rank 0's environment and problems are broadcast, every rank optimises its rows
    [lo, hi), the results are gathered to rank 0, which reports and writes the files."""
    env, tr = optimizer.env, optimizer.trajectory
    world, rank, _ = distributed.world_info()
    B = args.batch_size
    start, goal = batch_io.batch_problems(B, tr.robot.N_joints, args.seed)
    lo, hi = 0, B
    dev = "cpu"
    if world > 1:
        import torch
        dev = torch.device("cuda", args.device) if torch.distributed.get_backend() == "nccl" else "cpu"
        obs, start, goal = distributed.broadcast_environment(env.obstacles, start, goal, dev)
        env.obstacles = obs
        lo, hi = distributed.shard(B, world, rank)
    runtimes = []
    res = None
    for _ in range(args.n_measurements):
        st = time.time()
        for _ in range(args.n_times):
            res = optimizer.optimize_batch(start[lo:hi], goal[lo:hi], env.obstacles, series=args.extended_vis)
        et = time.time()
        if world > 1:
            et = st + distributed.reduce_timing(et - st, 0, dev)[0]
        runtimes.append(1000 * (et - st) / args.n_times)
        if rank == 0:
            print("took", 1000 * (et - st) / args.n_times, "ms")
    if args.n_measurements > 1 and rank == 0:
        print("runtimes in ms: mean", np.mean(runtimes), "stddev", np.std(runtimes))
    alpha, traj, stats = res[:3]
    series = res[3] if args.extended_vis else None
    if world > 1:
        parts = {"alpha": alpha, "traj": traj}
        parts.update({"stat_" + k: np.asarray(v) for k, v in stats.items()})
        if series is not None:
            parts["series"] = series
        full = distributed.gather_batch(parts, B, dev)  # rank 0 only
        if rank != 0:
            return alpha  # this rank's shard
        alpha, traj = full["alpha"], full["traj"]
        stats = {k[5:]: v for k, v in full.items() if k.startswith("stat_")}
        series = full.get("series")
    avg = tr.compute_trajectory_cost(alpha, env.obstacles, start, goal, 0, 0, 0)
    mx = tr.compute_trajectory_cost(alpha, env.obstacles, start, goal, 0, 0, 1)
    ok, _ = optimizer.context.constraints(alpha, start, goal)
    print("batch of", len(alpha), "problems" + (f" on {world} GPUs" if world > 1 else "") +
          ": constraint fulfiled", int(np.sum(ok)), "of", len(alpha),
          "; avg cost mean", float(np.mean(avg)), ", max cost mean", float(np.mean(mx)),
          "; inner iterations", int(np.sum(stats["inner_iterations"])))
    ok0 = tr.constraintsFulfilledVerbose(alpha[0], start[0], goal[0], verbose=True)
    print("result cost: ( avg", avg[0], ", max", mx[0], "). constraint fulfiled", ok0)
    batch_io.write_result(batch_io.RESULT, traj[0])
    batch_io.write_result_batch(batch_io.RESULT_BATCH, traj)
    batch_io.write_summary(batch_io.SUMMARY_BATCH, avg, mx, ok, stats)
    if series is not None:
        lens = stats["series_len"]
        frames0 = series[0][: int(lens[0])]
        print(frames0.shape)
        batch_io.write_series(batch_io.SERIES, frames0, tr.N_timesteps, tr.robot.N_joints)
        batch_io.write_series_batch(batch_io.SERIES_BATCH, series, lens)
    return alpha


def main(argv=None):
    args = parse_args(argv)
    world, _, local = distributed.world_info()
    if world > 1:  # torchrun: one process per GPU
        import torch
        import torch.distributed as dist
        # IRM_DIST_BACKEND=gloo: host-side collectives (e.g. several ranks sharing one GPU in tests)
        backend = os.environ.get("IRM_DIST_BACKEND", "nccl" if torch.cuda.is_available() else "gloo")
        ngpu = torch.cuda.device_count()
        args.device = local % max(1, ngpu)
        if not dist.is_initialized():
            if backend == "nccl":
                torch.cuda.set_device(args.device)
                dist.init_process_group("nccl", device_id=torch.device("cuda", args.device))
            else:
                dist.init_process_group("gloo")
    if args.optimizer_name == 'bls':
        optimizer = BacktrackingLineSearchOptimizer(args)
    elif args.optimizer_name == 'gd':
        optimizer = GradientDescentOptimizer(args)
    else:  # unreachable (argparse choices); kept for parity with main.py:113-115
        print("FATAL: not defined optimizer", args.optimizer_name)
        raise SystemExit(-1)
    if args.batch_size > 1:
        return run_batch(optimizer, args)

    def multiple_optimizations():
        runtimes = []
        result = None
        for _ in range(args.n_measurements):
            st = time.time()
            for _ in range(args.n_times):
                result = optimizer.optimize()
            et = time.time()
            runtimes.append(1000 * (et - st) / args.n_times)
            print("took", 1000 * (et - st) / args.n_times, "ms")
        if args.n_measurements > 1:
            print("runtimes in ms: mean", np.mean(runtimes), "stddev", np.std(runtimes))
        return result

    if args.extended_vis:
        result_alpha, p = multiple_optimizations()
    else:
        result_alpha = multiple_optimizations()
    if args.profiling:
        for k, v in optimizer.last_profile.items():
            print("profile", k, v)

    env, tr = optimizer.env, optimizer.trajectory
    avg_result_cost = tr.compute_trajectory_cost(result_alpha, env.obstacles, env.start_config, env.goal_config, 0, 0, 0)
    max_result_cost = tr.compute_trajectory_cost(result_alpha, env.obstacles, env.start_config, env.goal_config, 0, 0, 1)
    ok = tr.constraintsFulfilledVerbose(result_alpha, env.start_config, env.goal_config, verbose=True)
    print("result cost: ( avg", avg_result_cost, ", max", max_result_cost, "). constraint fulfiled", ok)

    np_trajectory = np.array(tr.evaluate(result_alpha, tr.km, tr.jac))
    np.savetxt("trajectory_result.txt", np_trajectory)
    if args.extended_vis:
        p_np = np.array(p)
        print(p_np.shape)
        np.savetxt("trajectory_series.txt", p_np.reshape((-1, tr.robot.N_joints * tr.N_timesteps)))
    return result_alpha


if __name__ == "__main__":
    main()
