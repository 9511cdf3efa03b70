"""Benchmark: GD inner-loop iterations/s for a batch of trajectories.

BASELINE.json metric "GD iterations/sec (batch of trajectories) at 1/2/4/8
MI355X; % HBM roofline", workload configs[2] (C3): per GPU a batch of 1024
random start/goal problems, N=128 waypoints, D=3 joints, the reference's 11
obstacles shared by the batch, GradientDescentOptimizer.  One step = one
optimize() of the whole batch (initTrajectory + the full inner loop) in one
persistent launch, inputs resident in HBM.  Bench mode runs every trajectory
for exactly --max-inner (200) iterations (loop_loss_reduction = -1e30,
max_outer_iteration = 1), so iterations/s = B·200/t.

Multi-GPU (torchrun, one rank per GPU): weak scaling, each rank owns a
1024-problem shard; the shared environment is broadcast from rank 0 over
RCCL (the only collective besides the timing/iteration reductions).

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

CONFIGS = {
    # name: (description, B per GPU, N, D, O, optimizer)
    "c3": ("batch of 1024 random start/goal trajectories, N=128, D=3, 11 shared obstacles, GD (BASELINE configs[2])",
           1024, 128, 3, 11, "gd"),
    "c4": ("batch of 1024 per GPU (8192 on 8), N=256, D=3, 50 random obstacles, GD (BASELINE configs[3])",
           1024, 256, 3, 50, "gd"),
    "c5": ("7-DoF arm, batch of 512 per GPU (4096 on 8), N=256, 11 obstacles, GD (BASELINE configs[4])",
           512, 256, 7, 11, "gd"),
    "c2": ("single trajectory, N=128, 10 obstacles, BLS (BASELINE configs[1])", 1, 128, 3, 10, "bls"),
    # north_star's stated target shape: a batch of 7-DoF, 128-waypoint trajectories
    "c7": ("north_star target: 7-DoF arm, batch of 1024 per GPU, N=128, 11 obstacles, GD", 1024, 128, 7, 11, "gd"),
    # the reference's default optimiser (main.py:27) on C3's batch: batched backtracking line search
    "c3bls": ("batch of 1024 random start/goal trajectories, N=128, D=3, 11 shared obstacles, BLS "
              "(the reference's default optimizer, main.py:27)", 1024, 128, 3, 11, "bls"),
    # diagnostic shapes (not BASELINE configurations): C3's batch at other trajectory lengths
    "c3n64": ("diagnostic: C3 batch at N=64", 1024, 64, 3, 11, "gd"),
    "c3n256": ("diagnostic: C3 batch at N=256", 1024, 256, 3, 11, "gd"),
    "c3o0": ("diagnostic: C3 batch without obstacles", 1024, 128, 3, 0, "gd"),
    "c3o44": ("diagnostic: C3 batch, the reference's obstacles ×4 (shifted copies)", 1024, 128, 3, 44, "gd"),
    "c3b8192": ("diagnostic: C3 problems, 8192 on one GPU (eight workgroups per CU in sequence)", 8192, 128, 3, 11, "gd"),
}

PEAK_FP32_TFLOPS = 157.3  # MI355X fp32 (vector = matrix), MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0


def make_problem(cfg, world, rank):
    """Synthetic inputs of SURVEY.md §8d (numpy default_rng), this rank's shard."""
    _, B, N, D, O, _ = CONFIGS[cfg]
    Btot = B * world
    if cfg == "c4":
        rng = np.random.default_rng(2)
        obs = []
        while len(obs) < O:
            o = rng.uniform(-3.5, 3.5, 2)
            if np.linalg.norm(o) >= 0.5:
                obs.append(o)
        obstacles = np.array(obs, np.float32)
        rs = np.random.default_rng(3)
    else:  # c3, c5, c2 and the diagnostic c3n* shapes
        from irm_motion_planning_amd.environment import OBSTACLES
        obstacles = OBSTACLES[:O].astype(np.float32)
        if O > len(OBSTACLES):  # diagnostic: shifted copies of the reference set
            reps = -(-O // len(OBSTACLES))
            obstacles = np.concatenate([OBSTACLES + 0.1 * i for i in range(reps)])[:O].astype(np.float32)
        rs = np.random.default_rng({"c5": 4, "c7": 7}.get(cfg, 1))  # c3bls: C3's problems
    start = rs.uniform(-0.5, 0.5, (Btot, D)).astype(np.float32)
    goal = rs.uniform(0.2, 1.6, (Btot, D)).astype(np.float32)
    if cfg == "c2":
        from irm_motion_planning_amd.environment import START_CONFIG, GOAL_CONFIG
        start[:] = START_CONFIG
        goal[:] = GOAL_CONFIG
    sl = slice(rank * B, (rank + 1) * B)
    return start[sl], goal[sl], obstacles


def make_args(cfg, faithful, max_inner):
    from irm_motion_planning_amd import main as irm_main
    _, B, N, D, O, opt = CONFIGS[cfg]
    argv = ["--optimizer-name", opt, "--n-timesteps", str(N), "--n-joints", str(D)]
    if D != 3:
        argv += ["--link-length"] + [str(3.0 / D)] * D
    if not faithful:
        argv += ["--loop-loss-reduction=-1e30", "--max-outer-iteration=1", f"--max-inner-iteration={max_inner}"]
        if D == 7:
            # The default first step size 2e-3 makes the 7-DoF GD diverge in exact arithmetic
            # (loss 3e28 after 200 steps; the faithful loop stops at the first increase).  Bench
            # mode forces every step to run, so C5 uses 1e-3 (converges, same work per step).
            argv += ["--gd-lr", "1e-3"]
    return irm_main.parse_args(argv)


def flops_per_iteration(N, D, O, R, split=False, lean=True, ranks=None, bls=False):
    """Algorithmic fp32 flops of one GD iteration of one trajectory.

    exec: what the optimiser kernel (waypoint-space rank-R iteration with the reference's fp32 α
    rounding) must do — stage 1 (y'' = Fᵀ[a; b]·Jᵀ, 2·R·N·D), the rounding residual z = V_Rᵀ·e'
    (2·Rz·N·D), stage 2 (the direction F·(y'' + z), 2·2N·Rf·D; G = V_R·y'', 2·N·Rg·D) — k_lean at
    R = 32 runs z and the direction at rank 16 and G at rank 24, k_optimize all at
    R —, the Jᵀ / J mixes of the gradient inputs and of the direction (2 × 2·2·N·D²), the α update
    with its residual (k_lean's two-FMA form 7·N·D, k_optimize's error-free one 14·N·D), the waypoint
    update (4·N·D), obstacle pairs (14·N·O), FK / Jacobian / penalties (24·N·D, sincos counted as 4 flops
    each).
    ref: SURVEY.md §8d's count of the reference formulation, 12N²D + 10ND² + 22NO.
    split: (direction round, trial round) — a BLS inner iteration is one direction round and one trial
    round per line-search trial; GD = one of each.  k_lean's BLS (bls=True): the direction round is
    stage 1, G and the gradient-input mix; every trial forms its fp32 iterate with the exact residual
    (14·N·D), projects the residual (z, 2·Rz·N·D) and runs the F tiles and the direction mix before its
    evaluation (round 4: each trial evaluated at its own iterate).
    """
    Rz, Rf, Rg = ranks if ranks is not None else ((16, 16, 24) if (lean and R == 32) else (R, R, R))
    ev_f = 4 * N * D + 14 * N * O + 24 * N * D
    if bls and lean:
        dir_f = 2 * R * N * D + 2 * Rg * N * D + 4 * N * D * D
        trial_f = 14 * N * D + 2 * Rz * N * D + 4 * Rf * N * D + 4 * N * D * D + ev_f
    else:
        dir_f = (2 * R * N * D + 2 * Rz * N * D + 4 * Rf * N * D + 2 * Rg * N * D + 8 * N * D * D
                 + (7 if lean else 14) * N * D)
        trial_f = ev_f
    ref_f = 12 * N * N * D + 10 * N * D * D + 22 * N * O
    if split:
        return dir_f, trial_f, ref_f
    return dir_f + trial_f, ref_f


def plan_label(plan):
    """Kernel label of the launch the library reports (irm_optimize_plan: filled in by its own launch
    dispatch, so the label and the flop model's ranks are those of the kernel that runs)."""
    flows = {0: "GD single loop", 1: "GD dual loop", 2: "BLS dual loop"}
    return (f"irm::{plan['kernel']} ({flows[plan['flow']]}, {plan['waypoints_per_lane']} waypoint(s) per lane, "
            f"{plan['traj_per_block']} trajectories per {plan['threads']}-thread workgroup, ranks z/dir/G "
            f"{plan['rank_z']}/{plan['rank_dir']}/{plan['rank_g']}; fp32 MFMA 16x16x4 + VALU)")


def cpu_baseline_port(args, start, goal, obstacles, cores, budget_s=12.0):
    """The scalar C oracle (restatement of the reference, fp64-accumulated contractions, OpenMP over
    trajectories) on a bounded sample: full optimize() of each problem."""
    from irm_motion_planning_amd.params import params_from_args
    from oracle.oracle import Oracle
    p = params_from_args(args)
    orc = Oracle(p)
    t0 = time.perf_counter()
    _, st1 = orc.optimize_batch(None, start[:1], goal[:1], obstacles, n_threads=1)
    t1 = time.perf_counter() - t0
    n = int(max(cores, min(len(start), budget_s / max(t1, 1e-6) * cores)))
    n = max(cores, (n // cores) * cores)
    n = min(n, len(start))
    t0 = time.perf_counter()
    _, st = orc.optimize_batch(None, start[:n], goal[:n], obstacles, n_threads=cores)
    dt = time.perf_counter() - t0
    iters = sum(s["grad_evals"] for s in st)
    return {"value": iters / dt, "value_1thread": st1[0]["grad_evals"] / t1, "cores": cores,
            "label": "scalar C oracle (oracle/irm_oracle.c), one problem per thread",
            "sample": f"{n} of the {len(start)} rank-0 problems, full optimize() each ({iters} iterations, "
                      f"{dt:.2f} s wall on {cores} threads); 1-thread rate {st1[0]['grad_evals'] / t1:.1f} it/s"}


def cpu_baseline_batched(args, start, goal, obstacles, cores, budget_s=10.0):
    """The vectorised fp32 restatement (oracle/batched_np.py): the whole sample's α as one N × (B·D)
    matrix per worker, every contraction an OpenBLAS sgemm as the reference's XLA path contracts,
    one worker process per core (forked before this process touches the GPU).  GD bench mode only."""
    from irm_motion_planning_amd.params import params_from_args
    from oracle import batched_np
    from oracle.oracle import Oracle
    if args.optimizer_name != "gd" or args.max_outer_iteration > 1 or args.loop_loss_reduction > -1e29:
        return None  # the batched restatement runs the GD single loop with every step accepted
    p = params_from_args(args)
    orc = Oracle(p)
    _, K, dK, J = orc.kernel_matrices()
    iters = int(args.max_inner_iteration)
    a0 = np.stack([orc.init_alpha(start[b], goal[b]) for b in range(len(start))])
    # calibrate on one core, then size the sample to the budget
    _, _, w = batched_np.run_processes(K, dK, J, p, a0[:16], start[:16], goal[:16], obstacles, 4, 1)
    rate1 = 16 * 4 / w
    n = int(min(len(start), max(cores, budget_s * rate1 * cores / iters)))
    n = max(cores, (n // cores) * cores) if n >= cores else n
    t0 = time.perf_counter()
    _, _, wmax = batched_np.run_processes(K, dK, J, p, a0[:n], start[:n], goal[:n], obstacles, iters, cores)
    wall = time.perf_counter() - t0
    return {"value": n * iters / wmax, "value_1core": rate1, "cores": cores,
            "label": "vectorised fp32 batch (oracle/batched_np.py): numpy + OpenBLAS sgemm over N x (B*D), "
                     "one process per core",
            "sample": f"{n} of the {len(start)} rank-0 problems x {iters} GD iterations, split over {cores} "
                      f"processes ({wmax:.2f} s in the slowest, {wall:.2f} s wall incl. start-up); "
                      f"1-core rate {rate1:.1f} it/s"}


# CPU-baseline budgets (seconds of timed CPU work: scalar oracle, batched numpy).  At world > 1 the other
# ranks wait in the rendezvous while rank 0 times them, so they are capped there (CPU_BUDGET_MULTI_S)
# and init_process_group's timeout is set explicitly to cover the wait (rendezvous_timeout).
CPU_BUDGET_S = (12.0, 10.0)
CPU_BUDGET_MULTI_S = (4.0, 3.0)


def cpu_budgets(world):
    return CPU_BUDGET_S if world <= 1 else CPU_BUDGET_MULTI_S


def rendezvous_timeout(world):
    """init_process_group's timeout: it bounds the rendezvous, where the other ranks wait for rank 0's
    capped CPU-baseline work (measured sample ≈ budget, plus the 1-thread calibration runs and the worker
    pool's start-up: ≤ 120 + 10 × the budgets with a wide margin), and it also becomes the timeout of every
    later collective (the barriers around the warm-up and the timed loop), so it is never below the RCCL
    default of 10 minutes: a slow rank in context set-up or warm-up does not trip the watchdog early."""
    import datetime
    return datetime.timedelta(seconds=max(600, int(120 + 10 * sum(cpu_budgets(world)))))


def cpu_baseline(cfg, args, start, goal, obstacles, world=1):
    """Both CPU restatements timed on this host (rank 0's shard); `value` is the faster one."""
    cores = max(1, min(16, len(os.sched_getaffinity(0))))
    b_port, b_batched = cpu_budgets(world)
    port = cpu_baseline_port(args, start, goal, obstacles, cores, budget_s=b_port)
    batched = cpu_baseline_batched(args, start, goal, obstacles, cores, budget_s=b_batched)
    best = port if batched is None or port["value"] >= batched["value"] else batched
    return {"value": best["value"], "unit": ("GD" if args.optimizer_name == "gd" else "BLS") + " iterations/s",
            "cores": cores, "kind": "port", "sample": best["label"] + ": " + best["sample"],
            "value_1thread": port["value_1thread"],  # 1-thread and all-cores rates
            "variants": {"scalar_oracle": port, "batched_fp32_numpy": batched}}


def pmc_traffic(cfg):
    """HBM bytes per optimiser launch from the newest profiles/*_pmc.json (rocprofv3 FETCH_SIZE /
    WRITE_SIZE passes of this bench command, tools/profile_round.sh), or None."""
    import glob
    files = sorted(glob.glob(os.path.join(HERE, "profiles", "*_pmc.json")))
    for path in reversed(files):
        with open(path) as f:
            d = json.load(f)
        if d.get("config", "c3") == cfg and not d.get("faithful") and d.get("hbm_bytes_per_launch"):
            return float(d["hbm_bytes_per_launch"]), os.path.relpath(path, HERE)
    return None, None


def pmc_flops(cfg):
    """Issued fp32 flops per optimiser launch from the newest profiles/*_flops.json (rocprofv3 SQ
    instruction counters of this bench command, tools/pmc_flops.sh), or None."""
    import glob
    for path in reversed(sorted(glob.glob(os.path.join(HERE, "profiles", "*_flops.json")))):
        with open(path) as f:
            d = json.load(f)
        if d.get("config", "c3") == cfg and d.get("flops_per_launch"):
            return float(d["flops_per_launch"]), os.path.relpath(path, HERE)
    return None, None


def config_record(a, args, desc, B, N, D, O, opt, world, info, plan=None):
    """The workload as run: shape, mode and every hyper-parameter that departs from main.py's defaults."""
    from irm_motion_planning_amd import main as irm_main
    defaults = vars(irm_main.parse_args([]))
    overrides = {k: v for k, v in vars(args).items() if k in defaults and defaults[k] != v
                 and k not in ("optimizer_name", "n_timesteps", "n_joints")}
    return {
        "workload": f"{a.config}: {desc}",
        "batch_per_gpu": B, "global_batch": B * world, "n_timesteps": N, "n_joints": D, "n_obstacles": O,
        "optimizer": opt,
        "mode": "faithful" if a.faithful else (f"bench ({a.max_inner} fixed GD iterations)" if opt == "gd" else
                                               f"bench ({a.max_inner} fixed BLS inner iterations, each with its "
                                               "line search)"),
        "gd_lr_first": float(args.gd_lr[0]),
        "overrides_vs_reference_defaults": overrides,
        "operator_rank": None if info is None else info["operator_rank"],
        "traj_per_block": None if plan is None else plan["traj_per_block"],
        "parallelism": f"dp{world} (batch sharded, env broadcast over {'gloo' if (a.dist_backend == 'gloo' or a.dry_run) else 'RCCL'})",
    }


def launch_ranks(a):
    """`bench.py --gpus N` outside torchrun: start N ranks under torch.distributed.run as a CHILD
    process (nothing in this process has touched HIP) and relay rank 0's JSON line."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "1"))
    p = subprocess.run(cmd, stdout=subprocess.PIPE, env=env, text=True)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{") and '"metric"' in ln]
    for ln in p.stdout.splitlines():
        if ln not in lines:
            print(ln, file=sys.stderr)
    if lines:
        print(lines[-1], flush=True)
    return p.returncode if lines or p.returncode else 1


def share_environment(obs_t, world):
    """Rank 0's obstacles to every rank (RCCL broadcast over xGMI; gloo in the CPU tests)."""
    if world > 1:
        import torch.distributed as dist
        dist.broadcast(obs_t, src=0)
    return obs_t


def aggregate(elapsed, iters_rank, world, device):
    """(max elapsed over ranks, Σ executed iterations over ranks) — the weak-scaling reduction."""
    import torch
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    it = torch.tensor([iters_rank], dtype=torch.float64, device=device)
    if world > 1:
        import torch.distributed as dist
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(it, op=dist.ReduceOp.SUM)
    return float(t.item()), float(it.item())


def rank_values(x, world, device):
    """x of every rank, in rank order (all_gather of one float64)."""
    import torch
    t = torch.tensor([x], dtype=torch.float64, device=device)
    if world == 1:
        return [float(x)]
    import torch.distributed as dist
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [float(v.item()) for v in out]


def dry_run(a, world, rank):
    """The multi-rank plumbing of main() without the device: shard, environment broadcast, the
    max-time / Σ-iterations reduction.  Prints the JSON line with value null."""
    import torch
    import torch.distributed as dist
    desc, B, N, D, O, opt = CONFIGS[a.config]
    args = make_args(a.config, a.faithful, a.max_inner)
    start, goal, obstacles = make_problem(a.config, world, rank)
    obs = share_environment(torch.from_numpy(obstacles + (0.0 if rank == 0 else 1.0)), world)
    elapsed_max, iters_all = aggregate(1.0 + rank, float(B * a.max_inner), world, "cpu")
    same = torch.tensor([float(np.array_equal(obs.numpy(), obstacles if rank == 0 else obstacles))])
    if world > 1:
        dist.all_reduce(same, op=dist.ReduceOp.MIN)
    shard = torch.tensor([float(start.sum())], dtype=torch.float64)
    shards = [torch.zeros_like(shard) for _ in range(world)] if world > 1 else [shard]
    if world > 1:
        dist.all_gather(shards, shard)
    # the global-batch rows this rank's shard holds (make_problem's slice), gathered in rank order
    rng = torch.tensor([rank * B, (rank + 1) * B], dtype=torch.int64)
    ranges = [torch.zeros_like(rng) for _ in range(world)] if world > 1 else [rng]
    if world > 1:
        dist.all_gather(ranges, rng)
    world_seen = dist.get_world_size() if world > 1 else 1
    if rank == 0:
        print(json.dumps({"metric": ("GD" if opt == "gd" else "BLS") + " iterations/sec (batch of trajectories)",
                          "value": None, "dry_run": True,
                          "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
                          "config": config_record(a, args, desc, B, N, D, O, opt, world, None),
                          "obstacles_equal_rank0": bool(same.item() == 1.0),
                          "elapsed_max": elapsed_max, "iterations_all": iters_all,
                          "shard_checksums": [float(x.item()) for x in shards],
                          "shard_ranges": [[int(v) for v in x.tolist()] for x in ranges],
                          "world_size": world_seen,
                          "rendezvous_timeout_s": rendezvous_timeout(world).total_seconds()}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--faithful", action="store_true", help="reference control flow (early exits) instead of 200 fixed")
    ap.add_argument("--max-inner", type=int, default=200)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--operator-rank", type=int, default=0)
    ap.add_argument("--tb", type=int, default=0, help="trajectories per workgroup (0 = auto)")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="gloo: rehearse the multi-rank path with host-side collectives, ranks may share a GPU")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher / collective plumbing only (no device, no kernel): CPU tests of --gpus N")
    a = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        return launch_ranks(a)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        print(f"bench: --gpus {a.gpus} but WORLD_SIZE={world}; reporting the launched world", file=sys.stderr)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    gloo = a.dist_backend == "gloo"
    if gloo:  # rehearsal: ranks may outnumber the GPUs of the box (counting devices does not init HIP)
        local = local % max(1, torch.cuda.device_count())
    desc, B, N, D, O, opt = CONFIGS[a.config]
    args = make_args(a.config, a.faithful, a.max_inner)
    start, goal, obstacles = make_problem(a.config, world, rank)
    # The CPU baselines run first, before this process touches the GPU — and, at world > 1, before the
    # process group exists: init_process_group("nccl", device_id=…) forms the RCCL communicator
    # eagerly, which initialises HIP on the device, and the batched baseline forks worker processes.
    # The other ranks wait for rank 0 in the rendezvous meanwhile.
    cpu = None
    if rank == 0 and not a.no_cpu_baseline and not a.dry_run:
        cpu = cpu_baseline(a.config, args, start, goal, obstacles, world)
    if world > 1:
        tmo = rendezvous_timeout(world)
        if gloo or a.dry_run:
            dist.init_process_group("gloo", timeout=tmo)
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=tmo)
    if a.dry_run:
        return dry_run(a, world, rank)

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    cdev = torch.device("cpu") if gloo else dev  # where the collectives' tensors live

    from irm_motion_planning_amd.context import Context, batch_dev
    from irm_motion_planning_amd._abi import IrmStats
    from irm_motion_planning_amd.params import params_from_args

    # shared environment: rank 0's obstacles broadcast over RCCL/xGMI
    obs_t = share_environment(torch.from_numpy(obstacles).to(cdev), world).to(dev)
    start_t = torch.from_numpy(start).to(dev)
    goal_t = torch.from_numpy(goal).to(dev)
    alpha_t = torch.empty((B, N, D), dtype=torch.float32, device=dev)
    traj_t = torch.empty_like(alpha_t)
    stats_t = torch.zeros((B, 8), dtype=torch.int32, device=dev)  # irm_stats = 8 × 4 bytes

    ctx = Context(params_from_args(args, operator_rank=a.operator_rank, device=local, traj_per_block=a.tb))
    info = ctx.info()
    bd = batch_dev(start=start_t.data_ptr(), goal=goal_t.data_ptr(), obstacles=obs_t.data_ptr(), n_obstacles=O,
                   batch=B, alpha_out=alpha_t.data_ptr(), traj_out=traj_t.data_ptr(), stats_out=stats_t.data_ptr())
    stream = torch.cuda.current_stream(dev)

    def step():
        ctx.optimize_dev(bd, stream.cuda_stream)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    t0 = time.perf_counter()
    for e0, e1 in evs:
        e0.record(stream)
        step()
        e1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = float(np.mean([e0.elapsed_time(e1) for e0, e1 in evs]))

    st = stats_t.cpu().numpy()
    iters_rank = float(st[:, 2].sum())  # grad_evals = executed inner iterations
    trials_rank = float(st[:, 4].sum())  # BLS line-search trials (one evaluation round each)
    elapsed_max, iters_all = aggregate(elapsed, iters_rank, world, cdev)
    value = iters_all * a.steps / elapsed_max
    kernel_ms_ranks = rank_values(kernel_ms, world, cdev)  # what each rank's launches took
    world_seen = dist.get_world_size() if world > 1 else 1  # the ranks the collectives ran over

    plan = ctx.launch_plan(B, O)
    kernel = plan_label(plan)
    dir_f, trial_f, ref_f = flops_per_iteration(N, D, O, info["operator_rank"], split=True, lean=bool(plan["lean"]),
                                                ranks=(plan["rank_z"], plan["rank_dir"], plan["rank_g"]),
                                                bls=opt == "bls")
    exec_f = dir_f + trial_f
    # GD: one trial per iteration; BLS: the trials the line searches ran
    launch_flops = dir_f * iters_rank + trial_f * (trials_rank if opt == "bls" else iters_rank)
    achieved = launch_flops / (kernel_ms * 1e-3) / 1e12
    dense_tflops = ref_f * iters_rank / (kernel_ms * 1e-3) / 1e12
    bytes_launch = B * (2 * D + 2 * N * D) * 4 + B * 32  # start/goal in; alpha/traj/stats out
    canonical = a.max_inner == 200 and not a.faithful and a.tb == 0 and a.operator_rank == 0
    traffic, traffic_src = pmc_traffic(a.config) if canonical else (None, None)
    counted, counted_src = pmc_flops(a.config) if canonical else (None, None)
    result = {
        "metric": ("GD" if opt == "gd" else "BLS") + " iterations/sec (batch of trajectories)",
        "value": value,
        "unit": "iterations/s",
        "n_gpus": world,
        "world_size": world_seen,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": 1000 * elapsed_max / a.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (SURVEY.md §8d seeds), reference environment",
        "config": config_record(a, args, desc, B, N, D, O, opt, world, info, plan),
        "roofline": {
            # achieved = the flops one launch of THIS algorithm executes (the rank-R trajectory-space
            # GD iteration, DESIGN.md §5: exec_f per trajectory-iteration × the iterations of the
            # launch) ÷ the launch's average duration (HIP events on the launch stream).
            "bound": "mfma",
            "achieved": achieved,
            "peak": PEAK_FP32_TFLOPS,
            "unit": "TFLOP/s",
            "frac": achieved / PEAK_FP32_TFLOPS,
            "traffic": traffic,
            "traffic_source": traffic_src,
            "kernel": kernel,
            "kernel_ms": kernel_ms,
            "kernel_ms_per_rank": kernel_ms_ranks,
            "flops_per_iteration": exec_f,
            "flops_per_launch": launch_flops,
            "bls_trials_per_launch": trials_rank if opt == "bls" else None,
            # what the hardware issued, from rocprofv3 PMC counters of the same command
            # (MFMA + f32 VALU lane operations, padding lanes/columns included; tools/pmc_flops.sh)
            "counted_flops_per_launch": counted,
            "counted_tflops": None if counted is None else counted / (kernel_ms * 1e-3) / 1e12,
            "counted_frac": None if counted is None else counted / (kernel_ms * 1e-3) / 1e12 / PEAK_FP32_TFLOPS,
            "counted_source": counted_src,
            # SURVEY.md §8d's count of the reference's dense alpha-space formulation, for comparison only:
            # the same iterations priced at 12N²D + 10ND² + 22NO flops each (this kernel does not execute them)
            "dense_equivalent_flops_per_iteration": ref_f,
            "dense_equivalent_tflops": dense_tflops,
            "dense_equivalent_frac": dense_tflops / PEAK_FP32_TFLOPS,
            "hbm_algorithmic_bytes_per_launch": bytes_launch,
            "hbm_achieved_gbs": bytes_launch / (kernel_ms * 1e-3) / 1e9,
            "hbm_frac": bytes_launch / (kernel_ms * 1e-3) / 1e9 / PEAK_HBM_GBS,
        },
        "cpu_baseline": cpu,  # rank 0's host cores, its own shard, every world size
        "iterations_per_step": iters_all,
    }
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
