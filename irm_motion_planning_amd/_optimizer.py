"""Shared body of the two optimizer classes (one persistent HIP launch per optimize())."""
import time

import numpy as np

from .environment import Environment
from .trajectory import Trajectory


class _PersistentOptimizer:
    """Reference object API: Optimizer(args); .optimize() -> α; .env; .trajectory.

    optimize() runs the whole outer/inner(/line-search) loop of the reference's
    jit variant in one persistent launch (k_lean or k_optimize, Context.launch_plan).
    With --extended-vis it also returns the per-iteration trajectory series the reference's plain loop
    records (in both loop modes — the reference supports it only with
    --jit-loop false).
    """

    kind = None

    def __init__(self, args, **overrides):
        self.args = args
        self.jitLoop = args.jit_loop
        self.extendedVis = args.extended_vis
        self.max_inner_iteration = args.max_inner_iteration
        self.max_outer_iteration = args.max_outer_iteration
        self.loop_loss_reduction = args.loop_loss_reduction
        self.lambda_constraint_increase = args.lambda_constraint_increase
        self.lambda_sg_constraint = args.lambda_sg_constraint
        self.lambda_jl_constraint = args.lambda_jl_constraint
        self.lambda_max_cost = args.lambda_max_cost
        self.lambda_reg = args.lambda_reg
        overrides.setdefault("record_series", 1 if self.extendedVis else 0)
        for knob in ("operator_rank", "device"):
            if hasattr(args, knob):
                overrides.setdefault(knob, getattr(args, knob))
        self.env = Environment()
        self.trajectory = Trajectory(args, **overrides)
        self.context = self.trajectory.context
        self.last_stats = None
        self.last_profile = {}
        t1 = time.time()
        self.optimize()  # the reference's warm-up (= XLA compile); here: first launch
        t2 = time.time()
        print("setup object, jit-compile took", 1000 * (t2 - t1), "ms")

    # ------------------------------------------------------------------ API
    def optimize(self):
        t0 = time.perf_counter()
        res = self.context.optimize(self.env.start_config, self.env.goal_config, self.env.obstacles,
                                    series=self.extendedVis)
        self.last_profile = {"optimize_ms": 1000 * (time.perf_counter() - t0)}
        if self.extendedVis:
            alpha, traj, stats, series = res
            self.last_stats = stats
            return alpha, [np.array(s) for s in series]
        alpha, traj, stats = res
        self.last_stats = stats
        self.last_trajectory = traj
        return alpha

    def optimize_batch(self, start, goal, obstacles=None, alpha0=None, obstacle_stride=0, series=False):
        """Batched optimize(): B independent start/goal problems (B×D each).

        Returns (alpha, traj, stats) — plus the B × S × N × D snapshot buffer with
        series=True (stats["series_len"] frames valid per problem)."""
        obstacles = self.env.obstacles if obstacles is None else obstacles
        start = np.asarray(start, np.float32).reshape(-1, self.trajectory.robot.N_joints)
        goal = np.asarray(goal, np.float32).reshape(-1, self.trajectory.robot.N_joints)
        res = self.context.optimize(start, goal, obstacles, alpha0=alpha0, obstacle_stride=obstacle_stride,
                                    series=series)
        self.last_stats = res[2]
        return res
