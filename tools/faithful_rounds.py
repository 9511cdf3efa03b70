"""Diagnostic: per-problem round counts of a faithful run (GPU box) — is the launch bound by its slowest
problem?  A round of k_lean is one evaluation of every live trajectory of a workgroup: GD — one
iteration (grad + step + cost); BLS — one line-search trial (the inner-loop head's direction is formed
in the round of trial 0), plus one resync round per outer iteration (α's exact trajectory and
constraintsFulfilled).  Prints the distribution over problems, the per-workgroup maximum (a workgroup
runs until its slowest trajectory stops), the share of trajectory-rounds that do work, and the time per
round of the timed launch.

    python tools/faithful_rounds.py [c3|c3bls] [--tb 4]
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.getcwd())
import bench  # noqa: E402
from irm_motion_planning_amd.context import Context  # noqa: E402
from irm_motion_planning_amd.params import params_from_args  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else "c3"
tb = int(sys.argv[sys.argv.index("--tb") + 1]) if "--tb" in sys.argv else 0
args = bench.make_args(cfg, True, 200)
s, g, obs = bench.make_problem(cfg, 1, 0)
c = Context(params_from_args(args, traj_per_block=tb))
plan = c.launch_plan(len(s), len(obs))
c.optimize(s, g, obs)  # warm-up
t0 = time.perf_counter()
_, _, st = c.optimize(s, g, obs)
wall = time.perf_counter() - t0
ge, oi, tr = (np.asarray(st[k]) for k in ("grad_evals", "outer_iterations", "bls_trials"))
bls = args.optimizer_name == "bls"
rounds = (tr if bls else ge) + oi
T = plan["traj_per_block"]
wg_max = np.array([rounds[i:i + T].max() for i in range(0, len(rounds), T)])
busy = rounds.sum() / (wg_max.repeat(T)[: len(rounds)].sum())
print(f"{cfg} faithful, {plan['kernel']}: {len(ge)} problems, {T} per workgroup")
print(f"  inner iterations (grad evals) mean {ge.mean():.1f} max {ge.max()}; outer mean {oi.mean():.2f} max {oi.max()}"
      + (f"; line-search trials mean {tr.mean():.1f} ({tr.sum() / ge.sum():.2f} per iteration)" if bls else ""))
print(f"  rounds per problem: mean {rounds.mean():.1f} p50 {np.percentile(rounds, 50):.0f} "
      f"p90 {np.percentile(rounds, 90):.0f} p99 {np.percentile(rounds, 99):.0f} max {rounds.max()}")
print(f"  per-workgroup max: mean {wg_max.mean():.1f} max {wg_max.max()}; trajectory-rounds doing work {busy:.1%} "
      f"of the workgroups' rounds, {rounds.sum() / (rounds.max() * len(rounds)):.1%} of the launch's")
print(f"  launch (host wall incl. copies) {wall * 1e3:.2f} ms = {wall * 1e6 / rounds.max():.2f} us per round of the "
      f"slowest problem")
