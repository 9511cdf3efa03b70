"""Diagnostic: the smoke() problem (reference environment, GD, N=50) — HIP vs the CPU oracle after
k = 1..20 steps from the same α0 (|traj − oracle|∞, differing α elements, losses)."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from irm_motion_planning_amd import main as irm_main  # noqa: E402
from irm_motion_planning_amd.context import Context  # noqa: E402
from irm_motion_planning_amd.environment import GOAL_CONFIG, OBSTACLES, START_CONFIG  # noqa: E402
from irm_motion_planning_amd.params import params_from_args  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402

obs = OBSTACLES.astype(np.float32)
for k in list(range(1, 21)):
    args = irm_main.parse_args(["--optimizer-name", "gd", "--max-outer-iteration", "1",
                                "--max-inner-iteration", str(k)])
    c = Context(params_from_args(args))
    o = Oracle(params_from_args(args))
    a0 = c.init_alpha(START_CONFIG, GOAL_CONFIG)
    al, tr, st = c.optimize(START_CONFIG, GOAL_CONFIG, obs, alpha0=a0)
    alo, sto = o.optimize(a0, obs, START_CONFIG, GOAL_CONFIG)
    tro = o.evaluate(alo)
    print(f"k={k:3d} |traj - oracle| {np.abs(tr - tro).max():.3e}  alpha differing {int(np.sum(al != alo)):4d}/{al.size} "
          f"max|dalpha| {np.abs(al - alo).max():.2e} loss {float(st['final_loss']):.7f} vs {sto['final_loss']:.7f}",
          flush=True)
    c.close()
