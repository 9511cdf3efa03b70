"""Diagnostic: does a problem's result depend on its workgroup neighbours?

Runs BASELINE C3 (1024 problems, four per workgroup) in bench mode, then the same batch
permuted, and reports how many trajectories are bit-equal to their unpermuted result."""
import os
import sys

import numpy as np

sys.path.insert(0, os.getcwd())
import bench  # noqa: E402
from irm_motion_planning_amd.context import Context  # noqa: E402
from irm_motion_planning_amd.params import params_from_args  # noqa: E402

if __name__ == "__main__":
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    general = len(sys.argv) > 2 and sys.argv[2] == "general"
    if general:
        os.environ["IRM_GENERAL_KERNEL"] = "1"
    args = bench.make_args(cfg, False, 200)
    s, g, obs = bench.make_problem(cfg, 1, 0)
    c = Context(params_from_args(args))
    _, traj, st = c.optimize(s, g, obs)
    perm = np.random.default_rng(3).permutation(len(s))
    _, traj_p, _ = c.optimize(s[perm], g[perm], obs)
    eq = np.all(traj_p == traj[perm], axis=(1, 2))
    print(f"{cfg} {'general' if general else 'lean'}: permuted batch bit-equal for {eq.mean():.3f} of problems, "
          f"max |dT| {np.abs(traj_p - traj[perm]).max():.2e}", flush=True)
