"""Diagnostic: bit-equality of the optimiser kernels across workgroup shapes.

For GD single-loop problems, compares the lean kernel (k_lean) and the general
kernel (IRM_GENERAL_KERNEL=1) with and without wave padding (IRM_PAD_WAVES) and at a
fixed trajectories-per-workgroup; prints the fraction of bit-equal trajectories."""
import os
import sys

import numpy as np

sys.path.insert(0, os.getcwd())
from irm_motion_planning_amd import main as irm_main  # noqa: E402
from irm_motion_planning_amd.context import Context  # noqa: E402
from irm_motion_planning_amd.environment import OBSTACLES  # noqa: E402
from irm_motion_planning_amd.params import params_from_args  # noqa: E402

obs = OBSTACLES.astype(np.float32)


def run(argv, B, pad, general, tb=0):
    os.environ["IRM_PAD_WAVES"] = "1" if pad else "0"
    if general:
        os.environ["IRM_GENERAL_KERNEL"] = "1"
    else:
        os.environ.pop("IRM_GENERAL_KERNEL", None)
    rng = np.random.default_rng(31)
    s = rng.uniform(-0.5, 0.5, (B, 3)).astype(np.float32)
    g = rng.uniform(0.2, 1.6, (B, 3)).astype(np.float32)
    c = Context(params_from_args(irm_main.parse_args(argv), traj_per_block=tb))
    return c.optimize(s, g, obs)


def cmp(tag, r1, r2):
    t1, t2 = r1[1], r2[1]
    print(tag, "bit-equal traj frac", np.mean(np.all(t1 == t2, axis=(1, 2))), "max", np.abs(t1 - t2).max(), flush=True)


if __name__ == "__main__":
    for N in (50, 128):
        argv = ["--optimizer-name", "gd", "--max-outer-iteration", "1", "--n-timesteps", str(N),
                "--loop-loss-reduction=-1e30", "--max-inner-iteration", "60"]
        for tb in (2, 4):
            cmp(f"N={N} tb={tb} lean vs general", run(argv, 48, 0, 0, tb), run(argv, 48, 0, 1, tb))
        cmp(f"N={N} lean tb=1 vs tb=4", run(argv, 48, 0, 0, 1), run(argv, 48, 0, 0, 4))
        cmp(f"N={N} general tb=1 vs tb=4", run(argv, 48, 0, 1, 1), run(argv, 48, 0, 1, 4))
        cmp(f"N={N} lean tb=1 pad vs nopad", run(argv, 48, 1, 0, 1), run(argv, 48, 0, 0, 1))
