"""Diagnostic: dense operator (--operator-rank -1) vs the rank-32 default vs the oracle, per problem, at an
N = 256 bench shape (GPU box).  python tools/dense_diag.py [c3n256|c5] [B] [iters]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.getcwd())
import bench  # noqa: E402
from irm_motion_planning_amd.context import Context  # noqa: E402
from irm_motion_planning_amd.params import params_from_args  # noqa: E402
from oracle.oracle import Oracle, compute_cost_vg  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3n256"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 16
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 100
args = bench.make_args(cfg, False, iters)
s, g, obs = bench.make_problem(cfg, 1, 0)
s, g = s[:B], g[:B]
cd = Context(params_from_args(args, operator_rank=-1))
c32 = Context(params_from_args(args))
a0 = cd.init_alpha(s, g)
_, td, std = cd.optimize(s, g, obs, alpha0=a0)
_, t32, st32 = c32.optimize(s, g, obs, alpha0=a0)
o = Oracle(params_from_args(args))
for b in range(B):
    ao, so = o.optimize(a0[b], obs, s[b], g[b])
    To = o.evaluate(ao)
    cv, _ = compute_cost_vg(o.fk(o.evaluate(a0[b])), obs)
    top = np.sort(cv)[::-1]
    print(f"{cfg}[{b:2d}]: dense-oracle {np.abs(td[b] - To).max():.2e}  r32-oracle {np.abs(t32[b] - To).max():.2e}  "
          f"dense-r32 {np.abs(td[b] - t32[b]).max():.2e}  losses {std['final_loss'][b]:.6f} {st32['final_loss'][b]:.6f} "
          f"{so['final_loss']:.6f}  argmax margin at a0 {(top[0] - top[1]) / top[0]:.1e}")
