"""Developer diagnostic (GPU box): how a bench-mode problem's HIP iterate departs from the CPU oracle's
step by step — gradual drift (an arithmetic error) or a jump (a max-cost argmax knife edge flipping).

    python tools/drift_diag.py c4 42 [64]        # config (suffix d: dense operator), problem, batch

For k in a ladder of step counts: |traj_HIP(k) − traj_oracle(k)|, the oracle's ±1-ulp spread at k, and
the max-cost waypoint of both runs with its margin over the runner-up (relative): a jump where the two
argmaxes part at a small margin is a knife edge of the max-cost term (trajectory.py:97)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import bench  # noqa: E402
from irm_motion_planning_amd.context import Context  # noqa: E402
from irm_motion_planning_amd.params import params_from_args  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402

name, b = sys.argv[1], int(sys.argv[2])
dense = name.endswith("d")
cfg = name[:-1] if dense else name
B = int(sys.argv[3]) if len(sys.argv) > 3 else 64
s, g, obs = bench.make_problem(cfg, 1, 0)
s, g = s[:B], g[:B]


def argmax_margin(o, traj):
    f = np.asarray(o.fk(np.asarray(traj, np.float32)), np.float64).reshape(2, -1)
    d2 = (f[0][:, None] - obs[None, :, 0]) ** 2 + (f[1][:, None] - obs[None, :, 1]) ** 2
    cv = (0.8 / (0.5 + 0.5 * d2)).sum(axis=1)
    i = np.argsort(cv)[::-1]
    return int(i[0]), int(i[1]), (cv[i[0]] - cv[i[1]]) / cv[i[0]]


ladder = [int(x) for x in os.environ.get("LADDER", "1,2,5,10,20,30,50,75,100,150,200").split(",")]
for k in ladder:
    args = bench.make_args(cfg, False, k)
    c = Context(params_from_args(args, operator_rank=-1 if dense else 0))
    a0 = c.init_alpha(s, g)
    _, traj, st = c.optimize(s, g, obs, alpha0=a0)
    o = Oracle(params_from_args(args))
    al, so = o.optimize(a0[b], obs, s[b], g[b])
    T = o.evaluate(al)
    sgn = np.random.default_rng(100).choice([-1.0, 1.0], a0[b].shape).astype(np.float32)
    ap = np.nextafter(a0[b], a0[b] + sgn * np.float32(np.inf)).astype(np.float32)
    ae, _ = o.optimize(ap, obs, s[b], g[b])
    spread = float(np.abs(o.evaluate(ae) - T).max())
    err = float(np.abs(traj[b] - T).max())
    mo, mh = argmax_margin(o, T), argmax_margin(o, traj[b])
    print(f"k={k:4d}  |HIP - oracle| {err:.3e}  spread {spread:.3e}  loss {float(st['final_loss'][b]):.7f} vs "
          f"{so['final_loss']:.7f}  argmax oracle {mo[0]} (2nd {mo[1]}, margin {mo[2]:.1e})  "
          f"HIP {mh[0]} (2nd {mh[1]}, margin {mh[2]:.1e})", flush=True)
