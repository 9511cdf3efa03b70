"""Developer diagnostic: lean vs general optimiser vs the exact-arithmetic iteration (GPU box)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from conftest import obstacles, params, ref_args  # noqa: E402
from irm_motion_planning_amd.context import Context  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402
from oracle.ref64 import Ref64  # noqa: E402
from irm_motion_planning_amd.params import params_from_args  # noqa: E402

for N, lm in ((256, "0"), (256, "0.5"), (128, "0")):
    argv = ["--optimizer-name", "gd", "--max-outer-iteration", "1", "--n-timesteps", str(N),
            "--loop-loss-reduction=-1e30", "--max-inner-iteration", "60", "--lambda-max-cost", lm]
    rng = np.random.default_rng(31)
    B = 16
    s = rng.uniform(-0.5, 0.5, (B, 3)).astype(np.float32)
    g = rng.uniform(0.2, 1.6, (B, 3)).astype(np.float32)
    lean = Context(params(*argv, traj_per_block=2))
    os.environ["IRM_GENERAL_KERNEL"] = "1"
    gen = Context(params(*argv, traj_per_block=2))
    del os.environ["IRM_GENERAL_KERNEL"]
    _, t1, _ = lean.optimize(s, g, obstacles())
    _, t2, _ = gen.optimize(s, g, obstacles())
    p = params_from_args(ref_args(*argv))
    o = Oracle(p)
    _, K, dK, J = o.kernel_matrices()
    r = Ref64(p, K, dK, J)
    e1 = e2 = 0.0
    for b in range(B):
        a0 = lean.init_alpha(s[b], g[b])
        a64, _, _ = r.gd_single(a0, obstacles(), s[b], g[b], 60)
        T64 = r.traj_vel(a64)[0]
        e1 = max(e1, float(np.abs(t1[b] - T64).max()))
        e2 = max(e2, float(np.abs(t2[b] - T64).max()))
    print(f"N={N} lmax={lm}: lean-vs-general {np.abs(t1 - t2).max():.2e}; vs exact: lean {e1:.2e} general {e2:.2e}",
          flush=True)
