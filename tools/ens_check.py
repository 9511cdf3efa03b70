"""Developer diagnostic (GPU box): how far a problem's HIP end state lies from the oracle, against the
oracle's own sensitivity measured with growing ±1-ulp ensembles on α0 (2, 4, 8 members) — whether a
test's band under-samples a chaotic problem or the HIP path is off.

    python tools/ens_check.py c4:21 c4:42 c5d:12 pp:4
(c4 / c3 / c5 / c7: bench mode, 200 steps; c5d: C5 dense operator, 100 steps, 16 problems; pp: the
per-problem-obstacle test's O = 7 case, 30 steps)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import bench  # noqa: E402
from irm_motion_planning_amd.context import Context  # noqa: E402
from irm_motion_planning_amd.params import params_from_args  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402


def ensemble(o, a0, obs, s, g, T, L, n):
    sp, lsp = [], []
    for seed in range(n):
        sgn = np.random.default_rng(100 + seed).choice([-1.0, 1.0], a0.shape).astype(np.float32)
        ap = np.nextafter(a0, a0 + sgn * np.float32(np.inf)).astype(np.float32)
        ae, se = o.optimize(ap, obs, s, g)
        sp.append(float(np.abs(o.evaluate(ae) - T).max()))
        lsp.append(abs(se["final_loss"] - L))
    return np.array(sp), np.array(lsp)


for spec in sys.argv[1:]:
    name, b = spec.split(":")
    b = int(b)
    if name == "pp":
        from conftest import oracle_for, params
        args = ("--optimizer-name", "gd", "--max-outer-iteration", 1, "--max-inner-iteration", 30)
        c, o = Context(params(*args)), oracle_for(*args)
        rng = np.random.default_rng(5)
        B = 5
        s = rng.uniform(-0.5, 0.5, (B, 3)).astype(np.float32)
        g = rng.uniform(0.2, 1.6, (B, 3)).astype(np.float32)
        for O in (0, 1, 7):
            obs_all = rng.uniform(-3.5, 3.5, (B, O, 2)).astype(np.float32)
        _, traj, st = c.optimize(s, g, obs_all, obstacle_stride=14)
        obs = obs_all[b]
        a0 = c.init_alpha(s[b], g[b])
    else:
        dense = name.endswith("d")
        cfg = name[:-1] if dense else name
        iters = 100 if dense else 200
        B = 16 if dense else 64
        args = bench.make_args(cfg, False, iters)
        s, g, obs = bench.make_problem(cfg, 1, 0)
        s, g = s[:B], g[:B]
        c = Context(params_from_args(args, operator_rank=-1 if dense else 0))
        a0s = c.init_alpha(s, g)
        _, traj, st = c.optimize(s, g, obs, alpha0=a0s)
        o = Oracle(params_from_args(args))
        a0 = a0s[b]
    al, so = o.optimize(a0, obs, s[b], g[b])
    T = o.evaluate(al)
    err = float(np.abs(traj[b] - T).max())
    lerr = abs(float(st["final_loss"][b]) - so["final_loss"])
    sp, lsp = ensemble(o, a0, obs, s[b], g[b], T, so["final_loss"], 8)
    print(f"{spec}: |HIP - oracle| {err:.3e}, loss diff {lerr:.3e} (rel {lerr / abs(so['final_loss']):.1e}); "
          f"ensemble spread n=2 {sp[:2].max():.3e}  n=4 {sp[:4].max():.3e}  n=8 {sp.max():.3e}; "
          f"loss spread n=8 {lsp.max():.3e}; members {np.array2string(sp, precision=2)}", flush=True)
