"""Diagnostic: operator rank vs accuracy and speed.

For each rank R, runs bench-mode GD (200 steps) on a slice of a BASELINE config and compares
each checked problem with the exact-arithmetic reference iteration (oracle/ref64.py), printing
|traj − exact| next to the exact iteration's own ±1-ulp sensitivity (the parity band of
tests/test_gpu_parity.py::_bench_vs_ref), then times the full-size launch."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.getcwd())
import bench  # noqa: E402
from irm_motion_planning_amd.context import Context  # noqa: E402
from irm_motion_planning_amd.params import params_from_args  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402
from oracle.ref64 import Ref64  # noqa: E402


def band(r, a0, obs, s, g, iters):
    a64, l64, _ = r.gd_single(a0, obs, s, g, iters)
    T64 = r.traj_vel(a64)[0]
    spread = 0.0
    for seed in range(2):
        sgn = np.random.default_rng(100 + seed).choice([-1.0, 1.0], a0.shape).astype(np.float32)
        ap = np.nextafter(a0, a0 + sgn * np.float32(np.inf)).astype(np.float32)
        ae, _, _ = r.gd_single(ap, obs, s, g, iters)
        spread = max(spread, float(np.abs(r.traj_vel(ae)[0] - T64).max()))
    return T64, l64, spread


if __name__ == "__main__":
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    ranks = [int(x) for x in sys.argv[2:]] or [32, 24, 16]
    args = bench.make_args(cfg, False, 200)
    s, g, obs = bench.make_problem(cfg, 1, 0)
    p0 = params_from_args(args)
    o = Oracle(p0)
    _, K, dK, J = o.kernel_matrices()
    r = Ref64(p0, K, dK, J)
    check = [0, 100, 500, 1000][: 3 if len(s) < 1001 else 4]
    ref = {}
    for R in ranks:
        c = Context(params_from_args(args, operator_rank=R))
        _, traj, st = c.optimize(s, g, obs)
        errs = []
        for b in check:
            a0 = c.init_alpha(s[b], g[b])
            if b not in ref:
                ref[b] = band(r, a0, obs, s[b], g[b], 200)
            T64, l64, spread = ref[b]
            errs.append((float(np.abs(traj[b] - T64).max()), spread, float(st["final_loss"][b]) - l64))
        import ctypes  # noqa: F401
        t0 = time.perf_counter()
        for _ in range(5):
            c.optimize(s, g, obs)
        dt = (time.perf_counter() - t0) / 5
        print(f"{cfg} R={R}: info rank {c.info()['operator_rank']}, host optimize {dt * 1e3:.2f} ms; "
              + "; ".join(f"err {e:.2e} spread {sp:.2e} dloss {dl:.1e}" for e, sp, dl in errs), flush=True)
