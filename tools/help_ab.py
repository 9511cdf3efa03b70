"""Developer check (GPU box): k_lean's BLS line-search helpers change no result — a whole batch (default:
C3-BLS faithful, 1024 problems) with the helpers on and off (IRM_LEAN_NOHELP) must agree bit for bit in α,
trajectory and every statistic; prints the launch times of both.

    python tools/help_ab.py [c3bls] [1024]
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.getcwd())
import bench  # noqa: E402
from irm_motion_planning_amd.context import Context  # noqa: E402
from irm_motion_planning_amd.params import params_from_args  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3bls"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
s, g, obs = bench.make_problem(cfg, 1, 0)
s, g = s[:B], g[:B]
res = []
for off in ("1", "0"):
    os.environ["IRM_LEAN_NOHELP"] = off
    c = Context(params_from_args(bench.make_args(cfg, True, 200)))
    c.optimize(s, g, obs)
    t0 = time.perf_counter()
    out = c.optimize(s, g, obs)
    res.append((out, time.perf_counter() - t0))
(a0, t0_, st0), w0 = res[0]
(a1, t1_, st1), w1 = res[1]
same = np.array_equal(a0, a1) and np.array_equal(t0_, t1_) and all(np.array_equal(st0[k], st1[k]) for k in st0)
print(f"{cfg} x{B}: helpers off {w0 * 1e3:.2f} ms, on {w1 * 1e3:.2f} ms (host wall); results bit-identical: {same}")
if not same:
    bad = np.nonzero(np.any((t0_ != t1_).reshape(B, -1), axis=1))[0]
    print("  differing problems:", bad[:20].tolist())
    sys.exit(1)
