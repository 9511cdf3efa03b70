"""Diagnostic: line-search log of one BLS problem (first NaN / inf in it), GPU box.

  [IRM_LIB=…] python tools/nan_diag.py <config> <problem> [out.npy]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.getcwd())
import bench  # noqa: E402
from irm_motion_planning_amd.context import Context  # noqa: E402
from irm_motion_planning_amd.params import params_from_args  # noqa: E402

cfg, b = sys.argv[1], int(sys.argv[2])
args = bench.make_args(cfg, True, 200)
args.optimizer_name = "bls"
s, g, obs = bench.make_problem(cfg, 1, 0)
c = Context(params_from_args(args))
c.bls_trace_enable(4096)
alpha, traj, st = c.optimize(s[b:b + 1], g[b:b + 1], obs)
tr = c.bls_trace(int(st["bls_trials"][0]))
print("stats", {k: v[0] for k, v in st.items()}, "nan in alpha:", bool(np.isnan(alpha).any()))
bad = np.where(~np.isfinite(tr).all(1))[0]
print("trials", len(tr), "first non-finite row", bad[:1])
lo = max(0, (bad[0] if len(bad) else len(tr)) - 12)
np.set_printoptions(linewidth=200, precision=6)
print("outer inner trial lr new_loss required accepted loss gnorm anorm")
print(tr[lo:lo + 16])
if len(sys.argv) > 3:
    np.save(sys.argv[3], tr)
