"""Developer diagnostic (GPU box): kernel rounds and helper rounds per problem of a BLS faithful batch
(IRM_TRACE_PROBLEM bit 29 makes k_lean report them in series_len: rounds | helper rounds << 16), with
the line-search trials each problem took, for the slowest problems.

    python tools/help_rounds.py [c3bls] [1024]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.getcwd())
import bench  # noqa: E402
from irm_motion_planning_amd.context import Context  # noqa: E402
from irm_motion_planning_amd.params import params_from_args  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3bls"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
s, g, obs = bench.make_problem(cfg, 1, 0)
s, g = s[:B], g[:B]
for off in ("1", "0"):
    os.environ["IRM_LEAN_NOHELP"] = off
    os.environ["IRM_TRACE_PROBLEM"] = str(1 << 29)
    c = Context(params_from_args(bench.make_args(cfg, True, 200)))
    _, _, st = c.optimize(s, g, obs)
    sl = np.asarray(st["series_len"])
    rounds, hm = sl & 0xFFFF, sl >> 16
    tr = np.asarray(st["bls_trials"]) + np.asarray(st["outer_iterations"])
    i = np.argsort(rounds)[::-1][:5]
    print(f"helpers {'off' if off == '1' else 'on'}: kernel rounds max {rounds.max()} mean {rounds.mean():.1f}; slowest: "
          + ", ".join(f"#{k} {rounds[k]} rounds ({hm[k]} helper rounds, {tr[k]} trials+outer)" for k in i))
