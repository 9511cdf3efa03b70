"""Diagnostic: per-problem iteration counts of the faithful C3 run (GPU box) — is the launch bound by
its slowest problem?  Prints mean / max executed iterations and outer iterations over the batch."""
import os
import sys

import numpy as np

sys.path.insert(0, os.getcwd())
import bench  # noqa: E402
from irm_motion_planning_amd.context import Context  # noqa: E402
from irm_motion_planning_amd.params import params_from_args  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
args = bench.make_args(cfg, True, 200)
s, g, obs = bench.make_problem(cfg, 1, 0)
c = Context(params_from_args(args))
_, _, st = c.optimize(s, g, obs)
ge, oi = np.asarray(st["grad_evals"]), np.asarray(st["outer_iterations"])
rounds = ge + oi  # one resync round per outer iteration
print(f"{cfg} faithful: {len(ge)} problems, iterations mean {ge.mean():.1f} max {ge.max()}, "
      f"outer mean {oi.mean():.2f} max {oi.max()}, rounds (iterations + resyncs) max {rounds.max()}, "
      f"p50 {np.percentile(rounds, 50):.0f} p90 {np.percentile(rounds, 90):.0f} p99 {np.percentile(rounds, 99):.0f}")
