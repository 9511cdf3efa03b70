"""Diagnostic: run-to-run determinism and padded-vs-unpadded bit-equality of generic (DynShape) shapes."""
import os, sys
import numpy as np
sys.path.insert(0, os.getcwd())
from irm_motion_planning_amd import main as irm_main
from irm_motion_planning_amd.context import Context
from irm_motion_planning_amd.params import params_from_args
from irm_motion_planning_amd.environment import OBSTACLES
obs = OBSTACLES.astype(np.float32)
for N, D, links in ((64, 5, [0.8, 0.7, 0.6, 0.5, 0.4]), (96, 4, [1.0, 0.8, 0.6, 0.4]), (33, 3, None)):
    for pad in ("1", "0"):
        os.environ["IRM_PAD_WAVES"] = pad
        argv = ["--optimizer-name", "gd", "--max-outer-iteration", "1", "--max-inner-iteration", "15",
                "--loop-loss-reduction=-1e30", "--lambda-max-cost", "0", "--n-timesteps", str(N), "--n-joints", str(D)]
        if links: argv += ["--link-length"] + [str(x) for x in links]
        c = Context(params_from_args(irm_main.parse_args(argv)))
        rng = np.random.default_rng(N + D)
        s = rng.uniform(-0.5, 0.5, (6, D)).astype(np.float32); g = rng.uniform(0.2, 1.6, (6, D)).astype(np.float32)
        outs = [c.optimize(s, g, obs)[1] for _ in range(8)]
        same = all(np.array_equal(outs[0], o) for o in outs[1:])
        print(f"N={N} D={D} pad={pad}: 8 runs bit-identical: {same}", flush=True)
        if pad == "1": ref = outs[0]
        else: print(f"   padded vs unpadded bit-identical: {np.array_equal(ref, outs[0])}, max {np.abs(ref-outs[0]).max():.2e}", flush=True)
