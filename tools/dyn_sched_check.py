"""Diagnostic (GPU box): the DynShape general kernel under two builds (default vs iterative-ILP machine
scheduler, libirm_hip_dynilp.so) on the shapes of test_generic_shapes_match_reference_iteration — the
scheduler only reorders instructions, so the results must be bit-identical.

    IRM_LIB=…/libirm_hip_dynilp.so python tools/dyn_sched_check.py run gpurun_out/dyn_ilp.npz
    python tools/dyn_sched_check.py run gpurun_out/dyn_def.npz
    python tools/dyn_sched_check.py cmp gpurun_out/dyn_def.npz gpurun_out/dyn_ilp.npz"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

SHAPES = [(33, 3, None), (100, 3, None), (96, 4, [1.0, 0.8, 0.6, 0.4]), (200, 2, [1.5, 1.0]),
          (64, 5, [0.8, 0.7, 0.6, 0.5, 0.4])]


def run(out):
    from conftest import obstacles, params
    from irm_motion_planning_amd.context import Context
    res = {}
    for N, D, links in SHAPES:
        argv = ["--optimizer-name", "gd", "--max-outer-iteration", "1", "--max-inner-iteration", "15",
                "--loop-loss-reduction=-1e30", "--lambda-max-cost", "0", "--n-timesteps", str(N), "--n-joints", str(D)]
        if links:
            argv += ["--link-length"] + [str(x) for x in links]
        c = Context(params(*argv))
        rng = np.random.default_rng(N + D)
        s = rng.uniform(-0.5, 0.5, (6, D)).astype(np.float32)
        g = rng.uniform(0.2, 1.6, (6, D)).astype(np.float32)
        alpha, traj, st = c.optimize(s, g, obstacles())
        res[f"{N}_{D}_alpha"], res[f"{N}_{D}_traj"] = alpha, traj
        res[f"{N}_{D}_loss"] = np.asarray(st["final_loss"])
        print(N, D, c.launch_plan(6, 11)["kernel"], flush=True)
    np.savez(out, **res)


def cmp(a, b):
    A, B = np.load(a), np.load(b)
    bad = 0
    for k in A.files:
        same = np.array_equal(A[k].view(np.uint32), B[k].view(np.uint32))
        d = float(np.abs(A[k] - B[k]).max())
        print(f"{k:16s} {'bit-identical' if same else f'DIFFERS (max {d:.3e})'}")
        bad += not same
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    {"run": lambda: run(sys.argv[2]), "cmp": lambda: cmp(sys.argv[2], sys.argv[3])}[sys.argv[1]]()
