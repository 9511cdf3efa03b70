"""Diagnostic: are the iterative-ILP-scheduled units bit-identical to the default scheduler?

  IRM_LIB=…/libirm_hip_defsched.so python tools/sched_check.py run gpurun_out/def.npz
  python tools/sched_check.py run gpurun_out/ilp.npz
  python tools/sched_check.py cmp gpurun_out/def.npz gpurun_out/ilp.npz

The machine scheduler only reorders instructions; a kernel whose results change with it has a
miscompile or an ordering bug, so every case below must compare bit for bit."""
import os
import sys

import numpy as np

sys.path.insert(0, os.getcwd())
import bench  # noqa: E402
from irm_motion_planning_amd.context import Context  # noqa: E402
from irm_motion_planning_amd.params import params_from_args  # noqa: E402

CASES = [  # (name, config, faithful, batch, general kernel, optimizer override)
    ("c3_bench_lean", "c3", False, 256, False, None),
    ("c3_bench_general", "c3", False, 256, True, None),
    ("c3_faithful", "c3", True, 256, False, None),
    ("c3_bls", "c3", True, 64, False, "bls"),
    ("c2_bls", "c2", True, 1, False, None),
    ("c4_bench_lean", "c4", False, 64, False, None),
    ("c4_faithful", "c4", True, 64, False, None),
    ("c5_bench_general", "c5", False, 32, True, None),
    ("c7_faithful", "c7", True, 64, False, None),
    ("c7_bls", "c7", True, 16, False, "bls"),
    ("c5_dense", "c5", False, 32, False, None, -1),  # (operator rank) k_optimize at R = N, L2 operands
    ("c3_dense_faithful", "c3", True, 32, False, None, -1),
    # the GD single loop at one wave per trajectory (N ≤ 64: no G tiles after the stage-2 barrier there)
    ("n50_bench_lean", "c3", False, 256, False, None, 0, {"n_timesteps": 50}),
    ("n64_bench_lean", "c3", False, 256, False, None, 0, {"n_timesteps": 64}),
    # the BLS flow: its bench mode (every trial round of 200 inner iterations, all-rejected searches going on
    # at the same α), the reference flow on a whole batch, and the one-wave-per-trajectory shapes
    ("c3bls_bench", "c3bls", False, 256, False, None),
    ("c3bls_faithful", "c3bls", True, 256, False, None),
    ("n64_bls", "c3", True, 64, False, "bls", 0, {"n_timesteps": 64}),
    ("n50_bls", "c3", True, 64, False, "bls", 0, {"n_timesteps": 50}),
]


def run(out):
    res = {}
    only = os.environ.get("IRM_CASES")
    for name, cfg, faithful, B, general, opt, *extra in CASES:
        if only and name not in only.split(","):
            continue
        rank = [extra[0]] if extra and extra[0] else []
        args = bench.make_args(cfg, faithful, 200)
        if opt:
            args.optimizer_name = opt
        for k, v in (extra[1] if len(extra) > 1 else {}).items():
            setattr(args, k, v)
        s, g, obs = bench.make_problem(cfg, 1, 0)
        if general:
            os.environ["IRM_GENERAL_KERNEL"] = "1"
        try:
            c = Context(params_from_args(args, operator_rank=rank[0]) if rank else params_from_args(args))
        finally:
            os.environ.pop("IRM_GENERAL_KERNEL", None)
        alpha, traj, st = c.optimize(s[:B], g[:B], obs)
        res[name + "_traj"] = traj
        res[name + "_alpha"] = alpha
        res[name + "_evals"] = np.asarray(st["grad_evals"])
        res[name + "_trials"] = np.asarray(st["bls_trials"])
        print(name, "done", flush=True)
    np.savez(out, **res)


def cmp(a, b):
    A, Bz = np.load(a), np.load(b)
    bad = 0
    for k in sorted(A.files):
        eq = np.array_equal(A[k], Bz[k])
        bad += not eq
        print(f"{k:28s} {'bit-equal' if eq else 'DIFFERS max ' + str(np.abs(A[k].astype(np.float64) - Bz[k]).max())}")
    print("all bit-equal" if bad == 0 else f"{bad} arrays differ")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2])
    else:
        cmp(sys.argv[2], sys.argv[3])
