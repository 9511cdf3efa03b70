"""Diagnostic: does the BLS step direction ĝ = G/‖G‖ (optimizer_BLS.py:165) equal the IEEE division?

    python -m irm_motion_planning_amd.build --divchk          (here: the IRM_DIV_CHECK library)
    IRM_LIB=…/libirm_hip_divchk.so python tools/div_check.py  (GPU box)

The IRM_DIV_CHECK build compares, for every element of every line-search trial the fused trial stages
form (bls_gz, irm_kernels_impl.hpp), the shipped quotient div_rcp(G, ‖G‖, rcp_rn_of(‖G‖, ·)) and round 5's
div_rcp(G, ‖G‖, rcp_refined(‖G‖)) against __fdiv_rn(G, ‖G‖), and counts per workgroup.  Runs the
reference's default flow (BLS, faithful) on all 1024 C3 problems and on C2."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from irm_motion_planning_amd.context import Context  # noqa: E402
from irm_motion_planning_amd.params import params_from_args  # noqa: E402


def count(cfg, B=None):
    args = bench.make_args(cfg, True, 200)
    s, g, obs = bench.make_problem(cfg, 1, 0)
    if B:
        s, g = s[:B], g[:B]
    c = Context(params_from_args(args))
    _, _, st = c.optimize(s, g, obs)
    nb, K = 4096, 24
    buf = (ctypes.c_uint64 * (nb * K))()
    n = c.lib.irm_debug_phase_profile(c.handle, buf, nb)
    assert n > 0, "not the IRM_DIV_CHECK library"
    p = np.frombuffer(buf, dtype=np.uint64, count=n * K).reshape(n, K)
    mis, mis5, tot = (int(p[:, i].sum()) for i in range(3))
    print(f"{cfg}: {s.shape[0]} problems, {int(np.sum(st['bls_trials']))} line-search trials, {tot} quotients ĝ_i: "
          f"{mis} differ from the IEEE division (shipped: RN(1/‖G‖) reciprocal), "
          f"{mis5} with round 5's Newton-refined reciprocal ({mis5 / max(tot, 1):.2e})", flush=True)
    return mis


if __name__ == "__main__":
    bad = count("c3bls") + count("c2")
    sys.exit(1 if bad else 0)
