"""Diagnostic (GPU box): where a batched C3-BLS problem's line-search log first parts from the oracle's.

    python tools/bls_flip.py 60 [64]

Runs problem P at batch slot 0 of the first `B` C3-BLS problems (four trajectories per workgroup), with the
line-search helpers on (helper rounds annotated: outer + 100, the helper's trial + 1000) and off
(IRM_LEAN_NOHELP=1), and the oracle from the same α0; prints the first decision flip of each log against
the oracle's (tests/test_gpu_parity.py::first_decision_flip) and the rows around it."""
import os
import sys

import numpy as np

sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "tests")]
import bench  # noqa: E402
from irm_motion_planning_amd.context import Context  # noqa: E402
from irm_motion_planning_amd.params import params_from_args  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402
from test_gpu_parity import first_decision_flip, loss_drift  # noqa: E402

P = int(sys.argv[1])
B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
s, g, obs = bench.make_problem("c3bls", 1, 0)
s, g = s[:B].copy(), g[:B].copy()
idx = np.arange(B)
idx[0], idx[P] = P, 0
args = bench.make_args("c3bls", True, 200)
np.set_printoptions(linewidth=220, precision=8, suppress=False)
o = None
for nohelp in ("0", "1"):
    os.environ["IRM_LEAN_NOHELP"] = nohelp
    os.environ["IRM_TRACE_PROBLEM"] = str(1 << 30)
    c = Context(params_from_args(args, traj_per_block=4))
    c.bls_trace_enable(4096)
    a0 = c.init_alpha(s[P], g[P])
    _, traj, st = c.optimize(s[idx], g[idx], obs)
    tr = c.bls_trace(int(st["bls_trials"][0]))
    if o is None:
        o = Oracle(params_from_args(args))
        _, so, tro = o.optimize_trace(a0, obs, s[P], g[P], cap=4096)
        print(f"oracle: {len(tro)} trials, grad evals {so['grad_evals']}, ok {so['constraints_ok']}")
    strip = tr.copy()
    strip[:, 0] %= 100
    strip[:, 2] %= 1000
    flip = first_decision_flip(strip, tro, float(args.loop_loss_reduction))
    drift = loss_drift(strip, tro, flip[0]) if flip else 0.0
    print(f"helpers {'off' if nohelp == '1' else 'on'}: {len(tr)} trials, grad evals {int(st['grad_evals'][0])}, "
          f"ok {int(st['constraints_ok'][0])}, first flip {flip}, drift {drift:.2e}")
    if nohelp == "0":
        np.savez(os.path.join("gpurun_out", f"flip{P}.npz"), a0=a0, tr=tr, tro=tro)
    if flip:
        k = flip[0]
        cols = "outer inner trial lr new_loss required acc loss |g| anorm"
        print("   kernel rows", max(0, k - 4), "..", k + 2, "(", cols, ")")
        print(tr[max(0, k - 4):k + 3])
        print("   oracle rows")
        print(tro[max(0, k - 4):k + 3])

# The max-cost argmax (trajectory.py:97) along both runs: the extended-vis frames (one per accepted inner
# iteration; the kernel's own waypoint state) of the kernel and the oracle from the same α0 — the first
# frame whose max-cost waypoints differ, and the two runs' relative potential gaps between them there.
from oracle.oracle import compute_cost_vg  # noqa: E402
os.environ["IRM_LEAN_NOHELP"] = "0"
os.environ.pop("IRM_TRACE_PROBLEM", None)
c = Context(params_from_args(args, traj_per_block=4))
_, _, st, ser = c.optimize(s[idx], g[idx], obs, series=True)
fk = ser[0][: int(st["series_len"][0])]
_, so, fo = o.optimize(a0, obs, s[P], g[P], max_series=4096)
n = min(len(fk), len(fo))
print(f"frames: kernel {len(fk)}, oracle {len(fo)}; |traj| diff at frames 0, 1, 2, 5, 10, 20, 30:",
      [f"{np.abs(fk[i] - fo[i]).max():.1e}" for i in (0, 1, 2, 5, 10, 20, 30) if i < n])
drift = 0.0
for i in range(n):
    cg = compute_cost_vg(o.fk(fk[i]), obs)[0]
    co = compute_cost_vg(o.fk(fo[i]), obs)[0]
    ag, ao = int(np.argmax(cg)), int(np.argmax(co))
    if ag != ao:
        m = min((cg[ag] - cg[ao]) / cg[ag], (co[ao] - co[ag]) / co[ao])
        print(f"frame {i}: max-cost waypoint kernel {ag} / oracle {ao}, margin {m:.2e}, potential drift before {drift:.2e}, "
              f"|traj| diff {np.abs(fk[i] - fo[i]).max():.2e}")
        break
    drift = max(drift, float(np.max(np.abs(cg - co)) / np.max(co)))
else:
    print(f"{n} frames: the same max-cost waypoint throughout")
