"""CPU model: how sparse the dense rounds' velocity half of stage 1 is (profiles/r06_pack_ab.txt).

    python tools/vsparse.py [c3]

Runs the reference's GD iteration in bench mode (oracle/batched_np.py, fp32 BLAS) on 64 problems for 200
steps and, per step and four-trajectory workgroup, asks whether any trajectory has an active joint-velocity
mask away from the endpoints (a dense round: b' ≠ 0 there, trajectory.py:251, 259-268) and which of the
16-waypoint k-quads hold such a row."""
import os
import sys

import numpy as np

sys.path.insert(0, os.getcwd())
import bench  # noqa: E402
from oracle.batched_np import BatchedGD  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402
from irm_motion_planning_amd.params import params_from_args  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
B = 64
args = bench.make_args(cfg, False, 200)
p = params_from_args(args)
o = Oracle(p)
s, g, obs = bench.make_problem(cfg, 1, 0)
s, g = s[:B], g[:B]
a = np.stack([o.init_alpha(s[b], g[b]) for b in range(B)])
_, K, dK, J = o.kernel_matrices()
bg = BatchedGD(K, dK, J, p)
thr = p.joint_safety_limit * p.max_joint_velocity
dense, rounds, frac = 0, 0, []
for _ in range(200):
    V = np.einsum("nm,bmd,de->bne", dK, a, J)
    act = (np.abs(V) > thr).any(axis=2)
    act[:, 0] = act[:, -1] = False  # the endpoint rows enter through their own MFMA
    for w in range(B // 4):
        m = act[4 * w:4 * w + 4].any(axis=0)
        rounds += 1
        if m.any():
            dense += 1
            frac.append(m.reshape(-1, 16).any(axis=1).mean())
    a, _ = bg.run(a, s, g, obs, 1)
print(f"{cfg}: dense rounds {dense / rounds:.2f}; in dense rounds, mean fraction of 16-waypoint k-quads "
      f"with an active row {np.mean(frac):.2f}")
