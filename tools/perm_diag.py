"""Developer diagnostic (GPU box): which problems of a batched BLS / GD-dual run change under a permutation of
the batch, with k_lean's line-search helpers on and off (IRM_LEAN_NOHELP), and whether the stage-1 dense
flag decides it (IRM_LEAN_DENSE=1 forces every round dense).

    python tools/perm_diag.py [c3bls] [64]
"""
import os
import sys

import numpy as np

sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "tests")]
import bench  # noqa: E402
from irm_motion_planning_amd.context import Context  # noqa: E402
from irm_motion_planning_amd.params import params_from_args  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3bls"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
s, g, obs = bench.make_problem(cfg, 1, 0)
s, g = s[:B], g[:B]
perm = np.random.default_rng(5).permutation(B)
for env in ({"IRM_LEAN_NOHELP": "0"}, {"IRM_LEAN_NOHELP": "1"}):
    os.environ.update(env)
    c = Context(params_from_args(bench.make_args(cfg, True, 200), traj_per_block=4))
    a, t, st = c.optimize(s, g, obs)
    ap, tp, stp = c.optimize(s[perm], g[perm], obs)
    inv = np.argsort(perm)
    d = np.abs(tp[inv] - t).reshape(B, -1).max(axis=1)
    bad = np.nonzero(d)[0]
    print(env, "problems differing under the permutation:", bad.tolist(), "max", d.max())
    for b in bad[:6]:
        k = int(inv[b])
        print(f"  problem {b} (slot {b % 4} of wg {b // 4}; permuted slot {k % 4} of wg {k // 4}): |dtraj| {d[b]:.2e}, "
              f"grad_evals {st['grad_evals'][b]} vs {stp['grad_evals'][k]}, trials {st['bls_trials'][b]} vs {stp['bls_trials'][k]}, "
              f"final_loss {st['final_loss'][b]:.7f} vs {stp['final_loss'][k]:.7f}")

# the line-search log of the first differing problem in both orders (helpers on): first divergent trial
os.environ["IRM_LEAN_NOHELP"] = "0"
c0 = Context(params_from_args(bench.make_args(cfg, True, 200), traj_per_block=4))
_, t0, _ = c0.optimize(s, g, obs)
_, tp0, _ = c0.optimize(s[perm], g[perm], obs)
inv = np.argsort(perm)
d = np.abs(tp0[inv] - t0).reshape(B, -1).max(axis=1)
bad = np.nonzero(d)[0]
if len(bad):
    b = int(bad[0])
    logs = []
    for order, idx in (("original", b), ("permuted", int(inv[b]))):
        os.environ["IRM_TRACE_PROBLEM"] = str(idx | (1 << 30))
        c = Context(params_from_args(bench.make_args(cfg, True, 200), traj_per_block=4))
        c.bls_trace_enable(4096)
        _, _, st = c.optimize(s if order == "original" else s[perm], g if order == "original" else g[perm], obs)
        logs.append(c.bls_trace(int(st["bls_trials"][idx])))
    a, p = logs
    n = min(len(a), len(p))
    strip = lambda x: np.concatenate([x[:, :1] % 100, x[:, 1:2], x[:, 2:3] % 1000, x[:, 3:]], axis=1)
    diff = np.nonzero(np.any(strip(a[:n]) != strip(p[:n]), axis=1))[0]
    k = int(diff[0]) if len(diff) else n
    print(f"problem {b}: logs {len(a)} / {len(p)} trials, first differing trial row {k}")
    np.set_printoptions(linewidth=200, precision=9, suppress=False)
    for r in range(max(0, k - 6), min(n, k + 3)):
        print("  orig", a[r].tolist())
        print("  perm", p[r].tolist())
