"""Diagnostic: the general kernel's BLS line-search log for one e2e case (default bls_n500, from the
reference's α0) against the oracle's over the whole run: per-outer-iteration summary and the first
trial whose decision differs, with the losses around it.

    python tools/bls_general_diverge.py [tag]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
from conftest import oracle_for, params, START, GOAL  # noqa: E402
from irm_motion_planning_amd.context import Context  # noqa: E402
from test_reference_bench import E2E_R02, e2e_alpha0, e2e_obstacles  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "bls_n500"
argv, src = E2E_R02[tag]
obs = e2e_obstacles(src)
CAP = 4096
c = Context(params(*argv))
print("plan", c.launch_plan(1, len(obs)))
c.bls_trace_enable(CAP)
a0 = e2e_alpha0(tag)
if a0 is None:
    a0 = c.init_alpha(START, GOAL)
al, _, st = c.optimize(START, GOAL, obs, alpha0=a0)
tr = c.bls_trace(int(st["bls_trials"]))
print("hip", {k: (np.asarray(v).tolist()) for k, v in st.items()})
o = oracle_for(*argv)
alo, so, tro = o.optimize_trace(a0, obs, START, GOAL, cap=CAP)
print("oracle", so)
print("alpha max |hip - oracle|", float(np.abs(np.asarray(al) - alo).max()))
for name, t in (("hip", tr), ("oracle", tro)):
    for oi in np.unique(t[:, 0]).astype(int):
        s = t[t[:, 0] == oi]
        print(f"  {name} outer {oi}: {len(s)} trials, inner max {int(s[:, 1].max())}, last loss {s[-1, 7]:.7g}")
n = min(len(tr), len(tro))
diff = np.nonzero((tr[:n, 6] != tro[:n, 6]) | (tr[:n, 0] != tro[:n, 0]) | (tr[:n, 1] != tro[:n, 1]))[0]
if len(diff) == 0:
    print(f"decisions identical over {n} trials")
else:
    k = int(diff[0])
    print(f"first differing trial {k}")
    for j in range(max(0, k - 4), min(n, k + 2)):
        print("   hip    " + " ".join(f"{x:.8g}" for x in tr[j]))
        print("   oracle " + " ".join(f"{x:.8g}" for x in tro[j]))
rel = np.abs(tr[:n, 4] - tro[:n, 4]) / np.abs(tro[:n, 4])
print("new_loss rel diff by trial (every 8th):", " ".join(f"{x:.1e}" for x in rel[::8]))
