"""Diagnostic: outcome spread of an e2e case under ±1-ulp perturbations of α0 (the reference
ensemble's scheme, oracle/tools/gen_golden.py), for the HIP path (default) or the oracle (--oracle).

    python tools/e2e_ensemble.py [tag] [--oracle] [--n 10]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
from conftest import oracle_for, params, START, GOAL  # noqa: E402
from conftest import e2e_reference  # noqa: E402
from test_reference_bench import E2E_R02, e2e_alpha0, e2e_obstacles  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
tag = args[0] if args else "bls_n500"
n = int(sys.argv[sys.argv.index("--n") + 1]) if "--n" in sys.argv else 10
use_oracle = "--oracle" in sys.argv
argv, src = E2E_R02[tag]
obs = e2e_obstacles(src)
if use_oracle:
    o = oracle_for(*argv)
    a0 = e2e_alpha0(tag)
    a0 = o.init_alpha(START, GOAL) if a0 is None else a0
else:
    from irm_motion_planning_amd.context import Context
    c = Context(params(*argv))
    o = oracle_for(*argv)
    a0 = e2e_alpha0(tag)
    a0 = c.init_alpha(START, GOAL) if a0 is None else a0
r = e2e_reference(tag)
print("reference grad calls:", {k: np.asarray(v["grad_calls"]).astype(int).tolist() for k, v in r.items()})
out = []
for seed in range(-1, n):
    if seed < 0:
        ap = a0
    else:
        sgn = np.random.default_rng(100 + seed).choice([-1.0, 1.0], a0.shape).astype(np.float32)
        ap = np.nextafter(a0, a0 + sgn * np.float32(np.inf)).astype(np.float32)
    if use_oracle:
        al, st = o.optimize(ap, obs, START, GOAL)
        ge = st["grad_evals"]
    else:
        al, _, st = c.optimize(START, GOAL, obs, alpha0=ap)
        ge = int(st["grad_evals"])
    al = np.asarray(al, np.float32)
    avg = o.cost(al, obs, START, GOAL, 0, 0, 0)
    ok = o.constraints(al, START, GOAL)[0]
    out.append(ge)
    print(f"seed {seed}: grad evals {ge}, avg {avg:.4f}, ok {ok}", flush=True)
print("grad evals", out, "min", min(out), "max", max(out))
