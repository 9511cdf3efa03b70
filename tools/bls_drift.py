"""HIP-vs-oracle loss drift of the BLS dual loop, trial for trial (GPU box).

For each traced C3-BLS problem (moved to batch index 0 of a 64-problem, four-per-workgroup faithful run,
so that the line-search log records it), the HIP log and the oracle's log from the same α0 are walked
together up to their first decision flip (tests/test_gpu_parity.py::first_decision_flip).  Along the
aligned prefix the relative drift of the losses — |new_loss_hip − new_loss_oracle| / |loss|, the same for
required_loss and the loss at α — is what a decision's margin must exceed to be decided identically; the
ratio of each first flip's margin to the drift before it sets the knife edge of the BLS end-state test
(tests/test_gpu_parity.py: BLS_KNIFE_FACTOR × loss_drift).

    python tools/bls_drift.py [n_problems=16] [out.txt]
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import bench  # noqa: E402
from irm_motion_planning_amd.context import Context  # noqa: E402
from irm_motion_planning_amd.params import params_from_args  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402
from test_gpu_parity import first_decision_flip  # noqa: E402


def main():
    nprob = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    out = sys.argv[2] if len(sys.argv) > 2 else None
    s, g, obs = bench.make_problem("c3bls", 1, 0)
    B = 64
    s, g = s[:B].copy(), g[:B].copy()
    args = bench.make_args("c3bls", True, 200)
    llr = float(args.loop_loss_reduction)
    c = Context(params_from_args(args, traj_per_block=4))
    c.bls_trace_enable(8192)
    o = Oracle(params_from_args(args))
    lines = []
    worst = []
    ratios = []
    for b in np.linspace(0, B - 1, nprob).astype(int):
        idx = np.arange(B)
        idx[0], idx[b] = b, 0
        _, _, st = c.optimize(s[idx], g[idx], obs)
        tr = c.bls_trace(int(st["bls_trials"][0]))
        _, _, tro = o.optimize_trace(c.init_alpha(s[b], g[b]), obs, s[b], g[b], cap=8192)
        flip = first_decision_flip(tr, tro, llr)
        n = flip[0] if flip is not None else min(len(tr), len(tro))
        a, r = tr[:n], tro[:n]
        den = np.maximum(np.abs(r[:, 7]), 1e-30)
        d_new = np.abs(a[:, 4] - r[:, 4]) / den
        d_req = np.abs(a[:, 5] - r[:, 5]) / den
        d_loss = np.abs(a[:, 7] - r[:, 7]) / den
        m = float(max(d_req.max(initial=0), d_loss.max(initial=0)))
        worst.append(m)
        if flip is not None:
            ratios.append(flip[1] / max(m, 1e-30))
        # the drift at the end of each outer iteration's first inner loops (where it accumulates)
        lines.append(f"problem {b:2d}: {len(tr)} trials (oracle {len(tro)}), aligned {n}, first flip "
                     f"{'none' if flip is None else f'at {flip[0]} margin {flip[1]:.2e}'}; max relative drift "
                     f"new_loss {d_new.max(initial=0):.2e} required {d_req.max(initial=0):.2e} loss "
                     f"{d_loss.max(initial=0):.2e}; median new_loss {np.median(d_new) if n else 0:.1e}")
    w = np.array(worst)
    lines.append(f"max relative drift of the loss at alpha / the Armijo threshold over the aligned prefixes: "
                 f"{w.max():.2e} (median over problems {np.median(w):.2e}); first-flip margin / drift before it: "
                 f"max {max(ratios, default=0):.2f}, median {np.median(ratios) if ratios else 0:.2f} "
                 f"({len(ratios)} flips)")
    text = "\n".join(lines)
    print(text)
    if out:
        with open(out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
