"""How many kernel rounds the C3-BLS faithful problems need with h line-search helpers (CPU, oracle logs).

Every problem of the bench batch is run through the C oracle's traced BLS dual loop
(optimizer_BLS.py:127-213); its line-search log gives the trials of each inner iteration.  A round of
k_lean evaluates one trial of a trajectory plus one per helper slot (a finished neighbour evaluating the
next trials lr·β, lr·β², ... — DESIGN.md §4), so an inner iteration with k trials takes ceil(k / (1 + h))
rounds, plus one resync round per outer iteration.  The model assumes the trajectory is alone in its
workgroup (helpers only serve a lone trajectory), so it bounds the rounds from below; the per-workgroup
simulation below plays the four problems of each workgroup together under several helper policies.

    python tools/bls_helper_sim.py [out.txt]
"""
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402
from irm_motion_planning_amd.params import params_from_args  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402

S, G, OBS = bench.make_problem("c3bls", 1, 0)
ARGS = bench.make_args("c3bls", True, 200)


def trials_per_iteration(idx):
    o = Oracle(params_from_args(ARGS))
    out = []
    for b in idx:
        _, _, tr = o.optimize_trace(o.init_alpha(S[b], G[b]), OBS, S[b], G[b], cap=16384)
        _, cnt = np.unique(tr[:, 0] * 100000 + tr[:, 1], return_counts=True)  # (outer, inner) groups
        nout = int(tr[:, 0].max()) + 1 if len(tr) else 0
        out.append((int(b), cnt, nout))
    return out


def main():
    res = []
    with ProcessPoolExecutor(min(8, os.cpu_count() or 1)) as ex:
        for r in ex.map(trials_per_iteration, np.array_split(np.arange(S.shape[0]), 32)):
            res += r
    lines = [f"C3-BLS faithful, {len(res)} problems (oracle line-search logs)"]
    for h in range(4):
        rounds = np.array([sum(int(np.ceil(c / (1 + h))) for c in cnt) + nout for _, cnt, nout in res])
        lines.append(f"helpers {h}: rounds per problem max {rounds.max()} p99 {np.percentile(rounds, 99):.0f} "
                     f"mean {rounds.mean():.0f}")
    # per workgroup (four consecutive problems, as the faithful launch places them): each round every live
    # trajectory runs one trial, plus its helpers' — "one": a done slot helps when exactly one is live (the
    # kernel's policy); "multi": every done slot helps a lone trajectory; "pair": each live trajectory gets a
    # done slot while there are enough
    res.sort(key=lambda r: r[0])

    def wg_rounds(wg, policy):
        qs = [[list(cnt) + [1] * nout, 0, 0] for _, cnt, nout in wg]
        rounds = 0
        while True:
            live = [i for i, q in enumerate(qs) if q[1] < len(q[0])]
            if not live:
                return rounds
            done = len(qs) - len(live)
            rounds += 1
            for r, i in enumerate(live):
                h = 0
                if policy == "one" and len(live) == 1:
                    h = 1
                elif policy == "multi" and len(live) == 1:
                    h = done
                elif policy == "pair" and r < done:
                    h = 1
                q = qs[i]
                q[2] += 1 + h
                if q[2] >= q[0][q[1]]:
                    q[1] += 1
                    q[2] = 0
    for policy in ("none", "one", "multi", "pair"):
        wr = [wg_rounds(res[w * 4:(w + 1) * 4], policy) for w in range(len(res) // 4)]
        lines.append(f"workgroups of four, helper policy {policy}: launch-bounding workgroup {max(wr)} rounds, "
                     f"mean {np.mean(wr):.0f}")
    cnt = np.concatenate([c for _, c, _ in res])
    lines.append(f"trials per inner iteration, histogram 0..11: {np.bincount(cnt)[:12].tolist()}")
    b, c, nout = max(res, key=lambda r: r[1].sum())
    lines.append(f"slowest problem {b}: {len(c)} inner iterations, {nout} outer, {c.sum()} trials, "
                 f"trials per iteration histogram {np.bincount(c)[:12].tolist()}")
    text = "\n".join(lines)
    print(text)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
