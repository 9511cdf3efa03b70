"""Developer diagnostic: per-phase cycle breakdown of k_optimize.

IRM_PROF_FIRST=<problem> moves that problem to batch slot 0 (the stamping wave is then its own) and,
with "cfg!f", reports block 0.

Needs the IRM_PHASE_PROFILE build (python -m irm_motion_planning_amd.build --prof);
run with IRM_LIB=<repo>/irm_motion_planning_amd/libirm_hip_prof.so on the GPU box.
"""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402
from irm_motion_planning_amd.context import Context  # noqa: E402
from irm_motion_planning_amd.params import params_from_args  # noqa: E402

PHASES = ["dir:stage1 barrier-wait", "dir: latch + endpoint reads", "dir:y rows + BLS norms", "dir:stage2 + barrier", "round-top (flags)",
          "dir:endpoint + stage1 mfma", "post-dir + resync + update", "E1 barrier-wait", "eval_waypoint",
          "eval reductions", "finalize+decide", "end barrier-wait", "grad inputs (mixed) + b flag", "#rounds with dense stage 1 (count)",
          "prologue", "accept+yacc+flags", "dP latch (after stage-2 barrier)", "resync check",
          "finalize: partial reads"]


LEAN_PHASES = ["round top: flags + latch reads", "stage-1 MFMA", "stage-1 barrier wait", "stage 2",
               "stage-2 barrier wait", "dP latch + update", "eval_waypoint", "reductions + endpoint rows",
               "E1 barrier wait", "finalize", "(unused)", "decide + grad inputs", "end barrier wait",
               "#rounds with dense stage 1 (count)", "prologue"] + ["(unused)"] * 9


def run(cfg, tb=0, rank=0, faithful=False):
    if faithful:  # k_lean's BLS flow reports each problem's kernel rounds (trace_b bit 29, series_len)
        os.environ["IRM_TRACE_PROBLEM"] = str(1 << 29)
    args = bench.make_args(cfg, faithful, 200)
    start, goal, obstacles = bench.make_problem(cfg, 1, 0)
    first = os.environ.get("IRM_PROF_FIRST")  # problem index moved to batch slot 0: its own waves stamp
    if first:
        idx = np.arange(start.shape[0])
        idx[0], idx[int(first)] = int(first), 0
        start, goal = start[idx], goal[idx]
    ctx = Context(params_from_args(args, traj_per_block=tb, operator_rank=rank))
    info = ctx.info()
    ctx.optimize(start, goal, obstacles)
    t0 = time.perf_counter()
    alpha, traj, st = ctx.optimize(start, goal, obstacles)
    dt = time.perf_counter() - t0
    nb = 4096
    K = 24
    buf = (ctypes.c_uint64 * (nb * K))()
    n = ctx.lib.irm_debug_phase_profile(ctx.handle, buf, nb)
    prof = np.frombuffer(buf, dtype=np.uint64, count=n * K).reshape(n, K).astype(np.float64)
    per = st["bls_trials"] if args.optimizer_name == "bls" else st["grad_evals"]  # one round per trial / step
    rounds = float(np.max(per) + np.max(st["outer_iterations"]))
    tot = prof.sum(1) - prof[:, 13]
    print(f"== {cfg} tb={info['traj_per_block']} R={info['operator_rank']} blocks={n} host {1000*dt:.2f} ms "
          f"rounds~{rounds:.0f} total cycles/block mean {tot.mean():.0f} -> {tot.mean()/rounds:.0f} per round")
    names = LEAN_PHASES if os.environ.get("IRM_PROFILE_LEAN") else PHASES
    for i, name in enumerate(names):
        c = prof[:, i].mean()
        if i == 13:
            print(f"   {name:22s} {c:9.1f} of {rounds:.0f} rounds")
        elif c > 0:
            print(f"   {name:22s} {c/rounds:9.0f} cyc/round  ({100*c/tot.mean():5.1f} %)")
    if faithful:  # the block that bounds the launch: its own rounds (its slowest problem's kernel rounds)
        k = 0 if first else int(np.argmax(tot))
        tbk = info["traj_per_block"]
        kr = (st["series_len"][k * tbk:(k + 1) * tbk] & 0xFFFF).max() if args.optimizer_name == "bls" else 0
        kr = float(kr) if kr > 0 else rounds
        print(f"   slowest block {k}: {tot[k]:.0f} cycles, {kr:.0f} kernel rounds -> {tot[k] / kr:.0f} per round")
        for i, name in enumerate(names):
            c = prof[k, i]
            if i != 13 and c > 0:
                print(f"     {name:22s} {c/kr:9.0f} cyc/round  ({100*c/tot[k]:5.1f} %)")


if __name__ == "__main__":
    for cfg in sys.argv[1:] or ["c3", "c2", "c5"]:  # "c5@-1": config at --operator-rank -1 (dense)
        faithful = cfg.endswith("!f")  # "c3bls!f": the reference's control flow
        name, _, rank = cfg.rstrip("!f").partition("@")
        run(name, rank=int(rank) if rank else 0, faithful=faithful)
