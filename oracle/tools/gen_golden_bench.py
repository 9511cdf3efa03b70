"""Reference-produced fixtures at the bench shapes, the BLS line-search log and the extra end-to-end runs.

TEST INFRASTRUCTURE ONLY — runs in the build container, never on the GPU box.  Like gen_golden.py it
imports the UNMODIFIED reference from /root/reference through oracle/tools/jaxshim (numpy adapter of
the jax API; eager jit / while_loop / cond) and commits only generated arrays:

  tests/golden/ref_bench_c3.npz   C3 (BASELINE configs[2]): 32 problems of bench.make_problem("c3"),
                                  N=128, the reference's 11 obstacles, GD single loop
                                  (optimizer_GD.py:68-97), bench mode (loop_loss_reduction=-1e30):
                                  α0, the 1..5-step trajectories and losses, the 200-step final
                                  trajectory and loss, and the same run from α0 ± 1 ulp (8 members)
                                  (trajectories as the reference evaluates them, K@α@J in fp32, and
                                  the fp32 α themselves, whose exact K@α@J the tests compare with)
  tests/golden/ref_bench_c4.npz   the same at C4's shape (N=256, 50 random obstacles), 8 problems, with
                                  the k-step iterates at k = 1..5, 10, 20, 50 (before the ±1-ulp
                                  spread of this chaotic shape grows) and an 8-member ensemble
  tests/golden/ref_bls_trials.npz the first inner iterations of jit_optimize (optimizer_BLS.py:
                                  135-179): per iteration loss, ‖g‖, alpha_norm; per trial lr,
                                  new_loss, required_loss, accepted — at N=50 and N=128, from the
                                  reference α0 and from a well-conditioned α
  tests/golden/ref_e2e_r02.npz    reference control flow end to end (as gen_golden.py's ref_e2e.npz):
                                  the GD λ_max table at N=50, GD at N=128 / 256, BLS at N=256 (C4
                                  obstacles), each with a ±1-ulp ensemble (avg / max cost, flag,
                                  gradient-call count)
  tests/golden/ref_e2e_n500.npz   the same for GD and BLS at N=500 (--only n500), with the reference's
                                  α0 (its fp32 LU solve differs from any other at this size: the runs
                                  under test start from it)

    PYTHONDONTWRITEBYTECODE=1 python oracle/tools/gen_golden_bench.py [--only c3,c4,bls,e2e]
    PYTHONDONTWRITEBYTECODE=1 python oracle/tools/gen_golden_bench.py --matmul exact --only c3,c4,bls,e2e,e2e1

--matmul exact runs the same reference with every `@` accumulated in fp64 and rounded once (the
correctly rounded contraction of this build's kernels and C oracle) and writes *_xm.npz: it separates
what the reference's fp32 BLAS summation noise contributes (its dual-loop inner-iteration counts are
set by it: gd_n50 takes 296 gradient calls with BLAS matmuls, 760 with exact ones) from the algorithm.
"""
import argparse
import contextlib
import io
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(1, REPO)

import gen_golden as gg  # noqa: E402  (load_reference, ref_args, make_opt, end_to_end, CallCounter)

OUT = gg.OUT


def perturb(a0, seed):
    """α0 with every entry moved by ±1 ulp (the floor of fp32 evaluation noise)."""
    sgn = np.random.default_rng(100 + seed).choice([-1.0, 1.0], a0.shape).astype(np.float32)
    return np.nextafter(a0, a0 + sgn * np.float32(np.inf)).astype(np.float32)


def gd_bench_fixture(refmain, ogd, cfg, n_problems, n_ens, steps=200, ks=(1, 2, 3, 4, 5)):
    """Reference GD single loop in bench mode on bench.make_problem(cfg)'s first problems."""
    import bench
    _, _, N, D, O, _ = bench.CONFIGS[cfg]
    start, goal, obstacles = bench.make_problem(cfg, 1, 0)
    start, goal = start[:n_problems], goal[:n_problems]
    base = dict(n_timesteps=N, optimizer_name="gd", max_outer_iteration=1, loop_loss_reduction=-1e30,
                jit_loop=True)
    out = {"start": start, "goal": goal, "obstacles": obstacles, "steps": np.array(steps), "ks": np.array(ks)}
    opts = {k: gg.make_opt(ogd, "GradientDescentOptimizer", gg.ref_args(refmain, max_inner_iteration=k, **base))
            for k in tuple(ks) + (steps,)}
    o = opts[steps]
    tr = o.trajectory
    lsg, ljl, lm = o.lambda_sg_constraint, o.lambda_jl_constraint, o.lambda_max_cost
    a0s, trajk, lossk, fin_t, fin_l, ens_t, ens_l = [], [], [], [], [], [], []
    alk, fin_a, ens_a, ens_ak = [], [], [], []

    def run(opt, a0, s, g):
        with contextlib.redirect_stdout(io.StringIO()):
            al = np.array(opt.jit_optimize(a0, obstacles, s, g), np.float32)
        t = np.array(tr.evaluate(al, tr.km, tr.jac), np.float32)
        loss = float(tr.compute_trajectory_cost(al, obstacles, s, g, lsg, ljl, lm))
        return t, loss, al

    for b in range(n_problems):
        s, g = start[b], goal[b]
        a0 = np.array(tr.initTrajectory(s, g), np.float32)
        a0s.append(a0)
        tk, lk, ak = zip(*[run(opts[k], a0, s, g) for k in ks])
        trajk.append(np.stack(tk))
        lossk.append(np.array(lk, np.float32))
        alk.append(np.stack(ak))
        # the k-step runs from α0 ± 1 ulp: the reference's own sensitivity after k steps
        ens_ak.append(np.stack([np.stack([run(opts[k], perturb(a0, e), s, g)[2] for k in ks]) for e in range(n_ens)]))
        t, l_, a_ = run(o, a0, s, g)
        fin_t.append(t)
        fin_l.append(l_)
        fin_a.append(a_)
        et, el, ea = zip(*[run(o, perturb(a0, e), s, g) for e in range(n_ens)])
        ens_t.append(np.stack(et))
        ens_l.append(np.array(el, np.float32))
        ens_a.append(np.stack(ea))
        print(f"{cfg} problem {b}: loss {l_:.6f}, ensemble [{min(el):.6f}, {max(el):.6f}], "
              f"spread {np.abs(np.stack(et) - t).max():.2e}", flush=True)
    out.update(alpha0=np.stack(a0s), traj_k=np.stack(trajk), loss_k=np.stack(lossk), traj_final=np.stack(fin_t),
               loss_final=np.array(fin_l, np.float32), ens_traj_final=np.stack(ens_t),
               ens_loss_final=np.stack(ens_l), alpha_k=np.stack(alk), alpha_final=np.stack(fin_a),
               ens_alpha_final=np.stack(ens_a), ens_alpha_k=np.stack(ens_ak))
    return out


class TrialLog:
    """Records the calls jit_optimize makes (patched on the Trajectory class, as gen_golden.CallCounter):
    an inner iteration is cost(α) → cost_g(α) → cost(α') per line-search trial (optimizer_BLS.py:
    163-164, 140), so the log reconstructs each trial's lr / new_loss / required_loss / accept."""

    def __init__(self, trajmod):
        self.calls = []
        cls = trajmod.Trajectory
        self.cls = cls
        self.orig = (cls.compute_trajectory_cost, cls.compute_trajectory_cost_g)
        c0, g0 = self.orig
        log = self

        def c(self_, *a, **k):
            r = c0(self_, *a, **k)
            log.calls.append(("c", float(r)))
            return r

        def g(self_, *a, **k):
            r = g0(self_, *a, **k)
            log.calls.append(("g", np.array(r, np.float32)))
            return r

        cls.compute_trajectory_cost = c
        cls.compute_trajectory_cost_g = g

    def restore(self):
        self.cls.compute_trajectory_cost, self.cls.compute_trajectory_cost_g = self.orig


def bls_trial_fixture(refmain, obls, trajmod, N, alpha_kind, n_iter):
    import jax.numpy as jnp  # the adapter: fp32 like the reference's own norm / sum
    args = gg.ref_args(refmain, n_timesteps=N, max_inner_iteration=n_iter, max_outer_iteration=1,
                       loop_loss_reduction=-1e30)
    o = gg.make_opt(obls, "BacktrackingLineSearchOptimizer", args)
    tr, env = o.trajectory, o.env
    if alpha_kind == "alpha0":
        a = np.array(tr.initTrajectory(env.start_config, env.goal_config), np.float32)
    else:  # well-conditioned: K@α is exact to fp32 rounding, so cost and gradient are too
        a = (np.random.default_rng(77 + N).standard_normal((N, 3)) * 0.05).astype(np.float32)
    log = TrialLog(trajmod)
    try:
        with contextlib.redirect_stdout(io.StringIO()):
            al = np.array(o.jit_optimize(a, env.obstacles, env.start_config, env.goal_config), np.float32)
    finally:
        log.restore()
    # parse: c(α) g(α) c(α'1) ... c(α'm) per inner iteration
    lr, calls, i = o.bls_lr_start, log.calls, 0
    it_rows, tr_rows = [], []
    while i < len(calls):
        assert calls[i][0] == "c" and calls[i + 1][0] == "g", calls[i:i + 2]
        loss, grad = calls[i][1], calls[i + 1][1]
        gn = float(jnp.linalg.norm(grad))
        anorm = float(jnp.sum(grad.T @ (grad / jnp.linalg.norm(grad))))
        i += 2
        it = len(it_rows)
        for j in range(o.bls_max_iter):
            new_loss = calls[i][1]
            i += 1
            required = float(np.float32(loss) - np.float32(o.bls_alpha) * np.float32(lr) * np.float32(anorm))
            acc = not (new_loss > required)
            tr_rows.append([it, j, lr, new_loss, required, float(acc)])
            lr = float(np.float32(lr) * np.float32(o.bls_beta_plus if acc else o.bls_beta_minus))
            if acc:
                break
        it_rows.append([loss, gn, anorm])
    print(f"BLS N={N} from {alpha_kind}: {len(it_rows)} iterations, {len(tr_rows)} trials, "
          f"accept pattern {[int(r[5]) for r in tr_rows]}", flush=True)
    return {"alpha_init": a, "alpha_final": al, "iterations": np.array(it_rows, np.float64),
            "trials": np.array(tr_rows, np.float64),
            "obstacles": np.array(env.obstacles, np.float32)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("reference", nargs="?", default="/root/reference")
    ap.add_argument("--only", default="c3,c4,bls,e2e")
    ap.add_argument("--matmul", default="blas", choices=("blas", "exact"),
                    help="exact: the reference with correctly rounded matmuls (jaxshim IRM_JAXSHIM_MATMUL), "
                         "fixtures suffixed _xm")
    a = ap.parse_args()
    if a.matmul == "exact":
        os.environ["IRM_JAXSHIM_MATMUL"] = "exact"
    sfx = "_xm" if a.matmul == "exact" else ""
    only = set(a.only.split(","))
    refmain, ogd, obls, trajmod = gg.load_reference(a.reference)
    os.makedirs(OUT, exist_ok=True)

    if "c3" in only:
        np.savez_compressed(os.path.join(OUT, f"ref_bench_c3{sfx}.npz"), **gd_bench_fixture(refmain, ogd, "c3", 32, 8))
    if "c4" in only:
        np.savez_compressed(os.path.join(OUT, f"ref_bench_c4{sfx}.npz"),
                            **gd_bench_fixture(refmain, ogd, "c4", 8, 8, ks=(1, 2, 3, 4, 5, 10, 20, 50)))
    if "bls" in only:
        bl = {}
        for N in (50, 128):
            for kind in ("alpha0", "wellcond"):
                for k, v in bls_trial_fixture(refmain, obls, trajmod, N, kind, 4).items():
                    bl[f"n{N}_{kind}__{k}"] = v
        np.savez_compressed(os.path.join(OUT, f"ref_bls_trials{sfx}.npz"), **bl)
    if "e2e" in only or "e2e1" in only or "n500" in only:
        import bench
        cnt = gg.CallCounter(trajmod)

        def record(e2e, tag, mod, cls, args, obstacles=None, ensemble=8, store_alpha0=False):
            o = gg.make_opt(mod, cls, args, obstacles)
            r = gg.end_to_end(o, cnt)
            for k, v in r.items():
                if k != "series":
                    e2e[f"{tag}__{k}"] = np.asarray(v)
            tr, env = o.trajectory, o.env
            init = tr.initTrajectory
            a0 = np.array(init(env.start_config, env.goal_config), np.float32)
            if store_alpha0:  # the reference's initTrajectory (its fp32 LU solve of the singular K)
                e2e[f"{tag}__alpha0"] = a0
            ens = {"avg_cost": [], "max_cost": [], "constraints_ok": [], "grad_calls": []}
            for seed in range(ensemble):
                tr.initTrajectory = lambda s_, g_, a=perturb(a0, seed): a.copy()
                rr = gg.end_to_end(o, cnt)
                for k in ens:
                    ens[k].append(rr[k])
            tr.initTrajectory = init
            for k, v in ens.items():
                e2e[f"{tag}__ens_{k}"] = np.asarray(v)
            print(f"{tag}: avg {r['avg_cost']:.4f} max {r['max_cost']:.4f} ok {r['constraints_ok']} "
                  f"grad {r['grad_calls']}; ensemble avg [{min(ens['avg_cost']):.4f}, {max(ens['avg_cost']):.4f}] "
                  f"grad {ens['grad_calls']}", flush=True)

        if "e2e" in only:
            e2e = {}
            for lm in (0.0, 0.25, 0.75, 1.0):  # the GD column of the blog's λ_max table (0.5 is gd_n50)
                record(e2e, f"gd_n50_lmax{lm}", ogd, "GradientDescentOptimizer",
                       gg.ref_args(refmain, n_timesteps=50, optimizer_name="gd", lambda_max_cost=lm))
            record(e2e, "gd_n128", ogd, "GradientDescentOptimizer",
                   gg.ref_args(refmain, n_timesteps=128, optimizer_name="gd"))
            record(e2e, "gd_n256", ogd, "GradientDescentOptimizer",
                   gg.ref_args(refmain, n_timesteps=256, optimizer_name="gd"))
            _, _, obs_c4 = bench.make_problem("c4", 1, 0)
            record(e2e, "bls_n256_c4obs", obls, "BacktrackingLineSearchOptimizer",
                   gg.ref_args(refmain, n_timesteps=256), obstacles=obs_c4, ensemble=6)
            np.savez_compressed(os.path.join(OUT, f"ref_e2e_r02{sfx}.npz"), **e2e)
        if "n500" in only:  # N > 256 (the blog's runtime study goes to N = 500): reference defaults
            e2e = {}
            record(e2e, "gd_n500", ogd, "GradientDescentOptimizer",
                   gg.ref_args(refmain, n_timesteps=500, optimizer_name="gd"), ensemble=4, store_alpha0=True)
            record(e2e, "bls_n500", obls, "BacktrackingLineSearchOptimizer",
                   gg.ref_args(refmain, n_timesteps=500), ensemble=4, store_alpha0=True)
            np.savez_compressed(os.path.join(OUT, f"ref_e2e_n500{sfx}.npz"), **e2e)
        if "e2e1" in only:  # gen_golden.py's end-to-end cases (ref_e2e.npz), here with exact matmuls
            assert sfx, "the BLAS variant of these cases is gen_golden.py's ref_e2e.npz"
            e2e = {}
            for lm in (0.0, 0.25, 0.5, 0.75, 1.0):
                record(e2e, f"bls_n50_lmax{lm}", obls, "BacktrackingLineSearchOptimizer",
                       gg.ref_args(refmain, n_timesteps=50, lambda_max_cost=lm))
            record(e2e, "gd_n50", ogd, "GradientDescentOptimizer", gg.ref_args(refmain, n_timesteps=50, optimizer_name="gd"))
            record(e2e, "bls_n128", obls, "BacktrackingLineSearchOptimizer", gg.ref_args(refmain, n_timesteps=128))
            o3 = np.array([[2, -3], [-2, 2], [3, 3]], np.int32)
            o10 = np.array([[2, -3], [-2, 2], [3, 3], [-1, -2], [-2, 1], [-1, -1], [-2, -3], [-2, 0], [1, 3], [3, 2]],
                           np.int32)
            record(e2e, "c1_gd_n64_o3", ogd, "GradientDescentOptimizer",
                   gg.ref_args(refmain, n_timesteps=64, optimizer_name="gd"), obstacles=o3)
            record(e2e, "c2_bls_n128_o10", obls, "BacktrackingLineSearchOptimizer", gg.ref_args(refmain, n_timesteps=128),
                   obstacles=o10)
            np.savez_compressed(os.path.join(OUT, f"ref_e2e{sfx}.npz"), **e2e)
    print("wrote", sorted(os.listdir(OUT)))


if __name__ == "__main__":
    main()
