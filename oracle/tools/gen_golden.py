"""Generate tests/golden/*.npz from the UNMODIFIED reference sources.

TEST INFRASTRUCTURE ONLY — runs in the build container, never on the GPU box.
The reference (simongroeger/irm_motion_planning, mounted read-only at
/root/reference) imports `jax`, which is not installed here; the numpy
adapter in oracle/tools/jaxshim provides the jax API it uses (fp32 default
dtypes, eager jit / while_loop / cond, legacy threefry PRNG).  Only the
generated arrays are committed; no reference source travels.

    PYTHONDONTWRITEBYTECODE=1 python oracle/tools/gen_golden.py [/root/reference]
"""
import argparse
import contextlib
import io
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(REPO, "tests", "golden")


def load_reference(ref):
    sys.dont_write_bytecode = True
    sys.path[:0] = [os.path.join(HERE, "jaxshim"), ref]
    import main as refmain  # noqa: E402  (reference main.py)
    import optimizer_BLS  # noqa: E402
    import optimizer_GD  # noqa: E402
    import trajectory  # noqa: E402
    return refmain, optimizer_GD, optimizer_BLS, trajectory


def ref_args(refmain, **kw):
    old = sys.argv
    sys.argv = ["main.py"]
    try:
        a = refmain.parse_args()
    finally:
        sys.argv = old
    for k, v in kw.items():
        setattr(a, k, v)
    return a


class CallCounter:
    """Counts compute_trajectory_cost(_g) calls.

    Patched on the Trajectory CLASS before any optimizer is built, so that
    bound methods the optimizers capture in __init__ (jit closures) count too.
    """

    def __init__(self, trajmod):
        self.cost = 0
        self.grad = 0
        cls = trajmod.Trajectory
        c0, g0 = cls.compute_trajectory_cost, cls.compute_trajectory_cost_g
        counter = self

        def c(self_, *a, **k):
            counter.cost += 1
            return c0(self_, *a, **k)

        def g(self_, *a, **k):
            counter.grad += 1
            return g0(self_, *a, **k)

        cls.compute_trajectory_cost = c
        cls.compute_trajectory_cost_g = g


def make_opt(mod, cls, args, obstacles=None):
    with contextlib.redirect_stdout(io.StringIO()):
        opt = getattr(mod, cls)(args)
    if obstacles is not None:
        opt.env.obstacles = obstacles
    return opt


def end_to_end(opt, counter=None):
    env, tr = opt.env, opt.trajectory
    if counter:
        counter.cost = counter.grad = 0
    with contextlib.redirect_stdout(io.StringIO()):
        res = opt.optimize()
    calls = (counter.cost, counter.grad) if counter else None
    alpha = res[0] if isinstance(res, tuple) else res
    series = np.array(res[1], np.float32) if isinstance(res, tuple) else None
    alpha = np.array(alpha, np.float32)
    traj = np.array(tr.evaluate(alpha, tr.km, tr.jac), np.float32)
    avg = float(tr.compute_trajectory_cost(alpha, env.obstacles, env.start_config, env.goal_config, 0, 0, 0))
    mx = float(tr.compute_trajectory_cost(alpha, env.obstacles, env.start_config, env.goal_config, 0, 0, 1))
    ok = bool(tr.constraintsFulfilled(alpha, env.start_config, env.goal_config))
    out = {"alpha": alpha, "traj": traj, "avg_cost": avg, "max_cost": mx, "constraints_ok": ok}
    if counter:
        out["cost_calls"], out["grad_calls"] = calls
    if series is not None:
        out["series"] = series
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("reference", nargs="?", default="/root/reference")
    a = ap.parse_args()
    refmain, ogd, obls, trajmod = load_reference(a.reference)
    os.makedirs(OUT, exist_ok=True)
    rng = np.random.default_rng(1234)

    # ---- setup: t, K, dK, J (trajectory.py:35-42) for several N
    setup = {}
    for N in (50, 64, 128, 256):
        tr = trajmod.Trajectory(ref_args(refmain, n_timesteps=N))
        K, dK = np.array(tr.km, np.float32), np.array(tr.dkm, np.float32)
        setup[f"t_{N}"] = np.array(tr.t, np.float32)
        if N <= 64:
            setup[f"K_{N}"] = K
            setup[f"dK_{N}"] = dK
        else:  # rows 0, N/2, N-1 are enough to pin the construction
            setup[f"Krows_{N}"] = K[[0, N // 2, N - 1]]
            setup[f"dKrows_{N}"] = dK[[0, N // 2, N - 1]]
    setup["J"] = np.array(tr.jac, np.float32)
    import jax  # the adapter
    setup["Z7"] = np.array(jax.random.normal(jax.random.PRNGKey(0), (7, 7)), np.float32)
    np.savez_compressed(os.path.join(OUT, "ref_setup.npz"), **setup)

    # ---- evaluation vectors at N=50 (trajectory.py:63-65, 73-78, 271-297, 129-137)
    N = 50
    opt = make_opt(obls, "BacktrackingLineSearchOptimizer", ref_args(refmain, n_timesteps=N))
    tr, env = opt.trajectory, opt.env
    alpha0 = np.array(tr.initTrajectory(env.start_config, env.goal_config), np.float32)
    alphas = {
        "alpha0": alpha0,
        "small1": (rng.standard_normal((N, 3)) * 0.05).astype(np.float32),
        "small2": (rng.standard_normal((N, 3)) * 0.2).astype(np.float32),
    }
    lams = np.array([[0.5, 0.1, 0.5], [50, 10, 0], [5, 1, 1], [0, 0, 0], [0, 0, 1]], np.float32)
    ev = {"lams": lams, "start": np.array(env.start_config, np.float32), "goal": np.array(env.goal_config, np.float32),
          "obstacles": np.array(env.obstacles, np.float32)}
    for name, al in alphas.items():
        ev[f"{name}"] = al
        ev[f"{name}_traj"] = np.array(tr.evaluate(al, tr.km, tr.jac), np.float32)
        ev[f"{name}_vel"] = np.array(tr.evaluate(al, tr.dkm, tr.jac), np.float32)
        ev[f"{name}_ok"] = np.array(bool(tr.constraintsFulfilled(al, env.start_config, env.goal_config)))
        costs, grads = [], []
        for lsg, ljl, lm in lams:
            costs.append(float(tr.compute_trajectory_cost(al, env.obstacles, env.start_config, env.goal_config,
                                                          float(lsg), float(ljl), float(lm))))
            grads.append(np.array(tr.compute_trajectory_cost_g(al, env.obstacles, env.start_config, env.goal_config,
                                                               float(lsg), float(ljl), float(lm)), np.float32))
        ev[f"{name}_cost"] = np.array(costs, np.float32)
        ev[f"{name}_grad"] = np.stack(grads)
        traj = ev[f"{name}_traj"]
        f = np.array(tr.robot.fk(traj), np.float32)
        ev[f"{name}_fk"] = f
        ev[f"{name}_jac"] = np.array(tr.robot.jacobian(traj), np.float32)
        import environment as refenv
        cv, cg = refenv.compute_cost_vg(f, env.obstacles)
        ev[f"{name}_cost_v"] = np.array(cv, np.float32)
        ev[f"{name}_cost_g"] = np.array(cg, np.float32)
    np.savez_compressed(os.path.join(OUT, "ref_eval_n50.npz"), **ev)

    # ---- first GD iterations (optimizer_GD.py:68-97, single loop) from alpha0
    gd = {}
    for k in range(1, 6):
        args = ref_args(refmain, n_timesteps=N, optimizer_name="gd", max_outer_iteration=1, max_inner_iteration=k,
                        jit_loop=True)
        o = make_opt(ogd, "GradientDescentOptimizer", args)
        with contextlib.redirect_stdout(io.StringIO()):
            al = np.array(o.jit_optimize(alpha0, o.env.obstacles, o.env.start_config, o.env.goal_config), np.float32)
        gd[f"traj_{k}"] = np.array(o.trajectory.evaluate(al, o.trajectory.km, o.trajectory.jac), np.float32)
        gd[f"loss_{k}"] = np.array(float(o.trajectory.compute_trajectory_cost(
            al, o.env.obstacles, o.env.start_config, o.env.goal_config, args.lambda_sg_constraint,
            args.lambda_jl_constraint, args.lambda_max_cost)), np.float32)
    gd["alpha0"] = alpha0
    np.savez_compressed(os.path.join(OUT, "ref_gd_steps_n50.npz"), **gd)

    # ---- end-to-end runs (reference control flow, default hyper-parameters)
    e2e = {}
    cnt = CallCounter(trajmod)

    def record(tag, mod, cls, args, obstacles=None, ensemble=8):
        o = make_opt(mod, cls, args, obstacles)
        r = end_to_end(o, cnt)
        for k, v in r.items():
            e2e[f"{tag}__{k}"] = np.asarray(v)
        print(tag, {k: (v if np.ndim(v) == 0 else np.shape(v)) for k, v in r.items()}, flush=True)
        if not ensemble:
            return
        # The loop is chaotic (BLS) / noise-terminated (late GD outer loops):
        # the same reference run from α0 with every entry moved by ±1 ulp —
        # the floor of fp32 evaluation noise — lands in a spread of outcomes.
        # Parity of another implementation is judged against that spread.
        tr, env = o.trajectory, o.env
        init = tr.initTrajectory
        a0 = np.array(init(env.start_config, env.goal_config), np.float32)
        ens = {"avg_cost": [], "max_cost": [], "constraints_ok": [], "grad_calls": []}
        for seed in range(ensemble):
            sgn = np.random.default_rng(100 + seed).choice([-1.0, 1.0], a0.shape).astype(np.float32)
            a0p = np.nextafter(a0, a0 + sgn * np.float32(np.inf)).astype(np.float32)
            tr.initTrajectory = lambda s_, g_, a=a0p: a.copy()
            rr = end_to_end(o, cnt)
            for k in ens:
                ens[k].append(rr[k])
        tr.initTrajectory = init
        for k, v in ens.items():
            e2e[f"{tag}__ens_{k}"] = np.asarray(v)
        print("   ensemble avg [%.4f, %.4f] max [%.4f, %.4f] ok %s grad %s" % (
            min(ens["avg_cost"]), max(ens["avg_cost"]), min(ens["max_cost"]), max(ens["max_cost"]),
            ens["constraints_ok"], ens["grad_calls"]), flush=True)

    for lm in (0.0, 0.25, 0.5, 0.75, 1.0):  # blog-post.html:546-581 (λ_max_cost table)
        record(f"bls_n50_lmax{lm}", obls, "BacktrackingLineSearchOptimizer",
               ref_args(refmain, n_timesteps=50, lambda_max_cost=lm))
    record("gd_n50", ogd, "GradientDescentOptimizer", ref_args(refmain, n_timesteps=50, optimizer_name="gd"))
    record("bls_n128", obls, "BacktrackingLineSearchOptimizer", ref_args(refmain, n_timesteps=128))
    # BASELINE configs[0]: N=64, 3 obstacles, GD;  configs[1]: N=128, 10 obstacles, BLS
    o3 = np.array([[2, -3], [-2, 2], [3, 3]], np.int32)
    o10 = np.array([[2, -3], [-2, 2], [3, 3], [-1, -2], [-2, 1], [-1, -1], [-2, -3], [-2, 0], [1, 3], [3, 2]], np.int32)
    record("c1_gd_n64_o3", ogd, "GradientDescentOptimizer", ref_args(refmain, n_timesteps=64, optimizer_name="gd"),
           obstacles=o3)
    record("c2_bls_n128_o10", obls, "BacktrackingLineSearchOptimizer", ref_args(refmain, n_timesteps=128),
           obstacles=o10)
    # extended-vis series of the plain BLS loop (optimizer_BLS.py:65-123)
    record("bls_n50_series", obls, "BacktrackingLineSearchOptimizer",
           ref_args(refmain, n_timesteps=50, jit_loop=False, extended_vis=True), ensemble=0)
    np.savez_compressed(os.path.join(OUT, "ref_e2e.npz"), **e2e)

    # ---- the reference's own committed output files (visualization/*.txt)
    vis = os.path.join(a.reference, "visualization")
    res = np.loadtxt(os.path.join(vis, "trajectory_result.txt")).astype(np.float32)
    ser = np.loadtxt(os.path.join(vis, "trajectory_series.txt")).astype(np.float32)
    np.savez_compressed(os.path.join(OUT, "ref_visualization.npz"), trajectory_result=res,
                        series_frames=ser[[0, 1, 2, len(ser) // 2, len(ser) - 1]],
                        series_frame_index=np.array([0, 1, 2, len(ser) // 2, len(ser) - 1]),
                        series_len=np.array(len(ser)))
    print("wrote", sorted(os.listdir(OUT)))


if __name__ == "__main__":
    main()
