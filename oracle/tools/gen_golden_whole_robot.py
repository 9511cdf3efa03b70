"""Golden vectors for the whole-robot obstacle cost.

TEST INFRASTRUCTURE ONLY — runs in the build container, never on the GPU box.

The reference optimises the end-effector cost only; its blog ("Insights:
Complete Robot Obstacle Avoidance", DevBlog-Theme/blog-post.html:491-498)
gives the whole-robot variant

    ObstacleCost_{t_i}(α) = Σ_{j=1}^{n_joints} costmap(fk_j(evaluate(K, J, α, t_i)))

with fk_j = Robot.fk_joint_j (robot.py:39-72).  This script composes that
formula from the UNMODIFIED reference functions (Robot.fk_joint_1..3,
environment.compute_cost, the max/mean weighting of
Trajectory.compute_point_cost, trajectory.py:81-88) through the numpy jax
adapter (oracle/tools/jaxshim), and records

  fkj_<name>         (3, 2, N)  fk_joint_1..3 of the golden trajectories
  cv_<name>          (N)        Σ_j compute_cost(fk_joint_j(traj)) in fp32
  loss_<name>        (3)        λmax·max + (1−λmax)·mean for λmax ∈ LMAX
  grad_<name>        (3, N, D)  d loss / d traj, central differences of the same
                                composition evaluated in fp64 (IRM_JAXSHIM_X64=1,
                                run as a child process), h = 1e-6

for the trajectories of tests/golden/ref_eval_n50.npz (alpha0, small1, small2).

    PYTHONDONTWRITEBYTECODE=1 python oracle/tools/gen_golden_whole_robot.py [/root/reference]
"""
import argparse
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(REPO, "tests", "golden")
NAMES = ("alpha0", "small1", "small2")
LMAX = (0.0, 0.5, 1.0)


def reference(ref):
    sys.dont_write_bytecode = True
    sys.path[:0] = [os.path.join(HERE, "jaxshim"), ref]
    import environment  # noqa: E402  (reference environment.py)
    import main as refmain  # noqa: E402
    import robot  # noqa: E402
    old = sys.argv
    sys.argv = ["main.py"]
    try:
        args = refmain.parse_args()
    finally:
        sys.argv = old
    return environment, robot.Robot(args)


def whole_robot_cv(env, rob, traj, obstacles):
    fks = [rob.fk_joint_1(traj), rob.fk_joint_2(traj), rob.fk_joint_3(traj)]
    cv = env.compute_cost(fks[0], obstacles)
    for f in fks[1:]:
        cv = cv + env.compute_cost(f, obstacles)
    return fks, cv


def point_loss(cv, lmax):
    """trajectory.py:81-88 on the summed per-waypoint cost."""
    import jax.numpy as jnp
    return lmax * jnp.max(cv) + (1 - lmax) * (jnp.sum(cv) / cv.shape[0])


def fd_child(ref, src, dst):
    """fp64 central differences of the composed loss (this process has IRM_JAXSHIM_X64=1)."""
    env, rob = reference(ref)
    with np.load(src) as z:
        trajs = {n: z[n].astype(np.float64) for n in NAMES}
        obstacles = z["obstacles"].astype(np.float64)
    h = 1e-6
    out = {}
    for name, traj in trajs.items():
        g = np.zeros((len(LMAX),) + traj.shape)
        for li, lm in enumerate(LMAX):
            for i in np.ndindex(traj.shape):
                tp, tm = traj.copy(), traj.copy()
                tp[i] += h
                tm[i] -= h
                lp = float(point_loss(whole_robot_cv(env, rob, tp, obstacles)[1], lm))
                lq = float(point_loss(whole_robot_cv(env, rob, tm, obstacles)[1], lm))
                g[(li,) + i] = (lp - lq) / (2 * h)
        out[name] = g
    np.savez(dst, **out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("reference", nargs="?", default="/root/reference")
    ap.add_argument("--fd-child", nargs=2, metavar=("SRC", "DST"))
    a = ap.parse_args()
    if a.fd_child:
        fd_child(a.reference, *a.fd_child)
        return
    env, rob = reference(a.reference)
    with np.load(os.path.join(OUT, "ref_eval_n50.npz")) as z:
        trajs = {n: z[n + "_traj"].astype(np.float32) for n in NAMES}
        obstacles = z["obstacles"].astype(np.float32)
    res = {"obstacles": obstacles, "lmax": np.array(LMAX, np.float32)}
    for name, traj in trajs.items():
        fks, cv = whole_robot_cv(env, rob, traj, obstacles)
        res[f"traj_{name}"] = traj
        res[f"fkj_{name}"] = np.stack([np.asarray(f, np.float32) for f in fks])
        res[f"cv_{name}"] = np.asarray(cv, np.float32)
        res[f"loss_{name}"] = np.array([float(point_loss(cv, lm)) for lm in LMAX], np.float32)
    tmp_in = "/tmp/irm_wr_in.npz"
    tmp_out = "/tmp/irm_wr_fd.npz"
    np.savez(tmp_in, obstacles=obstacles, **trajs)
    envx = dict(os.environ, IRM_JAXSHIM_X64="1", PYTHONDONTWRITEBYTECODE="1")
    subprocess.check_call([sys.executable, __file__, a.reference, "--fd-child", tmp_in, tmp_out], env=envx)
    with np.load(tmp_out) as z:
        for name in NAMES:
            res[f"grad_{name}"] = z[name].astype(np.float32)
    np.savez_compressed(os.path.join(OUT, "ref_whole_robot_n50.npz"), **res)
    print("wrote ref_whole_robot_n50.npz", {k: v.shape for k, v in res.items()})


if __name__ == "__main__":
    main()
