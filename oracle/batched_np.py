"""Vectorised fp32 CPU restatement of the reference's GD iteration for a batch of problems.

TEST / BASELINE INFRASTRUCTURE ONLY: bench.py's cpu_baseline leg times it next to the scalar C oracle
(oracle/irm_oracle.c); tests/test_oracle_golden.py pins it to that oracle.  The product package never
imports it.

The reference's XLA:CPU path contracts K@α@J with BLAS-style GEMMs (trajectory.py:63-65, :295); the
scalar oracle accumulates every contraction in fp64 one problem at a time, which understates what a
BLAS CPU path does per core.  Here the batch's α are one N × (B·D) matrix, so every contraction of one
GD iteration over the whole batch is a single fp32 sgemm (numpy → OpenBLAS, multi-threaded):

    iteration (optimizer_GD.py:76-91 / :180-195, bench mode: every step accepted)
      traj, vel = K@α@J, dK@α@J                    trajectory.py:63-65   (2 sgemm N×N×BD + J mixes)
      g = (Kᵀ ta + dKᵀ tb) @ Jᵀ                     trajectory.py:284-297 (2 sgemm)
      α' = (1 − λ_reg·lr)·α − lr·g                  optimizer_GD.py:81
      loss(α') → traj, vel at α' again              trajectory.py:271-281 (2 sgemm)

i.e. 6 N×N×(B·D) sgemms per batch-iteration = SURVEY.md §8d's 12·N²·D flop per trajectory-iteration,
plus the per-waypoint terms (robot.py:29-36, 75-87; environment.py:32-58; trajectory.py:81-268) as
vectorised fp32 numpy over B×N.
"""
import numpy as np


class BatchedGD:
    """The reference's GD single loop in bench mode (loop_loss_reduction = -inf: every step accepted,
    max_outer_iteration = 1) for B problems at once, fp32 throughout."""

    def __init__(self, K, dK, J, params):
        f = np.float32
        self.K = np.ascontiguousarray(K, f)
        self.dK = np.ascontiguousarray(dK, f)
        self.KT = np.ascontiguousarray(self.K.T)
        self.dKT = np.ascontiguousarray(self.dK.T)
        self.J = np.ascontiguousarray(J, f)
        p = params
        self.N, self.D = int(p.n_timesteps), int(p.n_joints)
        self.link = np.array(list(p.link_length)[: self.D], f)
        self.lmax = f(p.lambda_max_cost)
        self.lsg, self.ljl = f(p.lambda_sg_constraint), f(p.lambda_jl_constraint)
        self.lr = f(p.gd_lr[0])
        self.cf = f(1) - f(p.lambda_reg) * self.lr  # optimizer_GD.py:81 in fp32 (weakly typed λ_reg)
        mean = 0.5 * (float(p.max_joint_position) + float(p.min_joint_position))
        self.mean = f(mean)
        self.std = f(0.5 * (float(p.max_joint_position) - mean))  # trajectory.py:31-32
        self.hi = f(float(p.joint_safety_limit) * float(p.max_joint_position))
        self.lo = f(float(p.joint_safety_limit) * float(p.min_joint_position))
        self.vmax = f(p.max_joint_velocity)
        self.thr = f(float(p.joint_safety_limit) * float(p.max_joint_velocity))
        self.cvdl = bool(p.constraint_violating_dependant_loss)

    # State is kept waypoint-major, (N, B, D): every contraction over waypoints is then one sgemm on an
    # N × (B·D) view, and the D × D mixes one (N·B) × D × D sgemm, with no transposes in the loop.

    def _eval(self, M, a):
        """M@α@J for the whole batch (trajectory.py:63-65): sgemm N×N×(B·D), then the D×D mix."""
        N, B, D = a.shape
        t = M @ a.reshape(N, B * D)
        return np.einsum("md,dk->mk", t.reshape(N * B, D), self.J, optimize=True).reshape(N, B, D)

    def _terms(self, traj, vel, obs, s, g, grad):
        f = np.float32
        N = self.N
        c = np.cumsum(traj, axis=2, dtype=f)                        # robot.py:31
        sn, cs = np.sin(c), np.cos(c)
        fx = (cs * self.link).sum(axis=2, dtype=f)                  # robot.py:33-35, (N, B)
        fy = (sn * self.link).sum(axis=2, dtype=f)
        dx = fx[:, :, None] - obs[None, None, :, 0]                  # environment.py:32-58
        dy = fy[:, :, None] - obs[None, None, :, 1]
        den = f(0.5) + f(0.5) * (dx * dx + dy * dy)
        cv = (f(0.8) / den).sum(axis=2, dtype=f)                     # (N, B)
        toc = self.lmax * cv.max(axis=0) + (f(1) - self.lmax) * cv.mean(axis=0, dtype=f)  # trajectory.py:85-87
        e0, e1 = traj[0] - s, traj[N - 1] - g
        sgp = f(0.5) * (e0 * e0).sum(1) + f(0.5) * (e1 * e1).sum(1)                     # trajectory.py:183-188
        sgv = f(0.5) * (vel[0] ** 2).sum(1) + f(0.5) * (vel[N - 1] ** 2).sum(1)          # trajectory.py:201-204
        mp = (traj > self.hi) | (traj < self.lo) if self.cvdl else np.ones_like(traj, bool)
        mv = np.abs(vel) > self.thr if self.cvdl else np.ones_like(vel, bool)
        z = (traj - self.mean) / self.std
        jp = np.where(mp, f(0.5) * z * z, f(0)).sum(axis=(0, 2), dtype=f) / f(N)          # trajectory.py:215-227
        zv = vel / self.vmax
        jv = np.where(mv, f(0.5) * zv * zv, f(0)).sum(axis=(0, 2), dtype=f) / f(N)        # trajectory.py:245-255
        loss = toc + self.lsg * (sgp + sgv) + self.ljl * (jp + jv)                      # trajectory.py:281
        if not grad:
            return loss, None, None
        den2 = den * den
        gx = (f(-0.8) * dx / den2).sum(axis=2, dtype=f)
        gy = (f(-0.8) * dy / den2).sum(axis=2, dtype=f)
        idx = cv.argmax(axis=0)                                       # trajectory.py:97 (first index)
        w = np.full(cv.shape, (f(1) - self.lmax) * (f(1) / f(N)), f)
        w[idx, np.arange(len(idx))] += self.lmax
        xs, ys = -(self.link * sn), self.link * cs                    # robot.py:75-87
        jx = xs + xs.sum(2, keepdims=True) - np.cumsum(xs, axis=2, dtype=f)
        jy = ys + ys.sum(2, keepdims=True) - np.cumsum(ys, axis=2, dtype=f)
        ta = (w * gx)[:, :, None] * jx + (w * gy)[:, :, None] * jy    # trajectory.py:120-126
        tb = np.zeros_like(vel)
        ta[0] += self.lsg * e0                                         # trajectory.py:191-212
        ta[N - 1] += self.lsg * e1
        tb[0] += self.lsg * vel[0]
        tb[N - 1] += self.lsg * vel[N - 1]
        ta += self.ljl * np.where(mp, (traj - self.mean) / (self.std * self.std), f(0)) / f(N)  # :231-242
        tb += self.ljl * np.where(mv, vel / (self.vmax * self.vmax), f(0)) / f(N)               # :259-268
        return loss, ta, tb

    def _grad(self, ta, tb):
        """(Kᵀ ta + dKᵀ tb) @ Jᵀ (trajectory.py:295): two sgemms over the batch."""
        N, B, D = ta.shape
        u = self.KT @ ta.reshape(N, B * D) + self.dKT @ tb.reshape(N, B * D)
        return np.einsum("md,kd->mk", u.reshape(N * B, D), self.J, optimize=True).reshape(N, B, D)

    def run(self, alpha0, start, goal, obstacles, iters):
        """`iters` GD steps from alpha0 (B×N×D); returns (α as B×N×D, final loss per problem)."""
        f = np.float32
        a = np.ascontiguousarray(np.asarray(alpha0, f).transpose(1, 0, 2))  # waypoint-major
        s, g = np.asarray(start, f), np.asarray(goal, f)
        obs = np.asarray(obstacles, f).reshape(-1, 2)
        loss = None
        for _ in range(iters):
            traj, vel = self._eval(self.K, a), self._eval(self.dK, a)
            _, ta, tb = self._terms(traj, vel, obs, s, g, True)
            a = self.cf * a - self.lr * self._grad(ta, tb)             # optimizer_GD.py:81
            loss, _, _ = self._terms(self._eval(self.K, a), self._eval(self.dK, a), obs, s, g, False)
        return np.ascontiguousarray(a.transpose(1, 0, 2)), loss


def params_namespace(p):
    """The IrmParams fields BatchedGD reads, as a picklable namespace (worker processes)."""
    from types import SimpleNamespace
    keys = ("n_timesteps", "n_joints", "lambda_max_cost", "lambda_sg_constraint", "lambda_jl_constraint",
            "lambda_reg", "max_joint_position", "min_joint_position", "joint_safety_limit", "max_joint_velocity",
            "constraint_violating_dependant_loss")
    ns = SimpleNamespace(**{k: getattr(p, k) for k in keys})
    ns.gd_lr = list(p.gd_lr)
    ns.link_length = list(p.link_length)
    return ns


def _worker(job):
    K, dK, J, ns, a0, s, g, obs, iters = job
    from threadpoolctl import threadpool_limits
    with threadpool_limits(1):  # one core per worker: OpenBLAS' own threads oversubscribe (and thin sgemms crawl)
        bg = BatchedGD(K, dK, J, ns)
        bg.run(a0[:1], s[:1], g[:1], obs, 1)  # warm-up
        import time
        t0 = time.perf_counter()
        a, loss = bg.run(a0, s, g, obs, iters)
        return a, loss, time.perf_counter() - t0


def run_processes(K, dK, J, params, alpha0, start, goal, obstacles, iters, procs):
    """BatchedGD over the batch split into `procs` chunks, one worker process each (fork: call before
    the process touches the GPU).  Returns (α, loss, max worker seconds)."""
    import multiprocessing as mp
    ns = params_namespace(params)
    B = len(alpha0)
    cuts = np.linspace(0, B, procs + 1).astype(int)
    jobs = [(K, dK, J, ns, alpha0[a:b], start[a:b], goal[a:b], obstacles, iters)
            for a, b in zip(cuts[:-1], cuts[1:]) if b > a]
    with mp.get_context("fork").Pool(len(jobs)) as pool:
        out = pool.map(_worker, jobs)
    return np.concatenate([o[0] for o in out]), np.concatenate([o[1] for o in out]), max(o[2] for o in out)
