"""fp64 numpy restatement of the reference's cost, gradient and GD/BLS loops.

TEST INFRASTRUCTURE ONLY (like oracle.py).  Where the C oracle mirrors the
reference's fp32 arithmetic, this module runs the same algorithm in fp64, so
that tests can separate (a) fp32 rounding effects of the reference's α-space
iteration from (b) disagreements in the algorithm.  Citations as in
irm_oracle.c: trajectory.py:63-297, robot.py:29-113, environment.py:32-58,
optimizer_GD.py:68-97 / 386-445, optimizer_BLS.py:127-211.
"""
import numpy as np


class Ref64:
    def __init__(self, params, K, dK, J):
        p = params
        self.p = p
        self.N, self.D = int(p.n_timesteps), int(p.n_joints)
        self.K = np.asarray(K, np.float64)
        self.dK = np.asarray(dK, np.float64)
        self.J = np.asarray(J, np.float64)
        self.link = np.array([p.link_length[i] for i in range(self.D)], np.float64)
        self.mean = 0.5 * (p.max_joint_position + p.min_joint_position)
        self.std = 0.5 * (p.max_joint_position - self.mean)
        self.hi = p.joint_safety_limit * p.max_joint_position
        self.lo = p.joint_safety_limit * p.min_joint_position
        self.vthr = p.joint_safety_limit * p.max_joint_velocity

    def traj_vel(self, alpha):
        a = np.asarray(alpha, np.float64)
        return self.K @ a @ self.J, self.dK @ a @ self.J

    def _fk(self, q):
        c = np.cumsum(q, axis=1)
        x = (self.link * np.cos(c)).sum(1)
        y = (self.link * np.sin(c)).sum(1)
        sx = -(self.link * np.sin(c))
        cy = self.link * np.cos(c)
        jx = sx + sx.sum(1, keepdims=True) - np.cumsum(sx, axis=1)
        jy = cy + cy.sum(1, keepdims=True) - np.cumsum(cy, axis=1)
        return x, y, jx, jy

    def cost_tv(self, T, V, obs, s, g, lsg, ljl, lmax):
        p, N = self.p, self.N
        x, y, _, _ = self._fk(T)
        obs = np.asarray(obs, np.float64).reshape(-1, 2)
        d2 = (x[:, None] - obs[None, :, 0]) ** 2 + (y[:, None] - obs[None, :, 1]) ** 2
        cv = (0.8 / (0.5 + 0.5 * d2)).sum(1)
        toc = lmax * cv.max() + (1 - lmax) * cv.mean()
        sgp = 0.5 * np.sum((T[0] - s) ** 2) + 0.5 * np.sum((T[-1] - g) ** 2)
        sgv = 0.5 * np.sum(V[0] ** 2) + 0.5 * np.sum(V[-1] ** 2)
        z = (T - self.mean) / self.std
        mp = (T > self.hi) | (T < self.lo)
        jp = 0.5 * z ** 2
        if p.constraint_violating_dependant_loss:
            jp = np.where(mp, jp, 0.0)
        zv = V / p.max_joint_velocity
        mv = np.abs(V) > self.vthr
        jv = 0.5 * zv ** 2
        if p.constraint_violating_dependant_loss:
            jv = np.where(mv, jv, 0.0)
        return toc + lsg * (sgp + sgv) + ljl * (jp.sum() / N + jv.sum() / N)

    def grad_ab(self, T, V, obs, s, g, lsg, ljl, lmax):
        """∂cost/∂T (a) and ∂cost/∂V (b), per waypoint."""
        p, N = self.p, self.N
        x, y, jx, jy = self._fk(T)
        obs = np.asarray(obs, np.float64).reshape(-1, 2)
        dx = x[:, None] - obs[None, :, 0]
        dy = y[:, None] - obs[None, :, 1]
        den = 0.5 + 0.5 * (dx ** 2 + dy ** 2)
        cv = (0.8 / den).sum(1)
        gx = (-0.8 * dx / den ** 2).sum(1)
        gy = (-0.8 * dy / den ** 2).sum(1)
        w = np.full(N, (1 - lmax) / N)
        w[int(np.argmax(cv))] += lmax
        a = (w * gx)[:, None] * jx + (w * gy)[:, None] * jy
        b = np.zeros_like(V)
        a[0] += lsg * (T[0] - s)
        a[-1] += lsg * (T[-1] - g)
        b[0] += lsg * V[0]
        b[-1] += lsg * V[-1]
        mp = (T > self.hi) | (T < self.lo)
        jpg = (T - self.mean) / self.std ** 2 / N
        mv = np.abs(V) > self.vthr
        jvg = V / p.max_joint_velocity ** 2 / N
        if p.constraint_violating_dependant_loss:
            jpg = np.where(mp, jpg, 0.0)
            jvg = np.where(mv, jvg, 0.0)
        return a + ljl * jpg, b + ljl * jvg

    def cost(self, alpha, obs, s, g, lsg, ljl, lmax):
        T, V = self.traj_vel(alpha)
        return self.cost_tv(T, V, obs, s, g, lsg, ljl, lmax)

    def cost_g(self, alpha, obs, s, g, lsg, ljl, lmax):
        T, V = self.traj_vel(alpha)
        a, b = self.grad_ab(T, V, obs, s, g, lsg, ljl, lmax)
        return (self.K.T @ a + self.dK.T @ b) @ self.J.T

    def gd_single(self, alpha0, obs, s, g, iters, lr=None):
        """optimizer_GD.py:68-97 in fp64 (single loop, λ at their initial values)."""
        p = self.p
        lr = p.gd_lr[0] if lr is None else lr
        lsg, ljl, lmax = p.lambda_sg_constraint, p.lambda_jl_constraint, p.lambda_max_cost
        alpha = np.asarray(alpha0, np.float64).copy()
        last = self.cost(alpha, obs, s, g, lsg, ljl, lmax)
        n = 0
        for _ in range(iters):
            G = self.cost_g(alpha, obs, s, g, lsg, ljl, lmax)
            na = (1 - p.lambda_reg * lr) * alpha - lr * G
            nl = self.cost(na, obs, s, g, lsg, ljl, lmax)
            if last - nl < p.loop_loss_reduction:
                break
            alpha, last, n = na, nl, n + 1
        return alpha, last, n
