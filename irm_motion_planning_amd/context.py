"""numpy-facing wrapper of one irm_ctx (include/irm.h).

`Context` owns a device context for one (N, D, hyper-parameter) configuration
— the analogue of one reference `Trajectory` + optimizer object
(trajectory.py:23-42, optimizer_GD.py:15-51, optimizer_BLS.py:23-54).  Every
method calls a HIP kernel through the C ABI; there is no host fallback.
"""
import ctypes

import numpy as np

from . import _abi
from ._abi import IrmBatchDev, IrmInfo, IrmLaunchPlan, IrmParams, IrmStats, check, load_library

_fp = _abi.c_float_p


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def _ptr(a):
    return None if a is None else a.ctypes.data_as(_fp)


def stats_to_dict(stats):
    out = {name: np.array([getattr(s, name) for s in stats]) for name in _abi.STATS_FIELDS}
    return out


def default_jac(n_joints, jac_gaussian_mean=0.15, seed=0):
    """J = I + jgm·normal(PRNGKey(seed), (D, D)) — trajectory.py:42."""
    lib = load_library()
    out = np.zeros(n_joints * n_joints, np.float32)
    check(lib.irm_default_jac(n_joints, float(jac_gaussian_mean), seed, _ptr(out)))
    return out.reshape(n_joints, n_joints)


def default_params():
    p = IrmParams()
    load_library().irm_params_default(ctypes.byref(p))
    return p


class Context:
    def __init__(self, params):
        self.lib = load_library()
        self.params = params
        self.N, self.D = int(params.n_timesteps), int(params.n_joints)
        h = ctypes.c_void_p()
        check(self.lib.irm_ctx_create(ctypes.byref(h), ctypes.byref(params)))
        self._h = h

    @property
    def handle(self):
        return self._h

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            self.lib.irm_ctx_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------- queries
    def info(self):
        inf = IrmInfo()
        check(self.lib.irm_get_info(self._h, ctypes.byref(inf)))
        d = {name: getattr(inf, name) for name, _ in IrmInfo._fields_}
        d["device_name"] = d["device_name"].decode()
        d["arch"] = d["arch"].decode()
        d["build_id"] = d["build_id"].decode()
        return d

    def launch_plan(self, batch, n_obstacles=0, series=False):
        """The optimiser launch optimize() runs for `batch` problems (irm_optimize_plan: filled in by
        the library's own launch dispatch, nothing launched)."""
        pl = IrmLaunchPlan()
        check(self.lib.irm_optimize_plan(self._h, int(batch), int(n_obstacles), int(bool(series)), ctypes.byref(pl)))
        d = {name: getattr(pl, name) for name, _ in IrmLaunchPlan._fields_}
        d["kernel"] = d["kernel"].decode()
        return d

    def kernel_matrices(self):
        N, D = self.N, self.D
        t = np.zeros(N, np.float32)
        K = np.zeros((N, N), np.float32)
        dK = np.zeros((N, N), np.float32)
        J = np.zeros((D, D), np.float32)
        check(self.lib.irm_kernel_matrices(self._h, _ptr(t), _ptr(K), _ptr(dK), _ptr(J)))
        return t, K, dK, J

    def series_capacity(self):
        return int(self.lib.irm_series_capacity(self._h))

    # ---------------------------------------------------------- batched ops
    def _batch(self, a, tail):
        a = _f32(a)
        single = a.ndim == len(tail)
        if single:
            a = a[None]
        return a, single

    def init_alpha(self, start, goal):
        s, single = self._batch(start, (self.D,))
        g, _ = self._batch(goal, (self.D,))
        out = np.zeros((s.shape[0], self.N, self.D), np.float32)
        check(self.lib.irm_init_alpha(self._h, _ptr(s), _ptr(g), s.shape[0], _ptr(out)))
        return out[0] if single else out

    def evaluate(self, alpha, which=0):
        a, single = self._batch(alpha, (self.N, self.D))
        out = np.zeros_like(a)
        check(self.lib.irm_evaluate(self._h, _ptr(a), a.shape[0], int(which), _ptr(out)))
        return out[0] if single else out

    def _sg(self, start, goal, B):
        s = _f32(np.broadcast_to(_f32(start), (B, self.D)))
        g = _f32(np.broadcast_to(_f32(goal), (B, self.D)))
        return s, g

    def eval_cost(self, alpha, obstacles, start, goal, lsg, ljl, lmax):
        a, single = self._batch(alpha, (self.N, self.D))
        B = a.shape[0]
        s, g = self._sg(start, goal, B)
        obs = _f32(obstacles).reshape(-1, 2)
        out = np.zeros(B, np.float32)
        check(self.lib.irm_eval_cost(self._h, _ptr(a), _ptr(s), _ptr(g), _ptr(obs), obs.shape[0], B,
                                     float(lsg), float(ljl), float(lmax), _ptr(out)))
        return out[0] if single else out

    def eval_cost_grad(self, alpha, obstacles, start, goal, lsg, ljl, lmax, with_cost=False):
        a, single = self._batch(alpha, (self.N, self.D))
        B = a.shape[0]
        s, g = self._sg(start, goal, B)
        obs = _f32(obstacles).reshape(-1, 2)
        grad = np.zeros_like(a)
        cost = np.zeros(B, np.float32)
        check(self.lib.irm_eval_cost_grad(self._h, _ptr(a), _ptr(s), _ptr(g), _ptr(obs), obs.shape[0], B,
                                          float(lsg), float(ljl), float(lmax), _ptr(grad), _ptr(cost)))
        if single:
            grad, cost = grad[0], cost[0]
        return (grad, cost) if with_cost else grad

    def constraints(self, alpha, start, goal):
        a, single = self._batch(alpha, (self.N, self.D))
        B = a.shape[0]
        s, g = self._sg(start, goal, B)
        ok = np.zeros(B, np.uint8)
        rep = np.zeros((B, 11), np.float32)
        check(self.lib.irm_constraints(self._h, _ptr(a), _ptr(s), _ptr(g), B,
                                       ok.ctypes.data_as(_abi.c_uint8_p), _ptr(rep)))
        if single:
            return bool(ok[0]), rep[0]
        return ok.astype(bool), rep

    def fk(self, traj, with_jacobian=False):
        q, single = self._batch(traj, (self.N, self.D))
        B = q.shape[0]
        pos = np.zeros((B, 2, self.N), np.float32)
        jac = np.zeros((B, 2, self.N, self.D), np.float32) if with_jacobian else None
        check(self.lib.irm_fk(self._h, _ptr(q), B, _ptr(pos), _ptr(jac)))
        if single:
            pos = pos[0]
            jac = None if jac is None else jac[0]
        return (pos, jac) if with_jacobian else pos

    def fk_joints(self, traj):
        """Positions of every joint, B×D×2×N (robot.py:39-72 fk_joint_j for j = 1..D)."""
        q, single = self._batch(traj, (self.N, self.D))
        B = q.shape[0]
        pos = np.zeros((B, self.D, 2, self.N), np.float32)
        check(self.lib.irm_fk_joints(self._h, _ptr(q), B, _ptr(pos)))
        return pos[0] if single else pos

    def compute_cost_vg(self, f, obstacles, with_grad=True):
        x, single = self._batch(f, (2, self.N))
        B = x.shape[0]
        obs = _f32(obstacles).reshape(-1, 2)
        cv = np.zeros((B, self.N), np.float32)
        cg = np.zeros((B, 2, self.N), np.float32) if with_grad else None
        check(self.lib.irm_compute_cost_vg(self._h, _ptr(x), _ptr(obs), obs.shape[0], B, _ptr(cv), _ptr(cg)))
        if single:
            cv = cv[0]
            cg = None if cg is None else cg[0]
        return (cv, cg) if with_grad else cv

    def optimize(self, start, goal, obstacles, alpha0=None, obstacle_stride=0, series=False):
        """Batched Optimizer.optimize(): returns (alpha, traj, stats[, series])."""
        s, single = self._batch(start, (self.D,))
        g, _ = self._batch(goal, (self.D,))
        B = s.shape[0]
        obs = _f32(obstacles)
        O = obs.shape[-2] if obs.size else 0
        if obs.ndim == 3:  # per-problem obstacles B × O × 2: one row of 2·O floats per problem
            if obs.shape[0] != B or obs.shape[2] != 2:
                raise ValueError(f"per-problem obstacles must be ({B}, O, 2), got {obs.shape}")
            if obstacle_stride not in (0, 2 * O):
                raise ValueError(f"obstacle_stride {obstacle_stride} does not match obstacles {obs.shape}")
            obstacle_stride = 2 * O
        elif obs.size and (obs.ndim != 2 or obs.shape[1] != 2):
            raise ValueError(f"shared obstacles must be (O, 2), got {obs.shape}")
        elif obstacle_stride:
            raise ValueError("obstacle_stride needs per-problem obstacles of shape (B, O, 2)")
        a0 = None
        if alpha0 is not None:
            a0 = _f32(alpha0).reshape(B, self.N, self.D)
        alpha = np.zeros((B, self.N, self.D), np.float32)
        traj = np.zeros_like(alpha)
        stats = (IrmStats * B)()
        cap = self.series_capacity() if series else 0
        ser = np.zeros((B, cap, self.N, self.D), np.float32) if series else None
        check(self.lib.irm_optimize_batch(self._h, _ptr(a0), _ptr(s), _ptr(g), _ptr(obs), O, int(obstacle_stride),
                                          B, _ptr(alpha), _ptr(traj), stats, _ptr(ser)))
        st = stats_to_dict(stats)
        if single:
            alpha, traj = alpha[0], traj[0]
            st = {k: v[0] for k, v in st.items()}
            if series:
                ser = ser[0][: int(st["series_len"])]
        if series:
            return alpha, traj, st, ser
        return alpha, traj, st

    def bls_trace_enable(self, cap=256):
        """Record the line-search log of problem 0 of every later BLS optimize (diagnostics)."""
        check(self.lib.irm_debug_bls_trace_enable(self._h, int(cap)))
        self._trace_cap = int(cap)

    def bls_trace(self, n_trials):
        """The last run's log: n_trials × 10 (outer, inner, trial, lr, new_loss, required_loss,
        accepted, loss, ‖g‖, alpha_norm) — optimizer_BLS.py:139-149, 163-166."""
        cap = getattr(self, "_trace_cap", 0)
        out = np.zeros((cap, 10), np.float32)
        n = self.lib.irm_debug_bls_trace(self._h, _ptr(out), cap)
        if n < 0:
            check(n)
        return out[: min(int(n_trials), n)]

    def optimize_dev(self, batch_dev, stream=0):
        """Enqueue irm_optimize_batch_dev with device pointers (IrmBatchDev)."""
        check(self.lib.irm_optimize_batch_dev(self._h, ctypes.byref(batch_dev), ctypes.c_void_p(stream)))


def batch_dev(alpha0=0, start=0, goal=0, obstacles=0, n_obstacles=0, obstacle_stride=0, batch=0, alpha_out=0,
              traj_out=0, stats_out=0, series_out=0):
    """Build an IrmBatchDev from raw device addresses (e.g. torch data_ptr())."""
    b = IrmBatchDev()
    b.alpha0, b.start, b.goal, b.obstacles = alpha0 or None, start, goal, obstacles
    b.n_obstacles, b.obstacle_stride, b.batch = n_obstacles, obstacle_stride, batch
    b.alpha_out, b.traj_out, b.stats_out, b.series_out = alpha_out or None, traj_out or None, stats_out or None, \
        series_out or None
    return b
