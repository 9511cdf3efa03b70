"""Environment and obstacle potential — mirrors environment.py of the reference.

`Environment` holds the same start/goal configuration and 11 point obstacles
(environment.py:11-29).  `compute_cost` / `compute_cost_vg` evaluate the
inverse-quadratic potential (environment.py:32-58) with the HIP kernel
k_cost_vg through irm_compute_cost_vg.
"""
import numpy as np

from .context import Context, default_params

START_CONFIG = np.array([0.0, 0.0, 0.0], dtype=np.float32)  # environment.py:14
GOAL_CONFIG = np.array([1.2, 0.8, 0.3], dtype=np.float32)  # environment.py:15
OBSTACLES = np.array(  # environment.py:17-29 (int32 like the reference literal)
    [[2, -3], [-2, 2], [3, 3], [-1, -2], [-2, 1], [-1, -1], [-2, -3], [-2, 0], [1, 3], [3, 2], [2, 3]],
    dtype=np.int32,
)


class Environment:
    def __init__(self):
        self.start_config = START_CONFIG.copy()
        self.goal_config = GOAL_CONFIG.copy()
        self.obstacles = OBSTACLES.copy()


_CTX = {}


def _ctx_for(n_points):
    """A small context whose N matches the number of points (cached per N)."""
    n = int(n_points)
    if n not in _CTX:
        p = default_params()
        p.n_timesteps = max(2, n)
        _CTX[n] = Context(p)
    return _CTX[n]


def _as_f(f):
    f = np.ascontiguousarray(f, dtype=np.float32)
    if f.ndim != 2 or f.shape[0] != 2:
        raise ValueError("f must have shape (2, t_len)")
    return f


def compute_cost(f, obstacles):
    """cost_v[n] = Σ_o 0.8 / (0.5 + 0.5‖f_n − o‖²) — environment.py:32-43."""
    f = _as_f(f)
    return _ctx_for(f.shape[1]).compute_cost_vg(f, obstacles, with_grad=False)


def compute_cost_vg(f, obstacles):
    """(cost_v, cost_g) — environment.py:46-58."""
    f = _as_f(f)
    return _ctx_for(f.shape[1]).compute_cost_vg(f, obstacles, with_grad=True)


def compute_cost_g(f, obstacles):
    """cost_g only — environment.py:61-72."""
    return compute_cost_vg(f, obstacles)[1]
