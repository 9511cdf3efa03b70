"""Dynamic environments: re-plan a batch as obstacles move.

In the reference, obstacles, start and goal are traced arguments of the jitted
optimiser (`jit_optimize(alpha, obstacles, start, goal)`, optimizer_BLS.py:127-131,
optimizer_GD.py:173-177), so a new environment re-uses the compiled loop
(DevBlog-Theme/blog-post.html:353-354), but every optimize() restarts from the
straight line of initTrajectory (optimizer_BLS.py:57-62).

`Replanner` is the MPC-style form of that on the device:

* one context (K, dK, the low-rank operator, J) and one set of HBM buffers serve
  every call; only the new obstacles / start / goal are copied in;
* with warm_start the next plan starts from the previous plan's α, which never
  leaves HBM (α_out of call k is α0 of call k+1, double-buffered);
* each call is one optimiser launch (k_lean / k_optimize) through irm_optimize_batch_dev on the
  caller's stream (torch provides device memory and the stream).

The first call, or warm_start=False, is exactly Optimizer.optimize() for the batch.
A warm-started call equals irm_optimize_batch with alpha0 = the previous α_out bit for
bit (tests/test_gpu_parity.py::test_replanner_*).
"""
import numpy as np

from ._abi import STATS_FIELDS, IrmError
from .context import Context, batch_dev
from .params import params_from_args


class Replanner:
    def __init__(self, args, batch, n_obstacles, per_problem_obstacles=False, device=None, **overrides):
        import torch
        dev = int(device if device is not None else getattr(args, "device", 0))
        overrides.setdefault("device", dev)
        # raises IrmError without a gfx950 device: there is no CPU fallback
        self.context = Context(params_from_args(args, **overrides))
        self.N, self.D, self.B, self.O = self.context.N, self.context.D, int(batch), int(n_obstacles)
        self.per_problem = bool(per_problem_obstacles)
        self.torch = torch
        self.device = torch.device("cuda", dev)
        f32 = dict(dtype=torch.float32, device=self.device)
        B, N, D, O = self.B, self.N, self.D, self.O
        self.start = torch.zeros((B, D), **f32)
        self.goal = torch.zeros((B, D), **f32)
        self.obstacles = torch.zeros(((B if self.per_problem else 1) * max(O, 1), 2), **f32)
        self._alpha = [torch.zeros((B, N, D), **f32), torch.zeros((B, N, D), **f32)]
        self.traj = torch.zeros((B, N, D), **f32)
        self.stats = torch.zeros((B, len(STATS_FIELDS)), dtype=torch.int32, device=self.device)
        self.cur = 0          # index of the buffer holding the latest α
        self.planned = False  # is there a previous plan to warm-start from?
        self.calls = 0

    def _put(self, dst, x, shape):
        x = np.array(np.broadcast_to(np.asarray(x, np.float32), shape))  # writable copy
        dst.copy_(self.torch.from_numpy(x).reshape(dst.shape), non_blocking=False)

    def plan(self, obstacles, start=None, goal=None, warm_start=True, stream=None):
        """Optimise the batch against `obstacles` (O×2, or B×O×2 per problem).

        start / goal (B×D or D) are kept from the previous call when None.  Returns
        the per-problem statistics (dict of numpy arrays, irm_stats fields); the plan
        stays on the device (alpha(), trajectory())."""
        torch = self.torch
        B, D, O = self.B, self.D, self.O
        obs = np.asarray(obstacles, np.float32)
        want = (B, O, 2) if self.per_problem else (O, 2)
        if obs.shape != want:
            raise IrmError(f"obstacles must have shape {want}, got {obs.shape}")
        if start is not None:
            self._put(self.start, start, (B, D))
        if goal is not None:
            self._put(self.goal, goal, (B, D))
        if self.calls == 0 and (start is None or goal is None):
            raise IrmError("the first plan() needs start and goal")
        if O:
            self._put(self.obstacles, obs.reshape(-1, 2), self.obstacles.shape)
        warm = bool(warm_start) and self.planned
        a_in, a_out = self._alpha[self.cur], self._alpha[self.cur ^ 1]
        bd = batch_dev(alpha0=a_in.data_ptr() if warm else 0, start=self.start.data_ptr(),
                       goal=self.goal.data_ptr(), obstacles=self.obstacles.data_ptr(), n_obstacles=O,
                       obstacle_stride=2 * O if self.per_problem else 0, batch=B, alpha_out=a_out.data_ptr(),
                       traj_out=self.traj.data_ptr(), stats_out=self.stats.data_ptr())
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        self.context.optimize_dev(bd, s.cuda_stream)
        self.cur ^= 1
        self.planned = True
        self.calls += 1
        s.synchronize()
        st = self.stats.cpu().numpy()
        out = {name: st[:, i].copy() for i, name in enumerate(STATS_FIELDS)}
        out["final_loss"] = st[:, STATS_FIELDS.index("final_loss")].view(np.float32).copy()
        return out

    def alpha(self):
        """The latest plan's α (B×N×D, device tensor)."""
        return self._alpha[self.cur]

    def alpha_host(self):
        return self._alpha[self.cur].cpu().numpy()

    def trajectory(self):
        """K·α·J of the latest plan (B×N×D, device tensor)."""
        return self.traj

    def trajectory_host(self):
        return self.traj.cpu().numpy()

