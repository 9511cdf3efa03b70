"""RKHS trajectory — mirrors trajectory.py of the reference on the HIP backend.

Same attributes (robot, rbf_var, N_timesteps, t, c, km, dkm, jac,
mean/std_joint_position) and the same public methods with the same argument
meaning; every method runs a HIP kernel through the C ABI:

  evaluate                    trajectory.py:63-65   irm_evaluate
  initTrajectory              trajectory.py:73-78   irm_init_alpha
  compute_trajectory_cost     trajectory.py:271-281 irm_eval_cost
  compute_trajectory_cost_g   trajectory.py:284-297 irm_eval_cost_grad
  constraintsFulfilled        trajectory.py:129-137 irm_constraints
  constraintsFulfilledVerbose trajectory.py:140-180 irm_constraints (report)
All methods also accept a leading batch dimension.
"""
import numpy as np

from .context import Context
from .params import params_from_args
from .robot import Robot


class Trajectory:
    def __init__(self, args, context=None, **overrides):
        self.context = context if context is not None else Context(params_from_args(args, **overrides))
        self.robot = Robot(args, self.context)
        self.rbf_var = args.rbf_variance
        self.constraint_violating_dependant_loss = args.constraint_violating_dependant_loss
        self.joint_safety_limit = args.joint_safety_limit
        self.mean_joint_position = 0.5 * (self.robot.max_joint_position + self.robot.min_joint_position)
        self.std_joint_position = 0.5 * (self.robot.max_joint_position - self.mean_joint_position)
        self.N_timesteps = self.context.N
        t, km, dkm, jac = self.context.kernel_matrices()
        self.t = t
        self.c = 6 * t ** 5 - 15 * t ** 4 + 10 * t ** 3
        self.km, self.dkm, self.jac = km, dkm, jac

    # ------------------------------------------------------------ evaluation
    def evaluate(self, alpha, kernel_matrix, jac):
        """kernel_matrix @ alpha @ jac for kernel_matrix ∈ {km, dkm}."""
        if jac is not self.jac and not np.array_equal(np.asarray(jac), self.jac):
            raise ValueError("evaluate: only this trajectory's J is supported")
        if kernel_matrix is self.km:
            which = 0
        elif kernel_matrix is self.dkm:
            which = 1
        elif np.array_equal(np.asarray(kernel_matrix), self.km):
            which = 0
        elif np.array_equal(np.asarray(kernel_matrix), self.dkm):
            which = 1
        else:
            raise ValueError("evaluate: kernel_matrix must be this trajectory's km or dkm")
        return self.context.evaluate(alpha, which)

    def initTrajectory(self, start_config, goal_config):
        return self.context.init_alpha(start_config, goal_config)

    # ----------------------------------------------------------------- costs
    def compute_trajectory_cost(self, alpha, obstacles, start_config, goal_config, lambda_sg_constraint,
                                lambda_jl_constraint, lambda_max_cost):
        return self.context.eval_cost(alpha, obstacles, start_config, goal_config, lambda_sg_constraint,
                                      lambda_jl_constraint, lambda_max_cost)

    def compute_trajectory_cost_g(self, alpha, obstacles, start_config, goal_config, lambda_sg_constraint,
                                  lambda_jl_constraint, lambda_max_cost):
        return self.context.eval_cost_grad(alpha, obstacles, start_config, goal_config, lambda_sg_constraint,
                                           lambda_jl_constraint, lambda_max_cost)

    # ----------------------------------------------------------- constraints
    def constraintsFulfilled(self, alpha, start_config, goal_config):
        ok, _ = self.context.constraints(alpha, start_config, goal_config)
        return ok

    def constraintsFulfilledVerbose(self, alpha, start_config, goal_config, verbose=True):
        ok, r = self.context.constraints(alpha, start_config, goal_config)
        r = np.asarray(r, np.float32)
        f32 = np.float32
        if verbose:
            print(("ok" if r[7] else "violated") + " start goal position", f32(r[0]), f32(r[1]))
            print(("ok" if r[8] else "violated") + " start goal velocity", f32(r[2]), f32(r[3]))
            if r[9]:
                print("ok joint limit with", f32(r[4]), f32(r[5]))
            else:
                print("joint limit exceeded with", f32(r[4]), f32(r[5]))
            if r[10]:
                print("ok velocity limit with", f32(r[6]))
            else:
                print("joint velocity exceeded with", f32(r[6]))
        return bool(ok)
