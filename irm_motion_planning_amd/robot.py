"""Planar serial arm — mirrors robot.py of the reference.

fk / jacobian (robot.py:29-36, 75-87) run in the HIP kernel k_fk through
irm_fk; fk_joint_1..3 (robot.py:39-72, any joint 1..D) in k_fk_joints through
irm_fk_joints.  The constraint predicates (robot.py:90-113) compare a handful of
norms/extrema of arrays the caller already holds; constraintsFulfilled on a
whole α runs on the device (irm_constraints).
"""
import numpy as np

from ._abi import IrmError


class Robot:
    def __init__(self, args, context=None):
        self.max_joint_velocity = args.max_joint_velocity
        self.min_joint_position = args.min_joint_position
        self.max_joint_position = args.max_joint_position
        self.N_joints = args.n_joints
        self.link_length = np.array(args.link_length, dtype=np.float32)
        if self.N_joints != len(self.link_length):  # robot.py:21-23 (exit(-1) there)
            print("FATAL: n_joints and link_length do not match")
            raise IrmError("n_joints and link_length do not match")
        self.eps_velocity = args.eps_velocity
        self.eps_distance = args.eps_position
        self._ctx = context

    def fk(self, config):
        """End-effector (x, y) per waypoint: (2, N)."""
        return self._ctx.fk(np.asarray(config, np.float32).reshape(-1, self.N_joints))

    def fk_joint(self, config, joint_id):
        """Position of joint `joint_id` (FK of the first joint_id links): (2, N) — robot.py:39-72
        generalised to 1 ≤ joint_id ≤ D (k_fk_joints through irm_fk_joints)."""
        if not 1 <= int(joint_id) <= self.N_joints:
            raise IrmError(f"joint_id must be in 1..{self.N_joints}")
        pos = self._ctx.fk_joints(np.asarray(config, np.float32).reshape(-1, self.N_joints))
        return pos[int(joint_id) - 1]

    def fk_joint_1(self, config):  # robot.py:39-48
        return self.fk_joint(config, 1)

    def fk_joint_2(self, config):  # robot.py:51-60
        return self.fk_joint(config, 2)

    def fk_joint_3(self, config):  # robot.py:63-72
        return self.fk_joint(config, 3)

    def jacobian(self, config):
        """∂(x, y)/∂q per waypoint: (2, N, D)."""
        return self._ctx.fk(np.asarray(config, np.float32).reshape(-1, self.N_joints), with_jacobian=True)[1]

    def start_goal_position_constraint_fulfilled(self, s, g, start_config, goal_config):
        return bool(np.linalg.norm(np.float32(s) - start_config) < self.eps_distance and
                    np.linalg.norm(np.float32(g) - goal_config) < self.eps_distance)

    def start_goal_velocity_constraint_fulfilled(self, vs, vg):
        return bool(np.linalg.norm(vs) < self.eps_velocity and np.linalg.norm(vg) < self.eps_velocity)

    def joint_position_constraint(self, trajectory):
        t = np.asarray(trajectory)
        return bool(t.max() <= self.max_joint_position and t.min() >= self.min_joint_position)

    def joint_velocity_constraint(self, joint_velocity):
        return bool(np.abs(np.asarray(joint_velocity)).max() <= self.max_joint_velocity)
