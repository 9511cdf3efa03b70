"""argparse Namespace (main.py's surface, main.py:13-102) -> IrmParams."""
import ctypes

from . import _abi
from ._abi import IrmParams, IrmError
from .context import default_jac


def params_from_args(args, **overrides):
    """Map the reference's argument namespace onto the C-ABI parameter block.

    Extra build-only knobs (operator_rank, device, record_series, ...) come
    from `overrides` or from same-named attributes of `args` when present.
    """
    p = IrmParams()
    _abi.load_library().irm_params_default(ctypes.byref(p))
    N = int(round(float(args.n_timesteps)))  # main.py:33 parses it as float
    D = int(args.n_joints)
    if len(args.link_length) != D:
        raise IrmError("FATAL: n_joints and link_length do not match")  # robot.py:21-23
    if args.optimizer_name not in ("gd", "bls"):
        raise IrmError(f"FATAL: not defined optimizer {args.optimizer_name}")  # main.py:113-115
    if args.optimizer_name == "gd" and args.max_outer_iteration > len(args.gd_lr):
        raise IrmError("FATAL: max_outer_iteration and dual_lr do not match")  # optimizer_GD.py:34-36
    if len(args.gd_lr) > _abi.IRM_MAX_LR:
        raise IrmError(f"at most {_abi.IRM_MAX_LR} --gd-lr values are supported")
    p.n_timesteps = N
    p.n_joints = D
    p.optimizer = _abi.IRM_OPT_GD if args.optimizer_name == "gd" else _abi.IRM_OPT_BLS
    p.max_inner_iteration = int(args.max_inner_iteration)
    p.max_outer_iteration = int(args.max_outer_iteration)
    p.max_bls_iteration = int(args.max_bls_iteration)
    p.constraint_violating_dependant_loss = 1 if args.constraint_violating_dependant_loss else 0
    p.n_gd_lr = len(args.gd_lr)
    for i in range(_abi.IRM_MAX_LR):
        p.gd_lr[i] = float(args.gd_lr[i]) if i < len(args.gd_lr) else 0.0
    p.rbf_variance = float(args.rbf_variance)
    p.loop_loss_reduction = float(args.loop_loss_reduction)
    p.lambda_constraint_increase = float(args.lambda_constraint_increase)
    p.lambda_sg_constraint = float(args.lambda_sg_constraint)
    p.lambda_jl_constraint = float(args.lambda_jl_constraint)
    p.eps_position = float(args.eps_position)
    p.eps_velocity = float(args.eps_velocity)
    p.lambda_max_cost = float(args.lambda_max_cost)
    p.lambda_reg = float(args.lambda_reg)
    p.joint_safety_limit = float(args.joint_safety_limit)
    p.bls_lr_start = float(args.bls_lr_start)
    p.bls_alpha = float(args.bls_alpha)
    p.bls_beta_plus = float(args.bls_beta_plus)
    p.bls_beta_minus = float(args.bls_beta_minus)
    p.max_joint_velocity = float(args.max_joint_velocity)
    p.max_joint_position = float(args.max_joint_position)
    p.min_joint_position = float(args.min_joint_position)
    for i in range(_abi.IRM_MAX_JOINTS):
        p.link_length[i] = float(args.link_length[i]) if i < D else 0.0
    J = default_jac(D, float(args.jac_gaussian_mean), 0)  # trajectory.py:42
    for i in range(_abi.IRM_MAX_JOINTS * _abi.IRM_MAX_JOINTS):
        p.jac[i] = float(J.reshape(-1)[i]) if i < D * D else 0.0
    knobs = {
        "operator_rank": 0,
        "operator_tol": 1e-12,
        "device": 0,
        "record_series": 0,
        "max_series": 0,
        "traj_per_block": 0,
        "whole_robot_cost": 0,
    }
    for k, v in knobs.items():
        val = overrides.get(k, getattr(args, k, v))
        setattr(p, k, type(v)(val))
    if "jac" in overrides:
        Jo = overrides["jac"]
        for i in range(D * D):
            p.jac[i] = float(Jo.reshape(-1)[i])
    return p
