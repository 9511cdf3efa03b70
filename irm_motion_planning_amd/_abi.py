"""ctypes mirror of include/irm.h and the loader of libirm_hip.so.

The shared library is built in-tree by irm_motion_planning_amd.build (or
__graft_entry__.build()).  There is deliberately no CPU fallback: if the HIP
library is missing, or no gfx950 device is present when a context is created,
the calls raise IrmError.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("IRM_LIB") or os.path.join(HERE, "libirm_hip.so")

IRM_ABI_VERSION = 3
IRM_MAX_JOINTS = 8
IRM_MAX_TIMESTEPS = 512
IRM_MAX_OBSTACLES = 64
IRM_MAX_LR = 32

IRM_OPT_GD = 0
IRM_OPT_BLS = 1

c_float_p = ctypes.POINTER(ctypes.c_float)
c_int32_p = ctypes.POINTER(ctypes.c_int32)
c_uint8_p = ctypes.POINTER(ctypes.c_uint8)


class IrmError(RuntimeError):
    """Raised for a negative return code of the C ABI (message from irm_last_error)."""


class IrmParams(ctypes.Structure):
    _fields_ = [
        ("n_timesteps", ctypes.c_int32),
        ("n_joints", ctypes.c_int32),
        ("optimizer", ctypes.c_int32),
        ("max_inner_iteration", ctypes.c_int32),
        ("max_outer_iteration", ctypes.c_int32),
        ("max_bls_iteration", ctypes.c_int32),
        ("constraint_violating_dependant_loss", ctypes.c_int32),
        ("n_gd_lr", ctypes.c_int32),
        ("rbf_variance", ctypes.c_float),
        ("loop_loss_reduction", ctypes.c_float),
        ("lambda_constraint_increase", ctypes.c_float),
        ("lambda_sg_constraint", ctypes.c_float),
        ("lambda_jl_constraint", ctypes.c_float),
        ("eps_position", ctypes.c_float),
        ("eps_velocity", ctypes.c_float),
        ("lambda_max_cost", ctypes.c_float),
        ("lambda_reg", ctypes.c_float),
        ("joint_safety_limit", ctypes.c_float),
        ("bls_lr_start", ctypes.c_float),
        ("bls_alpha", ctypes.c_float),
        ("bls_beta_plus", ctypes.c_float),
        ("bls_beta_minus", ctypes.c_float),
        ("max_joint_velocity", ctypes.c_float),
        ("max_joint_position", ctypes.c_float),
        ("min_joint_position", ctypes.c_float),
        ("gd_lr", ctypes.c_float * IRM_MAX_LR),
        ("link_length", ctypes.c_float * IRM_MAX_JOINTS),
        ("jac", ctypes.c_float * (IRM_MAX_JOINTS * IRM_MAX_JOINTS)),
        ("operator_rank", ctypes.c_int32),
        ("operator_tol", ctypes.c_float),
        ("device", ctypes.c_int32),
        ("record_series", ctypes.c_int32),
        ("max_series", ctypes.c_int32),
        ("traj_per_block", ctypes.c_int32),
        ("whole_robot_cost", ctypes.c_int32),
    ]


class IrmStats(ctypes.Structure):
    _fields_ = [
        ("inner_iterations", ctypes.c_int32),
        ("outer_iterations", ctypes.c_int32),
        ("grad_evals", ctypes.c_int32),
        ("cost_evals", ctypes.c_int32),
        ("bls_trials", ctypes.c_int32),
        ("constraints_ok", ctypes.c_int32),
        ("series_len", ctypes.c_int32),
        ("final_loss", ctypes.c_float),
    ]


STATS_FIELDS = [f[0] for f in IrmStats._fields_]


class IrmInfo(ctypes.Structure):
    _fields_ = [
        ("abi_version", ctypes.c_int32),
        ("n_timesteps", ctypes.c_int32),
        ("n_joints", ctypes.c_int32),
        ("operator_rank", ctypes.c_int32),
        ("operator_trunc", ctypes.c_float),
        ("traj_per_block", ctypes.c_int32),
        ("num_cus", ctypes.c_int32),
        ("lds_bytes_optimize", ctypes.c_int32),
        ("device_name", ctypes.c_char * 64),
        ("arch", ctypes.c_char * 32),
        ("build_id", ctypes.c_char * 24),
    ]


class IrmLaunchPlan(ctypes.Structure):
    _fields_ = [
        ("kernel", ctypes.c_char * 128),
        ("lean", ctypes.c_int32),
        ("flow", ctypes.c_int32),
        ("waypoints_per_lane", ctypes.c_int32),
        ("threads", ctypes.c_int32),
        ("grid", ctypes.c_int32),
        ("lds_bytes", ctypes.c_int32),
        ("traj_per_block", ctypes.c_int32),
        ("rank_z", ctypes.c_int32),
        ("rank_dir", ctypes.c_int32),
        ("rank_g", ctypes.c_int32),
        ("lam16", ctypes.c_float),
        ("lam24", ctypes.c_float),
    ]


class IrmBatchDev(ctypes.Structure):
    _fields_ = [
        ("alpha0", ctypes.c_void_p),
        ("start", ctypes.c_void_p),
        ("goal", ctypes.c_void_p),
        ("obstacles", ctypes.c_void_p),
        ("n_obstacles", ctypes.c_int32),
        ("obstacle_stride", ctypes.c_int32),
        ("batch", ctypes.c_int32),
        ("pad_", ctypes.c_int32),
        ("alpha_out", ctypes.c_void_p),
        ("traj_out", ctypes.c_void_p),
        ("stats_out", ctypes.c_void_p),
        ("series_out", ctypes.c_void_p),
    ]


# name -> (restype, argtypes); every symbol include/irm.h declares.
PROTOTYPES = {
    "irm_params_default": (None, [ctypes.POINTER(IrmParams)]),
    "irm_default_jac": (ctypes.c_int, [ctypes.c_int32, ctypes.c_float, ctypes.c_uint32, c_float_p]),
    "irm_ctx_create": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(IrmParams)]),
    "irm_ctx_destroy": (None, [ctypes.c_void_p]),
    "irm_last_error": (ctypes.c_char_p, []),
    "irm_get_info": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(IrmInfo)]),
    "irm_kernel_matrices": (ctypes.c_int, [ctypes.c_void_p, c_float_p, c_float_p, c_float_p, c_float_p]),
    "irm_init_alpha": (ctypes.c_int, [ctypes.c_void_p, c_float_p, c_float_p, ctypes.c_int32, c_float_p]),
    "irm_evaluate": (ctypes.c_int, [ctypes.c_void_p, c_float_p, ctypes.c_int32, ctypes.c_int32, c_float_p]),
    "irm_eval_cost": (
        ctypes.c_int,
        [ctypes.c_void_p, c_float_p, c_float_p, c_float_p, c_float_p, ctypes.c_int32, ctypes.c_int32,
         ctypes.c_float, ctypes.c_float, ctypes.c_float, c_float_p],
    ),
    "irm_eval_cost_grad": (
        ctypes.c_int,
        [ctypes.c_void_p, c_float_p, c_float_p, c_float_p, c_float_p, ctypes.c_int32, ctypes.c_int32,
         ctypes.c_float, ctypes.c_float, ctypes.c_float, c_float_p, c_float_p],
    ),
    "irm_constraints": (
        ctypes.c_int, [ctypes.c_void_p, c_float_p, c_float_p, c_float_p, ctypes.c_int32, c_uint8_p, c_float_p]
    ),
    "irm_fk": (ctypes.c_int, [ctypes.c_void_p, c_float_p, ctypes.c_int32, c_float_p, c_float_p]),
    "irm_fk_joints": (ctypes.c_int, [ctypes.c_void_p, c_float_p, ctypes.c_int32, c_float_p]),
    "irm_compute_cost_vg": (
        ctypes.c_int, [ctypes.c_void_p, c_float_p, c_float_p, ctypes.c_int32, ctypes.c_int32, c_float_p, c_float_p]
    ),
    "irm_optimize_batch": (
        ctypes.c_int,
        [ctypes.c_void_p, c_float_p, c_float_p, c_float_p, c_float_p, ctypes.c_int32, ctypes.c_int32,
         ctypes.c_int32, c_float_p, c_float_p, ctypes.POINTER(IrmStats), c_float_p],
    ),
    "irm_optimize_batch_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(IrmBatchDev), ctypes.c_void_p]),
    "irm_series_capacity": (ctypes.c_int32, [ctypes.c_void_p]),
    "irm_optimize_plan": (
        ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(IrmLaunchPlan)]
    ),
    "irm_build_id": (ctypes.c_char_p, []),
    "irm_debug_phase_profile": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int32]),
    "irm_debug_bls_trace_enable": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32]),
    "irm_debug_bls_trace": (ctypes.c_int, [ctypes.c_void_p, c_float_p, ctypes.c_int32]),
}

_LIB = None


def load_library(path=None):
    """Load libirm_hip.so (in-tree build).  Raises IrmError if it is missing."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    path = path or LIB_PATH
    if not os.path.exists(path):
        raise IrmError(
            f"{path} not found: build the HIP library first "
            "(python -c 'import __graft_entry__ as g; g.build()')"
        )
    # One HIP runtime per process.  torch ships its own libamdhip64 (SONAME libamdhip64.so.7,
    # but torch's libraries NEED it as "libamdhip64.so"): loaded after ours, the loader maps a
    # second runtime and torch then finds "No HIP GPUs".  Loaded first, ours resolves to torch's
    # copy by SONAME.  So torch, when present, is imported before the library.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(path)
    for name, (res, args) in PROTOTYPES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path == LIB_PATH:
        _LIB = lib
    return lib


def check(rc):
    if rc != 0:
        msg = load_library().irm_last_error()
        raise IrmError(f"irm error {rc}: {msg.decode() if msg else ''}")
    return rc
