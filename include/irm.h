/*
 * irm.h — C ABI of the MI355X-native RKHS trajectory optimiser
 * (drop-in for the hot path of simongroeger/irm_motion_planning).
 *
 * The reference has no FFI layer: its de-facto operator boundary is the
 * Python object API that main.py drives:
 *   Optimizer(args) / .optimize()        main.py:109-122, optimizer_GD.py:54-65,
 *                                        optimizer_BLS.py:57-62
 *   Trajectory.evaluate                  trajectory.py:63-65
 *   Trajectory.initTrajectory            trajectory.py:73-78
 *   Trajectory.compute_trajectory_cost   trajectory.py:271-281
 *   Trajectory.compute_trajectory_cost_g trajectory.py:284-297
 *   Trajectory.constraintsFulfilled      trajectory.py:129-137
 *   Robot.fk / Robot.jacobian            robot.py:29-36, 75-87
 *   environment.compute_cost(_vg)        environment.py:32-58
 * Each entry point below names the reference symbol it replaces.  The
 * Python host layer (irm_motion_planning_amd/) binds these with ctypes.
 *
 * Conventions
 *   - Arrays are C-contiguous float32, row-major.  A batch of B trajectories
 *     of N waypoints and D joints is B×N×D (waypoint-major, as np.savetxt
 *     writes a reference trajectory).  Obstacles are O×2.
 *   - Host-pointer entry points copy in, compute on the context's device and
 *     synchronise before returning.  *_dev entry points take device pointers
 *     and a hipStream_t (as void*) and only enqueue.
 *   - Return 0 on success, a negative IRM_E* code on failure; the message is
 *     available from irm_last_error() (thread-local).  Nothing here calls
 *     exit(); the reference's exit(-1) cases are reported as IRM_EINVAL.
 *   - One context per device per thread.  There is no CPU fallback: a
 *     context cannot be created without a gfx950 device.
 */
#ifndef IRM_H_
#define IRM_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define IRM_ABI_VERSION 3

#define IRM_MAX_JOINTS 8       /* D  */
#define IRM_MAX_TIMESTEPS 512  /* N  */
#define IRM_MAX_OBSTACLES 64   /* O  */
#define IRM_MAX_LR 32          /* len(--gd-lr) */

#define IRM_OK 0
#define IRM_EINVAL (-22)
#define IRM_ENOMEM (-12)
#define IRM_EDEVICE (-19)
#define IRM_EKERNEL (-5)

#define IRM_OPT_GD 0  /* optimizer_GD.GradientDescentOptimizer            */
#define IRM_OPT_BLS 1 /* optimizer_BLS.BacktrackingLineSearchOptimizer    */

/* Hyper-parameters: every field of main.py's argparser (main.py:13-102) that
 * reaches the optimiser, with the same meaning.  Fill with irm_params_default
 * and override. */
typedef struct irm_params {
    int32_t n_timesteps;         /* --n-timesteps (N), main.py:33          */
    int32_t n_joints;            /* --n-joints (D), main.py:89             */
    int32_t optimizer;           /* IRM_OPT_GD | IRM_OPT_BLS, main.py:27   */
    int32_t max_inner_iteration; /* main.py:41                             */
    int32_t max_outer_iteration; /* main.py:47                             */
    int32_t max_bls_iteration;   /* main.py:73                             */
    int32_t constraint_violating_dependant_loss; /* bool, main.py:67      */
    int32_t n_gd_lr;             /* number of valid entries in gd_lr      */
    float rbf_variance;          /* σ of the RBF kernel, main.py:35        */
    float loop_loss_reduction;   /* main.py:43                             */
    float lambda_constraint_increase; /* main.py:49                        */
    float lambda_sg_constraint;  /* main.py:52                             */
    float lambda_jl_constraint;  /* main.py:54                             */
    float eps_position;          /* main.py:57                             */
    float eps_velocity;          /* main.py:59                             */
    float lambda_max_cost;       /* main.py:63                             */
    float lambda_reg;            /* main.py:65                             */
    float joint_safety_limit;    /* main.py:69                             */
    float bls_lr_start;          /* main.py:75                             */
    float bls_alpha;             /* main.py:77                             */
    float bls_beta_plus;         /* main.py:79                             */
    float bls_beta_minus;        /* main.py:81                             */
    float max_joint_velocity;    /* main.py:93                             */
    float max_joint_position;    /* main.py:95                             */
    float min_joint_position;    /* main.py:97                             */
    float gd_lr[IRM_MAX_LR];     /* --gd-lr, main.py:85                    */
    float link_length[IRM_MAX_JOINTS];           /* main.py:91             */
    float jac[IRM_MAX_JOINTS * IRM_MAX_JOINTS];  /* J (D×D), trajectory.py:42;
                                                    irm_default_jac fills it */
    /* --- build-only knobs (no reference counterpart) --- */
    int32_t operator_rank;  /* rank R of the kernel operator used inside the
                               optimiser loop: 0 = auto (smallest multiple of
                               16 whose truncation is below operator_tol),
                               -1 = dense (exact [K;dK]), >0 = explicit. */
    float operator_tol;     /* auto-rank tolerance on σ_R²/σ_0² (1e-12)   */
    int32_t device;         /* HIP device ordinal                          */
    int32_t record_series;  /* keep per-iteration snapshots (--extended-vis) */
    int32_t max_series;     /* snapshot capacity per trajectory (0 = auto) */
    int32_t traj_per_block; /* trajectories per workgroup (0 = auto)       */
    /* --- additive cost variant (ABI 2) --- */
    int32_t whole_robot_cost; /* 0: end-effector obstacle cost (the reference's,
                                 trajectory.py:113-126); 1: summed over every
                                 joint position fk_j, j = 1..D (robot.py:39-72;
                                 DevBlog-Theme/blog-post.html:491-498)       */
} irm_params;

/* Per-trajectory statistics of one optimize() call. */
typedef struct irm_stats {
    int32_t inner_iterations; /* accepted inner-loop steps, all outer iterations */
    int32_t outer_iterations; /* outer (λ) iterations executed               */
    int32_t grad_evals;       /* compute_trajectory_cost_g equivalents       */
    int32_t cost_evals;       /* compute_trajectory_cost equivalents         */
    int32_t bls_trials;       /* BLS trial evaluations (0 for GD)            */
    int32_t constraints_ok;   /* constraintsFulfilled at exit (0/1)          */
    int32_t series_len;       /* snapshots written (record_series)           */
    float final_loss;         /* loss at the returned α with the final λ's   */
} irm_stats;

/* Context / device facts (filled by irm_get_info). */
typedef struct irm_info {
    int32_t abi_version;
    int32_t n_timesteps;
    int32_t n_joints;
    int32_t operator_rank;      /* R actually used                         */
    float operator_trunc;       /* σ_R²/σ_0² dropped by the truncation     */
    int32_t traj_per_block;     /* TB used by the optimiser kernel         */
    int32_t num_cus;
    int32_t lds_bytes_optimize; /* LDS per optimiser workgroup             */
    char device_name[64];
    char arch[32];
    char build_id[24];          /* = irm_build_id(): source hash of the build */
} irm_info;

/* Device-pointer batch for irm_optimize_batch_dev.  All pointers are device
 * pointers; nullable outputs may be 0. */
typedef struct irm_batch_dev {
    const float* alpha0;   /* B×N×D initial α (or 0: start from the straight
                              line of initTrajectory, computed on device)    */
    const float* start;    /* B×D                                            */
    const float* goal;     /* B×D                                            */
    const float* obstacles;/* O×2 (obstacle_stride 0) or B×O×2               */
    int32_t n_obstacles;   /* O                                              */
    int32_t obstacle_stride; /* 0: shared environment; else floats between
                                consecutive trajectories' obstacle sets      */
    int32_t batch;         /* B                                              */
    int32_t pad_;
    float* alpha_out;      /* B×N×D final α (nullable)                       */
    float* traj_out;       /* B×N×D final K α J (nullable)                   */
    irm_stats* stats_out;  /* B (nullable)                                   */
    float* series_out;     /* B×max_series×N×D snapshots (nullable)          */
} irm_batch_dev;

typedef struct irm_ctx irm_ctx;

/* Defaults of main.py's argparser (main.py:13-102), N=50, D=3, BLS. */
void irm_params_default(irm_params* p);

/* J = I + jgm·normal(PRNGKey(seed), (D,D)), legacy threefry2x32 as
 * jax.random.normal draws it — trajectory.py:42. */
int irm_default_jac(int32_t n_joints, float jac_gaussian_mean, uint32_t seed, float* jac_out);

int irm_ctx_create(irm_ctx** out, const irm_params* params);
void irm_ctx_destroy(irm_ctx* ctx);
const char* irm_last_error(void);
int irm_get_info(const irm_ctx* ctx, irm_info* out);

/* t (N), K (N×N), dK (N×N), J (D×D) exactly as Trajectory.__init__ builds
 * them — trajectory.py:14-19, 35-48 (any output may be NULL). */
int irm_kernel_matrices(const irm_ctx* ctx, float* t, float* km, float* dkm, float* jac);

/* Trajectory.initTrajectory — trajectory.py:73-78: α0 = solve(K, line·J⁻¹)
 * for B start/goal pairs (B×D each) → B×N×D. */
int irm_init_alpha(irm_ctx* ctx, const float* start, const float* goal, int32_t batch, float* alpha_out);

/* Trajectory.evaluate — trajectory.py:63-65: out = M·α·J with M = K
 * (which = 0) or dK (which = 1), for B trajectories. */
int irm_evaluate(irm_ctx* ctx, const float* alpha, int32_t batch, int32_t which, float* out);

/* Trajectory.compute_trajectory_cost — trajectory.py:271-281. */
int irm_eval_cost(irm_ctx* ctx, const float* alpha, const float* start, const float* goal,
                  const float* obstacles, int32_t n_obstacles, int32_t batch,
                  float lambda_sg, float lambda_jl, float lambda_max, float* cost_out);

/* Trajectory.compute_trajectory_cost_g — trajectory.py:284-297 (cost_out
 * nullable: the cost at α is produced by the same pass). */
int irm_eval_cost_grad(irm_ctx* ctx, const float* alpha, const float* start, const float* goal,
                       const float* obstacles, int32_t n_obstacles, int32_t batch,
                       float lambda_sg, float lambda_jl, float lambda_max,
                       float* grad_out, float* cost_out);

/* Trajectory.constraintsFulfilled(Verbose) — trajectory.py:129-180 with
 * robot.py:90-113.  report_out (nullable) holds, per trajectory, the 7
 * numbers constraintsFulfilledVerbose prints: ‖τ0−s‖, ‖τN−1−g‖, ‖v0‖,
 * ‖vN−1‖, max τ, min τ, max|v|, plus the 4 sub-flags as floats (11). */
int irm_constraints(irm_ctx* ctx, const float* alpha, const float* start, const float* goal,
                    int32_t batch, uint8_t* ok_out, float* report_out);

/* Robot.fk + Robot.jacobian — robot.py:29-36, 75-87: pos_out B×2×N,
 * jac_out B×2×N×D (nullable). */
int irm_fk(irm_ctx* ctx, const float* traj, int32_t batch, float* pos_out, float* jac_out);

/* Robot.fk_joint_1..3 — robot.py:39-72 (generalised to j = 1..D): position of
 * joint j (FK of the first j links) for every waypoint, pos_out B×D×2×N
 * (pos_out[b][j-1] = fk_joint_j(traj[b]); fk_joint_D = fk).  ABI 2. */
int irm_fk_joints(irm_ctx* ctx, const float* traj, int32_t batch, float* pos_out);

/* environment.compute_cost_vg — environment.py:46-58 (cost_g nullable ⇒
 * compute_cost, environment.py:32-43): f B×2×N → cost_v B×N, cost_g B×2×N. */
int irm_compute_cost_vg(irm_ctx* ctx, const float* f, const float* obstacles, int32_t n_obstacles,
                        int32_t batch, float* cost_v, float* cost_g);

/* Optimizer.optimize() for a batch — optimizer_GD.py:54-232 /
 * optimizer_BLS.py:57-213 (jit variants), one persistent launch.  alpha0 may
 * be NULL (start from initTrajectory on device).  Outputs nullable. */
int irm_optimize_batch(irm_ctx* ctx, const float* alpha0, const float* start, const float* goal,
                       const float* obstacles, int32_t n_obstacles, int32_t obstacle_stride,
                       int32_t batch, float* alpha_out, float* traj_out, irm_stats* stats_out,
                       float* series_out);

/* Same, device pointers, enqueue-only on `stream` (hipStream_t). */
int irm_optimize_batch_dev(irm_ctx* ctx, const irm_batch_dev* args, void* stream);

/* Workspace sizing for irm_optimize_batch_dev callers that pass series_out. */
int32_t irm_series_capacity(const irm_ctx* ctx);

/* The optimiser launch that irm_optimize_batch(_dev) runs for `batch` problems with n_obstacles
 * obstacles (record_series: series_out passed; the context's own irm_params.record_series counts
 * too, as in the launch).  Filled in by the launch dispatch itself with nothing launched, so it
 * names the kernel that actually runs (bench.py's flop model and kernel label come from here).
 * The plan assumes one obstacle table shared by the batch (obstacle_stride 0): per-problem tables
 * take more LDS per workgroup and may run fewer trajectories per workgroup.  ABI 3; no reference
 * counterpart. */
typedef struct irm_launch_plan {
    char kernel[128];           /* template instance, e.g. k_lean<FixShape<3,128,32>,512,1,FULL,GD1> */
    int32_t lean;               /* 1: k_lean, 0: k_optimize                                */
    int32_t flow;               /* 0 GD single loop, 1 GD dual loop, 2 BLS                 */
    int32_t waypoints_per_lane;
    int32_t threads;            /* per workgroup                                           */
    int32_t grid;               /* workgroups                                              */
    int32_t lds_bytes;          /* per workgroup                                           */
    int32_t traj_per_block;
    int32_t rank_z;             /* operator rank of the rounding-residual projection (0: V_R = I) */
    int32_t rank_dir;           /* ... of the waypoint direction F·y''                     */
    int32_t rank_g;             /* ... of the α-space gradient G = V_R·y'' (0: V_R = I, a copy) */
    float lam16;                /* λ_16/λ_0 of [K; dK]ᵀ[K; dK] as built (0: not in the operator) */
    float lam24;                /* λ_24/λ_0                                                */
} irm_launch_plan;
int irm_optimize_plan(const irm_ctx* ctx, int32_t batch, int32_t n_obstacles, int32_t record_series,
                      irm_launch_plan* out);

/* Build id of the library: the first 16 hex digits of the SHA-256 over every file of
 * irm_motion_planning_amd/csrc and include/irm.h, the compile flags of every unit and the build
 * variant (build.py source_hash); "unknown" otherwise.
 * __graft_entry__.smoke() compares it with the checked-out sources.  ABI 3. */
const char* irm_build_id(void);

/* Diagnostics: per-workgroup phase cycle counters of the last optimize
 * launch (24 uint64 per workgroup).  Only a library built with
 * -DIRM_PHASE_PROFILE records them; otherwise returns IRM_EINVAL.  Returns
 * the number of workgroups written. */
int irm_debug_phase_profile(irm_ctx* ctx, uint64_t* out, int32_t max_blocks);

/* Diagnostics: line-search log of problem 0 of every later BLS optimize on this
 * context — one record of 10 floats per trial, the values optimizer_BLS.py
 * computes at optimizer_BLS.py:139-149 (trial) and :163-166 (inner-loop head):
 * outer, inner, trial, lr, new_loss, required_loss, accepted, loss, ‖g‖,
 * alpha_norm.  cap records are kept (0 disables).  The record count of a run is
 * that problem's irm_stats.bls_trials (at most cap are stored). */
int irm_debug_bls_trace_enable(irm_ctx* ctx, int32_t cap);
/* Copy up to cap records of the last run's log; returns the number copied. */
int irm_debug_bls_trace(irm_ctx* ctx, float* out, int32_t cap);

#ifdef __cplusplus
}
#endif

#endif /* IRM_H_ */
