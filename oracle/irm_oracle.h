/*
 * irm_oracle.h — CPU restatement of the reference algorithm (TEST
 * INFRASTRUCTURE: only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it; the product never links it).
 *
 * Restates simongroeger/irm_motion_planning's α-space fp32 computation
 * (trajectory.py, robot.py, environment.py, optimizer_GD.py,
 * optimizer_BLS.py) in plain C with the reference's operation order.
 * Pinned against golden vectors produced by running the unmodified reference
 * (tests/golden/, oracle/tools/gen_golden.py) and the blog's published λ table.
 */
#ifndef IRM_ORACLE_H_
#define IRM_ORACLE_H_

#include <stdint.h>

#include "../include/irm.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_ctx orc_ctx;

orc_ctx* orc_create(const irm_params* p);
void orc_destroy(orc_ctx* c);

void orc_kernel_matrices(const orc_ctx* c, float* t, float* km, float* dkm, float* jac);
void orc_default_jac(int32_t D, float jgm, uint32_t seed, float* jac_out);

void orc_evaluate(const orc_ctx* c, const float* alpha, int32_t which, float* out);
void orc_fk(const orc_ctx* c, const float* traj, float* pos);
void orc_fk_joint(const orc_ctx* c, const float* traj, int32_t j, float* pos);
void orc_jacobian(const orc_ctx* c, const float* traj, float* jac);
void orc_compute_cost_vg(int32_t N, const float* f, const float* obstacles, int32_t O, float* cost_v,
                         float* cost_g);
float orc_cost(const orc_ctx* c, const float* alpha, const float* obstacles, int32_t O, const float* s,
               const float* g, float lsg, float ljl, float lmax);
void orc_cost_g(const orc_ctx* c, const float* alpha, const float* obstacles, int32_t O, const float* s,
                const float* g, float lsg, float ljl, float lmax, float* grad);
int32_t orc_constraints(const orc_ctx* c, const float* alpha, const float* s, const float* g, float* report);
void orc_init_alpha(const orc_ctx* c, const float* s, const float* g, float* alpha_out);

/* One optimize() (jit-loop semantics); series (nullable) receives
 * snapshots as the plain loop's extended-vis records them. */
void orc_optimize(const orc_ctx* c, const float* alpha0, const float* obstacles, int32_t O, const float* s,
                  const float* g, float* alpha_out, irm_stats* stats, float* series, int32_t max_series);

/* orc_optimize plus the BLS line-search log: ORC_TRACE_W floats per trial (outer, inner, trial, lr,
 * new_loss, required_loss, accepted, loss, ‖g‖, alpha_norm), at most trace_cap records; returns the
 * number of trials (may exceed trace_cap). */
#define ORC_TRACE_W 10
int32_t orc_trial_iterate(const orc_ctx* c, const float* alpha0, const float* obstacles, int32_t O, const float* s,
                          const float* g, int32_t row, float* out);
int32_t orc_optimize_trace(const orc_ctx* c, const float* alpha0, const float* obstacles, int32_t O, const float* s,
                           const float* g, float* alpha_out, irm_stats* stats, float* series, int32_t max_series,
                           float* trace, int32_t trace_cap);

/* Batch driver (OpenMP over trajectories; n_threads <= 0: all). */
void orc_optimize_batch(const orc_ctx* c, const float* alpha0, const float* start, const float* goal,
                        const float* obstacles, int32_t O, int32_t obstacle_stride, int32_t B,
                        float* alpha_out, irm_stats* stats, int32_t n_threads);

#ifdef __cplusplus
}
#endif
#endif
