/*
 * irm_oracle.c — plain-C fp32 restatement of the reference's α-space
 * optimiser.  TEST INFRASTRUCTURE ONLY (see irm_oracle.h).
 *
 * Every function follows the reference line it cites; arithmetic is fp32
 * (JAX x64 disabled), sequential in the order the reference expression is
 * written, compiled with -ffp-contract=off.  Matrix products are plain
 * left-to-right dot products (XLA:CPU uses Eigen; ordering differences are
 * the ~1e-4 waypoint noise SURVEY.md Appendix A.1 documents).
 */
#include "irm_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* A hyper-parameter the reference holds as a Python double (argparse) reaches this library as a
   float: recover the double the decimal argument denotes — the shortest decimal that round-trips the
   float (0.1f → "0.1" → 0.1) — so derived constants such as fp32(2·σ²) round as the reference's do
   (trajectory.py:14-19: 2*rbf_var**2 is a double, weakly typed to fp32 in the division). */
static double decimal_double(float f) {
    char buf[32];
    for (int prec = 6; prec <= 9; ++prec) {
        snprintf(buf, sizeof buf, "%.*g", prec, (double)f);
        if (strtof(buf, NULL) == f) return strtod(buf, NULL);
    }
    return (double)f;
}

struct orc_ctx {
    irm_params p;
    int N, D;
    float* t;   /* N     */
    float* c;   /* N: 6t^5-15t^4+10t^3 */
    float* K;   /* N×N   */
    float* dK;  /* N×N   */
    float J[IRM_MAX_JOINTS * IRM_MAX_JOINTS];
    float mean_pos, std_pos; /* trajectory.py:31-32 (fp32 of the Python doubles) */
};

/* ------------------------------------------------------------------ setup */

/* jnp.linspace(0,1,N) in fp32: t_i = 0*(1-i/div) + 1*(i/div), last = 1. */
static void linspace01(int N, float* t) {
    if (N == 1) { t[0] = 0.f; return; }
    float div = (float)(N - 1);
    for (int i = 0; i < N - 1; ++i) {
        float step = (float)i / div;
        t[i] = 0.f * (1.f - step) + 1.f * step;
    }
    t[N - 1] = 1.f;
}

orc_ctx* orc_create(const irm_params* p) {
    orc_ctx* c = (orc_ctx*)calloc(1, sizeof(orc_ctx));
    c->p = *p;
    int N = c->N = p->n_timesteps;
    c->D = p->n_joints;
    c->t = (float*)malloc(sizeof(float) * N);
    c->c = (float*)malloc(sizeof(float) * N);
    c->K = (float*)malloc(sizeof(float) * N * N);
    c->dK = (float*)malloc(sizeof(float) * N * N);
    linspace01(N, c->t); /* trajectory.py:35 */
    for (int i = 0; i < N; ++i) { /* trajectory.py:38: 6 t^5 - 15 t^4 + 10 t^3 */
        float t = c->t[i];
        float t3 = t * t * t, t4 = t3 * t, t5 = t4 * t;
        c->c[i] = 6.f * t5 - 15.f * t4 + 10.f * t3;
    }
    /* trajectory.py:14-19,40-48: a,b = meshgrid(t,t) -> a[i][j]=t_j, b[i][j]=t_i;
       K = exp(-(a-b)^2/(2σ^2)), dK = (a-b)/σ^2 * exp(...). σ enters as a
       Python double: 2*rbf_var**2 and rbf_var**2 are doubles cast to fp32. */
    double sig = decimal_double(p->rbf_variance);
    float two_s2 = (float)(2.0 * sig * sig), s2 = (float)(sig * sig);
    for (int i = 0; i < N; ++i)
        for (int j = 0; j < N; ++j) {
            float d = c->t[j] - c->t[i];
            float e = expf(-(d * d) / two_s2);
            c->K[i * N + j] = e;
            c->dK[i * N + j] = d / s2 * e;
        }
    memcpy(c->J, p->jac, sizeof(c->J));
    double mean = 0.5 * ((double)p->max_joint_position + (double)p->min_joint_position);
    c->mean_pos = (float)mean;
    c->std_pos = (float)(0.5 * ((double)p->max_joint_position - mean));
    return c;
}

void orc_destroy(orc_ctx* c) {
    if (!c) return;
    free(c->t); free(c->c); free(c->K); free(c->dK);
    free(c);
}

void orc_kernel_matrices(const orc_ctx* c, float* t, float* km, float* dkm, float* jac) {
    int N = c->N, D = c->D;
    if (t) memcpy(t, c->t, sizeof(float) * N);
    if (km) memcpy(km, c->K, sizeof(float) * N * N);
    if (dkm) memcpy(dkm, c->dK, sizeof(float) * N * N);
    if (jac)
        for (int i = 0; i < D; ++i)
            for (int j = 0; j < D; ++j) jac[i * D + j] = c->J[i * D + j];
}

/* ---- trajectory.py:42: J = I + jgm * jax.random.normal(PRNGKey(seed),(D,D)).
   Legacy threefry2x32 (jax/_src/prng.py, published algorithm). */
static uint32_t rotl32(uint32_t v, int r) { return (v << r) | (v >> (32 - r)); }

static void threefry2x32(uint32_t k0, uint32_t k1, uint32_t* x0, uint32_t* x1) {
    static const int rot[2][4] = {{13, 15, 26, 6}, {17, 29, 16, 24}};
    uint32_t ks[3] = {k0, k1, k0 ^ k1 ^ 0x1BD11BDAu};
    uint32_t a = *x0 + ks[0], b = *x1 + ks[1];
    static const int inj[5][2] = {{1, 2}, {2, 0}, {0, 1}, {1, 2}, {2, 0}};
    for (int i = 0; i < 5; ++i) {
        for (int r = 0; r < 4; ++r) {
            a += b;
            b = rotl32(b, rot[i % 2][r]);
            b ^= a;
        }
        a += ks[inj[i][0]];
        b += ks[inj[i][1]] + (uint32_t)(i + 1);
    }
    *x0 = a; *x1 = b;
}

static double erfinv_d(double y) {
    /* Newton on erf(x) - y from a Winitzki start; fp64 then rounded (the
       survey's adapter does the same: ≤1 ulp from JAX's fp32 erf_inv). */
    if (y <= -1.0) return -INFINITY;
    if (y >= 1.0) return INFINITY;
    double a = 0.147, ln = log(1.0 - y * y);
    double t1 = 2.0 / (M_PI * a) + ln / 2.0;
    double x = copysign(sqrt(sqrt(t1 * t1 - ln / a) - t1), y);
    for (int it = 0; it < 60; ++it) {
        double err = erf(x) - y;
        double step = err / (2.0 / sqrt(M_PI) * exp(-x * x));
        x -= step;
        if (fabs(step) < 1e-17 * (1.0 + fabs(x))) break;
    }
    return x;
}

void orc_default_jac(int32_t D, float jgm, uint32_t seed, float* jac_out) {
    int n = D * D, odd = n & 1, half = (n + odd) / 2;
    uint32_t* cnt = (uint32_t*)calloc((size_t)(2 * half), sizeof(uint32_t));
    for (int i = 0; i < n; ++i) cnt[i] = (uint32_t)i;
    uint32_t* bits = (uint32_t*)calloc((size_t)(2 * half), sizeof(uint32_t));
    for (int i = 0; i < half; ++i) {
        uint32_t x0 = cnt[i], x1 = cnt[half + i];
        threefry2x32(0u, seed, &x0, &x1);
        bits[i] = x0;
        bits[half + i] = x1;
    }
    float lo = nextafterf(-1.f, 0.f);
    for (int i = 0; i < n; ++i) {
        uint32_t fb = (bits[i] >> 9) | 0x3F800000u;
        float f;
        memcpy(&f, &fb, 4);
        f -= 1.f;
        float u = f * (1.f - lo) + lo;
        if (u < lo) u = lo;
        float z = (float)sqrt(2.0) * (float)erfinv_d((double)u);
        float eye = (i / D == i % D) ? 1.f : 0.f;
        jac_out[i] = eye + jgm * z;
    }
    free(cnt);
    free(bits);
}

/* ------------------------------------------------------------- evaluation */

/* C(m×n) = A(m×k) @ B(k×n) on fp32 operands; each dot product accumulates in
   fp64 and is rounded once to fp32.  The reference's contractions are XLA/BLAS
   blocked fp32 GEMMs whose summation order is unspecified; with the singular K
   (|α| ≈ 1e3 after initTrajectory, larger after the dual loop escalates λ) a
   plain sequential fp32 sum drifts by >1e-2 in waypoint space late in the dual
   loop and sends the chaotic BLS into another basin.
   The correctly-rounded product is order independent and matches the
   reference run with fp64 *or* BLAS evaluation (tests/golden c2 case). */
static void matmul(const float* A, const float* B, float* C, int m, int k, int n) {
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < n; ++j) {
            double s = 0.0;
            for (int l = 0; l < k; ++l) s += (double)A[i * k + l] * (double)B[l * n + j];
            C[i * n + j] = (float)s;
        }
}

/* trajectory.py:63-65: kernel_matrix @ alpha @ jac (left to right). */
static void evaluate_m(const orc_ctx* c, const float* M, const float* alpha, float* out) {
    int N = c->N, D = c->D;
    float tmp[IRM_MAX_TIMESTEPS * IRM_MAX_JOINTS];
    matmul(M, alpha, tmp, N, N, D);
    matmul(tmp, c->J, out, N, D, D);
}

void orc_evaluate(const orc_ctx* c, const float* alpha, int32_t which, float* out) {
    evaluate_m(c, which ? c->dK : c->K, alpha, out);
}

/* robot.py:29-36: c = cumsum(config, axis=1); pos = (L @ cos(c).T, L @ sin(c).T). */
void orc_fk(const orc_ctx* c, const float* traj, float* pos) {
    int N = c->N, D = c->D;
    for (int n = 0; n < N; ++n) {
        float cs = 0.f, px = 0.f, py = 0.f;
        for (int l = 0; l < D; ++l) {
            cs += traj[n * D + l];
            px += c->p.link_length[l] * cosf(cs);
            py += c->p.link_length[l] * sinf(cs);
        }
        pos[n] = px;
        pos[N + n] = py;
    }
}

/* robot.py:39-72 fk_joint_j (generalised to j = 1..D): FK of the first j links, i.e. the
   position of joint j (fk_joint_D = fk). */
void orc_fk_joint(const orc_ctx* c, const float* traj, int32_t j, float* pos) {
    int N = c->N, D = c->D;
    for (int n = 0; n < N; ++n) {
        float cs = 0.f, px = 0.f, py = 0.f;
        for (int l = 0; l < j; ++l) {
            cs += traj[n * D + l];
            px += c->p.link_length[l] * cosf(cs);
            py += c->p.link_length[l] * sinf(cs);
        }
        pos[n] = px;
        pos[N + n] = py;
    }
}

/* robot.py:75-87: x = -L*sin(c); rc_x = x + sum(x) - cumsum(x); y = L*cos(c). */
void orc_jacobian(const orc_ctx* c, const float* traj, float* jac) {
    int N = c->N, D = c->D;
    for (int n = 0; n < N; ++n) {
        float cs = 0.f, x[IRM_MAX_JOINTS], y[IRM_MAX_JOINTS], sx = 0.f, sy = 0.f;
        for (int l = 0; l < D; ++l) {
            cs += traj[n * D + l];
            x[l] = -(c->p.link_length[l] * sinf(cs));
            y[l] = c->p.link_length[l] * cosf(cs);
            sx += x[l];
            sy += y[l];
        }
        float cx = 0.f, cy = 0.f;
        for (int l = 0; l < D; ++l) {
            cx += x[l];
            cy += y[l];
            jac[(0 * N + n) * D + l] = (x[l] + sx) - cx;
            jac[(1 * N + n) * D + l] = (y[l] + sy) - cy;
        }
    }
}

/* environment.py:32-58: r2 = Σ_dim (f-o)^2; cost_v = Σ_o 0.8/(0.5+0.5 r2);
   cost_g = Σ_o (-0.8 (f-o)) / (0.5+0.5 r2)^2. */
void orc_compute_cost_vg(int32_t N, const float* f, const float* obstacles, int32_t O, float* cost_v,
                         float* cost_g) {
    for (int n = 0; n < N; ++n) {
        float cv = 0.f, gx = 0.f, gy = 0.f;
        for (int o = 0; o < O; ++o) {
            float dx = f[n] - obstacles[2 * o], dy = f[N + n] - obstacles[2 * o + 1];
            float r2 = dx * dx + dy * dy;
            float den = 0.5f + 0.5f * r2;
            cv += 0.8f / den;
            float den2 = den * den;
            gx += (-0.8f * dx) / den2;
            gy += (-0.8f * dy) / den2;
        }
        cost_v[n] = cv;
        if (cost_g) {
            cost_g[n] = gx;
            cost_g[N + n] = gy;
        }
    }
}

/* Per-waypoint obstacle potential.  End effector (the reference, trajectory.py:82,115):
   compute_cost(fk(traj)).  Whole robot (blog "Insights", DevBlog-Theme/blog-post.html:491-498):
   Σ_{j=1..D} compute_cost(fk_joint_j(traj)), summed in j order. */
static void point_costs(const orc_ctx* c, const float* traj, const float* obs, int O, float* cv) {
    int N = c->N;
    float f[2 * IRM_MAX_TIMESTEPS], cj[IRM_MAX_TIMESTEPS];
    if (!c->p.whole_robot_cost) {
        orc_fk(c, traj, f);
        orc_compute_cost_vg(N, f, obs, O, cv, NULL);
        return;
    }
    for (int j = 1; j <= c->D; ++j) {
        orc_fk_joint(c, traj, j, f);
        orc_compute_cost_vg(N, f, obs, O, j == 1 ? cv : cj, NULL);
        if (j > 1)
            for (int n = 0; n < N; ++n) cv[n] += cj[n];
    }
}

/* trajectory.py:81-88 (+113-117): obstacle cost of one trajectory. */
static float obstacle_cost(const orc_ctx* c, const float* traj, const float* obs, int O, float lmax) {
    int N = c->N;
    float cv[IRM_MAX_TIMESTEPS];
    point_costs(c, traj, obs, O, cv);
    float mx = cv[0], sum = 0.f;
    for (int n = 0; n < N; ++n) {
        if (cv[n] > mx) mx = cv[n];
        sum += cv[n];
    }
    float avg = sum / (float)N;
    return lmax * mx + (1.f - lmax) * avg;
}

/* Whole-robot gradient: trajectory.py:91-110 + 120-126 applied to every joint position, the
   Jacobian of fk_joint_j being robot.py:75-87's reverse cumsum over links 0..j-1 (zero for
   angles k >= j); the max/mean weights come from the summed per-waypoint cost. */
static void obstacle_cost_g_whole(const orc_ctx* c, const float* traj, const float* obs, int O, float lmax,
                                  float* grad) {
    int N = c->N, D = c->D;
    float f[2 * IRM_MAX_TIMESTEPS], cv[IRM_MAX_TIMESTEPS], cj[IRM_MAX_TIMESTEPS], cg[2 * IRM_MAX_TIMESTEPS];
    point_costs(c, traj, obs, O, cv);
    int idx = 0; /* jnp.argmax: first maximal index */
    for (int n = 1; n < N; ++n)
        if (cv[n] > cv[idx]) idx = n;
    float avg_w = (1.f - lmax) * (1.f / (float)N);
    for (int i = 0; i < N * D; ++i) grad[i] = 0.f;
    for (int j = 1; j <= D; ++j) {
        orc_fk_joint(c, traj, j, f);
        orc_compute_cost_vg(N, f, obs, O, cj, cg);
        for (int n = 0; n < N; ++n) {
            float w = lmax * (n == idx ? 1.f : 0.f) + avg_w;
            float wx = w * cg[n], wy = w * cg[N + n];
            float cs = 0.f, x[IRM_MAX_JOINTS], y[IRM_MAX_JOINTS], sx = 0.f, sy = 0.f;
            for (int l = 0; l < j; ++l) {
                cs += traj[n * D + l];
                x[l] = -(c->p.link_length[l] * sinf(cs));
                y[l] = c->p.link_length[l] * cosf(cs);
                sx += x[l];
                sy += y[l];
            }
            float cx = 0.f, cy = 0.f;
            for (int k = 0; k < j; ++k) {
                cx += x[k];
                cy += y[k];
                grad[n * D + k] += wx * ((x[k] + sx) - cx) + wy * ((y[k] + sy) - cy);
            }
        }
    }
}

/* trajectory.py:91-110 + 120-126: obstacle gradient w.r.t. waypoints. */
static void obstacle_cost_g(const orc_ctx* c, const float* traj, const float* obs, int O, float lmax,
                            float* grad) {
    int N = c->N, D = c->D;
    float f[2 * IRM_MAX_TIMESTEPS], cv[IRM_MAX_TIMESTEPS], cg[2 * IRM_MAX_TIMESTEPS];
    float jac[2 * IRM_MAX_TIMESTEPS * IRM_MAX_JOINTS];
    if (c->p.whole_robot_cost) {
        obstacle_cost_g_whole(c, traj, obs, O, lmax, grad);
        return;
    }
    orc_fk(c, traj, f);
    orc_compute_cost_vg(N, f, obs, O, cv, cg);
    int idx = 0; /* jnp.argmax: first maximal index */
    for (int n = 1; n < N; ++n)
        if (cv[n] > cv[idx]) idx = n;
    float avg_w = (1.f - lmax) * (1.f / (float)N);
    orc_jacobian(c, traj, jac);
    for (int n = 0; n < N; ++n) {
        float w = lmax * (n == idx ? 1.f : 0.f) + avg_w;
        float wx = w * cg[n], wy = w * cg[N + n];
        for (int k = 0; k < D; ++k) grad[n * D + k] = wx * jac[n * D + k] + wy * jac[(N + n) * D + k];
    }
}

/* trajectory.py:215-227 / 245-255: masked joint-limit penalties. */
static float jpl_cost(const orc_ctx* c, const float* traj) {
    int ND = c->N * c->D;
    float hi = (float)(c->p.joint_safety_limit * (double)c->p.max_joint_position);
    float lo = (float)(c->p.joint_safety_limit * (double)c->p.min_joint_position);
    float s = 0.f;
    for (int i = 0; i < ND; ++i) {
        float z = (traj[i] - c->mean_pos) / c->std_pos;
        float e = 0.5f * (z * z);
        if (c->p.constraint_violating_dependant_loss && !(traj[i] > hi || traj[i] < lo)) e = 0.f;
        s += e;
    }
    return s / (float)c->N;
}

static float jvl_cost(const orc_ctx* c, const float* vel) {
    int ND = c->N * c->D;
    float vmax = c->p.max_joint_velocity;
    float thr = (float)(c->p.joint_safety_limit * (double)c->p.max_joint_velocity);
    float s = 0.f;
    for (int i = 0; i < ND; ++i) {
        float z = vel[i] / vmax;
        float e = 0.5f * (z * z);
        if (c->p.constraint_violating_dependant_loss && !(fabsf(vel[i]) > thr)) e = 0.f;
        s += e;
    }
    return s / (float)c->N;
}

/* trajectory.py:271-281 */
static float cost_traj(const orc_ctx* c, const float* traj, const float* vel, const float* obs, int O,
                       const float* s, const float* g, float lsg, float ljl, float lmax) {
    int N = c->N, D = c->D;
    float toc = obstacle_cost(c, traj, obs, O, lmax);
    float a = 0.f, b = 0.f; /* trajectory.py:183-188 */
    for (int k = 0; k < D; ++k) {
        float d0 = traj[k] - s[k], d1 = traj[(N - 1) * D + k] - g[k];
        a += d0 * d0;
        b += d1 * d1;
    }
    float sgpc = 0.5f * a + 0.5f * b;
    a = b = 0.f; /* trajectory.py:201-204 */
    for (int k = 0; k < D; ++k) {
        a += vel[k] * vel[k];
        b += vel[(N - 1) * D + k] * vel[(N - 1) * D + k];
    }
    float sgvc = 0.5f * a + 0.5f * b;
    float jpc = jpl_cost(c, traj), jvc = jvl_cost(c, vel);
    return toc + lsg * (sgpc + sgvc) + ljl * (jpc + jvc);
}

float orc_cost(const orc_ctx* c, const float* alpha, const float* obstacles, int32_t O, const float* s,
               const float* g, float lsg, float ljl, float lmax) {
    float traj[IRM_MAX_TIMESTEPS * IRM_MAX_JOINTS], vel[IRM_MAX_TIMESTEPS * IRM_MAX_JOINTS];
    evaluate_m(c, c->K, alpha, traj);
    evaluate_m(c, c->dK, alpha, vel);
    return cost_traj(c, traj, vel, obstacles, O, s, g, lsg, ljl, lmax);
}

/* trajectory.py:284-297 */
void orc_cost_g(const orc_ctx* c, const float* alpha, const float* obstacles, int32_t O, const float* s,
                const float* g, float lsg, float ljl, float lmax, float* grad) {
    int N = c->N, D = c->D, ND = N * D;
    float traj[IRM_MAX_TIMESTEPS * IRM_MAX_JOINTS], vel[IRM_MAX_TIMESTEPS * IRM_MAX_JOINTS];
    float toc_g[IRM_MAX_TIMESTEPS * IRM_MAX_JOINTS], ta[IRM_MAX_TIMESTEPS * IRM_MAX_JOINTS],
        tb[IRM_MAX_TIMESTEPS * IRM_MAX_JOINTS], tmp[IRM_MAX_TIMESTEPS * IRM_MAX_JOINTS];
    evaluate_m(c, c->K, alpha, traj);
    evaluate_m(c, c->dK, alpha, vel);
    obstacle_cost_g(c, traj, obstacles, O, lmax, toc_g);
    float hi = (float)(c->p.joint_safety_limit * (double)c->p.max_joint_position);
    float lo = (float)(c->p.joint_safety_limit * (double)c->p.min_joint_position);
    float thr = (float)(c->p.joint_safety_limit * (double)c->p.max_joint_velocity);
    float std2 = c->std_pos * c->std_pos;
    float vmax2 = c->p.max_joint_velocity * c->p.max_joint_velocity;
    for (int i = 0; i < ND; ++i) {
        int n = i / D, k = i % D;
        /* start_goal_cost_g / start_goal_velocity_cost_g, trajectory.py:191-212 */
        float sgp = 0.f, sgv = 0.f;
        if (n == 0) { sgp = traj[i] - s[k]; sgv = vel[i]; }
        if (n == N - 1) { sgp = traj[i] - g[k]; sgv = vel[i]; }
        /* joint_position_limit_cost_g, trajectory.py:231-242 */
        float jp = (traj[i] - c->mean_pos) / std2;
        if (c->p.constraint_violating_dependant_loss && !(traj[i] > hi || traj[i] < lo)) jp = 0.f;
        jp = jp / (float)N;
        /* joint_velocity_limit_cost_g, trajectory.py:259-268 */
        float jv = vel[i] / vmax2;
        if (c->p.constraint_violating_dependant_loss && !(fabsf(vel[i]) > thr)) jv = 0.f;
        jv = jv / (float)N;
        ta[i] = toc_g[i] + lsg * sgp + ljl * jp;
        tb[i] = lsg * sgv + ljl * jv;
    }
    /* (K^T @ ta + dK^T @ tb) @ J^T */
    for (int n = 0; n < N; ++n)
        for (int k = 0; k < D; ++k) {
            double u = 0.0, v = 0.0; /* fp64 accumulation, rounded once (see matmul) */
            for (int m = 0; m < N; ++m) u += (double)c->K[m * N + n] * (double)ta[m * D + k];
            for (int m = 0; m < N; ++m) v += (double)c->dK[m * N + n] * (double)tb[m * D + k];
            tmp[n * D + k] = (float)u + (float)v;
        }
    for (int n = 0; n < N; ++n)
        for (int k = 0; k < D; ++k) {
            float u = 0.f;
            for (int l = 0; l < D; ++l) u += tmp[n * D + l] * c->J[k * D + l];
            grad[n * D + k] = u;
        }
}

static float norm_row(const float* x, const float* y, int D) {
    float s = 0.f;
    for (int k = 0; k < D; ++k) {
        float d = y ? x[k] - y[k] : x[k];
        s += d * d;
    }
    return sqrtf(s);
}

/* trajectory.py:129-180 with robot.py:90-113. report: 7 values + 4 flags. */
static int32_t constraints_traj(const orc_ctx* c, const float* traj, const float* vel, const float* s,
                                const float* g, float* report) {
    int N = c->N, D = c->D, ND = N * D;
    float ds = norm_row(traj, s, D), dg = norm_row(traj + (N - 1) * D, g, D);
    float vs = norm_row(vel, NULL, D), vg = norm_row(vel + (N - 1) * D, NULL, D);
    float mx = traj[0], mn = traj[0], va = fabsf(vel[0]);
    for (int i = 1; i < ND; ++i) {
        if (traj[i] > mx) mx = traj[i];
        if (traj[i] < mn) mn = traj[i];
        if (fabsf(vel[i]) > va) va = fabsf(vel[i]);
    }
    int f0 = ds < c->p.eps_position && dg < c->p.eps_position;
    int f1 = vs < c->p.eps_velocity && vg < c->p.eps_velocity;
    int f2 = mx <= c->p.max_joint_position && mn >= c->p.min_joint_position;
    int f3 = va <= c->p.max_joint_velocity;
    if (report) {
        float r[11] = {ds, dg, vs, vg, mx, mn, va, (float)f0, (float)f1, (float)f2, (float)f3};
        memcpy(report, r, sizeof(r));
    }
    return f0 && f1 && f2 && f3;
}

int32_t orc_constraints(const orc_ctx* c, const float* alpha, const float* s, const float* g, float* report) {
    float traj[IRM_MAX_TIMESTEPS * IRM_MAX_JOINTS], vel[IRM_MAX_TIMESTEPS * IRM_MAX_JOINTS];
    evaluate_m(c, c->K, alpha, traj);
    evaluate_m(c, c->dK, alpha, vel);
    return constraints_traj(c, traj, vel, s, g, report);
}

/* fp32 LU with partial pivoting in LAPACK's recursive order (sgetrf2: factor the left half of the
   columns, swap, triangular solve, Schur update, factor the right half) followed by sgetrs's
   substitutions.  numpy.linalg.solve — what trajectory.py:77 runs — is LAPACK sgesv; K is
   numerically singular (cond ≈ 1e19), so α0's null-space part is rounding noise whose size depends
   on the elimination order: the recursive order keeps |α0| at the reference's ~1e3 where the
   right-looking textbook loop reached 4e4 (N=50), with K·α0·J within 3e-4 of the reference's. */
static void getrf2_f32(int m, int n, float* A, int lda, int* ipiv) {
    if (n == 1) {
        int p = 0;
        for (int i = 1; i < m; ++i)
            if (fabsf(A[(size_t)i * lda]) > fabsf(A[(size_t)p * lda])) p = i;
        ipiv[0] = p;
        if (p != 0) {
            float t = A[0];
            A[0] = A[(size_t)p * lda];
            A[(size_t)p * lda] = t;
        }
        if (A[0] != 0.f) {
            const float r = 1.f / A[0]; /* LAPACK scales by the reciprocal */
            for (int i = 1; i < m; ++i) A[(size_t)i * lda] *= r;
        }
        return;
    }
    const int n1 = (m < n ? m : n) / 2, n2 = n - n1;
    getrf2_f32(m, n1, A, lda, ipiv);
    for (int i = 0; i < n1; ++i) /* row swaps of the left panel on the right columns */
        if (ipiv[i] != i)
            for (int j = n1; j < n; ++j) {
                float t = A[(size_t)i * lda + j];
                A[(size_t)i * lda + j] = A[(size_t)ipiv[i] * lda + j];
                A[(size_t)ipiv[i] * lda + j] = t;
            }
    for (int i = 1; i < n1; ++i) /* A12 = L11⁻¹·A12 (unit lower) */
        for (int k = 0; k < i; ++k) {
            const float l = A[(size_t)i * lda + k];
            for (int j = n1; j < n; ++j) A[(size_t)i * lda + j] -= l * A[(size_t)k * lda + j];
        }
    for (int i = n1; i < m; ++i) /* A22 −= A21·A12 */
        for (int j = n1; j < n; ++j) {
            float s = 0.f;
            for (int k = 0; k < n1; ++k) s += A[(size_t)i * lda + k] * A[(size_t)k * lda + j];
            A[(size_t)i * lda + j] -= s;
        }
    getrf2_f32(m - n1, n2, A + (size_t)n1 * lda + n1, lda, ipiv + n1);
    for (int i = n1; i < (m < n ? m : n); ++i) {
        ipiv[i] += n1;
        if (ipiv[i] != i) /* the right factorisation's swaps on the left columns */
            for (int j = 0; j < n1; ++j) {
                float t = A[(size_t)i * lda + j];
                A[(size_t)i * lda + j] = A[(size_t)ipiv[i] * lda + j];
                A[(size_t)ipiv[i] * lda + j] = t;
            }
    }
}

/* A·X = B, A n×n, B / X n×nrhs, row-major; returns 0 if a pivot is exactly 0. */
static int lu_solve_f32(int n, const float* A_in, const float* B_in, int nrhs, float* X) {
    float* A = (float*)malloc(sizeof(float) * (size_t)n * n);
    int* ipiv = (int*)malloc(sizeof(int) * (size_t)n);
    int ok = 1;
    memcpy(A, A_in, sizeof(float) * (size_t)n * n);
    memcpy(X, B_in, sizeof(float) * (size_t)n * nrhs);
    getrf2_f32(n, n, A, n, ipiv);
    for (int i = 0; i < n; ++i) {
        if (A[(size_t)i * n + i] == 0.f) ok = 0;
        if (ipiv[i] != i)
            for (int j = 0; j < nrhs; ++j) {
                float t = X[(size_t)i * nrhs + j];
                X[(size_t)i * nrhs + j] = X[(size_t)ipiv[i] * nrhs + j];
                X[(size_t)ipiv[i] * nrhs + j] = t;
            }
    }
    if (ok) {
        for (int j = 0; j < nrhs; ++j) {
            for (int i = 1; i < n; ++i) {
                float s = X[(size_t)i * nrhs + j];
                for (int k = 0; k < i; ++k) s -= A[(size_t)i * n + k] * X[(size_t)k * nrhs + j];
                X[(size_t)i * nrhs + j] = s;
            }
            for (int i = n - 1; i >= 0; --i) {
                float s = X[(size_t)i * nrhs + j];
                for (int k = i + 1; k < n; ++k) s -= A[(size_t)i * n + k] * X[(size_t)k * nrhs + j];
                X[(size_t)i * nrhs + j] = s / A[(size_t)i * n + i];
            }
        }
    }
    free(A);
    free(ipiv);
    return ok;
}

/* trajectory.py:73-78: α0 = solve(K, (s + (g-s) c) @ inv(J)). */
void orc_init_alpha(const orc_ctx* c, const float* s, const float* g, float* alpha_out) {
    int N = c->N, D = c->D;
    float eye[IRM_MAX_JOINTS * IRM_MAX_JOINTS], Jinv[IRM_MAX_JOINTS * IRM_MAX_JOINTS];
    for (int i = 0; i < D * D; ++i) eye[i] = (i / D == i % D) ? 1.f : 0.f;
    float Jl[IRM_MAX_JOINTS * IRM_MAX_JOINTS];
    for (int i = 0; i < D; ++i)
        for (int j = 0; j < D; ++j) Jl[i * D + j] = c->J[i * D + j];
    lu_solve_f32(D, Jl, eye, D, Jinv);
    float* line = (float*)malloc(sizeof(float) * N * D);
    float* rhs = (float*)malloc(sizeof(float) * N * D);
    for (int n = 0; n < N; ++n)
        for (int k = 0; k < D; ++k) line[n * D + k] = s[k] + (g[k] - s[k]) * c->c[n];
    matmul(line, Jinv, rhs, N, D, D);
    lu_solve_f32(N, c->K, rhs, D, alpha_out);
    free(line);
    free(rhs);
}

/* ------------------------------------------------------------- optimisers */

static void snapshot(const orc_ctx* c, const float* alpha, float* series, int32_t max_series, int32_t* len) {
    if (!series || *len >= max_series) return;
    evaluate_m(c, c->K, alpha, series + (size_t)(*len) * c->N * c->D);
    (*len)++;
}

/* optimizer_GD.py:173-232 (jit_dual_optimize); with max_outer_iteration == 1
   it reduces to jit_optimize (optimizer_GD.py:68-97). */
static void optimize_gd(const orc_ctx* c, float* alpha, const float* obs, int O, const float* s,
                        const float* g, irm_stats* st, float* series, int32_t max_series) {
    const irm_params* p = &c->p;
    int ND = c->N * c->D;
    float lsg = p->lambda_sg_constraint, ljl = p->lambda_jl_constraint;
    float grad[IRM_MAX_TIMESTEPS * IRM_MAX_JOINTS], na[IRM_MAX_TIMESTEPS * IRM_MAX_JOINTS];
    int fulfilled = 0, outer = 0;
    /* dualOptimization = max_outer_iteration > 1 (optimizer_GD.py:18); otherwise the single loop
       (:54-65) runs once, whatever max_outer_iteration is */
    const int max_outer = p->max_outer_iteration > 1 ? p->max_outer_iteration : 1;
    while (outer < max_outer && !fulfilled) {
        float lr = p->gd_lr[outer];
        float last = orc_cost(c, alpha, obs, O, s, g, lsg, ljl, p->lambda_max_cost); /* :93 / :210 */
        st->cost_evals++;
        int it = 0, minimized = 0;
        while (it < p->max_inner_iteration && !minimized) { /* :76-91 / :180-195 */
            orc_cost_g(c, alpha, obs, O, s, g, lsg, ljl, p->lambda_max_cost, grad);
            st->grad_evals++;
            float cf = 1.f - p->lambda_reg * lr;
            for (int i = 0; i < ND; ++i) na[i] = cf * alpha[i] - lr * grad[i];
            float nl = orc_cost(c, na, obs, O, s, g, lsg, ljl, p->lambda_max_cost);
            st->cost_evals++;
            if (last - nl < p->loop_loss_reduction) {
                minimized = 1;
            } else {
                it++;
                memcpy(alpha, na, sizeof(float) * ND);
                last = nl;
                st->inner_iterations++;
                snapshot(c, alpha, series, max_series, &st->series_len); /* optimizer_GD.py:153-154 */
            }
        }
        fulfilled = orc_constraints(c, alpha, s, g, NULL); /* :214 */
        st->outer_iterations++;
        if (!fulfilled) {
            outer++;
            lsg *= p->lambda_constraint_increase;
            ljl *= p->lambda_constraint_increase;
        }
        st->final_loss = last;
    }
    st->constraints_ok = fulfilled;
}

/* optimizer_BLS.py:126-213 (jit_optimize). */
/* Line-search log (tests): per trial ORC_TRACE_W floats — outer, inner, trial, lr, new_loss,
   required_loss, accepted, loss, ‖g‖, alpha_norm (optimizer_BLS.py:139-149, 163-166). */
typedef struct {
    float* buf;
    int32_t cap, n;
    int32_t snap_row; /* orc_trial_iterate: the trial iterate of log row snap_row goes to snap */
    float* snap;
} bls_trace;

static void trace_put(bls_trace* tr, int outer, int inner, int trial, float lr, float nl, float req, int acc,
                      float loss, float gn, float an) {
    if (!tr || !tr->buf || tr->n >= tr->cap) {
        if (tr) tr->n++;
        return;
    }
    float* r = tr->buf + (size_t)tr->n * ORC_TRACE_W;
    r[0] = (float)outer; r[1] = (float)inner; r[2] = (float)trial; r[3] = lr; r[4] = nl; r[5] = req;
    r[6] = (float)acc; r[7] = loss; r[8] = gn; r[9] = an;
    tr->n++;
}

static void optimize_bls(const orc_ctx* c, float* alpha, const float* obs, int O, const float* s,
                         const float* g, irm_stats* st, float* series, int32_t max_series, bls_trace* trc) {
    const irm_params* p = &c->p;
    int N = c->N, D = c->D, ND = N * D;
    float lsg = p->lambda_sg_constraint, ljl = p->lambda_jl_constraint;
    float grad[IRM_MAX_TIMESTEPS * IRM_MAX_JOINTS], ng[IRM_MAX_TIMESTEPS * IRM_MAX_JOINTS],
        na[IRM_MAX_TIMESTEPS * IRM_MAX_JOINTS];
    int fulfilled = 0, outer = 0;
    while (outer < p->max_outer_iteration && !fulfilled) {
        float lr = p->bls_lr_start; /* :193 */
        int it = 0, minimized = 0;
        float loss = 0.f;
        while (it < p->max_inner_iteration && !minimized) { /* :159-179 */
            loss = orc_cost(c, alpha, obs, O, s, g, lsg, ljl, p->lambda_max_cost);
            st->cost_evals++;
            orc_cost_g(c, alpha, obs, O, s, g, lsg, ljl, p->lambda_max_cost, grad);
            st->grad_evals++;
            float nrm = 0.f;
            for (int i = 0; i < ND; ++i) nrm += grad[i] * grad[i];
            nrm = sqrtf(nrm);
            for (int i = 0; i < ND; ++i) ng[i] = grad[i] / nrm;
            /* alpha_norm = sum(grad^T @ n_grad) over all D×D entries (:166) */
            float anorm = 0.f;
            for (int a = 0; a < D; ++a)
                for (int b = 0; b < D; ++b) {
                    float e = 0.f;
                    for (int n = 0; n < N; ++n) e += grad[n * D + a] * ng[n * D + b];
                    anorm += e;
                }
            float new_loss = loss;
            for (int j = 0; j < p->max_bls_iteration; ++j) { /* :131-150 */
                float cf = 1.f - p->lambda_reg * lr;
                for (int i = 0; i < ND; ++i) na[i] = cf * alpha[i] - lr * ng[i];
                float nl = orc_cost(c, na, obs, O, s, g, lsg, ljl, p->lambda_max_cost);
                st->cost_evals++;
                st->bls_trials++;
                float required = loss - p->bls_alpha * lr * anorm;
                if (trc && trc->snap && trc->n == trc->snap_row) memcpy(trc->snap, na, sizeof(float) * ND);
                trace_put(trc, outer, it, j, lr, nl, required, !(nl > required), loss, nrm, anorm);
                if (nl > required) {
                    lr = lr * p->bls_beta_minus;
                } else {
                    memcpy(alpha, na, sizeof(float) * ND);
                    lr = lr * p->bls_beta_plus;
                    new_loss = nl;
                    break;
                }
            }
            if (loss - new_loss < p->loop_loss_reduction) { /* :178 */
                minimized = 1;
                loss = new_loss;
            } else {
                it++;
                st->inner_iterations++;
                loss = new_loss;
                snapshot(c, alpha, series, max_series, &st->series_len); /* optimizer_BLS.py:106-107 */
            }
        }
        fulfilled = orc_constraints(c, alpha, s, g, NULL); /* :196 */
        st->outer_iterations++;
        st->final_loss = loss;
        if (!fulfilled) {
            outer++;
            lsg *= p->lambda_constraint_increase;
            ljl *= p->lambda_constraint_increase;
        }
    }
    /* max_outer_iteration <= 0: the outer while_loop never runs and α0 is returned (:184-186, 210-213);
       the flag reported is constraintsFulfilled(α0), as main.py:143 would print it */
    if (p->max_outer_iteration <= 0) {
        fulfilled = orc_constraints(c, alpha, s, g, NULL);
        st->final_loss = orc_cost(c, alpha, obs, O, s, g, lsg, ljl, p->lambda_max_cost);
    }
    st->constraints_ok = fulfilled;
}

int32_t orc_optimize_trace(const orc_ctx* c, const float* alpha0, const float* obstacles, int32_t O, const float* s,
                           const float* g, float* alpha_out, irm_stats* stats, float* series, int32_t max_series,
                           float* trace, int32_t trace_cap) {
    irm_stats st;
    memset(&st, 0, sizeof(st));
    bls_trace tr = {trace, trace_cap, 0, -1, NULL};
    memcpy(alpha_out, alpha0, sizeof(float) * c->N * c->D);
    snapshot(c, alpha_out, series, max_series, &st.series_len); /* row 0 = initial trajectory */
    if (c->p.optimizer == IRM_OPT_BLS)
        optimize_bls(c, alpha_out, obstacles, O, s, g, &st, series, max_series, &tr);
    else
        optimize_gd(c, alpha_out, obstacles, O, s, g, &st, series, max_series);
    if (stats) *stats = st;
    return tr.n;
}

/* Test diagnostics: the fp32 trial iterate α_j = (1 − λ_reg·lr)·α − lr·ĝ of line-search log row `row`
   (optimizer_BLS.py:139) of a BLS run from alpha0 — e.g. to find the loss's penalty-mask thresholds
   (trajectory.py:221-222, 251) near a trial whose accept / reject two runs decide differently.
   Returns 1 if the run reached that row. */
int32_t orc_trial_iterate(const orc_ctx* c, const float* alpha0, const float* obstacles, int32_t O, const float* s,
                          const float* g, int32_t row, float* out) {
    irm_stats st;
    memset(&st, 0, sizeof(st));
    float a[IRM_MAX_TIMESTEPS * IRM_MAX_JOINTS];
    bls_trace tr = {NULL, 0, 0, row, out};
    memcpy(a, alpha0, sizeof(float) * c->N * c->D);
    if (c->p.optimizer != IRM_OPT_BLS) return 0;
    optimize_bls(c, a, obstacles, O, s, g, &st, NULL, 0, &tr);
    return tr.n > row ? 1 : 0;
}

void orc_optimize(const orc_ctx* c, const float* alpha0, const float* obstacles, int32_t O, const float* s,
                  const float* g, float* alpha_out, irm_stats* stats, float* series, int32_t max_series) {
    (void)orc_optimize_trace(c, alpha0, obstacles, O, s, g, alpha_out, stats, series, max_series, NULL, 0);
}

void orc_optimize_batch(const orc_ctx* c, const float* alpha0, const float* start, const float* goal,
                        const float* obstacles, int32_t O, int32_t obstacle_stride, int32_t B,
                        float* alpha_out, irm_stats* stats, int32_t n_threads) {
    int ND = c->N * c->D, D = c->D;
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
    for (int b = 0; b < B; ++b) {
        float a0[IRM_MAX_TIMESTEPS * IRM_MAX_JOINTS];
        if (alpha0)
            memcpy(a0, alpha0 + (size_t)b * ND, sizeof(float) * ND);
        else
            orc_init_alpha(c, start + b * D, goal + b * D, a0);
        orc_optimize(c, a0, obstacles + (size_t)b * obstacle_stride, O, start + b * D, goal + b * D,
                     alpha_out + (size_t)b * ND, stats ? stats + b : NULL, NULL, 0);
    }
    (void)n_threads;
}
