// irm_host.cpp — C ABI (include/irm.h) of the MI355X trajectory optimiser.
//
// Context creation builds, once per configuration, everything
// Trajectory.__init__ builds (trajectory.py:23-42) plus the device-side
// operators of the trajectory-space formulation:
//   L = [K; dK]                (2N × N, fp32 exactly as the reference)
//   F = L·V_R                  (V_R: top-R eigenvectors of LᵀL, fp64 Jacobi)
// packed into the 16x16x4 MFMA A-fragment layout and uploaded to HBM.
// All per-call numerics run in irm_kernels.hip; there is no CPU fallback.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/irm.h"
#include "irm_kernels.hpp"

using irm::KParams;

namespace {
/* A hyper-parameter the reference holds as a Python double (argparse) reaches this library as a
   float: recover the double the decimal argument denotes — the shortest decimal that round-trips the
   float (0.1f → "0.1" → 0.1) — so derived constants such as fp32(2·σ²) round as the reference's do
   (trajectory.py:14-19: 2*rbf_var**2 is a double, weakly typed to fp32 in the division). */
double decimal_double(float f) {
    char buf[32];
    for (int prec = 6; prec <= 9; ++prec) {
        snprintf(buf, sizeof buf, "%.*g", prec, (double)f);
        if (strtof(buf, nullptr) == f) return strtod(buf, nullptr);
    }
    return (double)f;
}

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                          \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess) return fail(IRM_EKERNEL, "%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

// ------------------------------------------------------------- host linalg
// Cyclic Jacobi eigen-decomposition of a symmetric n×n matrix (fp64).
// On return a's diagonal holds the eigenvalues and v the eigenvectors (columns).
// The rotations work on copies with a padded row stride (a power-of-two stride put every element of a
// column rotation into one cache set) and accumulate the eigenvectors as rows (vᵀ: each rotation updates
// two contiguous rows): the same operations in the same order as the plain n-stride form, so the result
// is bit-identical, 4.6× faster at n = 512 (108 → 23 s on one core; the context of an N = 512 trajectory).
void jacobi_eigen(std::vector<double>& a_io, int n, std::vector<double>& v_out) {
    const int ld = n + 8;
    std::vector<double> a((size_t)n * ld), vt((size_t)n * ld, 0.0);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) a[(size_t)i * ld + j] = a_io[(size_t)i * n + j];
    for (int i = 0; i < n; ++i) vt[(size_t)i * ld + i] = 1.0;
    double fro = 0.0;
    for (double x : a_io) fro += x * x;
    fro = sqrt(fro);
    for (int sweep = 0; sweep < 64; ++sweep) {
        double off = 0.0;
        for (int p = 0; p < n; ++p)
            for (int q = p + 1; q < n; ++q) off += a[(size_t)p * ld + q] * a[(size_t)p * ld + q];
        if (sqrt(off) <= 1e-17 * fro) break;
        for (int p = 0; p < n; ++p) {
            for (int q = p + 1; q < n; ++q) {
                double apq = a[(size_t)p * ld + q];
                if (fabs(apq) <= 1e-300) continue;
                double app = a[(size_t)p * ld + p], aqq = a[(size_t)q * ld + q];
                double theta = (aqq - app) / (2.0 * apq);
                double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
                for (int k = 0; k < n; ++k) {  // rotate columns p, q
                    double akp = a[(size_t)k * ld + p], akq = a[(size_t)k * ld + q];
                    a[(size_t)k * ld + p] = c * akp - s * akq;
                    a[(size_t)k * ld + q] = s * akp + c * akq;
                }
                double* ap = &a[(size_t)p * ld];
                double* aq = &a[(size_t)q * ld];
                for (int k = 0; k < n; ++k) {  // rotate rows p, q
                    double apk = ap[k], aqk = aq[k];
                    ap[k] = c * apk - s * aqk;
                    aq[k] = s * apk + c * aqk;
                }
                double* vp = &vt[(size_t)p * ld];
                double* vq = &vt[(size_t)q * ld];
                for (int k = 0; k < n; ++k) {  // eigenvector columns p, q (rows of vᵀ)
                    double vkp = vp[k], vkq = vq[k];
                    vp[k] = c * vkp - s * vkq;
                    vq[k] = s * vkp + c * vkq;
                }
            }
        }
    }
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) a_io[(size_t)i * n + j] = a[(size_t)i * ld + j];
    v_out.assign((size_t)n * n, 0.0);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) v_out[(size_t)i * n + j] = vt[(size_t)j * ld + i];
}

// Eigen-decompositions of the operator Gram matrices already computed in this process, keyed by the
// matrix itself (a context of the same N, σ and time grid reuses it: N = 512 takes ≈ 20 s to factorise).
struct EigenMemo {
    int n;
    std::vector<double> g, a, v;  // input, decomposed a (eigenvalues on the diagonal), eigenvectors
};
std::mutex g_eigen_mu;
std::vector<EigenMemo> g_eigen_memo;

void jacobi_eigen_memo(std::vector<double>& a, int n, std::vector<double>& v) {
    {
        std::lock_guard<std::mutex> lk(g_eigen_mu);
        for (const EigenMemo& m : g_eigen_memo)
            if (m.n == n && m.g == a) {
                a = m.a;
                v = m.v;
                return;
            }
    }
    EigenMemo m{n, a, {}, {}};
    jacobi_eigen(a, n, v);
    m.a = a;
    m.v = v;
    std::lock_guard<std::mutex> lk(g_eigen_mu);
    if (g_eigen_memo.size() >= 8) g_eigen_memo.erase(g_eigen_memo.begin());
    g_eigen_memo.push_back(std::move(m));
}

/* fp32 LU with partial pivoting in LAPACK's recursive order (sgetrf2: factor the left half of the
   columns, swap, triangular solve, Schur update, factor the right half) followed by sgetrs's
   substitutions.  numpy.linalg.solve — what trajectory.py:77 runs — is LAPACK sgesv; K is
   numerically singular (cond ≈ 1e19), so α0's null-space part is rounding noise whose size depends
   on the elimination order: the recursive order keeps |α0| at the reference's ~1e3 where the
   right-looking textbook loop reached 4e4 (N=50), with K·α0·J within 3e-4 of the reference's. */
void getrf2_f32(int m, int n, float* A, int lda, int* ipiv) {
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

/* A·X = B, A n×n, B / X n×nrhs, row-major; returns false if a pivot is exactly 0. */
bool lu_solve_f32(int n, const float* A_in, const float* B_in, int nrhs, float* X) {
    float* A = (float*)malloc(sizeof(float) * (size_t)n * n);
    int* ipiv = (int*)malloc(sizeof(int) * (size_t)n);
    bool ok = true;
    memcpy(A, A_in, sizeof(float) * (size_t)n * n);
    memcpy(X, B_in, sizeof(float) * (size_t)n * nrhs);
    getrf2_f32(n, n, A, n, ipiv);
    for (int i = 0; i < n; ++i) {
        if (A[(size_t)i * n + i] == 0.f) ok = false;
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

// ------------------------------------------------ legacy threefry (J)
uint32_t rotl32(uint32_t v, int r) { return (v << r) | (v >> (32 - r)); }

void threefry2x32(uint32_t k0, uint32_t k1, uint32_t& x0, uint32_t& x1) {
    static const int rot[2][4] = {{13, 15, 26, 6}, {17, 29, 16, 24}};
    static const int inj[5][2] = {{1, 2}, {2, 0}, {0, 1}, {1, 2}, {2, 0}};
    const uint32_t ks[3] = {k0, k1, k0 ^ k1 ^ 0x1BD11BDAu};
    uint32_t a = x0 + ks[0], b = x1 + ks[1];
    for (int i = 0; i < 5; ++i) {
        for (int r = 0; r < 4; ++r) {
            a += b;
            b = rotl32(b, rot[i % 2][r]);
            b ^= a;
        }
        a += ks[inj[i][0]];
        b += ks[inj[i][1]] + (uint32_t)(i + 1);
    }
    x0 = a;
    x1 = b;
}

double erfinv_f64(double y) {
    if (y <= -1.0) return -INFINITY;
    if (y >= 1.0) return INFINITY;
    const double a = 0.147, ln = log(1.0 - y * y);
    const double t1 = 2.0 / (M_PI * a) + ln / 2.0;
    double x = copysign(sqrt(sqrt(t1 * t1 - ln / a) - t1), y);
    for (int it = 0; it < 60; ++it) {  // Newton on erf(x) = y
        const double step = (erf(x) - y) / (2.0 / sqrt(M_PI) * exp(-x * x));
        x -= step;
        if (fabs(step) < 1e-17 * (1.0 + fabs(x))) break;
    }
    return x;
}

void fill_frag(std::vector<float>& out, int M, int K, const std::vector<double>& A /*row-major M×K*/,
               bool kperm = false) {
    out.assign((size_t)irm::frag_floats(M, K), 0.f);
    for (int r = 0; r < M; ++r)
        for (int k = 0; k < K; ++k)
            out[(size_t)(kperm ? irm::frag_index_kp(r, k, K) : irm::frag_index(r, k, K))] = (float)A[(size_t)r * K + k];
}

int round_up(int x, int m) { return (x + m - 1) / m * m; }

}  // namespace

// ================================================================ context
struct irm_ctx {
    irm_params p{};
    int N = 0, D = 0, R = 0, NK = 0, MP = 0, RP = 0;
    float trunc = 0.f;
    // λ_16/λ_0, λ_24/λ_0 of the operator actually built (0 where the component is not in it): the
    // lean kernel's per-stage rank cuts (direction / residual at rank 16, G at rank 24) are exact to
    // fp32 only while these are at fp32 noise, so they gate it (lean_rank_cut_ok)
    float lam16 = 0.f, lam24 = 0.f;
    std::vector<float> t, cvec, K, dK, J;
    KParams kp{};
    // device
    float *d_K = nullptr, *d_dK = nullptr, *d_Kt = nullptr, *d_dKt = nullptr, *d_F1 = nullptr, *d_F2 = nullptr,
          *d_F1p = nullptr, *d_F2p = nullptr, *d_Fbot = nullptr, *d_Vr = nullptr, *d_H = nullptr, *d_u = nullptr, *d_w = nullptr,
          *d_VTp = nullptr, *d_VNp = nullptr, *d_HV = nullptr, *d_VTs = nullptr, *d_VNs = nullptr;
    // host-API staging
    void* d_io = nullptr;
    size_t io_bytes = 0;
    hipStream_t stream = nullptr;
    int num_cus = 0;
    char name[64] = {0}, arch[32] = {0};
    int tb_opt = 1, ops_lds = 0, lds_opt = 0;
    int max_series = 0;
    unsigned long long* d_prof = nullptr;  // IRM_PHASE_PROFILE builds only
    int prof_blocks = 0, prof_cap = 0;
    float* d_trace = nullptr;  // BLS line-search log of problem 0 (irm_debug_bls_trace)
    int trace_cap = 0;
};

namespace {

// Thresholds of the lean kernel's rank cuts on λ_r/λ_0 (see irm_ctx_create): the direction keeps its
// terms to ≤ 1e-6 relative (fp32 rounding of the direction itself is 6e-8), G to σ_24/σ_0 ≤ 1e-7.
constexpr float kLam16Max = 1e-6f, kLam24Max = 1e-14f;
bool lean_rank_cut_ok(float lam16, float lam24) { return lam16 <= kLam16Max && lam24 <= kLam24Max; }

int ensure_io(irm_ctx* c, size_t bytes) {
    if (bytes <= c->io_bytes) return 0;
    if (c->d_io) (void)hipFree(c->d_io);
    c->d_io = nullptr;
    c->io_bytes = 0;
    bytes = std::max<size_t>(bytes, 1 << 20);
    HIP_TRY(hipMalloc(&c->d_io, bytes));
    c->io_bytes = bytes;
    return 0;
}

int upload(float** dst, const std::vector<float>& src) {
    HIP_TRY(hipMalloc(dst, std::max<size_t>(src.size(), 4) * sizeof(float)));
    if (!src.empty()) HIP_TRY(hipMemcpy(*dst, src.data(), src.size() * sizeof(float), hipMemcpyHostToDevice));
    return 0;
}

// Workgroup shape for a launch of B trajectories: one lane per (trajectory,
// waypoint), NW = N rounded up to 64 lanes per trajectory, TB trajectories
// per workgroup with TB·D ≤ 16 MFMA columns and TB·NW ≤ 1024 threads.  For
// the optimiser TB defaults to ⌈B / #CU⌉ (one workgroup per CU when B is
// small) and the operator fragments are staged into LDS when they fit.
int choose_shape(const irm_ctx* c, int B, bool optimizer, KParams& kp, int* lds_bytes_out) {
    const int D = c->D;
    kp.NW = round_up(c->N, 64);
    // D ≥ 5 needs > 128 VGPRs per lane: keep those workgroups at ≤ 512 threads
    const int maxthreads = (D >= 5) ? 512 : irm::kMaxThreads;
    // Optimiser workgroups of N ≤ 128 stay at ≤ 512 threads: the 1024-thread variants are capped at
    // 128 VGPRs and spill (C3 with five trajectories per workgroup: 1.47 ms vs 0.79 ms for four), so a
    // large batch is better served by more 4-trajectory workgroups (bench.py --tb 5 vs default).
    const int cap = (optimizer && kp.NW <= 128) ? std::min(maxthreads, 512) : maxthreads;
    const int tbmax = std::max(1, std::min(irm::kCols / D, cap / kp.NW));
    int tb = tbmax;
    if (optimizer && c->p.traj_per_block > 0) tb = std::min(c->p.traj_per_block, tbmax);
    else if (optimizer) tb = std::min(tbmax, std::max(1, (B + c->num_cus - 1) / std::max(1, c->num_cus)));
    tb = std::max(1, std::min(tb, std::max(1, B)));
    const size_t lds_cap = 160 * 1024;
    // Under-filled GPU (fewer workgroups than half the CUs: small batches, C2's single
    // trajectory): pad the optimiser's workgroup with waves that take no trajectory
    // (tvalid = false in the kernels) up to 512 threads.  They share the MFMA stages (stage-2
    // tiles and stage-1 units are distributed over all waves), which shortens every round's
    // latency chain; the per-tile arithmetic is unchanged, so results are bit-identical.
    const char* pw = getenv("IRM_PAD_WAVES");
    const bool pad_ok = optimizer && !(pw && pw[0] == '0');
    for (; tb >= 1; --tb) {
        kp.TB = tb;
        kp.BT = tb * kp.NW;
        if (pad_ok && 2 * ((B + tb - 1) / tb) <= c->num_cus && kp.BT < 512) kp.BT = 512;
        kp.nsplit = irm::stage1_splits(kp.NK);
        // the lean kernel (k_lean) runs one stage-1 unit per wave and is instantiated for 256- and
        // 512-thread workgroups: smaller optimiser workgroups get idle waves up to that size (e.g.
        // one N = 128 trajectory per workgroup: 2 → 4 waves), so that the lean kernel — and its
        // fp32-α rounding — serves them; the general kernel runs padded workgroups bit-identically
        if (optimizer && kp.BT < 512) {
            kp.BT = std::max(kp.BT, std::min(512, 64 * (kp.RP / 16) * kp.nsplit));
            kp.BT = kp.BT <= 256 ? 256 : 512;
        }
        if (optimizer) {
            kp.regops = irm::regops_fit(kp) ? 1 : 0;
            irm::Plan a = irm::plan_lds(kp, true, true);
            if ((size_t)a.total * 4 <= lds_cap) {
                kp.ops_in_lds = 1;
                if (lds_bytes_out) *lds_bytes_out = a.total * 4;
                return tb;
            }
            irm::Plan b = irm::plan_lds(kp, false, true);
            if ((size_t)b.total * 4 <= lds_cap) {
                kp.ops_in_lds = 0;
                kp.regops = 0;
                if (lds_bytes_out) *lds_bytes_out = b.total * 4;
                return tb;
            }
        } else {
            irm::Plan a = irm::plan_lds(kp, false, false);
            if ((size_t)a.total * 4 <= lds_cap) {
                if (lds_bytes_out) *lds_bytes_out = a.total * 4;
                return tb;
            }
        }
    }
    return 0;
}

int set_device(const irm_ctx* c) {
    HIP_TRY(hipSetDevice(c->p.device));
    return 0;
}

}  // namespace

extern "C" {

void irm_params_default(irm_params* p) {
    memset(p, 0, sizeof(*p));
    p->n_timesteps = 50;
    p->n_joints = 3;
    p->optimizer = IRM_OPT_BLS;
    p->max_inner_iteration = 200;
    p->max_outer_iteration = 10;
    p->max_bls_iteration = 20;
    p->constraint_violating_dependant_loss = 1;
    const float lr[10] = {2e-3f, 1e-4f, 1e-5f, 1e-6f, 1e-7f, 1e-8f, 1e-8f, 1e-8f, 1e-8f, 1e-8f};
    p->n_gd_lr = 10;
    for (int i = 0; i < 10; ++i) p->gd_lr[i] = lr[i];
    p->rbf_variance = 0.1f;
    p->loop_loss_reduction = 1e-3f;
    p->lambda_constraint_increase = 10.f;
    p->lambda_sg_constraint = 0.5f;
    p->lambda_jl_constraint = 0.1f;
    p->eps_position = 0.01f;
    p->eps_velocity = 0.01f;
    p->lambda_max_cost = 0.5f;
    p->lambda_reg = 1e-4f;
    p->joint_safety_limit = 0.98f;
    p->bls_lr_start = 0.2f;
    p->bls_alpha = 0.01f;
    p->bls_beta_plus = 1.2f;
    p->bls_beta_minus = 0.5f;
    p->max_joint_velocity = 7.f;
    p->max_joint_position = 2.f;
    p->min_joint_position = -1.f;
    p->link_length[0] = 1.5f;
    p->link_length[1] = 1.0f;
    p->link_length[2] = 0.5f;
    irm_default_jac(3, 0.15f, 0u, p->jac);
    p->operator_rank = 0;
    p->operator_tol = 1e-12f;
    p->device = 0;
}

int irm_default_jac(int32_t D, float jgm, uint32_t seed, float* jac_out) {
    if (D < 1 || D > IRM_MAX_JOINTS || !jac_out) return fail(IRM_EINVAL, "irm_default_jac: bad arguments");
    const int n = D * D, odd = n & 1, half = (n + odd) / 2;
    std::vector<uint32_t> cnt(2 * half, 0u), bits(2 * half, 0u);
    for (int i = 0; i < n; ++i) cnt[i] = (uint32_t)i;
    for (int i = 0; i < half; ++i) {
        uint32_t x0 = cnt[i], x1 = cnt[half + i];
        threefry2x32(0u, seed, x0, x1);  // PRNGKey(seed) = [0, seed]
        bits[i] = x0;
        bits[half + i] = x1;
    }
    const float lo = nextafterf(-1.f, 0.f);
    for (int i = 0; i < n; ++i) {
        uint32_t fb = (bits[i] >> 9) | 0x3F800000u;
        float f;
        memcpy(&f, &fb, 4);
        f -= 1.f;
        float u = std::max(lo, f * (1.f - lo) + lo);
        float z = (float)sqrt(2.0) * (float)erfinv_f64((double)u);
        jac_out[i] = ((i / D) == (i % D) ? 1.f : 0.f) + jgm * z;
    }
    return IRM_OK;
}

const char* irm_last_error(void) { return g_err.c_str(); }

int irm_ctx_create(irm_ctx** out, const irm_params* p) {
    if (!out || !p) return fail(IRM_EINVAL, "irm_ctx_create: null argument");
    *out = nullptr;
    const int N = p->n_timesteps, D = p->n_joints;
    if (N < 2 || N > IRM_MAX_TIMESTEPS) return fail(IRM_EINVAL, "n_timesteps=%d outside [2, %d]", N, IRM_MAX_TIMESTEPS);
    if (D < 1 || D > IRM_MAX_JOINTS) return fail(IRM_EINVAL, "n_joints=%d outside [1, %d]", D, IRM_MAX_JOINTS);
    if (p->optimizer != IRM_OPT_GD && p->optimizer != IRM_OPT_BLS) return fail(IRM_EINVAL, "unknown optimizer %d", p->optimizer);
    if (p->optimizer == IRM_OPT_GD && p->max_outer_iteration > p->n_gd_lr)
        return fail(IRM_EINVAL, "max_outer_iteration and dual_lr do not match");  // optimizer_GD.py:34-36
    if (p->n_gd_lr > IRM_MAX_LR) return fail(IRM_EINVAL, "at most %d --gd-lr entries", IRM_MAX_LR);
    if (p->max_bls_iteration < 1 && p->optimizer == IRM_OPT_BLS) return fail(IRM_EINVAL, "max_bls_iteration must be >= 1");
    if (!(p->rbf_variance > 0.f)) return fail(IRM_EINVAL, "rbf_variance must be > 0");

    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= p->device || p->device < 0)
        return fail(IRM_EDEVICE, "no HIP device %d (found %d): this library has no CPU fallback", p->device, ndev);
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, p->device));
    if (!strstr(prop.gcnArchName, "gfx950"))
        return fail(IRM_EDEVICE, "device %d is %s; this build targets gfx950 (MI355X) only", p->device, prop.gcnArchName);
    HIP_TRY(hipSetDevice(p->device));

    irm_ctx* c = new irm_ctx();
    c->p = *p;
    c->N = N;
    c->D = D;
    c->num_cus = prop.multiProcessorCount;
    snprintf(c->name, sizeof(c->name), "%s", prop.name);
    snprintf(c->arch, sizeof(c->arch), "%s", prop.gcnArchName);

    // ---- Trajectory.__init__ (trajectory.py:31-42), fp32 as the reference
    c->t.resize(N);
    c->cvec.resize(N);
    {
        const float div = (float)(N - 1);
        for (int i = 0; i < N - 1; ++i) {
            const float st = (float)i / div;
            c->t[i] = 0.f * (1.f - st) + 1.f * st;
        }
        c->t[N - 1] = 1.f;
        for (int i = 0; i < N; ++i) {
            const float tt = c->t[i], t3 = tt * tt * tt, t4 = t3 * tt, t5 = t4 * tt;
            c->cvec[i] = 6.f * t5 - 15.f * t4 + 10.f * t3;
        }
    }
    c->K.resize((size_t)N * N);
    c->dK.resize((size_t)N * N);
    {
        const double sig = decimal_double(p->rbf_variance);
        const float two_s2 = (float)(2.0 * sig * sig), s2 = (float)(sig * sig);
        for (int i = 0; i < N; ++i)
            for (int j = 0; j < N; ++j) {
                const float d = c->t[j] - c->t[i];
                const float e = expf(-(d * d) / two_s2);
                c->K[(size_t)i * N + j] = e;
                c->dK[(size_t)i * N + j] = d / s2 * e;
            }
    }
    c->J.assign(p->jac, p->jac + (size_t)D * D);

    // ---- operator factorisation F = L·V_R
    // optimiser row layout: position half rows 0..N-1, velocity half from row NK
    const int NK = round_up(N, 16), MP = 2 * NK;
    std::vector<double> Ld((size_t)2 * N * N);
    for (int i = 0; i < N; ++i)
        for (int j = 0; j < N; ++j) {
            Ld[(size_t)i * N + j] = c->K[(size_t)i * N + j];
            Ld[(size_t)(N + i) * N + j] = c->dK[(size_t)i * N + j];
        }
    int R = 0, RP = 0;
    std::vector<double> Vd;  // N × RP
    if (p->operator_rank < 0) {  // dense: F = L, V = I
        R = N;
        RP = NK;
        Vd.assign((size_t)N * RP, 0.0);
        for (int i = 0; i < N; ++i) Vd[(size_t)i * RP + i] = 1.0;
        c->trunc = 0.f;
    } else {
        std::vector<double> G((size_t)N * N, 0.0), Vfull, LdT((size_t)N * 2 * N);
        for (int m = 0; m < 2 * N; ++m)  // Lᵀ rows: the Gram sums read contiguously (same sums, same order)
            for (int i = 0; i < N; ++i) LdT[(size_t)i * 2 * N + m] = Ld[(size_t)m * N + i];
        for (int i = 0; i < N; ++i)
            for (int j = i; j < N; ++j) {
                double s = 0.0;
                const double* li = &LdT[(size_t)i * 2 * N];
                const double* lj = &LdT[(size_t)j * 2 * N];
                for (int m = 0; m < 2 * N; ++m) s += li[m] * lj[m];
                G[(size_t)i * N + j] = G[(size_t)j * N + i] = s;
            }
        jacobi_eigen_memo(G, N, Vfull);
        std::vector<int> order(N);
        for (int i = 0; i < N; ++i) order[i] = i;
        std::sort(order.begin(), order.end(),
                  [&](int a, int b) { return G[(size_t)a * N + a] > G[(size_t)b * N + b]; });
        const double l0 = G[(size_t)order[0] * N + order[0]];
        if (p->operator_rank > 0) {
            R = std::min(p->operator_rank, N);
        } else {
            const double tol = p->operator_tol > 0.f ? p->operator_tol : 1e-12;
            R = N;
            for (int r = 16; r < N; r += 16) {
                const double lr = std::max(0.0, G[(size_t)order[r] * N + order[r]]);
                if (lr / l0 < tol) { R = r; break; }
            }
        }
        RP = round_up(R, 16);
        c->trunc = (R < N) ? (float)(std::max(0.0, G[(size_t)order[R] * N + order[R]]) / l0) : 0.f;
        auto lam = [&](int r) { return (r < R) ? (float)(std::max(0.0, G[(size_t)order[r] * N + order[r]]) / l0) : 0.f; };
        c->lam16 = lam(16);
        c->lam24 = lam(24);
        Vd.assign((size_t)N * RP, 0.0);
        // Rank slot of component r.  At RP = 32 the second k-quad interleaves components 16-23 and
        // 24-31 so that the lean kernel's MFMAs 2 and 3 of that quad (k-permuted fragments: MFMA j
        // covers rows j, 4+j, 8+j, 12+j of a quad) see only components 24-31, whose singular values
        // are at fp32 noise (σ_24/σ_0 ≈ 3e-8 at N = 128) — k_lean skips those two MFMAs (rank 24 in
        // stage 2).  Every other use is a sum over all slots, so the order does not matter there.
        auto slot = [&](int r) {
            if (RP != 32 || r < 16) return r;
            const int j = r - 16, hi = j >= 8, q = j & 7;  // q-th of the 8 components of its half
            return 16 + 4 * (q >> 1) + (q & 1) + (hi ? 2 : 0);
        };
        for (int i = 0; i < N; ++i)
            for (int r = 0; r < R; ++r) Vd[(size_t)i * RP + slot(r)] = Vfull[(size_t)i * N + order[r]];
    }
    c->R = R;
    c->RP = RP;
    c->NK = NK;
    c->MP = MP;
    std::vector<double> F((size_t)2 * N * RP, 0.0);  // F = L·V
    for (int m = 0; m < 2 * N; ++m)
        for (int r = 0; r < RP; ++r) {
            double s = 0.0;
            for (int j = 0; j < N; ++j) s += Ld[(size_t)m * N + j] * Vd[(size_t)j * RP + r];
            F[(size_t)m * RP + r] = s;
        }

    // fragments
    std::vector<double> A;
    std::vector<float> frag;
    int rc = 0;
    {  // K, dK and their transposes, row-major fp32: the correctly rounded α-space
       // contractions (eval_exact / grad_exact) read one coalesced row per k-step
        std::vector<float> kt((size_t)N * N), dkt((size_t)N * N);
        for (int i = 0; i < N; ++i)
            for (int j = 0; j < N; ++j) {
                kt[(size_t)j * N + i] = c->K[(size_t)i * N + j];
                dkt[(size_t)j * N + i] = c->dK[(size_t)i * N + j];
            }
        rc |= upload(&c->d_K, c->K);
        rc |= upload(&c->d_dK, c->dK);
        rc |= upload(&c->d_Kt, kt);
        rc |= upload(&c->d_dKt, dkt);
    }
    // F rows m < N (K part) → row m, m = N + j (dK part) → row NK + j
    auto frow = [&](int m) { return m < N ? m : NK + (m - N); };
    // Fᵀ (RP × MP): stage 1 contracts y = Fᵀ·[a; b].  The endpoint velocity rows (m = N, 2N−1)
    // are left out: the optimiser adds b'[0], b'[N−1] through their own operator columns (Hend,
    // Fbot) in every round, so a round whose stage 1 is dense because of a neighbour adds exact
    // zeros for them and a problem's arithmetic never depends on its workgroup neighbours.
    A.assign((size_t)RP * MP, 0.0);
    for (int m = 0; m < 2 * N; ++m) {
        if (m == N || m == 2 * N - 1) continue;
        for (int r = 0; r < RP; ++r) A[(size_t)r * MP + frow(m)] = F[(size_t)m * RP + r];
    }
    fill_frag(frag, RP, MP, A);
    rc |= upload(&c->d_F1, frag);
    fill_frag(frag, RP, MP, A, true);
    rc |= upload(&c->d_F1p, frag);
    A.assign((size_t)MP * RP, 0.0);  // F (MP × RP)
    for (int m = 0; m < 2 * N; ++m)
        for (int r = 0; r < RP; ++r) A[(size_t)frow(m) * RP + r] = F[(size_t)m * RP + r];
    fill_frag(frag, MP, RP, A);
    rc |= upload(&c->d_F2, frag);
    fill_frag(frag, MP, RP, A, true);
    rc |= upload(&c->d_F2p, frag);
    std::vector<float> fb((size_t)N * RP), vr((size_t)N * RP);
    for (int n = 0; n < N; ++n)
        for (int r = 0; r < RP; ++r) {
            fb[(size_t)n * RP + r] = (float)F[(size_t)(N + n) * RP + r];
            vr[(size_t)n * RP + r] = (float)Vd[(size_t)n * RP + r];
        }
    rc |= upload(&c->d_Fbot, fb);
    rc |= upload(&c->d_Vr, vr);
    {  // the lean kernel's α-space terms: V_Rᵀ (RP × NK) and V_R (NK × RP), k-permuted fragments,
       // and G's endpoint velocity columns hv_e = V_R·F[N+e]ᵀ (e ∈ {0, N−1}), NK each
        A.assign((size_t)RP * NK, 0.0);
        for (int n = 0; n < N; ++n)
            for (int r = 0; r < RP; ++r) A[(size_t)r * NK + n] = Vd[(size_t)n * RP + r];
        fill_frag(frag, RP, NK, A, true);
        rc |= upload(&c->d_VTp, frag);
        fill_frag(frag, RP, NK, A);
        rc |= upload(&c->d_VTs, frag);
        A.assign((size_t)NK * RP, 0.0);
        for (int n = 0; n < N; ++n)
            for (int r = 0; r < RP; ++r) A[(size_t)n * RP + r] = Vd[(size_t)n * RP + r];
        fill_frag(frag, NK, RP, A, true);
        rc |= upload(&c->d_VNp, frag);
        fill_frag(frag, NK, RP, A);
        rc |= upload(&c->d_VNs, frag);
        std::vector<float> hv((size_t)2 * NK, 0.f);
        for (int e = 0; e < 2; ++e) {
            const int me = N + (e ? N - 1 : 0);
            for (int n = 0; n < N; ++n) {
                double acc = 0.0;
                for (int r = 0; r < RP; ++r) acc += Vd[(size_t)n * RP + r] * F[(size_t)me * RP + r];
                hv[(size_t)e * NK + n] = (float)acc;
            }
        }
        rc |= upload(&c->d_HV, hv);
    }
    {  // h_e = F·F[N+e]ᵀ for the endpoint velocity rows e ∈ {0, N−1}, kernel row layout
        std::vector<float> h((size_t)2 * MP, 0.f);
        for (int e = 0; e < 2; ++e) {
            const int me = N + (e ? N - 1 : 0);
            for (int m = 0; m < 2 * N; ++m) {
                double acc = 0.0;
                for (int r = 0; r < RP; ++r) acc += F[(size_t)m * RP + r] * F[(size_t)me * RP + r];
                h[(size_t)e * MP + frow(m)] = (float)acc;
            }
        }
        rc |= upload(&c->d_H, h);
    }
    // initTrajectory basis: u = K⁻¹(1−c), w = K⁻¹c (fp32 LU, trajectory.py:77)
    {
        std::vector<float> rhs((size_t)N * 2), X((size_t)N * 2);
        for (int n = 0; n < N; ++n) {
            rhs[(size_t)n * 2] = 1.f - c->cvec[n];
            rhs[(size_t)n * 2 + 1] = c->cvec[n];
        }
        if (!lu_solve_f32(N, c->K.data(), rhs.data(), 2, X.data())) {
            irm_ctx_destroy(c);
            return fail(IRM_EINVAL, "kernel matrix K is exactly singular in fp32 LU");
        }
        std::vector<float> u(N), w(N);
        for (int n = 0; n < N; ++n) {
            u[n] = X[(size_t)n * 2];
            w[n] = X[(size_t)n * 2 + 1];
        }
        rc |= upload(&c->d_u, u);
        rc |= upload(&c->d_w, w);
    }
    if (rc) {
        std::string e = g_err;
        irm_ctx_destroy(c);
        return fail(IRM_ENOMEM, "%s", e.c_str());
    }

    // ---- kernel parameter template
    KParams& kp = c->kp;
    kp.N = N;
    kp.D = D;
    kp.R = R;
    kp.NK = NK;
    kp.MP = MP;
    kp.RP = RP;
    kp.v_ident = p->operator_rank < 0 ? 1 : 0;
    kp.O = 0;
    kp.optimizer = p->optimizer;
    kp.max_inner = p->max_inner_iteration;
    kp.max_outer = p->max_outer_iteration;
    kp.max_bls = p->max_bls_iteration;
    kp.cvdl = p->constraint_violating_dependant_loss ? 1 : 0;
    kp.llr = p->loop_loss_reduction;
    kp.lci = p->lambda_constraint_increase;
    kp.lsg0 = p->lambda_sg_constraint;
    kp.ljl0 = p->lambda_jl_constraint;
    kp.eps_p = p->eps_position;
    kp.eps_v = p->eps_velocity;
    kp.lmax = p->lambda_max_cost;
    kp.lreg = p->lambda_reg;
    // GD weight decay (1 − λ_reg·lr) per outer iteration, in fp32 as the reference evaluates it:
    // lr = dual_lr[k] is an fp32 array element (optimizer_GD.py:38-39, :209) and the Python float
    // λ_reg enters weakly typed, so both the product and the difference round to fp32
    // (optimizer_GD.py:81, :185).  The product is rounded through a volatile: clang contracts across
    // statements under -ffp-contract=fast, so only the missing FMA of the default host target kept the
    // two roundings apart before (a -march with FMA would have fused them into one)
    for (int i = 0; i < IRM_MAX_LR; ++i) {
        volatile float prod = p->lambda_reg * p->gd_lr[i];
        kp.gd_c[i] = 1.f - prod;
    }
    kp.bls_lr0 = p->bls_lr_start;
    kp.bls_a = p->bls_alpha;
    kp.bls_bp = p->bls_beta_plus;
    kp.bls_bm = p->bls_beta_minus;
    kp.vmax = p->max_joint_velocity;
    kp.pmax = p->max_joint_position;
    kp.pmin = p->min_joint_position;
    {  // trajectory.py:31-32, 221-222, 251 (Python doubles → fp32)
        const double mean = 0.5 * ((double)p->max_joint_position + (double)p->min_joint_position);
        const double stdp = 0.5 * ((double)p->max_joint_position - mean);
        kp.mean_pos = (float)mean;
        kp.std_pos = (float)stdp;
        kp.std2 = kp.std_pos * kp.std_pos;
        kp.vmax2 = kp.vmax * kp.vmax;
        kp.thr_hi = (float)((double)p->joint_safety_limit * (double)p->max_joint_position);
        kp.thr_lo = (float)((double)p->joint_safety_limit * (double)p->min_joint_position);
        kp.thr_v = (float)((double)p->joint_safety_limit * (double)p->max_joint_velocity);
        // --constraint-violating-dependant-loss false (trajectory.py:221-222, 251: the penalties apply to
        // every element): thresholds that every finite joint position / velocity passes, so the kernels
        // form the masks without the flag (one scalar op fewer per mask element and round).  Deliberate
        // deviation: a NaN joint value fails every compare, so its penalty term is masked
        // off (0) where the reference's unmasked penalty would carry the NaN into the loss — only a diverged
        // trajectory (non-finite state) can see the difference, and its loss is non-finite either way
        if (!p->constraint_violating_dependant_loss) {
            kp.thr_hi = -INFINITY;
            kp.thr_lo = INFINITY;
            kp.thr_v = -1.f;
        }
        kp.invN = 1.f / (float)N;
        kp.inv_std_pos = 1.f / kp.std_pos;
        kp.inv_vmax = 1.f / kp.vmax;
        kp.inv_std2 = 1.f / kp.std2;
        kp.inv_vmax2 = 1.f / kp.vmax2;
        kp.Nmagic = (uint32_t)((((uint64_t)1 << 32) + (uint64_t)N - 1) / (uint64_t)N);
        kp.NDmagic = (uint32_t)((((uint64_t)1 << 32) + (uint64_t)(N * D) - 1) / (uint64_t)(N * D));
    }
    for (int i = 0; i < IRM_MAX_LR; ++i) kp.gd_lr[i] = p->gd_lr[i];
    for (int i = 0; i < IRM_MAX_JOINTS; ++i) kp.link[i] = p->link_length[i];
    {
        std::vector<double> Jd((size_t)D * D), JtJ((size_t)D * D, 0.0);
        for (int i = 0; i < D * D; ++i) Jd[i] = p->jac[i];
        for (int a = 0; a < D; ++a)
            for (int b = 0; b < D; ++b) {
                double s = 0.0;
                for (int k = 0; k < D; ++k) s += Jd[(size_t)k * D + a] * Jd[(size_t)k * D + b];
                JtJ[(size_t)a * D + b] = s;
            }
        std::vector<float> eye((size_t)D * D, 0.f), Jinv((size_t)D * D);
        for (int i = 0; i < D; ++i) eye[(size_t)i * D + i] = 1.f;
        if (!lu_solve_f32(D, p->jac, eye.data(), D, Jinv.data())) {
            irm_ctx_destroy(c);
            return fail(IRM_EINVAL, "J is singular");
        }
        // (JᵀJ)⁻¹ by Gauss-Jordan in fp64, and w = (JᵀJ)⁻¹·Jᵀ1 (BLS norms from y' = y·JᵀJ)
        std::vector<double> Mi((size_t)D * D, 0.0), Mw(JtJ);
        for (int i = 0; i < D; ++i) Mi[(size_t)i * D + i] = 1.0;
        for (int col = 0; col < D; ++col) {
            int piv = col;
            for (int r = col + 1; r < D; ++r)
                if (std::fabs(Mw[(size_t)r * D + col]) > std::fabs(Mw[(size_t)piv * D + col])) piv = r;
            for (int k = 0; k < D; ++k) {
                std::swap(Mw[(size_t)col * D + k], Mw[(size_t)piv * D + k]);
                std::swap(Mi[(size_t)col * D + k], Mi[(size_t)piv * D + k]);
            }
            const double d = Mw[(size_t)col * D + col];
            for (int k = 0; k < D; ++k) {
                Mw[(size_t)col * D + k] /= d;
                Mi[(size_t)col * D + k] /= d;
            }
            for (int r = 0; r < D; ++r) {
                if (r == col) continue;
                const double f = Mw[(size_t)r * D + col];
                for (int k = 0; k < D; ++k) {
                    Mw[(size_t)r * D + k] -= f * Mw[(size_t)col * D + k];
                    Mi[(size_t)r * D + k] -= f * Mi[(size_t)col * D + k];
                }
            }
        }
        for (int a = 0; a < D; ++a) {
            double w = 0.0;
            for (int b = 0; b < D; ++b) {
                double u = 0.0;
                for (int i = 0; i < D; ++i) u += (double)p->jac[(size_t)i * D + b];
                w += Mi[(size_t)a * D + b] * u;
            }
            kp.wal[a] = (float)w;
        }
        for (int i = 0; i < D * D; ++i) kp.Minv[i] = (float)Mi[i];
        for (int i = 0; i < D * D; ++i) {
            kp.J[i] = p->jac[i];
            kp.JtJ[i] = (float)JtJ[i];
            kp.Jinv[i] = Jinv[i];
        }
    }
    kp.Km = c->d_K;
    kp.dKm = c->d_dK;
    kp.Kt = c->d_Kt;
    kp.dKt = c->d_dKt;
    kp.F1frag = c->d_F1;
    kp.F2frag = c->d_F2;
    kp.F1p = c->d_F1p;
    kp.F2p = c->d_F2p;
    kp.Fbot = c->d_Fbot;
    kp.Vr = c->d_Vr;
    kp.Hend = c->d_H;
    kp.VTp = c->d_VTp;
    kp.VNp = c->d_VNp;
    kp.HV = c->d_HV;
    kp.VTs = c->d_VTs;
    kp.VNs = c->d_VNs;
    kp.uvec = c->d_u;
    kp.wvec = c->d_w;
    kp.lam_max = p->lambda_max_cost;
    kp.one_m_lmax = (float)(1.0 - (double)p->lambda_max_cost);
    kp.record_series = p->record_series ? 1 : 0;
    kp.whole_robot = p->whole_robot_cost ? 1 : 0;
    {
        const char* g = getenv("IRM_GENERAL_KERNEL");  // diagnostics: force the general optimiser
        kp.lean_ok = (g && g[0] == '1') ? 0 : 1;
        // k_lean drops the components 16-31 from the waypoint direction (terms ∝ λ_r) and the residual
        // projection, and 24-31 from G (∝ σ_r): only where those are at fp32 noise (σ = 0.1: λ16/λ0 ≈
        // 1.5e-7, λ24/λ0 ≈ 6e-16).  A flatter spectrum (smaller --rbf-variance, e.g. 0.07: 4e-4 / 7e-9)
        // still selects R = 32; it runs the general kernel at the full rank instead.
        if (!lean_rank_cut_ok(c->lam16, c->lam24)) kp.lean_ok = 0;
        const char* w = getenv("IRM_LEAN_WPL");
        kp.lean_wpl = w ? atoi(w) : 0;
        const char* nh = getenv("IRM_LEAN_NOHELP");
        kp.lean_nohelp = (nh && nh[0] == '1') ? 1 : 0;
        const char* tp = getenv("IRM_TRACE_PROBLEM");
        kp.trace_b = tp ? atoi(tp) : 0;
    }
    c->max_series = p->max_series > 0 ? p->max_series : 1 + p->max_outer_iteration * p->max_inner_iteration;
    kp.max_series = c->max_series;

    {
        KParams probe = c->kp;
        probe.O = IRM_MAX_OBSTACLES;
        c->tb_opt = choose_shape(c, 1 << 20, true, probe, &c->lds_opt);
        c->ops_lds = probe.ops_in_lds;
    }
    if (c->tb_opt <= 0) {
        irm_ctx_destroy(c);
        return fail(IRM_EINVAL, "configuration N=%d D=%d R=%d does not fit the 160 KiB LDS", N, D, R);
    }
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        irm_ctx_destroy(c);
        return fail(IRM_EDEVICE, "hipStreamCreate failed");
    }
    *out = c;
    return IRM_OK;
}

void irm_ctx_destroy(irm_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->p.device);
    float* bufs[] = {c->d_K, c->d_dK, c->d_Kt, c->d_dKt, c->d_F1,   c->d_F2, c->d_F1p, c->d_F2p,
                     c->d_Fbot, c->d_Vr, c->d_H, c->d_u, c->d_w, c->d_VTp, c->d_VNp, c->d_HV, c->d_VTs, c->d_VNs};
    for (float* b : bufs)
        if (b) (void)hipFree(b);
    if (c->d_io) (void)hipFree(c->d_io);
    if (c->d_prof) (void)hipFree(c->d_prof);
    if (c->d_trace) (void)hipFree(c->d_trace);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int irm_get_info(const irm_ctx* c, irm_info* out) {
    if (!c || !out) return fail(IRM_EINVAL, "irm_get_info: null argument");
    memset(out, 0, sizeof(*out));
    out->abi_version = IRM_ABI_VERSION;
    out->n_timesteps = c->N;
    out->n_joints = c->D;
    out->operator_rank = c->R;
    out->operator_trunc = c->trunc;
    out->traj_per_block = c->tb_opt;
    out->num_cus = c->num_cus;
    out->lds_bytes_optimize = c->lds_opt;
    snprintf(out->device_name, sizeof(out->device_name), "%s", c->name);
    snprintf(out->arch, sizeof(out->arch), "%s", c->arch);
    snprintf(out->build_id, sizeof(out->build_id), "%s", irm_build_id());
    return IRM_OK;
}

int32_t irm_series_capacity(const irm_ctx* c) { return c ? c->max_series : 0; }

int irm_debug_bls_trace_enable(irm_ctx* c, int32_t cap) {
    if (!c || cap < 0) return fail(IRM_EINVAL, "irm_debug_bls_trace_enable: bad argument");
    if (set_device(c)) return IRM_EDEVICE;
    if (c->d_trace) (void)hipFree(c->d_trace);
    c->d_trace = nullptr;
    c->trace_cap = 0;
    if (cap == 0) return IRM_OK;
    HIP_TRY(hipMalloc(&c->d_trace, (size_t)cap * irm::kTraceW * sizeof(float)));
    HIP_TRY(hipMemset(c->d_trace, 0, (size_t)cap * irm::kTraceW * sizeof(float)));
    c->trace_cap = cap;
    return IRM_OK;
}

int irm_debug_bls_trace(irm_ctx* c, float* out, int32_t cap) {
    if (!c || !out || cap < 0) return fail(IRM_EINVAL, "irm_debug_bls_trace: bad argument");
    if (!c->d_trace) return fail(IRM_EINVAL, "line-search log not enabled (irm_debug_bls_trace_enable)");
    if (set_device(c)) return IRM_EDEVICE;
    const int n = std::min(cap, c->trace_cap);
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(out, c->d_trace, (size_t)n * irm::kTraceW * sizeof(float), hipMemcpyDeviceToHost));
    return n;
}

int irm_debug_phase_profile(irm_ctx* c, uint64_t* out, int32_t max_blocks) {
    if (!c || !out) return fail(IRM_EINVAL, "null argument");
#if defined(IRM_PHASE_PROFILE) || defined(IRM_DIV_CHECK)
    if (set_device(c)) return IRM_EDEVICE;
    const int n = std::min(max_blocks, c->prof_blocks);
    if (n <= 0 || !c->d_prof) return 0;
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(out, c->d_prof, (size_t)n * irm::kProfPhases * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return n;
#else
    (void)max_blocks;
    return fail(IRM_EINVAL, "library built without IRM_PHASE_PROFILE");
#endif
}

int irm_kernel_matrices(const irm_ctx* c, float* t, float* km, float* dkm, float* jac) {
    if (!c) return fail(IRM_EINVAL, "null context");
    if (t) memcpy(t, c->t.data(), sizeof(float) * c->N);
    if (km) memcpy(km, c->K.data(), sizeof(float) * c->K.size());
    if (dkm) memcpy(dkm, c->dK.data(), sizeof(float) * c->dK.size());
    if (jac) memcpy(jac, c->J.data(), sizeof(float) * c->J.size());
    return IRM_OK;
}

// ----------------------------------------------------- host-pointer calls
namespace {

struct Stage {
    irm_ctx* c;
    size_t off = 0;
    char* base() { return (char*)c->d_io; }
    // reserve 256-B aligned slice
    size_t take(size_t bytes) {
        size_t o = off;
        off += (bytes + 255) & ~(size_t)255;
        return o;
    }
};

int check_obs(int O) {
    if (O < 0 || O > IRM_MAX_OBSTACLES) return fail(IRM_EINVAL, "n_obstacles=%d outside [0, %d]", O, IRM_MAX_OBSTACLES);
    return 0;
}

// obstacle_stride: 0 = one shared O×2 table, else floats between consecutive problems' tables (≥ 2·O)
int check_stride(int O, int stride) {
    if (stride != 0 && (stride < 2 * O || stride < 0))
        return fail(IRM_EINVAL, "obstacle_stride=%d must be 0 (shared) or >= 2*n_obstacles=%d", stride, 2 * O);
    return 0;
}

// Run one forward-family kernel on B host trajectories.
int run_forward(irm_ctx* c, int mode, const float* alpha, const float* start, const float* goal, const float* obs,
                int O, int B, float lsg, float ljl, float lmax, int which, float* out0, float* out1, uint8_t* ok) {
    if (set_device(c)) return IRM_EDEVICE;
    if (B < 0 || !alpha) return fail(IRM_EINVAL, "bad batch arguments");
    if (check_obs(O)) return IRM_EINVAL;
    if (B == 0) return IRM_OK;
    const int N = c->N, D = c->D;
    const size_t nd = (size_t)B * N * D;
    Stage st{c};
    const size_t o_alpha = st.take(nd * 4), o_s = st.take((size_t)B * D * 4), o_g = st.take((size_t)B * D * 4),
                 o_obs = st.take((size_t)std::max(O, 1) * 8), o_out0 = st.take(std::max(nd, (size_t)B * 11) * 4),
                 o_out1 = st.take(nd * 4), o_ok = st.take((size_t)B);
    if (ensure_io(c, st.off)) return IRM_ENOMEM;
    char* d = st.base();
    hipStream_t s = c->stream;
    std::vector<float> zeros;
    if (!start || !goal) zeros.assign((size_t)B * D, 0.f);
    HIP_TRY(hipMemcpyAsync(d + o_alpha, alpha, nd * 4, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d + o_s, start ? start : zeros.data(), (size_t)B * D * 4, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d + o_g, goal ? goal : zeros.data(), (size_t)B * D * 4, hipMemcpyHostToDevice, s));
    if (O > 0 && obs) HIP_TRY(hipMemcpyAsync(d + o_obs, obs, (size_t)O * 8, hipMemcpyHostToDevice, s));
    KParams kp = c->kp;
    kp.B = B;
    kp.O = (obs ? O : 0);
    kp.obs_stride = 0;
    kp.alpha0 = (const float*)(d + o_alpha);
    kp.start = (const float*)(d + o_s);
    kp.goal = (const float*)(d + o_g);
    kp.obstacles = (const float*)(d + o_obs);
    kp.lam_sg = lsg;
    kp.lam_jl = ljl;
    kp.lam_max = lmax;
    kp.one_m_lmax = (float)(1.0 - (double)lmax);
    kp.which = which;
    kp.out0 = (float*)(d + o_out0);
    kp.out1 = (float*)(d + o_out1);
    kp.out_ok = (uint8_t*)(d + o_ok);
    if (choose_shape(c, B, false, kp, nullptr) <= 0) return fail(IRM_EINVAL, "no workgroup shape fits LDS");
    HIP_TRY(irm::launch_forward(kp, mode, s));
    if (out0) {
        size_t bytes = (mode == 0) ? nd * 4 : (mode == 3 ? (size_t)B * 11 * 4 : (size_t)B * 4);
        HIP_TRY(hipMemcpyAsync(out0, d + o_out0, bytes, hipMemcpyDeviceToHost, s));
    }
    if (out1) HIP_TRY(hipMemcpyAsync(out1, d + o_out1, nd * 4, hipMemcpyDeviceToHost, s));
    if (ok) HIP_TRY(hipMemcpyAsync(ok, d + o_ok, (size_t)B, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return IRM_OK;
}

}  // namespace

int irm_evaluate(irm_ctx* c, const float* alpha, int32_t B, int32_t which, float* out) {
    if (!c || !out) return fail(IRM_EINVAL, "irm_evaluate: null argument");
    return run_forward(c, 0, alpha, nullptr, nullptr, nullptr, 0, B, 0.f, 0.f, 0.f, which ? 1 : 0, out, nullptr,
                       nullptr);
}

int irm_eval_cost(irm_ctx* c, const float* alpha, const float* start, const float* goal, const float* obstacles,
                  int32_t O, int32_t B, float lsg, float ljl, float lmax, float* cost_out) {
    if (!c || !cost_out || !start || !goal) return fail(IRM_EINVAL, "irm_eval_cost: null argument");
    return run_forward(c, 1, alpha, start, goal, obstacles, O, B, lsg, ljl, lmax, 0, cost_out, nullptr, nullptr);
}

int irm_eval_cost_grad(irm_ctx* c, const float* alpha, const float* start, const float* goal, const float* obstacles,
                       int32_t O, int32_t B, float lsg, float ljl, float lmax, float* grad_out, float* cost_out) {
    if (!c || !grad_out || !start || !goal) return fail(IRM_EINVAL, "irm_eval_cost_grad: null argument");
    return run_forward(c, 2, alpha, start, goal, obstacles, O, B, lsg, ljl, lmax, 0, cost_out, grad_out, nullptr);
}

int irm_constraints(irm_ctx* c, const float* alpha, const float* start, const float* goal, int32_t B, uint8_t* ok_out,
                    float* report_out) {
    if (!c || !ok_out || !start || !goal) return fail(IRM_EINVAL, "irm_constraints: null argument");
    return run_forward(c, 3, alpha, start, goal, nullptr, 0, B, 0.f, 0.f, 0.f, 0, report_out, nullptr, ok_out);
}

int irm_fk(irm_ctx* c, const float* traj, int32_t B, float* pos_out, float* jac_out) {
    if (!c || !traj || !pos_out) return fail(IRM_EINVAL, "irm_fk: null argument");
    if (set_device(c)) return IRM_EDEVICE;
    if (B <= 0) return B == 0 ? IRM_OK : fail(IRM_EINVAL, "negative batch");
    const int N = c->N, D = c->D;
    const size_t nd = (size_t)B * N * D;
    Stage st{c};
    const size_t o_q = st.take(nd * 4), o_p = st.take((size_t)B * 2 * N * 4), o_j = st.take(2 * nd * 4);
    if (ensure_io(c, st.off)) return IRM_ENOMEM;
    char* d = st.base();
    KParams kp = c->kp;
    kp.B = B;
    HIP_TRY(hipMemcpyAsync(d + o_q, traj, nd * 4, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(irm::launch_fk(kp, (const float*)(d + o_q), (float*)(d + o_p), jac_out ? (float*)(d + o_j) : nullptr,
                           c->stream));
    HIP_TRY(hipMemcpyAsync(pos_out, d + o_p, (size_t)B * 2 * N * 4, hipMemcpyDeviceToHost, c->stream));
    if (jac_out) HIP_TRY(hipMemcpyAsync(jac_out, d + o_j, 2 * nd * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return IRM_OK;
}

int irm_fk_joints(irm_ctx* c, const float* traj, int32_t B, float* pos_out) {
    if (!c || !traj || !pos_out) return fail(IRM_EINVAL, "irm_fk_joints: null argument");
    if (set_device(c)) return IRM_EDEVICE;
    if (B <= 0) return B == 0 ? IRM_OK : fail(IRM_EINVAL, "negative batch");
    const int N = c->N, D = c->D;
    const size_t nd = (size_t)B * N * D;
    Stage st{c};
    const size_t o_q = st.take(nd * 4), o_p = st.take(2 * nd * 4);
    if (ensure_io(c, st.off)) return IRM_ENOMEM;
    char* d = st.base();
    KParams kp = c->kp;
    kp.B = B;
    HIP_TRY(hipMemcpyAsync(d + o_q, traj, nd * 4, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(irm::launch_fk_joints(kp, (const float*)(d + o_q), (float*)(d + o_p), c->stream));
    HIP_TRY(hipMemcpyAsync(pos_out, d + o_p, 2 * nd * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return IRM_OK;
}

int irm_compute_cost_vg(irm_ctx* c, const float* f, const float* obstacles, int32_t O, int32_t B, float* cost_v,
                        float* cost_g) {
    if (!c || !f || !cost_v || (O > 0 && !obstacles)) return fail(IRM_EINVAL, "irm_compute_cost_vg: null argument");
    if (check_obs(O)) return IRM_EINVAL;
    if (set_device(c)) return IRM_EDEVICE;
    if (B <= 0) return B == 0 ? IRM_OK : fail(IRM_EINVAL, "negative batch");
    const int N = c->N;
    Stage st{c};
    const size_t o_f = st.take((size_t)B * 2 * N * 4), o_o = st.take((size_t)std::max(O, 1) * 8),
                 o_v = st.take((size_t)B * N * 4), o_g = st.take((size_t)B * 2 * N * 4);
    if (ensure_io(c, st.off)) return IRM_ENOMEM;
    char* d = st.base();
    KParams kp = c->kp;
    kp.B = B;
    kp.O = O;
    kp.obstacles = (const float*)(d + o_o);
    HIP_TRY(hipMemcpyAsync(d + o_f, f, (size_t)B * 2 * N * 4, hipMemcpyHostToDevice, c->stream));
    if (O > 0) HIP_TRY(hipMemcpyAsync(d + o_o, obstacles, (size_t)O * 8, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(irm::launch_cost_vg(kp, (const float*)(d + o_f), (float*)(d + o_v), cost_g ? (float*)(d + o_g) : nullptr,
                                c->stream));
    HIP_TRY(hipMemcpyAsync(cost_v, d + o_v, (size_t)B * N * 4, hipMemcpyDeviceToHost, c->stream));
    if (cost_g) HIP_TRY(hipMemcpyAsync(cost_g, d + o_g, (size_t)B * 2 * N * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return IRM_OK;
}

int irm_init_alpha(irm_ctx* c, const float* start, const float* goal, int32_t B, float* alpha_out) {
    if (!c || !start || !goal || !alpha_out) return fail(IRM_EINVAL, "irm_init_alpha: null argument");
    if (set_device(c)) return IRM_EDEVICE;
    if (B <= 0) return B == 0 ? IRM_OK : fail(IRM_EINVAL, "negative batch");
    const int N = c->N, D = c->D;
    const size_t nd = (size_t)B * N * D;
    Stage st{c};
    const size_t o_s = st.take((size_t)B * D * 4), o_g = st.take((size_t)B * D * 4), o_a = st.take(nd * 4);
    if (ensure_io(c, st.off)) return IRM_ENOMEM;
    char* d = st.base();
    KParams kp = c->kp;
    kp.B = B;
    kp.start = (const float*)(d + o_s);
    kp.goal = (const float*)(d + o_g);
    HIP_TRY(hipMemcpyAsync(d + o_s, start, (size_t)B * D * 4, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(d + o_g, goal, (size_t)B * D * 4, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(irm::launch_init_alpha(kp, (float*)(d + o_a), c->stream));
    HIP_TRY(hipMemcpyAsync(alpha_out, d + o_a, nd * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return IRM_OK;
}

int irm_optimize_batch_dev(irm_ctx* c, const irm_batch_dev* a, void* stream) {
    if (!c || !a) return fail(IRM_EINVAL, "irm_optimize_batch_dev: null argument");
    if (a->batch < 0 || !a->start || !a->goal) return fail(IRM_EINVAL, "bad batch arguments");
    if (check_obs(a->n_obstacles) || check_stride(a->n_obstacles, a->obstacle_stride)) return IRM_EINVAL;
    if (a->n_obstacles > 0 && !a->obstacles) return fail(IRM_EINVAL, "obstacles pointer missing");
    if (set_device(c)) return IRM_EDEVICE;
    if (a->batch == 0) return IRM_OK;
    KParams kp = c->kp;
    kp.B = a->batch;
    kp.O = a->n_obstacles;
    kp.obs_stride = a->obstacle_stride;
    kp.alpha0 = a->alpha0;
    kp.start = a->start;
    kp.goal = a->goal;
    kp.obstacles = a->obstacles;
    kp.alpha_out = a->alpha_out;
    kp.traj_out = a->traj_out;
    kp.stats = a->stats_out;
    kp.series = a->series_out;
    kp.trace = c->d_trace;
    kp.trace_cap = c->trace_cap;
    if (choose_shape(c, a->batch, true, kp, nullptr) <= 0) return fail(IRM_EINVAL, "no workgroup shape fits LDS");
#if defined(IRM_PHASE_PROFILE) || defined(IRM_DIV_CHECK)
    {  // (IRM_DIV_CHECK: per-block counters of the BLS division check, zeroed per launch)
        const int grid = (a->batch + kp.TB - 1) / kp.TB;
        if (grid > c->prof_cap) {
            if (c->d_prof) (void)hipFree(c->d_prof);
            c->d_prof = nullptr;
            HIP_TRY(hipMalloc(&c->d_prof, (size_t)grid * irm::kProfPhases * sizeof(unsigned long long)));
            c->prof_cap = grid;
        }
        c->prof_blocks = grid;
        kp.prof = c->d_prof;
#ifdef IRM_DIV_CHECK
        HIP_TRY(hipMemsetAsync(c->d_prof, 0, (size_t)grid * irm::kProfPhases * sizeof(unsigned long long), (hipStream_t)stream));
#endif
    }
#endif
    HIP_TRY(irm::launch_optimize(kp, (hipStream_t)stream));
    return IRM_OK;
}

int irm_optimize_plan(const irm_ctx* c, int32_t batch, int32_t n_obstacles, int32_t record_series,
                      irm_launch_plan* out) {
    if (!c || !out || batch <= 0) return fail(IRM_EINVAL, "irm_optimize_plan: bad argument");
    if (check_obs(n_obstacles)) return IRM_EINVAL;
    memset(out, 0, sizeof(*out));
    KParams kp = c->kp;
    kp.B = batch;
    kp.O = n_obstacles;
    // the series flow runs when the context records it (irm_params.record_series) or the call asks
    // for the series (irm_optimize_batch with series_out) — as in irm_optimize_batch(_dev)
    kp.record_series = (c->kp.record_series || record_series) ? 1 : 0;
    if (choose_shape(c, batch, true, kp, nullptr) <= 0) return fail(IRM_EINVAL, "no workgroup shape fits LDS");
    irm::LaunchDesc d{};
    d.describe_only = true;
    HIP_TRY(irm::launch_optimize(kp, nullptr, &d));  // the dispatch fills d and launches nothing
    snprintf(out->kernel, sizeof(out->kernel), "%s", d.kernel);
    out->lean = d.lean;
    out->flow = d.flow;
    out->waypoints_per_lane = d.wpl;
    out->threads = d.threads;
    out->grid = d.grid;
    out->lds_bytes = d.lds_bytes;
    out->traj_per_block = d.traj_per_block;
    out->rank_z = d.rank_z;
    out->rank_dir = d.rank_dir;
    out->rank_g = d.rank_g;
    out->lam16 = c->lam16;
    out->lam24 = c->lam24;
    return IRM_OK;
}

const char* irm_build_id(void) {
#ifdef IRM_SOURCE_HASH
    return IRM_SOURCE_HASH;
#else
    return "unknown";
#endif
}

int irm_optimize_batch(irm_ctx* c, const float* alpha0, const float* start, const float* goal, const float* obstacles,
                       int32_t O, int32_t obstacle_stride, int32_t B, float* alpha_out, float* traj_out,
                       irm_stats* stats_out, float* series_out) {
    if (!c || !start || !goal) return fail(IRM_EINVAL, "irm_optimize_batch: null argument");
    if (check_obs(O) || check_stride(O, obstacle_stride)) return IRM_EINVAL;
    if (set_device(c)) return IRM_EDEVICE;
    if (B <= 0) return B == 0 ? IRM_OK : fail(IRM_EINVAL, "negative batch");
    const int N = c->N, D = c->D;
    const size_t nd = (size_t)B * N * D;
    const size_t nobs = obstacle_stride ? (size_t)B * obstacle_stride : (size_t)O * 2;
    const size_t nser = series_out ? (size_t)B * c->max_series * N * D : 0;
    Stage st{c};
    const size_t o_a0 = st.take(nd * 4), o_s = st.take((size_t)B * D * 4), o_g = st.take((size_t)B * D * 4),
                 o_o = st.take(std::max<size_t>(nobs, 1) * 4), o_ao = st.take(nd * 4), o_to = st.take(nd * 4),
                 o_st = st.take((size_t)B * sizeof(irm_stats)), o_se = st.take(std::max<size_t>(nser, 1) * 4);
    if (ensure_io(c, st.off)) return IRM_ENOMEM;
    char* d = st.base();
    hipStream_t s = c->stream;
    if (alpha0) HIP_TRY(hipMemcpyAsync(d + o_a0, alpha0, nd * 4, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d + o_s, start, (size_t)B * D * 4, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d + o_g, goal, (size_t)B * D * 4, hipMemcpyHostToDevice, s));
    if (nobs && obstacles) HIP_TRY(hipMemcpyAsync(d + o_o, obstacles, nobs * 4, hipMemcpyHostToDevice, s));
    irm_batch_dev a{};
    a.alpha0 = alpha0 ? (const float*)(d + o_a0) : nullptr;
    a.start = (const float*)(d + o_s);
    a.goal = (const float*)(d + o_g);
    a.obstacles = (const float*)(d + o_o);
    a.n_obstacles = O;
    a.obstacle_stride = obstacle_stride;
    a.batch = B;
    a.alpha_out = (float*)(d + o_ao);
    a.traj_out = (float*)(d + o_to);
    a.stats_out = (irm_stats*)(d + o_st);
    a.series_out = series_out ? (float*)(d + o_se) : nullptr;
    KParams save = c->kp;
    if (series_out) c->kp.record_series = 1;
    int rc = irm_optimize_batch_dev(c, &a, s);
    c->kp = save;
    if (rc) return rc;
    if (alpha_out) HIP_TRY(hipMemcpyAsync(alpha_out, d + o_ao, nd * 4, hipMemcpyDeviceToHost, s));
    if (traj_out) HIP_TRY(hipMemcpyAsync(traj_out, d + o_to, nd * 4, hipMemcpyDeviceToHost, s));
    if (stats_out) HIP_TRY(hipMemcpyAsync(stats_out, d + o_st, (size_t)B * sizeof(irm_stats), hipMemcpyDeviceToHost, s));
    if (series_out) HIP_TRY(hipMemcpyAsync(series_out, d + o_se, nser * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return IRM_OK;
}

}  // extern "C"
