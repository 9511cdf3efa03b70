// irm_kernels.hpp — launch-side interface between the C-ABI host code
// (irm_host.cpp) and the gfx950 kernels (irm_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/irm.h"

namespace irm {

constexpr int kCols = 16;         // MFMA 16x16x4 column tile = TB·D columns
constexpr int kLd = 17;           // LDS row stride of [row][16] buffers: odd, so a lane-per-row
                                  // access (lane n → row n) hits 32 different banks
constexpr int kMaxThreads = 1024; // one lane per (trajectory, waypoint): TB·NW ≤ 1024

// Per-trajectory phases of the on-device optimiser state machine.
// PH_RESYNC: an inner loop has ended; α is materialised in fp32, [T; V] is
// re-evaluated from it exactly and constraintsFulfilled(α) decides the outer step.
enum Phase : int32_t {
    PH_OUTER_START = 0,
    PH_GD_INNER = 1,
    PH_BLS_TRIAL = 2,
    PH_DONE = 3,
    PH_BLS_REEVAL = 4,
    PH_RESYNC = 5
};

// Everything a kernel needs, passed by value (kernarg segment).
struct KParams {
    // shapes
    int32_t N, D, R, TB, B, O, obs_stride;
    int32_t NK;   // N rounded up to 16 (k extent of N-contractions)
    int32_t MP;   // 2·NK: rows of [K; dK] / [a; b] / [T; V], velocity half from row NK
    int32_t RP;   // R (multiple of 16)
    int32_t ops_in_lds;  // operator fragments staged into LDS
    int32_t NW;          // lanes per trajectory = N rounded up to 64 (whole waves)
    int32_t BT;          // threads per workgroup = TB·NW
    int32_t nsplit;      // stage-1 split-K factor
    int32_t regops;      // operator A-fragments held in VGPRs (k_optimize<…, REGOPS>)
    int32_t v_ident;     // V_R = I (dense operator, --operator-rank -1): G = y'' rows, no G-tile MFMAs
    // optimiser
    int32_t optimizer, max_inner, max_outer, max_bls, cvdl, record_series, max_series;
    int32_t lean_ok;  // k_gd_single may serve GD single-loop launches (IRM_GENERAL_KERNEL=1 clears it)
    int32_t lean_wpl; // diagnostics: IRM_LEAN_WPL=2 forces two waypoints per lane at N ≤ 128
    int32_t lean_nohelp;  // diagnostics: IRM_LEAN_NOHELP=1 turns k_lean's BLS line-search helpers off
    int32_t trace_b;      // diagnostics: the batch index whose line search is logged (IRM_TRACE_PROBLEM, default 0)
    float llr, lci, lsg0, ljl0, eps_p, eps_v, lmax, lreg;
    float bls_lr0, bls_a, bls_bp, bls_bm, vmax, pmax, pmin, pad1;
    // derived fp32 constants (reference casts its Python doubles to fp32)
    float mean_pos, std_pos, std2, vmax2, thr_hi, thr_lo, thr_v, invN;
    float inv_std_pos, inv_vmax, inv_std2, inv_vmax2;  // reciprocals: x/c → x·(1/c) in the hot loops
    uint32_t Nmagic, NDmagic;  // ⌈2³²/N⌉, ⌈2³²/(N·D)⌉: exact __umulhi division for dividends < 2¹⁶
    float gd_lr[IRM_MAX_LR];
    float gd_c[IRM_MAX_LR];  // GD weight decay fp32(1 − λ_reg·lr_k), from the Python doubles (optimizer_GD.py:81)
    float link[IRM_MAX_JOINTS];
    float J[IRM_MAX_JOINTS * IRM_MAX_JOINTS];    // J (D×D, row-major, stride D)
    float JtJ[IRM_MAX_JOINTS * IRM_MAX_JOINTS];  // JᵀJ
    float Jinv[IRM_MAX_JOINTS * IRM_MAX_JOINTS]; // J⁻¹
    float Minv[IRM_MAX_JOINTS * IRM_MAX_JOINTS]; // (JᵀJ)⁻¹
    float wal[IRM_MAX_JOINTS];                   // (JᵀJ)⁻¹·Jᵀ1: alpha_norm·‖G‖ = Σ_r (y'_r·wal)²
    // operators (device, fp32)
    const float* Km;      // K, row-major                 (N × N)
    const float* dKm;     // dK, row-major                (N × N)
    const float* Kt;      // Kᵀ, row-major                (N × N)
    const float* dKt;     // dKᵀ, row-major               (N × N)
    const float* F1frag;  // A-fragments of Fᵀ            (RP × MP)
    const float* F2frag;  // A-fragments of F             (MP × RP)
    const float* F1p;     // Fᵀ / F in the k-permuted fragment layout (frag_index_kp) of the
    const float* F2p;     //   lean kernel, whose B operands are 4 consecutive rows per lane
    const float* Fbot;    // F rows N..2N-1, row-major    (N × RP)
    const float* Vr;      // V_R, row-major               (N × RP)
    const float* Hend;    // F·F[NK]ᵀ, F·F[NK+N−1]ᵀ: operator columns of the endpoint velocity rows (2 × MP)
    // V_R in the k-permuted fragment layouts of the lean kernel's fp32-α rounding terms
    const float* VTp;     // V_Rᵀ (RP × NK): z = V_Rᵀ·e' (the rounding residual of α into waypoint space)
    const float* VNp;     // V_R (NK × RP):  G = V_R·y'·J⁻¹ (the α-space gradient, per waypoint)
    const float* HV;      // V_R·F[NK]ᵀ, V_R·F[NK+N−1]ᵀ: G's endpoint velocity columns (2 × NK)
    const float* VTs;     // V_Rᵀ / V_R in the standard fragment layout (frag_index) of the general
    const float* VNs;     //   kernel's GD rounding terms
    const float* uvec;    // K⁻¹(1-c)   (N)  initTrajectory basis
    const float* wvec;    // K⁻¹c       (N)
    // batch I/O
    const float* alpha0;
    const float* start;
    const float* goal;
    const float* obstacles;
    float* alpha_out;
    float* traj_out;
    irm_stats* stats;
    float* series;
    // cost weights of the current call (optimiser: lam_max = --lambda-max-cost)
    float lam_sg, lam_jl, lam_max, one_m_lmax;  // one_m_lmax = fp32(1 − λmax in double)
    int32_t which;
    int32_t whole_robot;  // obstacle cost over every joint position (irm_params.whole_robot_cost)
    float* out0;   // evaluate: B×N×D; cost: B; constraints report: B×11
    float* out1;   // grad: B×N×D
    uint8_t* out_ok;
    unsigned long long* prof;  // IRM_PHASE_PROFILE builds: per-block phase cycle counters
    // diagnostics: BLS line-search log of problem 0 (irm_debug_bls_trace), kTraceW floats per trial
    float* trace;
    int32_t trace_cap;
};

constexpr int kTraceW = 10;  // outer, inner, trial, lr, new_loss, required_loss, accepted, loss, ‖g‖, alpha_norm

constexpr int kProfPhases = 24;

// Operator fragment sizes (floats) for the layout of mfma_frag_index.
__host__ __device__ inline int64_t frag_floats(int M, int K) {
    int MT = (M + 15) / 16, KQ = (K + 15) / 16;
    return (int64_t)MT * KQ * 64 * 4;
}

// Element (row, k) of a row-major M×K matrix in the 16x16x4 A-fragment layout:
// block (row/16, k/16), lane = row%16 + 16*(k%4), float slot j = (k%16)/4.
__host__ __device__ inline int64_t frag_index(int row, int k, int K) {
    int KQ = (K + 15) / 16;
    int mt = row / 16, kq = k / 16, kk = k % 16;
    int lane = (row % 16) + 16 * (kk % 4), j = kk / 4;
    return (((int64_t)mt * KQ + kq) * 64 + lane) * 4 + j;
}

// k-permuted variant: MFMA j of k-group kq takes k = 16·kq + 4·(lane>>4) + j, so a lane's four
// B values of a k-group are 4 consecutive rows (one ds_read_b128 from a column-major buffer).
__host__ __device__ inline int64_t frag_index_kp(int row, int k, int K) {
    int KQ = (K + 15) / 16;
    int mt = row / 16, kq = k / 16, kk = k % 16;
    int lane = (row % 16) + 16 * (kk / 4), j = kk % 4;
    return (((int64_t)mt * KQ + kq) * 64 + lane) * 4 + j;
}

// LDS layout of the optimiser / eval workgroups (float offsets, 16-B aligned).
struct Plan {
    int f1, f2, fb;              // staged operators F_topᵀ, F, F_bot (optimiser, ops_in_lds)
    int alist, acnt;             // per-wave lists of active sparse rows (optimiser)
    int X, Bs;                   // MFMA B operand: a (NK × 16) and b (N × 16) / [a; b] (MP × 16)
    int dP;                      // MFMA output rows (MP × 16)
    int Ypart, Ydir, Ymix, Yacc; // stage-1 partials, y, y·JᵀJ, Σ steps·y
    int red, sg, wp;             // wave partials, start/goal rows, BLS Gram partials
    int flags, act, list;        // per-trajectory flags, active sparse rows
    int obs;                     // obstacles (shared or per trajectory)
    int total;
};

__host__ __device__ constexpr int al4(int x) { return (x + 3) & ~3; }

// Head of the LDS layout: every region whose size depends only on the shape
// (MP, RP, nsplit), plus fixed-capacity per-wave / per-trajectory records, so that
// a shape-specialised kernel sees compile-time offsets.  Obstacles follow; the
// staged operator fragments (non-REGOPS, ops_in_lds) come last.
constexpr int kMaxWaves = kMaxThreads / 64;
constexpr int kMaxTraj = kCols;  // TB·D ≤ 16
struct Head {
    int X, dP, Ypart, Ymix, red, sg, wp, flags, cold, obs;
};
// LDS "cold" parameter block of k_optimize (word offsets)
enum ColdWord : int {
    C_GDLR = 0,  // IRM_MAX_LR words
    C_LCI = 32, C_EPSP, C_EPSV, C_PMAX, C_PMIN, C_VMAX, C_BLR0, C_BA, C_BP, C_BM, C_MAXOUT, C_MAXBLS, C_MAXSER,
    C_TRCAP = 45,   // line-search log capacity (records)
    C_PTR = 46,     // 5 pointers × 2 words: series, Vr, Kt, dKt, trace
    C_MINV = 56,    // (JᵀJ)⁻¹, D×D
    C_WAL = 120,    // D
    C_JINV = 128,   // J⁻¹, D×D
    C_J = 192,      // J, D×D
    kColdWords = 256
};
// column stride of k_lean's stage-1 partials ([split][column][r]): ≡ 8 mod 64 like its other strides
// (conflict-free b128 tile reads and stores with the row swizzle r ^ (c & 4), see k_lean)
__host__ __device__ constexpr int lean_ldy(int RP) { return RP + 8 + (64 - (RP + 8) % 64 + 8) % 64; }
// lean: the layout of k_lean (stage-1 partials [split][column][r], stride lean_ldy(RP)) instead of
// k_optimize's [split][r][column] (stride kLd) — 640 instead of 544 floats per split at RP = 32,
// which decides whether N = 512 fits the general kernel's 160 KiB.
__host__ __device__ constexpr Head plan_head(int MP, int RP, int nsplit, bool optimizer, bool lean = false) {
    Head H{};
    H.X = 0;
    H.dP = H.X + al4(MP * kLd);
    int off = H.dP + al4(MP * kLd);
    H.Ypart = H.Ymix = 0;
    if (optimizer) {
        H.Ypart = off;
        off += al4(nsplit * (lean ? 16 * lean_ldy(RP) : RP * kLd));
        H.Ymix = off;
        off += al4(RP * kLd);
    }
    H.red = off;
    off += kMaxWaves * 8;
    H.sg = off;
    off += kMaxTraj * 4;
    H.wp = off;
    off += kMaxWaves * 2;
    H.flags = off;
    off += 8;
    H.cold = 0;
    if (optimizer) {
        H.cold = off;
        off += kColdWords;
    }
    H.obs = off;
    return H;
}

__host__ __device__ inline Plan plan_lds(const KParams& p, bool ops_lds, bool optimizer, bool lean = false) {
    const Head H = plan_head(p.MP, p.RP, p.nsplit, optimizer, lean);
    Plan L{};
    L.X = H.X;
    L.Bs = L.X + p.NK * kLd;
    L.dP = H.dP;
    L.Ypart = H.Ypart;
    L.Ymix = H.Ymix;
    L.Ydir = L.Yacc = L.alist = L.acnt = L.act = L.list = L.fb = 0;
    L.red = H.red;
    L.sg = H.sg;
    L.wp = H.wp;
    L.flags = H.flags;
    L.obs = H.obs;
    int off = H.obs + al4((p.obs_stride ? p.TB : 1) * ((p.O + 3) & ~3) * 2 + 4);
    L.f1 = L.f2 = 0;
    if (optimizer && ops_lds && !p.regops) {  // with REGOPS the A-fragments live in VGPRs
        L.f1 = off;
        off += al4((int)frag_floats(p.RP, p.MP));
        L.f2 = off;
        off += al4((int)frag_floats(p.MP, p.RP));
    }
    L.total = off;
    return L;
}


// LDS of the lean kernel (k_lean) beyond the optimiser head + obstacles (`base`): the V_R fragments
// (when staged: vlds), the rounding residual rows e' ([column][waypoint], stride NK + 8), its stage-1
// partials zp ([split][column][r], stride RP + 8), the gradient rows G ([column][waypoint]) and the
// compact endpoint velocity rows ep ([trajectory][2][kEpS]) + a zero word.
// k-splits of k_lean's residual projection z = V_Rᵀ·e' (rank 16: one row tile, see k_lean): twice
// the stage-1 splits where the LDS allows (vlds shapes: N ≤ 128, D ≤ 3), so the units stay one per wave
__host__ __device__ constexpr int lean_zsplit(int nsplit, bool vlds) { return vlds ? 2 * nsplit : nsplit; }
struct LeanX {
    int vt, vn, eb, zp, gb, ep, ep0, ss, hp, aj, ts, total;
};
// BLS flow of k_lean: the trial's residual projection z = V_Rᵀ·e' is formed by the G-tile waves, one
// partial per wave, stored quad-major (partial w, row quad rq, column c at w·256 + rq·64 + c·4: a lane's
// f32x4 of an MFMA tile — b128 stores and B-operand reads conflict-free); at most 8 waves (MAXT ≤ 512)
__host__ __device__ constexpr int lean_bls_nzp(int NK) { return NK / 16 < 8 ? NK / 16 : 8; }
// per-slot trial scalars of the BLS flow (TS): lr, ‖G‖, "in a line search" flag, spare
constexpr int kTsW = 4;
// compact copy of each trajectory's endpoint velocity rows b'[0], b'[N−1] of X (k_lean): kEpS floats each
constexpr int kEpS = 8;
__host__ __device__ constexpr int lean_ld(int NK) { return NK + 8; }
// help_threads > 0: the BLS line-search helpers' exchange regions (k_lean, kHelp): a trajectory's α, T, V
// rows by thread ([3·D][threads], ss) and its per-round scalars (8 words per trajectory slot, hp)
constexpr int kHpW = 8;
// bls: the BLS flow's regions — α rows (Ab, in e.eb's place), the trial iterate's rows (Aj), the z partials
// (quad-major, lean_bls_nzp) and the per-slot trial scalars (TS) instead of the GD flows' e' / z regions
__host__ __device__ inline LeanX lean_extra(int base, int MP, int NK, int RP, int nsplit, bool vlds, int D = 0,
                                            int help_threads = 0, bool bls = false, bool dense = false) {
    LeanX e{};
    int off = base;
    e.vt = e.vn = 0;
    if (vlds) {
        e.vt = off;
        off += al4((int)frag_floats(RP, NK));
        e.vn = off;
        off += al4((int)frag_floats(NK, RP));
    }
    e.eb = off;
    off += al4(16 * lean_ld(NK));
    e.aj = e.ts = 0;
    if (bls) {
        e.aj = off;
        off += al4(16 * lean_ld(NK));
        e.zp = off;
        off += lean_bls_nzp(NK) * 256;
        e.ts = off;
        off += kMaxTraj * kTsW;
    } else if (!dense) {
        e.zp = off;
        off += al4(lean_zsplit(nsplit, vlds) * 16 * lean_ldy(RP));
    }
    e.gb = off;  // (dense: G is y'' itself — no G rows, no z partials)
    if (!dense) off += al4(16 * lean_ld(NK));
    e.ep = off;
    off += kMaxTraj * 2 * kEpS;
    e.ep0 = off;  // one zero word (the endpoint MFMA's B for k = 2, 3)
    off += 4;
    e.ss = e.hp = 0;
    if (help_threads > 0) {
        e.ss = off;
        off += al4(3 * D * help_threads);
        e.hp = off;
        off += kMaxTraj * kHpW;
    }
    e.total = off;
    return e;
}
// V_R fragments staged in LDS for the lean kernel: N ≤ 128 at D ≤ 3 in 512-thread workgroups (117 KiB
// at N = 128).  256-thread workgroups run two per CU (76 KiB each without them) and every N = 256
// shape reads them from L2 instead: LDS budget.
__host__ __device__ constexpr bool lean_vlds(int NK, int D, int threads) { return NK <= 128 && D <= 3 && threads > 256; }

// Stage-1 split-K factor: units of 4 k-quads over the position half.
__host__ __device__ constexpr int stage1_splits(int NK) { return (NK / 16 + 3) / 4; }

// Can the operator A-fragments live in VGPRs (k_optimize<…, REGOPS=true>)?
// Mirrors kS1Q / kS2T in irm_kernels.hip.
inline bool regops_fit(const KParams& p) {
    const int nw = p.BT / 64, MT1 = p.RP / 16, KQa = p.NK / 16, KQ2 = p.RP / 16, MT2 = p.MP / 16;
    if (p.BT > 512 || KQ2 > 2 || MT1 * p.nsplit > nw) return false;
    const int s1q = p.BT <= 256 ? 8 : 4, s2t = p.BT <= 256 ? 8 : 2;  // kS1Q / kS2T
    const int kq_per_unit = (KQa + p.nsplit - 1) / p.nsplit;  // stage 1 keeps the position half in VGPRs
    const int tiles_per_wave = (MT2 + nw - 1) / nw;
    return kq_per_unit <= s1q && tiles_per_wave <= s2t;
}

// What an optimiser launch runs, filled in by the launch dispatch itself (launch_optimize_shape), so
// that irm_optimize_plan reports the kernel that a launch of the same arguments would run — not a
// re-derivation of the dispatch rules.  describe_only: fill the record, launch nothing.
struct LaunchDesc {
    bool describe_only;
    char kernel[128];  // template instance, e.g. "k_lean<FixShape<3,128,32>,512,1,FULL,GD1>"
    int lean;          // 1: k_lean, 0: k_optimize
    int flow;          // 0 GD single loop, 1 GD dual loop, 2 BLS (the lean kernel's LeanFlow)
    int wpl;           // waypoints per lane
    int threads, grid, lds_bytes, traj_per_block;
    int rank_z, rank_dir, rank_g;  // operator rank of the residual projection, the waypoint direction, G
};

// launchers (return hipError_t)
hipError_t launch_init_alpha(const KParams& p, float* alpha_out, hipStream_t s);
hipError_t launch_optimize(const KParams& p, hipStream_t s, LaunchDesc* desc = nullptr);
hipError_t launch_forward(const KParams& p, int mode, hipStream_t s);  // mode: 0 evaluate, 1 cost, 2 cost+grad, 3 constraints
hipError_t launch_fk(const KParams& p, const float* traj, float* pos, float* jac, hipStream_t s);
hipError_t launch_fk_joints(const KParams& p, const float* traj, float* pos, hipStream_t s);
hipError_t launch_cost_vg(const KParams& p, const float* f, float* cv, float* cg, hipStream_t s);

}  // namespace irm
