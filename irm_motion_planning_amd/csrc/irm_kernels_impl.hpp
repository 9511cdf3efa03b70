// irm_kernels_impl.hpp — gfx950 (CDNA4) kernel templates of the RKHS trajectory optimiser.
// Included by irm_kernels.hip (host-API kernels, launch dispatch) and by the instantiation
// units irm_opt_inst.hip (one k_optimize shape / k_forward D per object, compiled in parallel).
//
// Hot path of simongroeger/irm_motion_planning: optimizer_GD.py:173-232 and
// optimizer_BLS.py:126-213 over trajectory.py:271-297 / robot.py:29-87 /
// environment.py:32-58.  DESIGN.md describes the formulation:
//   * the optimiser state is kept in trajectory space, T = K·α·J and
//     V = dK·α·J (the reference keeps α, |α|≈1e3, which cancels in fp32);
//   * the α-space step α' = c·α − s·G, G = (Kᵀa + dKᵀb)Jᵀ, becomes
//     [T';V'] = c·[T;V] − s·L·Lᵀ[a;b]·JᵀJ with L = [K;dK];
//   * L·Lᵀ is applied as F·(Fᵀ[a;b]) with F = L·V_R (V_R = top-R right
//     singular vectors of L; R = N, V = I is the exact dense operator);
//   * both contractions run on v_mfma_f32_16x16x4_f32 with the TB·D
//     (trajectory, joint) columns of a workgroup as the 16 MFMA columns;
//   * one lane per (trajectory, waypoint): the trajectory's waypoints and
//     velocities live in that lane's registers for the whole optimisation;
//     FK / obstacle potential / penalties are VALU, per-trajectory
//     reductions are DPP wave reductions + a cross-wave LDS combine;
//   * the GD / BLS control flow is a per-trajectory state machine whose
//     scalar state is replicated in the trajectory's lanes (every lane takes
//     the same decision from the same reduced values), inside one persistent
//     launch per optimize().
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>

#include <type_traits>

#include "irm_kernels.hpp"

namespace irm {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// The kernels are compiled with -ffp-contract=off (build.py): every fused multiply-add is written
// as one, so the arithmetic does not depend on the compiler's contraction choices.
__device__ __forceinline__ f32x2 pkfma(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }

// ------------------------------------------------------------ LDS planning

// ------------------------------------------------------------ wave helpers
// DPP row reductions (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror,
// row_mirror) leave each 16-lane row reduced in all its lanes; the four
// rows are then combined from v_readlane (uniform result, no LDS).
// Every control used here is an in-row permutation (no lane reads outside its row), so the old value
// is never kept: mov_dpp (old undefined, bound_ctrl) lets the compiler fold the move into the consuming
// VALU op as a DPP source (v_add_f32_dpp …) instead of v_mov_b32 + v_mov_b32_dpp + the op.
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
    static_assert(CTRL == 0xB1 || CTRL == 0x4E || CTRL == 0x141 || CTRL == 0x140, "in-row permutations only");
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
template <int CTRL>
__device__ __forceinline__ int dppi(int v) {
    static_assert(CTRL == 0xB1 || CTRL == 0x4E || CTRL == 0x141 || CTRL == 0x140, "in-row permutations only");
    return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, true);
}
// s + (row_bcast:15 of s) in rows 1 and 3 (ROW = 15), s + (row_bcast:31 of s) in rows 2 and 3 (ROW = 31);
// the other rows keep s.  As one v_add_f32_dpp (the compiler's DPP combine leaves the float add with a
// partial row mask as a v_mov_b32_dpp + v_add_f32 pair); s_nop 1: the VALU-write → DPP-read hazard.
template <int ROW>
__device__ __forceinline__ float bcast_add(float s) {
    static_assert(ROW == 15 || ROW == 31, "row broadcasts");
    if constexpr (ROW == 15)
        asm volatile("s_nop 1\n\tv_add_f32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf" : "+v"(s));
    else
        asm volatile("s_nop 1\n\tv_add_f32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf" : "+v"(s));
    return s;
}
// max of floats that are ≥ +0 or −inf, on their bit patterns (signed-int order = float order there):
// no NaN canonicalisation, and the DPP move folds into v_max_i32_dpp
__device__ __forceinline__ float maxpos(float a, float b) {
    return __int_as_float(max(__float_as_int(a), __float_as_int(b)));
}
__device__ __forceinline__ float lanef(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ float wred_sum(float v) {
    v += dppf<0xB1>(v);
    v += dppf<0x4E>(v);
    v += dppf<0x141>(v);
    v += dppf<0x140>(v);
    return (lanef(v, 0) + lanef(v, 16)) + (lanef(v, 32) + lanef(v, 48));
}
__device__ __forceinline__ float wred_max(float v) {
    v = fmaxf(v, dppf<0xB1>(v));
    v = fmaxf(v, dppf<0x4E>(v));
    v = fmaxf(v, dppf<0x141>(v));
    v = fmaxf(v, dppf<0x140>(v));
    return fmaxf(fmaxf(lanef(v, 0), lanef(v, 16)), fmaxf(lanef(v, 32), lanef(v, 48)));
}
__device__ __forceinline__ float wred_min(float v) {
    v = fminf(v, dppf<0xB1>(v));
    v = fminf(v, dppf<0x4E>(v));
    v = fminf(v, dppf<0x141>(v));
    v = fminf(v, dppf<0x140>(v));
    return fminf(fminf(lanef(v, 0), lanef(v, 16)), fminf(lanef(v, 32), lanef(v, 48)));
}
// max with first-index tie break (jnp.argmax, trajectory.py:97)
__device__ __forceinline__ void amax_step(float& v, int& i, float ov, int oi) {
    if (ov > v || (ov == v && oi < i)) {
        v = ov;
        i = oi;
    }
}
template <int CTRL>
__device__ __forceinline__ void amax_dpp(float& v, int& i) {
    float ov = dppf<CTRL>(v);
    int oi = dppi<CTRL>(i);
    amax_step(v, i, ov, oi);
}
__device__ __forceinline__ void wred_argmax(float& v, int& i) {
    amax_dpp<0xB1>(v, i);
    amax_dpp<0x4E>(v, i);
    amax_dpp<0x141>(v, i);
    amax_dpp<0x140>(v, i);
    float bv = lanef(v, 0);
    int bi = __builtin_amdgcn_readlane(i, 0);
#pragma unroll
    for (int r = 16; r < 64; r += 16) amax_step(bv, bi, lanef(v, r), __builtin_amdgcn_readlane(i, r));
    v = bv;
    i = bi;
}

// ---------------------------------------------------- phase profiler (diag)
// Built with -DIRM_PHASE_PROFILE: thread 0 of each workgroup accumulates the
// shader-clock cycles (s_memtime) between consecutive stamps per phase into
// P.prof[block][phase].  In the shipped build every stamp is empty.
struct Prof {
#ifdef IRM_PHASE_PROFILE
    unsigned long long last, acc[kProfPhases];
    __device__ __forceinline__ void init() {
        last = __builtin_amdgcn_s_memtime();
#pragma unroll
        for (int i = 0; i < kProfPhases; ++i) acc[i] = 0;
    }
    __device__ __forceinline__ void stamp(int ph) {
        unsigned long long now = __builtin_amdgcn_s_memtime();
        acc[ph] += now - last;
        last = now;
    }
    __device__ __forceinline__ void count(int ph, bool c) {
        if (c) acc[ph] += 1;
    }
    __device__ __forceinline__ void flush(unsigned long long* out) {
        if (out)
            for (int i = 0; i < kProfPhases; ++i) out[(size_t)blockIdx.x * kProfPhases + i] = acc[i];
    }
#else
    __device__ __forceinline__ void init() {}
    __device__ __forceinline__ void stamp(int) {}
    __device__ __forceinline__ void count(int, bool) {}
    __device__ __forceinline__ void flush(unsigned long long*) {}
#endif
};
#ifdef IRM_ISA_MARKS  // analysis builds: phase markers in the emitted assembly
#define IRM_STAMP(ph) asm volatile("; IRM_PHASE " #ph)
#define IRM_COUNT(ph, c)
#else
#define IRM_STAMP(ph)                         \
    do {                                      \
        if (threadIdx.x == 0) prof.stamp(ph); \
    } while (0)
#define IRM_COUNT(ph, c)                          \
    do {                                          \
        if (threadIdx.x == 0) prof.count(ph, c);  \
    } while (0)
#endif

// ---------------------------------------------------------- MFMA contraction
// D layout of 16x16x4: lane l holds rows 4*(l>>4)+i, column l&15.
// Callers keep every tile inside the buffer (row extents are multiples of 16).
__device__ __forceinline__ void store_tile(float* out, int tile, f32x4 acc, unsigned colmask) {
    const int lane = threadIdx.x & 63;
    const int col = lane & 15;
    if (!((colmask >> col) & 1u)) return;
    float* o = out + (tile * 16 + 4 * (lane >> 4)) * kLd + col;
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i * kLd] = acc[i];
}

// ------------------------------------------------ per-waypoint physics
// sin/cos for robot.py's joint angles: Cody-Waite reduction by π/2 (3-part
// split, fma) and the cephes single-precision minimax polynomials on
// [−π/4, π/4]; ≈1 ulp, branch-free.  |x| > 1e4 rad falls back to sincosf.
__device__ __forceinline__ void sincos_poly(float x, float& sn, float& cs) {
    // k = round(x·2/π) by the 1.5·2²³ shifter: one fma rounds the exact product to an integer (ties to
    // even), whose low bits are k's two's-complement bits in t's mantissa (|k| < 2²² here); kf = k as a
    // float.  (rintf(fl(x·2/π)) differs only where x·2/π lies within an ulp of a half-integer — then r
    // sits at ±π/4 either way, inside the polynomials' accurate range.)
    const float t = fmaf(x, 0.636619772f, 12582912.0f);
    const float kf = t - 12582912.0f;
    float r = fmaf(kf, -1.57079637050628662109375f, x);
    r = fmaf(kf, 4.371138828673793e-08f, r);
    r = fmaf(kf, 1.7151245100058819e-15f, r);
    const float z = r * r;
    const float sp = fmaf(r * z, fmaf(z, fmaf(z, -1.9515295891e-4f, 8.3321608736e-3f), -1.6666654611e-1f), r);
    const float cp = fmaf(z * z, fmaf(z, fmaf(z, 2.443315711809948e-5f, -1.388731625493765e-3f), 4.166664568298827e-2f),
                          fmaf(-0.5f, z, 1.0f));
    // quadrant q = kf mod 4: swap on odd q, sin negated for q ∈ {2, 3}, cos for q ∈ {1, 2} — the sign
    // flips as bit 1 of q (resp. q + 1) moved to the sign bit (an xor; −x and the flip agree bit for bit)
    const int qi = __float_as_int(t);  // k mod 4 in the low bits
    const float s0 = (qi & 1) ? cp : sp;
    const float c0 = (qi & 1) ? sp : cp;
    sn = __uint_as_float(__float_as_uint(s0) ^ (((unsigned)qi << 30) & 0x80000000u));
    cs = __uint_as_float(__float_as_uint(c0) ^ (((unsigned)(qi + 1) << 30) & 0x80000000u));
}
__device__ __forceinline__ void sincos_fast(float x, float& sn, float& cs) {
    if (__builtin_expect(fabsf(x) > 1.0e4f, 0)) {
        sincosf(x, &sn, &cs);
        return;
    }
    sincos_poly(x, sn, cs);
}

template <int D>
struct WP {
    float cv, gx, gy;        // obstacle potential and its gradient at the end effector
    float jp, jv;            // masked joint-position / joint-velocity penalty terms (LEAN: Σ zm², Σ zvm²)
    float tx, tn, va;        // max/min joint position, max |joint velocity|
    float jx[D], jy[D];      // end-effector Jacobian row
    float fx, fy;            // end-effector position (eval_waypoint<…, POT = false>: potential not yet added)
    float zm[D], zvm[D];     // LEAN: masked (q − μ)/σ_q and v/v_max (0 where the limit mask is off)
};

// robot.py:29-36 (fk), 75-87 (jacobian); environment.py:46-58
// (compute_cost_vg); trajectory.py:215-227, 245-255 (penalty elements).
// WHOLE: the potential is summed over every joint position p_j = fk_joint_j
// (robot.py:39-72; DevBlog-Theme/blog-post.html:491-498) instead of the end
// effector only.  Its gradient w.r.t. angle k is Σ_{l≥k} (X_l·GX_l + Y_l·GY_l)
// with (X_l, Y_l) = L_l·(−sin c_l, cos c_l) and GX_l = Σ_{j≥l} ∂cost/∂p_j; it is
// returned as w.jx (with w.gx = 1, w.jy = w.gy = 0) so grad_waypoint is shared.
// POT = false (end-effector cost only): everything but the obstacle potential, whose inputs are left
// in w.fx / w.fy (potential_pair evaluates two waypoints' potentials in one pass over the obstacles).
// LEAN evaluations keep zm / zvm for the gradient inputs at D ≤ 3; at D = 7 the 14 values live across
// the evaluation barrier pushed the spill-free 7-DoF bench kernels into scratch, so the gradient inputs
// recompute them there (lean_pen: the same arithmetic, the same values)
template <int D>
constexpr bool kLeanKeep = D <= 3;
template <int D>
__device__ __forceinline__ void lean_pen(const KParams& P, const float (&q)[D], const float (&v)[D], float (&zm)[D],
                                         float (&zvm)[D]) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
        const float z = (q[d] - P.mean_pos) * P.inv_std_pos;
        const bool m = (q[d] > P.thr_hi) || (q[d] < P.thr_lo);
        const float zv = v[d] * P.inv_vmax;
        const bool mv = fabsf(v[d]) > P.thr_v;
        zm[d] = m ? z : 0.f;  // (cvdl off: the host's thresholds make every mask true)
        zvm[d] = mv ? zv : 0.f;
    }
}

// LEAN (the optimiser kernels): the penalty terms in the form the loss and the gradient inputs share —
// zm = mask·(q − μ)/σ_q and zvm = mask·v/v_max per joint, w.jp = Σ zm², w.jv = Σ zvm² (the ½ and the
// 1/N of trajectory.py:215-227, 245-255 go into the per-trajectory weights, grad_waypoint_lean); the
// host-API kernels keep the reference's element order (½·z² per element, summed).
template <int D, bool WHOLE = false, bool POT = true, bool LEAN = false>
__device__ __forceinline__ void eval_waypoint(const KParams& P, const float (&q)[D], const float (&v)[D],
                                              const float* __restrict__ ob, WP<D>& w,
                                              const f32x4* oreg = nullptr) {  // oreg: the 12-obstacle
                                                                              // table held in VGPRs
    float fx = 0.f, fy = 0.f, Sx = 0.f, Sy = 0.f;
    float xs[D], ys[D], px[D], py[D], cum[D], snv[D], csv[D];
    bool big = false;
#pragma unroll
    for (int d = 0; d < D; ++d) {
        cum[d] = d ? cum[d - 1] + q[d] : q[d];
        big |= fabsf(cum[d]) > 1.0e4f;
    }
    // One wave-uniform branch for all joints: the D polynomial chains share a basic block (the
    // scheduler interleaves them); a wave with any |angle| > 1e4 takes the per-lane form, whose
    // small-angle lanes compute the same polynomial, so every lane's value is that of sincos_fast.
#ifdef IRM_X_NOSC
    big = true;
#endif
    if (__builtin_expect(__ballot(big) != 0ull, 0)) {
#pragma unroll
        for (int d = 0; d < D; ++d) sincos_fast(cum[d], snv[d], csv[d]);
    } else {
#pragma unroll
        for (int d = 0; d < D; ++d) sincos_poly(cum[d], snv[d], csv[d]);
    }
#pragma unroll
    for (int d = 0; d < D; ++d) {
        const float sn = snv[d], cs = csv[d];
        fx = fmaf(P.link[d], cs, fx);
        fy = fmaf(P.link[d], sn, fy);
        px[d] = fx;
        py[d] = fy;
        xs[d] = -(P.link[d] * sn);
        ys[d] = P.link[d] * cs;
        Sx = d ? Sx + xs[d] : xs[d];
        Sy = d ? Sy + ys[d] : ys[d];
    }
    // Obstacles are staged in LDS in pairs (x_a, x_b, y_a, y_b), padded to a multiple of 4
    // with sentinels at (1e20, 1e20): r² overflows to +inf, rcp → 0, so a sentinel adds
    // exactly 0.  Two obstacles per packed-fp32 instruction; the even- and odd-numbered
    // obstacles accumulate separately and are added at the end.
    const f32x4* o4 = reinterpret_cast<const f32x4*>(ob);
    const int nq = (P.O + 3) >> 2;
    // Per pair of obstacles: e = 1 + dx² + dy² (= 2·den), u = rcp(e); the potential's constants are
    // applied once at the end: cost = 0.8/den = 1.6·Σu, ∂cost/∂f = −0.8·d/den² = −3.2·Σ d·u².
    auto potential = [&](float x, float y, float& cv, float& ax, float& ay) {
        f32x2 cv2 = {0.f, 0.f}, ax2 = {0.f, 0.f}, ay2 = {0.f, 0.f};
        const f32x2 fx2 = {x, x}, fy2 = {y, y}, one = {1.f, 1.f};
        auto pair2 = [&](f32x2 ox, f32x2 oy) {
            const f32x2 dx = fx2 - ox, dy = fy2 - oy;
            const f32x2 e = pkfma(dy, dy, pkfma(dx, dx, one));
            const f32x2 u = {__builtin_amdgcn_rcpf(e.x), __builtin_amdgcn_rcpf(e.y)};
            cv2 += u;
            const f32x2 u2 = u * u;
            ax2 = pkfma(dx, u2, ax2);
            ay2 = pkfma(dy, u2, ay2);
        };
#ifdef IRM_X_NOOBS
        if (false) {
#else
        if (nq == 3) {  // 9-12 obstacles (the reference's 11): one straight-line block, all 12 rcps
                        // issued back to back, then the sums in pair2's order
#endif
            f32x2 dx[6], dy[6], u[6];
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const f32x4 p = oreg ? oreg[i] : o4[i];
                dx[i] = fx2 - p.xy;
                dy[i] = fy2 - p.zw;
                const f32x2 e = pkfma(dy[i], dy[i], pkfma(dx[i], dx[i], one));
                u[i] = f32x2{__builtin_amdgcn_rcpf(e.x), __builtin_amdgcn_rcpf(e.y)};
            }
            // (the sums start from the first pair, not from +0: the same values, two instructions fewer)
            cv2 = u[0];
            ax2 = dx[0] * (u[0] * u[0]);
            ay2 = dy[0] * (u[0] * u[0]);
#pragma unroll
            for (int i = 1; i < 6; ++i) {
                cv2 += u[i];
                const f32x2 u2 = u[i] * u[i];
                ax2 = pkfma(dx[i], u2, ax2);
                ay2 = pkfma(dy[i], u2, ay2);
            }
        } else {
            for (int c = 0; c < nq; ++c) {
                const f32x4 p0 = o4[2 * c], p1 = o4[2 * c + 1];
                pair2(p0.xy, p0.zw);
                pair2(p1.xy, p1.zw);
            }
        }
        cv = 1.6f * (cv2.x + cv2.y);
        ax = -3.2f * (ax2.x + ax2.y);
        ay = -3.2f * (ay2.x + ay2.y);
    };
    if constexpr (!WHOLE) {
        float Cx = 0.f, Cy = 0.f;
#pragma unroll
        for (int d = 0; d < D; ++d) {
            Cx = d ? Cx + xs[d] : xs[d];
            Cy = d ? Cy + ys[d] : ys[d];
            w.jx[d] = (xs[d] + Sx) - Cx;
            w.jy[d] = (ys[d] + Sy) - Cy;
        }
        if constexpr (POT) {
            potential(fx, fy, w.cv, w.gx, w.gy);
        } else {
            w.fx = fx;
            w.fy = fy;
        }
    } else {
        float cvt = 0.f, gxj[D], gyj[D];
#pragma unroll
        for (int j = 0; j < D; ++j) {
            float cvj;
            potential(px[j], py[j], cvj, gxj[j], gyj[j]);
            cvt += cvj;
        }
        float GX = 0.f, GY = 0.f, acc = 0.f;
#pragma unroll
        for (int l = D - 1; l >= 0; --l) {
            GX += gxj[l];
            GY += gyj[l];
            acc = fmaf(xs[l], GX, fmaf(ys[l], GY, acc));
            w.jx[l] = acc;
            w.jy[l] = 0.f;
        }
        w.cv = cvt;
        w.gx = 1.f;
        w.gy = 0.f;
    }
    float jp = 0.f, jv = 0.f, tx = -INFINITY, tn = INFINITY, va = 0.f;
#pragma unroll
    for (int d = 0; d < D; ++d) {
        const float z = (q[d] - P.mean_pos) * P.inv_std_pos;
        const bool m = (q[d] > P.thr_hi) || (q[d] < P.thr_lo);
        const float zv = v[d] * P.inv_vmax;
        const bool mv = fabsf(v[d]) > P.thr_v;
        if constexpr (LEAN) {
            const float zm = m ? z : 0.f, zvm = mv ? zv : 0.f;  // (cvdl: folded into the thresholds)
            if constexpr (kLeanKeep<D>) {
                w.zm[d] = zm;
                w.zvm[d] = zvm;
            }
            jp = fmaf(zm, zm, jp);
            jv = fmaf(zvm, zvm, jv);
        } else {
            jp += m ? 0.5f * (z * z) : 0.f;
            jv += mv ? 0.5f * (zv * zv) : 0.f;
        }
        tx = fmaxf(tx, q[d]);
        tn = fminf(tn, q[d]);
        va = fmaxf(va, fabsf(v[d]));
    }
    w.jp = jp;
    w.jv = jv;
    w.tx = tx;
    w.tn = tn;
    w.va = va;
}

// The obstacle potential of two waypoints (w0.fx/fy, w1.fx/fy) in one pass over the LDS obstacle table:
// each obstacle pair is loaded once and both waypoints' terms are formed from it (independent chains
// that interleave).  Per waypoint the arithmetic and the accumulation order are eval_waypoint's.
template <int D>
__device__ __forceinline__ void potential_pair(const KParams& P, const float* __restrict__ ob, WP<D>& w0, WP<D>& w1) {
    const f32x4* o4 = reinterpret_cast<const f32x4*>(ob);
    const int nq = (P.O + 3) >> 2;
    f32x2 cv0 = {0.f, 0.f}, ax0 = {0.f, 0.f}, ay0 = {0.f, 0.f}, cv1 = cv0, ax1 = cv0, ay1 = cv0;
    const f32x2 x0 = {w0.fx, w0.fx}, y0 = {w0.fy, w0.fy}, x1 = {w1.fx, w1.fx}, y1 = {w1.fy, w1.fy};
    const f32x2 one = {1.f, 1.f};
    auto pair2 = [&](const f32x2& fx2, const f32x2& fy2, f32x2 ox, f32x2 oy, f32x2& cv2, f32x2& ax2, f32x2& ay2) {
        const f32x2 dx = fx2 - ox, dy = fy2 - oy;
        const f32x2 e = pkfma(dy, dy, pkfma(dx, dx, one));
        const f32x2 u = {__builtin_amdgcn_rcpf(e.x), __builtin_amdgcn_rcpf(e.y)};
        cv2 += u;
        const f32x2 u2 = u * u;
        ax2 = pkfma(dx, u2, ax2);
        ay2 = pkfma(dy, u2, ay2);
    };
    for (int c = 0; c < nq; ++c) {
        const f32x4 p0 = o4[2 * c], p1 = o4[2 * c + 1];
        pair2(x0, y0, p0.xy, p0.zw, cv0, ax0, ay0);
        pair2(x1, y1, p0.xy, p0.zw, cv1, ax1, ay1);
        pair2(x0, y0, p1.xy, p1.zw, cv0, ax0, ay0);
        pair2(x1, y1, p1.xy, p1.zw, cv1, ax1, ay1);
    }
    w0.cv = 1.6f * (cv0.x + cv0.y);
    w0.gx = -3.2f * (ax0.x + ax0.y);
    w0.gy = -3.2f * (ay0.x + ay0.y);
    w1.cv = 1.6f * (cv1.x + cv1.y);
    w1.gx = -3.2f * (ax1.x + ax1.y);
    w1.gy = -3.2f * (ay1.x + ay1.y);
}

// eval_waypoint with the cost variant chosen at run time (host-API kernels, DynShape optimiser).
template <int D>
__device__ __forceinline__ void eval_waypoint_rt(const KParams& P, const float (&q)[D], const float (&v)[D],
                                                 const float* __restrict__ ob, WP<D>& w) {
    if (P.whole_robot) eval_waypoint<D, true>(P, q, v, ob, w);
    else eval_waypoint<D, false>(P, q, v, ob, w);
}

// Gradient inputs a (→ Kᵀ) and b (→ dKᵀ) of one waypoint, trajectory.py:91-126
// (obstacle), 191-212 (start/goal), 231-242 / 259-268 (joint limits).
template <int D>
__device__ __forceinline__ void grad_waypoint(const KParams& P, const WP<D>& w, const float (&q)[D],
                                              const float (&v)[D], int n, int idx, float lsg, float ljl,
                                              const float (&s)[D], const float (&g)[D], float (&a)[D],
                                              float (&b)[D]) {
    const int N = P.N;
    const float wt = (n == idx ? P.lam_max : 0.f) + P.one_m_lmax * P.invN;
    const float wx = wt * w.gx, wy = wt * w.gy;
#pragma unroll
    for (int d = 0; d < D; ++d) {
        float sgp = 0.f, sgv = 0.f;
        if (n == 0) {
            sgp = q[d] - s[d];
            sgv = v[d];
        }
        if (n == N - 1) {
            sgp = q[d] - g[d];
            sgv = v[d];
        }
        float jpg = 0.f, jvg = 0.f;
        const bool m = (q[d] > P.thr_hi) || (q[d] < P.thr_lo);
        if (m) jpg = ((q[d] - P.mean_pos) * P.inv_std2) * P.invN;
        const bool mv = fabsf(v[d]) > P.thr_v;
        if (mv) jvg = (v[d] * P.inv_vmax2) * P.invN;
        a[d] = fmaf(ljl, jpg, fmaf(lsg, sgp, fmaf(wx, w.jx[d], wy * w.jy[d])));
        b[d] = fmaf(lsg, sgv, ljl * jvg);
    }
}

// Per-trajectory weights of the LEAN evaluation (uniform; ljl changes with the outer iteration):
// the loss's mean / penalty terms u = c_mean·cv + c_pen·(Σzm² + Σzvm²) (trajectory.py:85-87, 281 with
// ½ and 1/N folded), the gradient's penalty slopes k_pos = λjl/(σ_q·N), k_vel = λjl/(v_max·N)
// (trajectory.py:231-242, 259-268: (q − μ)/σ_q²/N = zm·(1/σ_q)/N).
struct LeanW {
    float c_mean, c_pen, k_pos, k_vel;
};
__device__ __forceinline__ LeanW lean_weights(const KParams& P, float ljl) {
    LeanW c;
    c.c_mean = P.one_m_lmax * P.invN;
    c.c_pen = (0.5f * ljl) * P.invN;
    c.k_pos = (ljl * P.inv_std_pos) * P.invN;
    c.k_vel = (ljl * P.inv_vmax) * P.invN;
    return c;
}

// Gradient inputs a, b of one waypoint from a LEAN evaluation (grad_waypoint's terms, the penalty
// masks and normalised deviations reused from the evaluation).  lsg_ep = λsg on rows 0 and N−1, else
// 0 (per lane); tg the row's start / goal.
template <int D>
__device__ __forceinline__ void grad_waypoint_lean(const KParams& P, const WP<D>& w, const float (&q)[D],
                                                   const float (&v)[D], bool isidx, float lsg_ep,
                                                   const LeanW& c, const float (&tg)[D], float (&a)[D],
                                                   float (&b)[D]) {
    const float wt = (isidx ? P.lam_max : 0.f) + c.c_mean;
    const float wx = wt * w.gx, wy = wt * w.gy;
    float zm[D], zvm[D];
    if constexpr (kLeanKeep<D>) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            zm[d] = w.zm[d];
            zvm[d] = w.zvm[d];
        }
    } else {
        lean_pen<D>(P, q, v, zm, zvm);
    }
#pragma unroll
    for (int d = 0; d < D; ++d) {
        a[d] = fmaf(c.k_pos, zm[d], fmaf(lsg_ep, q[d] - tg[d], fmaf(wx, w.jx[d], wy * w.jy[d])));
        b[d] = fmaf(lsg_ep, v[d], c.k_vel * zvm[d]);
    }
}

// Result of one cost evaluation of one trajectory (reduced over waypoints).
struct EvalOut {
    float loss, ds, dg, vs, vg, tmax, tmin, vabs;
    int idx;
};

// Wave-reduce this lane's waypoint terms; lane 0 of each wave stores the
// partials, the lanes of rows 0 / N−1 store the start/goal terms.  Must be
// reached by the whole wave (a wave never straddles two trajectories).
template <int D>
__device__ __forceinline__ void eval_partials(const KParams& P, bool live, const WP<D>& w, int n, int wave,
                                              const float (&q)[D], const float (&v)[D], const float (&s)[D],
                                              const float (&g)[D], float* red, float* sg, int t) {
    float cmax = live ? w.cv : -INFINITY;
    int cidx = live ? n : 0x7fffffff;
    wred_argmax(cmax, cidx);
    const float csum = wred_sum(live ? w.cv : 0.f);
    const float jps = wred_sum(live ? w.jp : 0.f);
    const float jvs = wred_sum(live ? w.jv : 0.f);
    const float tx = wred_max(live ? w.tx : -INFINITY);
    const float tn = wred_min(live ? w.tn : INFINITY);
    const float va = wred_max(live ? w.va : 0.f);
    if ((threadIdx.x & 63) == 0) {
        float* r = red + wave * 10;
        r[0] = cmax;
        r[1] = __int_as_float(cidx);
        r[2] = csum;
        r[3] = jps;
        r[4] = jvs;
        r[5] = tx;
        r[6] = tn;
        r[7] = va;
    }
    if (live && (n == 0 || n == P.N - 1)) {  // trajectory.py:183-204 rows 0 and N−1
        float a = 0.f, bb = 0.f;
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const float e = q[d] - (n == 0 ? s[d] : g[d]);
            a += e * e;
            bb += v[d] * v[d];
        }
        sg[t * 4 + (n == 0 ? 0 : 2)] = a;
        sg[t * 4 + (n == 0 ? 1 : 3)] = bb;
    }
}

// Combine the trajectory's wave partials (fixed order) into loss + stats.
__device__ __forceinline__ EvalOut eval_finalize(const KParams& P, const float* red, const float* sg, int t,
                                                 int wave0, int nwt, float lsg, float ljl) {
    const float* r = red + wave0 * 10;
    float cmax = r[0];
    int cidx = __float_as_int(r[1]);
    float csum = r[2], jps = r[3], jvs = r[4], tx = r[5], tn = r[6], va = r[7];
    for (int w = 1; w < nwt; ++w) {
        const float* q = red + (wave0 + w) * 10;
        amax_step(cmax, cidx, q[0], __float_as_int(q[1]));
        csum += q[2];
        jps += q[3];
        jvs += q[4];
        tx = fmaxf(tx, q[5]);
        tn = fminf(tn, q[6]);
        va = fmaxf(va, q[7]);
    }
    const float a0 = sg[t * 4 + 0], b0 = sg[t * 4 + 1], a1 = sg[t * 4 + 2], b1 = sg[t * 4 + 3];
    const float nN = (float)P.N;
    const float sgpc = 0.5f * a0 + 0.5f * a1;                          // trajectory.py:187
    const float sgvc = 0.5f * b0 + 0.5f * b1;                          // trajectory.py:203
    const float toc = P.lam_max * cmax + P.one_m_lmax * (csum / nN);    // trajectory.py:85-87
    EvalOut e;
    e.loss = toc + lsg * (sgpc + sgvc) + ljl * (jps / nN + jvs / nN);  // trajectory.py:281
    e.idx = cidx;
    e.ds = sqrtf(a0);
    e.dg = sqrtf(a1);
    e.vs = sqrtf(b0);
    e.vg = sqrtf(b1);
    e.tmax = tx;
    e.tmin = tn;
    e.vabs = va;
    return e;
}

// Obstacles into LDS: one shared set (obs_stride 0) or one per trajectory,
// each padded to obs_pitch floats with zero-contribution sentinels.
__host__ __device__ inline int obs_pitch(int O) { return ((O + 3) & ~3) * 2; }
__device__ inline void stage_obstacles(const KParams& P, int tb0, int ntb, float* obsL) {
    const int pitch = obs_pitch(P.O), nsets = P.obs_stride ? P.TB : 1;
    for (int e = threadIdx.x; e < nsets * pitch; e += P.BT) {
        const int tt = e / pitch, r = e - tt * pitch;
        // r = 4·pair + 2·coord + j  →  obstacle 2·pair + j, coordinate coord
        const int o = 2 * (r >> 2) + (r & 1), coord = (r >> 1) & 1;
        float val = 1.0e20f;
        if (o < P.O) {
            const int src = 2 * o + coord;
            if (!P.obs_stride) val = P.obstacles[src];
            else if (tt < ntb) val = P.obstacles[(size_t)(tb0 + tt) * P.obs_stride + src];
        }
        obsL[e] = val;
    }
}

// α0 of the block's trajectories into X[n][tD+d] (rows ≥ N / unused columns 0).
template <int D>
__device__ void stage_alpha(const KParams& P, int tb0, int ntb, float* X, int xrows) {
    const int N = P.N;
    for (int e = threadIdx.x; e < xrows * 16; e += P.BT) {
        const int n = e >> 4, c = e & 15, t = c / D, d = c - t * D;
        float* dst = X + n * kLd + c;
        float val = 0.f;
        if (n < N && t < ntb) {
            const size_t b = (size_t)(tb0 + t);
            if (P.alpha0) {
                val = P.alpha0[(b * N + n) * D + d];
            } else {  // trajectory.py:73-78 via K⁻¹(1−c), K⁻¹c (linearity of solve)
                float sj = 0.f, gj = 0.f;
                for (int e2 = 0; e2 < D; ++e2) {
                    sj += P.start[b * D + e2] * P.Jinv[e2 * D + d];
                    gj += P.goal[b * D + e2] * P.Jinv[e2 * D + d];
                }
                val = P.uvec[n] * sj + P.wvec[n] * gj;
            }
        }
        *dst = val;
    }
}

// ------------------------------------------- correctly rounded α-space maps
// The reference's K@α@J (trajectory.py:63-65) contracts over N waypoints with
// |α| ≈ 1e3 (singular K): a plain fp32 sum carries ~1e-4 (positions) and
// ~1e-3 (velocities) of order-dependent noise.  Here every product of two
// fp32 values is exact in fp64 and the N-term sum accumulates in fp64 (same
// sequential order as oracle/irm_oracle.c), then rounds once — the result is
// the correctly rounded fp32 value, bit-identical to the CPU oracle.  Used off
// the hot loop: host-API evaluation and the optimiser's prologue / resyncs.
//
// Lane n of trajectory column block Xa (LDS, rows m = 0..N-1, stride kLd):
//   q = fp32(fp32(K·α)[n]·J), v = fp32(fp32(dK·α)[n]·J).
// (rs, cs: row / column strides of Xa — [row][16] LDS buffers by default, the lean kernel's
// column-major buffers with rs = 1, cs = column stride)
// U: K / dK rows per software-pipelined batch (8 in the prologue / epilogue; the optimiser loop's resync
// rounds use 2, which keeps the register peak of the dual-loop / BLS instantiations low — spill-free —
// at the cost of less latency hiding in a round that runs once per outer iteration)
// JL: J (D×D) from Jm, an LDS copy (inside the optimiser loop, whose reads are not hoisted: the D² fp64
// conversions of P.J hoisted out of the round loop held 2·D² VGPRs), else from P.J.  A compile-time
// choice: a run-time select between &P.J and an LDS address takes the kernel argument's address, and the
// compiler then copies all of KParams into scratch and reads every parameter from there (1.8 KB of
// scratch and ≈60 scratch loads in the dual-loop / BLS rounds, round 4)
template <int D, int U = 8, bool JL = false>
__device__ void eval_exact(const KParams& P, const float* __restrict__ Xa, int n, float (&q)[D], float (&v)[D],
                           const float* Kt = nullptr, const float* dKt = nullptr, int rs = kLd, int cs = 1,
                           const float* Jm = nullptr) {
    const float* J;
    if constexpr (JL) J = Jm;
    else J = P.J;
    const int N = P.N;
    double aq[D], av[D];
#pragma unroll
    for (int d = 0; d < D; ++d) aq[d] = av[d] = 0.0;
    // wave-uniform bases and 32-bit element offsets (global loads with an SGPR base and a VGPR
    // offset): inside the optimiser loop a per-lane 64-bit pointer would be hoisted out of the loop
    // and held (or spilled) across every round
    const float* kt = Kt ? Kt : P.Kt;
    const float* dkt = dKt ? dKt : P.dKt;
    const unsigned un = (unsigned)n, uN = (unsigned)N;
    // K / dK rows come from L2 / HBM: software-pipelined batches of U rows (the next batch's 2U
    // loads are in flight while this one is summed; the sum stays in the sequential order
    // m = 0, 1, …, N−1 of the oracle)
    const int nb = N / U;
    int m0 = nb * U;
    if (nb > 0) {
        float kq[U], kv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            kq[u] = kt[(unsigned)u * uN + un];
            kv[u] = dkt[(unsigned)u * uN + un];
        }
        for (int bi = 0; bi < nb; ++bi) {
            const int mb = bi * U;
            float nq[U], nv[U];
            const int mn = (bi + 1 < nb) ? mb + U : mb;  // (the last batch re-reads itself: no branch)
#pragma unroll
            for (int u = 0; u < U; ++u) {
                nq[u] = kt[(unsigned)(mn + u) * uN + un];   // K[n][m]
                nv[u] = dkt[(unsigned)(mn + u) * uN + un];  // dK[n][m]
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const float* xr = Xa + (mb + u) * rs;
#pragma unroll
                for (int d = 0; d < D; ++d) {
                    const double x = (double)xr[d * cs];
                    aq[d] = fma((double)kq[u], x, aq[d]);
                    av[d] = fma((double)kv[u], x, av[d]);
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                kq[u] = nq[u];
                kv[u] = nv[u];
            }
        }
    }
    for (int m = m0; m < N; ++m) {
        const double kq = (double)kt[(unsigned)m * uN + un], kv = (double)dkt[(unsigned)m * uN + un];
        const float* xr = Xa + m * rs;
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const double x = (double)xr[d * cs];
            aq[d] = fma(kq, x, aq[d]);
            av[d] = fma(kv, x, av[d]);
        }
    }
    float tq[D], tv[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
        tq[d] = (float)aq[d];
        tv[d] = (float)av[d];
    }
#pragma unroll
    for (int k = 0; k < D; ++k) {
        double sq = 0.0, sv = 0.0;
#pragma unroll
        for (int d = 0; d < D; ++d) {
            sq = fma((double)tq[d], (double)J[d * D + k], sq);
            sv = fma((double)tv[d], (double)J[d * D + k], sv);
        }
        q[k] = (float)sq;
        v[k] = (float)sv;
    }
}

// eval_exact for one lane inside the optimiser loop (the lean kernel's resyncs at D > 3): the same sums
// in the same order, as one loop over m whose K / dK loads run PF rows ahead, J read from LDS (Jl).
// eval_exact's batched form kept ~80 more VGPRs live around the resync at D = 7 (its fp64 J products
// hoisted out of the round loop, and the batch's addressing): the 7-DoF dual-loop / BLS kernels spilled.
template <int D, int PF>
__device__ __forceinline__ void eval_exact_loop(const KParams& P, const float* __restrict__ Xc, int ldc, int n, int N,
                                                const float* Jl, float (&q)[D], float (&v)[D]) {
    const unsigned un = (unsigned)n, uN = (unsigned)N;
    double aq[D], av[D];
#pragma unroll
    for (int d = 0; d < D; ++d) aq[d] = av[d] = 0.0;
    float kq = P.Kt[un], kv = P.dKt[un];
#pragma unroll 1
    for (int m = 0; m < N; m += PF) {
        float nq[PF], nv[PF];
#pragma unroll
        for (int u = 0; u < PF; ++u) {  // rows m+1 … m+PF (clamped: the last rows re-read row N − 1)
            const unsigned mn = (unsigned)min(m + 1 + u, N - 1);
            nq[u] = P.Kt[mn * uN + un];
            nv[u] = P.dKt[mn * uN + un];
        }
#pragma unroll
        for (int u = 0; u < PF; ++u) {
            if (PF == 1 || m + u < N) {
#pragma unroll
                for (int d = 0; d < D; ++d) {
                    const double x = (double)Xc[d * ldc + m + u];
                    aq[d] = fma((double)kq, x, aq[d]);
                    av[d] = fma((double)kv, x, av[d]);
                }
            }
            kq = nq[u];
            kv = nv[u];
        }
    }
    float tq[D], tv[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
        tq[d] = (float)aq[d];
        tv[d] = (float)av[d];
    }
#pragma unroll
    for (int k = 0; k < D; ++k) {
        // one column of J at a time: without the barrier the scheduler hoists all D² LDS reads and their fp64
        // conversions (2·D² = 98 VGPRs at D = 7) ahead of the first product — the resync's register peak
        __builtin_amdgcn_sched_barrier(0);
        double sq = 0.0, sv = 0.0;
#pragma unroll
        for (int d = 0; d < D; ++d) {
            sq = fma((double)tq[d], (double)Jl[d * D + k], sq);
            sv = fma((double)tv[d], (double)Jl[d * D + k], sv);
        }
        q[k] = (float)sq;
        v[k] = (float)sv;
    }
}

// G[n] = (fp32(Kᵀa)[n] + fp32(dKᵀb)[n])·Jᵀ  (trajectory.py:295), the N-sums
// in fp64 as above, the fp32 add and the D-term J product unfused in fp32
// (the oracle's order).  Xa: a in rows 0..N-1, b in rows N..2N-1.
template <int D>
__device__ void grad_exact(const KParams& P, const float* __restrict__ Xa, int n, float (&G)[D]) {
    const int N = P.N;
    double ga[D], gb[D];
#pragma unroll
    for (int d = 0; d < D; ++d) ga[d] = gb[d] = 0.0;
    const float* km = P.Km + n;
    const float* dkm = P.dKm + n;
    for (int m = 0; m < N; ++m) {
        const double ka = (double)km[(size_t)m * N], kb = (double)dkm[(size_t)m * N];  // K[m][n], dK[m][n]
        const float* xa = Xa + m * kLd;
        const float* xb = Xa + (N + m) * kLd;
#pragma unroll
        for (int d = 0; d < D; ++d) {
            ga[d] = fma(ka, (double)xa[d], ga[d]);
            gb[d] = fma(kb, (double)xb[d], gb[d]);
        }
    }
    float tmp[D];
#pragma unroll
    for (int d = 0; d < D; ++d) tmp[d] = __fadd_rn((float)ga[d], (float)gb[d]);
#pragma unroll
    for (int k = 0; k < D; ++k) {
        float u = 0.f;
#pragma unroll
        for (int l = 0; l < D; ++l) u = __fadd_rn(u, __fmul_rn(tmp[l], P.J[k * D + l]));
        G[k] = u;
    }
}

// ------------------------------------------------------------ optimiser
// Wave reduction of one evaluation's per-waypoint terms.
// usum: Σ_n [(1−λmax)/N·cost_v[n] + λjl/N·(jp[n] + jv[n])], the mean-obstacle and
// joint-limit terms of trajectory.py:281 folded into one sum; cmax with the
// first-index argmax of jnp.argmax (trajectory.py:97) from a ballot of the lanes
// holding the wave maximum.  tx/tn/va (constraint extrema) only when `ext`.
// Lane 0 stores the wave's record at red[wave·8].
__device__ __forceinline__ void ered_store(bool live, float cv, float us, float tx, float tn, float va, bool ext,
                                           int n0, float* red, int wave) {
    float m = live ? cv : -INFINITY, s = live ? us : 0.f;  // cv ≥ +0 (a sum of reciprocals): maxpos
    m = maxpos(m, dppf<0xB1>(m));
    s += dppf<0xB1>(s);
    m = maxpos(m, dppf<0x4E>(m));
    s += dppf<0x4E>(s);
    m = maxpos(m, dppf<0x141>(m));
    s += dppf<0x141>(s);
    m = maxpos(m, dppf<0x140>(m));
    s += dppf<0x140>(s);
    // cross-row combine with the GFX9 row broadcasts: row_bcast:15 into rows 1 and 3, row_bcast:31 into
    // rows 2 and 3, so lane 63 holds (r3 ∘ r2) ∘ (r1 ∘ r0) — the association of the readlane form
    // (lanes 0, 16, 32, 48), fp addition being commutative; read back as a wave-uniform value
    float wm, ws;
    {
        m = maxpos(m, __int_as_float(__builtin_amdgcn_update_dpp((int)0x80000000, __float_as_int(m), 0x142, 0xA, 0xF, false)));
        s = bcast_add<15>(s);
        m = maxpos(m, __int_as_float(__builtin_amdgcn_update_dpp((int)0x80000000, __float_as_int(m), 0x143, 0xC, 0xF, false)));
        s = bcast_add<31>(s);
        wm = lanef(m, 63);
        ws = lanef(s, 63);
    }
    const unsigned long long hit = __ballot(live && cv == wm);
    const int idx = hit ? n0 + __builtin_ctzll(hit) : 0x7fffffff;
    float ox = 0.f, on = 0.f, oa = 0.f;
    if (ext) {
        ox = wred_max(live ? tx : -INFINITY);
        on = wred_min(live ? tn : INFINITY);
        oa = wred_max(live ? va : 0.f);
    }
    if ((threadIdx.x & 63) == 0) {
        float* q = red + wave * 8;
        q[0] = wm;
        q[1] = __int_as_float(idx);
        q[2] = ws;
        q[3] = ox;
        q[4] = on;
        q[5] = oa;
    }
}

// A value the compiler may not fuse into a neighbouring operation (hipcc contracts a·b − c into
// an fma even under `#pragma clang fp contract(off)` when the product comes from __fmul_rn).
__device__ __forceinline__ float unfused(float x) {
    asm("" : "+v"(x));
    return x;
}

// a/b through a reciprocal refined by one Newton step (r = rcp_refined(b)): q = a·r, then q + (a − q·b)·r —
// the correctly rounded quotient but in rare near-ties, in 3 VALU per quotient once r is known (the IEEE
// division expands to ~10 with its scaling and fix-up).  The BLS trial stages form ĝ = G/‖G‖ with it
// (optimizer_BLS.py:165); its operands are normal numbers there.
__device__ __forceinline__ float rcp_refined(float b) {
    const float r0 = __builtin_amdgcn_rcpf(b);
    return fmaf(fmaf(-b, r0, 1.f), r0, r0);
}
__device__ __forceinline__ float div_rcp(float a, float b, float r) {
    const float q = a * r;
    return fmaf(fmaf(-q, b, a), r, q);
}
// The IEEE quotient a/b in div_rcp's 3 VALU (round 6): with r = RN(1/b), the correctly rounded reciprocal
// (shared by every quotient of the same divisor), q = RN(a·r) is within an ulp of a/b and the fma
// correction RN(q + (a − q·b)·r) is the correctly rounded a/b (Markstein's theorem; normal operands, and a
// remainder a − q·b above the subnormal range).  RN(1/b) itself: one Newton step from v_rcp_f32 (faithful,
// ≤ 1 ulp) is the correctly rounded reciprocal for every divisor but those with an all-ones mantissa
// (b = 2^e·(2 − 2^-23)), whose RN(1/b) = 2^(−e−1)·(1 + 2^-23) has the bit pattern 0x7F000000 − bits(b) (b > 0)
// and is selected there (branch-free; a branch here split the trial stage's block).
// tests/test_division.py checks both statements on the host (every divisor mantissa); the IRM_DIV_CHECK build
// counts the kernel's mismatches against __fdiv_rn (tools/div_check.py → profiles/r06_div_check.txt: 0).
// The BLS step direction ĝ = G/‖G‖ (optimizer_BLS.py:165) uses it (b = ‖G‖ > 0, normal).
__device__ __forceinline__ float rcp_rn_of(float b, float r) {  // r = rcp_refined(b)
#ifdef IRM_X_RCP_OLD
    return r;
#else
    const unsigned u = __float_as_uint(b);
    return (u & 0x7fffffu) == 0x7fffffu ? __uint_as_float(0x7F000000u - u) : r;
#endif
}

// One f32x4 of an operator fragment array through a buffer descriptor: the per-lane part of the address in
// one VGPR (voff, shared by every load of a stream), the wave-uniform part (tile, k-quad) in soff — a
// streamed operator holds no 64-bit address per load (the dense stages' unrolled k-loops spilled them)
__device__ __forceinline__ f32x4 ld_frag(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}

// Smallest step a rounding residual is folded with (e' = −e/step): |e'| ≤ 1e-3·2^80 ≈ 1e21 stays
// finite where a tiny BLS step (lr/‖G‖ after many rejected trials, or --gd-lr 0) would give ±inf.
constexpr float kMinRefStep = 8.271806e-25f;  // 2^-80

// One fp32 α element of the reference's GD / BLS update and its rounding residual:
//   α' = fl(fl(c·α) − fl(lr·ĝ))                        (optimizer_GD.py:81, optimizer_BLS.py:139)
//   e  = α' − (c·α − step·G)  exactly (to fp32 rounding of e itself), where c·[T; V] − step·F·y'
//        is the waypoint-space update the kernel applies (ĝ = G for GD, G/‖G‖ for BLS).
// Products and the subtraction are rounded separately (the reference's arithmetic, no fma); the
// residuals come from fma (c·α − fl(c·α) is exact) and TwoSum.
__device__ __forceinline__ float alpha_step(float al, float c, float lr, float gh, float step, float G, float& e) {
    const float p1 = unfused(c * al), p2 = unfused(lr * gh);
    const float an = unfused(p1 - p2);
    const float ep1 = fmaf(c, al, -p1);                 // c·α − p1
    const float bb = an - p1;                           // TwoSum(p1, −p2) = an + es
    const float es = (p1 - (an - bb)) + (-p2 - bb);
    const float p = unfused(step * G);
    const float ep = fmaf(step, G, -p);                 // step·G − p
    e = (((p - p2) - es) + ep) - ep1;                   // α' − (c·α − step·G)
    return an;
}

// alpha_step for GD (ĝ = G, step = lr): step·G is the reference's own product p2, so its term drops.
// α' = fl(fl(c·α) − fl(lr·G)) (optimizer_GD.py:81) and the scaled residual the direction folds in,
// e' = −(α' − (c·α − lr·G))/lr = (c·α − α')/lr − G, as u = fl(c·α − α') (one rounding, |u| ≈ |lr·G|) and
// e' = fl(u·(1/lr) − G) (ne = −1/lr): the residual to 2^-24 of |G| (i.e. the waypoint state to 2^-24 of a
// step per step, below the rank-16 direction's own 1.5e-7) in two FMAs instead of TwoSum and the two
// product errors (alpha_step_gd: 9 more VALU per component on the round's critical path)
__device__ __forceinline__ float alpha_step_gd2(float al, float c, float lr, float G, float ne, float& eo) {
    const float p1 = unfused(c * al), p2 = unfused(lr * G);
    const float an = unfused(p1 - p2);
    const float u = fmaf(c, al, -an);
    eo = fmaf(-u, ne, -G);
    return an;
}
__device__ __forceinline__ float alpha_step_gd(float al, float c, float lr, float G, float& e) {
    const float p1 = unfused(c * al), p2 = unfused(lr * G);
    const float an = unfused(p1 - p2);
    const float ep1 = fmaf(c, al, -p1);
    const float bb = an - p1;
    const float es = (p1 - (an - bb)) + (-p2 - bb);
    const float ep = fmaf(lr, G, -p2);                  // lr·G − p2
    e = ((-es) + ep) - ep1;
    return an;
}

// Operator fragments a wave keeps in VGPRs across all rounds (REGOPS).
// Capacities mirror regops_fit (irm_kernels.hpp): a 512-thread workgroup (8 waves) keeps 4 stage-1
// k-quads and 2 stage-2 tiles per wave (N ≤ 128 at R = 32), a 256-thread one up to 8 of each.

// Problem shape of an optimiser launch.  FixShape: compile-time N / R (and everything derived,
// incl. the LDS layout head) for the common shapes; DynShape: any shape, read from KParams.
template <int D_, int N_, int RP_>
struct FixShape {
    static constexpr int D = D_, N = N_, NK = (N_ + 15) / 16 * 16, MP = 2 * NK, RP = RP_;
    static constexpr int NW = (N_ + 63) / 64 * 64, WPT = NW / 64, NSPLIT = stage1_splits(NK);
    static constexpr bool kVariants = false;  // end-effector cost only (the reference's)
    static constexpr bool kDense = false;
    static constexpr int kNW = NW;             // lanes per trajectory (0: only known at run time)
    // stage-1 k-quads per split-K unit when the split is even (else 0: checked per quad)
    static constexpr int KQU = (NK / 16) % NSPLIT == 0 ? (NK / 16) / NSPLIT : 0;
    __device__ explicit FixShape(const KParams&) {}
};
// The dense operator (--operator-rank -1: R = N, F = L = [K; dK], V_R = I, so G = y'' and z = e') of a
// fixed shape, for k_lean's GD single loop: one split, every operator fragment streamed from L2.
template <int D_, int N_>
struct DenseShape {
    static constexpr int D = D_, N = N_, NK = (N_ + 15) / 16 * 16, MP = 2 * NK, RP = NK;
    static constexpr int NW = (N_ + 63) / 64 * 64, WPT = NW / 64, NSPLIT = 1;
    static constexpr bool kVariants = false;
    static constexpr bool kDense = true;
    static constexpr int kNW = NW;
    static constexpr int KQU = 0;
    __device__ explicit DenseShape(const KParams&) {}
};
template <int D_>
struct DynShape {
    static constexpr int D = D_;
    static constexpr bool kVariants = true;  // cost variants chosen at run time (whole_robot)
    static constexpr bool kDense = false;
    static constexpr int kNW = 0;
    static constexpr int KQU = 0;
    int N, NK, MP, RP, NW, WPT, NSPLIT;
    __device__ explicit DynShape(const KParams& P)
        : N(P.N), NK(P.NK), MP(P.MP), RP(P.RP), NW(P.NW), WPT(P.NW >> 6), NSPLIT(P.nsplit) {}
};
constexpr int kS1Q(int maxt) { return maxt <= 256 ? 8 : 4; }   // stage-1 float4 per wave
constexpr int kS2T(int maxt) { return maxt <= 256 ? 8 : 2; }   // stage-2 tiles per wave (KQ2 ≤ 2)
// MP of a shape-specialised shape (0 for DynShape, whose MP is a run-time value)
template <class S>
constexpr int shape_mp() {
    if constexpr (S::kNW > 0) return S::MP;
    else return 0;
}

// Row layout of the optimiser's [a; b] / [T; V] buffers and of F: the velocity
// half starts at row NK (= N rounded up to 16), so the position half is whole
// k-quads of its own and stage 1 can skip the velocity half when b is zero
// away from the two endpoint rows (the usual case); the endpoint rows then enter
// through the precomputed operator columns h0 = F·F[NK]ᵀ, h1 = F·F[NK+N−1]ᵀ.
//
// One round of a workgroup (TB trajectories, one lane per waypoint):
//   stage 1   y' = Fᵀ·[a'; b']          (MFMA, split-K over the waves → Ypart)
//             a' = a·JᵀJ, b' = b·JᵀJ were mixed per lane when written, so y' = y·JᵀJ
//   stage 2   G = (V_R·y')·J⁻¹ (MFMA tile set); GD also Δ[T; V] = F·y' (B operand = Σ partials,
//             summed on load)
//   update    GD:  [T; V]' = c·[T; V] − s·Δ  (Δ latched in registers per direction)
//             BLS: [T; V]' = eval_exact(α_j), the trial's fp32 iterate (below)
//   evaluate  cost at the trial point; gradient inputs for the next direction
//   decide    the reference's accept / reject / λ logic per trajectory
//   GD accept α' = fl(fl(c·α) − fl(lr·G)) per lane in fp32 with the reference's rounding, the rounding
//             residual folded into the next direction through z = V_Rᵀ·e' (k_lean's scheme)
// BLS: every trial's α_j = fl(fl(c_j·α) − fl(lr_j·ĝ)), ĝ = G/‖G‖ (optimizer_BLS.py:139, 165) is formed
// per lane and its trajectory evaluated exactly, as the reference evaluates it: at N ≳ 500 (|α| ≈ 1e3,
// singular K) one ulp of α moves the endpoint velocities by ~2e-3, so a trajectory that takes a trial's
// rounding one step late (the GD scheme) decides a noise-dominated line search on other losses than the
// reference (tools/e2e_ensemble.py: 47-67 gradient evaluations against the reference's 89-122 at
// N = 500); the exact evaluation costs 2·N²·D fp64 FMAs per trial, this path's shapes are the small
// batches outside k_lean's set.  Accepting a trial takes α_j and its [T; V] as they are.
// When an inner loop ends (PH_RESYNC) [T; V] is replaced by eval_exact(α).
// FULL (shape-specialised REGOPS launches of exactly MAXT threads): the stage-2 tiles per wave are
// known exactly, so only those operator fragments occupy VGPRs (as in k_gd_single<…, FULL>).
template <class S, int MAXT, bool OPS_LDS, bool REGOPS, bool BLS, bool FULL = false>
// 256-thread workgroups without register-resident operators fit two per CU (≤ 256 VGPRs); the
// REGOPS variants need more and keep one (they are launched one per CU anyway).
__global__ __launch_bounds__(MAXT, (MAXT <= 256 && !REGOPS) ? 2 : 1) void k_optimize(KParams P) {
    constexpr int D = S::D;
    static_assert(!FULL || (REGOPS && S::kNW > 0), "FULL: shape-specialised REGOPS variants only");
    constexpr int S1Q = kS1Q(MAXT);
    constexpr int S2T = FULL ? (shape_mp<S>() / 16 + MAXT / 64 - 1) / (MAXT / 64) : kS2T(MAXT);
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const S sh(P);
    const Head H = plan_head(sh.MP, sh.RP, sh.NSPLIT, true);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nwaves = FULL ? MAXT / 64 : P.BT >> 6;
    const int N = sh.N, NW = sh.NW, TB = P.TB, RP = sh.RP, MP = sh.MP, NK = sh.NK;
    const int WPT = sh.WPT;             // waves per trajectory
    const int t = wave / WPT;           // this lane's trajectory (wave-uniform)
    const int n = tid - t * NW;         // this lane's waypoint (and row r of y for n < RP)
    const int n0 = (wave - t * WPT) * 64;  // first waypoint of this wave
    const int tb0 = blockIdx.x * TB;
    const int ntb = min(TB, P.B - tb0);
    if (ntb <= 0) return;
    const bool tvalid = t < ntb;
    const bool valid = tvalid && n < N;
    const bool yrow = tvalid && n < RP;
    const size_t b = (size_t)(tb0 + (tvalid ? t : 0));
    constexpr bool bls = BLS;
    const bool rec = P.record_series && P.series;
    Prof prof;
    if (tid == 0) prof.init();

    float* X = smem + H.X;    // [a'; b'] (rows 0..N-1, NK..NK+N-1) × 16 columns
    float* dP = smem + H.dP;  // Δ[T; V], same row layout
    float* Ypart = smem + H.Ypart;
    float* Ymix = smem + H.Ymix;
    float* red = smem + H.red;
    float* sg = smem + H.sg;
    float* wp = smem + H.wp;
    // [0,1] direction masks (bit per column) and [3,4] resync masks (bit per trajectory) by
    // round parity; [2] done mask; [5,6] "b' non-zero away from the endpoints" by round parity
    unsigned* flagw = reinterpret_cast<unsigned*>(smem + H.flags);
    float* obsL = smem + H.obs;
    const float* F1 = P.F1frag;
    const float* F2 = P.F2frag;

    const int KQ1 = MP / 16, KQa = NK / 16, MT1 = RP / 16;  // stage 1: (RP × MP)·(MP × 16)
    const int KQ2 = RP / 16, MT2 = MP / 16;                 // stage 2: (MP × RP)·(RP × 16)
    const int nsplit = sh.NSPLIT;
    // stage-1 unit of this wave (split-K over the position half): tile, k-quads [kq0, kq1)
    const bool has1 = wave < MT1 * nsplit;
    const int tile1 = wave % MT1, sp1 = wave / MT1;
    const int kq0 = (KQa * sp1) / nsplit, kq1 = (KQa * (sp1 + 1)) / nsplit;

    // ----------------------------------------------------------- prologue
    if (OPS_LDS && !REGOPS) {
        const Plan L = plan_lds(P, OPS_LDS, true);
        const int n1 = (int)frag_floats(RP, MP) / 4, n2 = (int)frag_floats(MP, RP) / 4;
        const f32x4* g1 = reinterpret_cast<const f32x4*>(P.F1frag);
        const f32x4* g2 = reinterpret_cast<const f32x4*>(P.F2frag);
        f32x4* l1 = reinterpret_cast<f32x4*>(smem + L.f1);
        f32x4* l2 = reinterpret_cast<f32x4*>(smem + L.f2);
        for (int e = tid; e < n1; e += P.BT) l1[e] = g1[e];
        for (int e = tid; e < n2; e += P.BT) l2[e] = g2[e];
        F1 = smem + L.f1;
        F2 = smem + L.f2;
    }
    // RV: the velocity half of stage 1's fragments is register-resident too (dense rounds, where
    // b' is non-zero away from the endpoints, then read no operator from memory)
    constexpr bool RV = REGOPS && MAXT > 256 && !BLS;  // (the BLS state leaves no room: spills)
    f32x4 a1[REGOPS ? S1Q : 1], a2[REGOPS ? S2T * 2 : 1], a1v[RV ? S1Q : 1];
    if (REGOPS) {  // operator A-fragments resident in VGPRs for the whole launch
        const f32x4* g1 = reinterpret_cast<const f32x4*>(P.F1frag);
        const f32x4* g2 = reinterpret_cast<const f32x4*>(P.F2frag);
#pragma unroll
        for (int i = 0; i < S1Q; ++i) {
            a1[i] = f32x4{0.f, 0.f, 0.f, 0.f};
            if (has1 && kq0 + i < kq1) a1[i] = g1[((size_t)tile1 * KQ1 + kq0 + i) * 64 + lane];
            if constexpr (RV) {
                a1v[i] = f32x4{0.f, 0.f, 0.f, 0.f};
                if (has1 && kq0 + i < kq1) a1v[i] = g1[((size_t)tile1 * KQ1 + KQa + kq0 + i) * 64 + lane];
            }
        }
#pragma unroll
        for (int j = 0; j < S2T; ++j)
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                a2[j * 2 + i] = f32x4{0.f, 0.f, 0.f, 0.f};
                const int tile = wave + j * nwaves;
                if (tile < MT2 && i < KQ2) a2[j * 2 + i] = g2[((size_t)tile * KQ2 + i) * 64 + lane];
            }
    }
    // endpoint-velocity operator columns for this lane's rows (sparse stage 1), and the
    // F rows of the two endpoint velocities for the BLS norms (rows r = n < RP)
    const float h0T = valid ? P.Hend[n] : 0.f, h1T = valid ? P.Hend[MP + n] : 0.f;
    const float h0V = valid ? P.Hend[NK + n] : 0.f, h1V = valid ? P.Hend[MP + NK + n] : 0.f;
    const float fb0 = yrow ? P.Fbot[(size_t)0 * RP + n] : 0.f;
    const float fb1 = yrow ? P.Fbot[(size_t)(N - 1) * RP + n] : 0.f;
    stage_obstacles(P, tb0, ntb, obsL);
    for (int e = tid; e < RP * kLd; e += P.BT) Ymix[e] = 0.f;
    // GD: the rounding residual rows e' live in dP's direction columns between an accepted step and the
    // next stage 1 (stage 2 rewrites dP only after the stage-1 barrier); none pending at start
    if constexpr (!BLS)
        for (int e = tid; e < MP * kLd; e += P.BT) dP[e] = 0.f;
    // G's endpoint velocity columns for this lane's row (G = V_R·y'·J⁻¹, see the latch)
    const float hv0 = valid ? P.HV[n] : 0.f, hv1 = valid ? P.HV[NK + n] : 0.f;
    if (tid < 8) flagw[tid] = 0u;
    // Parameters used only on rare paths (outer-loop step, line search, resync, series) live in
    // LDS so that they hold no SGPRs across the loop.
    float* cold = smem + H.cold;
    for (int i = tid; i < kColdWords; i += P.BT) {
        float val = 0.f;
        if (i < IRM_MAX_LR) val = P.gd_lr[i];
        else if (i == C_LCI) val = P.lci;
        else if (i == C_EPSP) val = P.eps_p;
        else if (i == C_EPSV) val = P.eps_v;
        else if (i == C_PMAX) val = P.pmax;
        else if (i == C_PMIN) val = P.pmin;
        else if (i == C_VMAX) val = P.vmax;
        else if (i == C_BLR0) val = P.bls_lr0;
        else if (i == C_BA) val = P.bls_a;
        else if (i == C_BP) val = P.bls_bp;
        else if (i == C_BM) val = P.bls_bm;
        else if (i == C_MAXOUT) val = __int_as_float(P.max_outer);
        else if (i == C_MAXBLS) val = __int_as_float(P.max_bls);
        else if (i == C_MAXSER) val = __int_as_float(P.max_series);
        else if (i == C_TRCAP) val = __int_as_float(P.trace ? P.trace_cap : 0);
        else if (i >= C_PTR && i < C_PTR + 10) {
            const int w = i - C_PTR;
            const void* ptrs[5] = {P.series, P.Vr, P.Kt, P.dKt, P.trace};
            const uint64_t a = reinterpret_cast<uint64_t>(ptrs[w >> 1]);
            val = __uint_as_float((w & 1) ? (uint32_t)(a >> 32) : (uint32_t)a);
        } else if (i >= C_MINV && i < C_MINV + D * D) val = P.Minv[i - C_MINV];
        else if (i >= C_WAL && i < C_WAL + D) val = P.wal[i - C_WAL];
        else if (i >= C_JINV && i < C_JINV + D * D) val = P.Jinv[i - C_JINV];
        else if (i >= C_J && i < C_J + D * D) val = P.J[i - C_J];
        cold[i] = val;
    }
    auto cold_ptr = [&](int w) -> float* {
        const uint64_t lo = __float_as_uint(cold[C_PTR + 2 * w]), hi = __float_as_uint(cold[C_PTR + 2 * w + 1]);
        return reinterpret_cast<float*>(lo | (hi << 32));
    };
    auto cold_int = [&](int i) { return __float_as_int(cold[i]); };
    stage_alpha<D>(P, tb0, ntb, X, NK);
    __syncthreads();
    // T0 = (K·α0)·J, V0 = (dK·α0)·J  (trajectory.py:63-65), correctly rounded.
    // ab: this lane's row of the α the state is expressed against (α0, then the α
    // materialised at the last resync).
    float q[D], v[D], s[D], g[D], ab[D], dT[D], dV[D], Gl[D];
#pragma unroll
    for (int k = 0; k < D; ++k) {
        q[k] = v[k] = 0.f;
        dT[k] = dV[k] = Gl[k] = 0.f;
        ab[k] = valid ? X[n * kLd + t * D + k] : 0.f;
        s[k] = tvalid ? P.start[b * D + k] : 0.f;
        g[k] = tvalid ? P.goal[b * D + k] : 0.f;
    }
    if (valid) {
        eval_exact<D>(P, X + t * D, n, q, v);
        if (rec) {
#pragma unroll
            for (int k = 0; k < D; ++k) P.series[(b * P.max_series) * N * D + n * D + k] = q[k];
        }
    }
    __syncthreads();  // every lane has read α0 from X
    for (int e = tid; e < MP * kLd; e += P.BT) X[e] = 0.f;
    const float* obs = obsL + (P.obs_stride ? t * obs_pitch(P.O) : 0);

    // stage 1 over the units of this wave: Ypart[s] = Fᵀ·[a'; b'] (velocity half if `full`)
    auto stage1 = [&](bool full) {
        const float* xl = X + (lane >> 4) * kLd + (lane & 15);
        // QB k-quads per batch: their operator fragments (L2) and B rows (LDS) in flight together, then
        // the MFMAs in the sequential order (dense / large-N operators; the REGOPS shapes keep QB = 1)
        auto quads = [&](const f32x4* ap, int qoff, int k0, int k1, f32x4& acc0, f32x4& acc1) {
            constexpr int QB = REGOPS ? 1 : 4;
            for (int kq = k0; kq < k1; kq += QB) {
                f32x4 a[QB];
                float bq[QB][4];
#pragma unroll
                for (int j = 0; j < QB; ++j) {
                    const bool in = kq + j < k1;
                    const float* xb = xl + (qoff + kq + j) * 16 * kLd;
                    a[j] = in ? ap[(size_t)(kq + j) * 64] : f32x4{0.f, 0.f, 0.f, 0.f};
                    bq[j][0] = in ? xb[0] : 0.f;
                    bq[j][1] = in ? xb[4 * kLd] : 0.f;
                    bq[j][2] = in ? xb[8 * kLd] : 0.f;
                    bq[j][3] = in ? xb[12 * kLd] : 0.f;
                }
#pragma unroll
                for (int j = 0; j < QB; ++j) {
                    if (kq + j < k1) {
                        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j][0], bq[j][0], acc0, 0, 0, 0);
                        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j][1], bq[j][1], acc1, 0, 0, 0);
                        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j][2], bq[j][2], acc0, 0, 0, 0);
                        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j][3], bq[j][3], acc1, 0, 0, 0);
                    }
                }
            }
        };
        if (REGOPS) {  // one unit per wave (regops_fit), position-half fragments in VGPRs
            if (has1) {
                // k-quads of this unit: compile-time count for the shape-specialised kernels
                constexpr bool kFix = S::KQU > 0 && S::KQU <= S1Q;
                constexpr int KQU = kFix ? S::KQU : S1Q;
                auto in = [&](int i) { return kFix ? i < KQU : kq0 + i < kq1; };
                float bv[KQU][4], bw[RV ? KQU : 1][4];
#pragma unroll
                for (int i = 0; i < KQU; ++i) {
                    const float* xb = xl + (kq0 + i) * 16 * kLd;
                    bv[i][0] = in(i) ? xb[0] : 0.f;
                    bv[i][1] = in(i) ? xb[4 * kLd] : 0.f;
                    bv[i][2] = in(i) ? xb[8 * kLd] : 0.f;
                    bv[i][3] = in(i) ? xb[12 * kLd] : 0.f;
                }
                if constexpr (RV) {
                    if (full) {
#pragma unroll
                        for (int i = 0; i < KQU; ++i) {
                            const float* xb = xl + (KQa + kq0 + i) * 16 * kLd;
                            bw[i][0] = in(i) ? xb[0] : 0.f;
                            bw[i][1] = in(i) ? xb[4 * kLd] : 0.f;
                            bw[i][2] = in(i) ? xb[8 * kLd] : 0.f;
                            bw[i][3] = in(i) ? xb[12 * kLd] : 0.f;
                        }
                    }
                }
                f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int i = 0; i < KQU; ++i) {
                    if (in(i)) {
                        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[i][0], bv[i][0], acc0, 0, 0, 0);
                        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[i][1], bv[i][1], acc1, 0, 0, 0);
                        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[i][2], bv[i][2], acc0, 0, 0, 0);
                        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[i][3], bv[i][3], acc1, 0, 0, 0);
                    }
                }
                if constexpr (RV) {
                    if (full) {
#pragma unroll
                        for (int i = 0; i < KQU; ++i) {
                            if (in(i)) {
                                acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1v[i][0], bw[i][0], acc0, 0, 0, 0);
                                acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1v[i][1], bw[i][1], acc1, 0, 0, 0);
                                acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1v[i][2], bw[i][2], acc0, 0, 0, 0);
                                acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1v[i][3], bw[i][3], acc1, 0, 0, 0);
                            }
                        }
                    }
                } else if (full) {
                    quads(reinterpret_cast<const f32x4*>(F1) + ((size_t)tile1 * KQ1 + KQa) * 64 + lane, KQa, kq0,
                          kq1, acc0, acc1);
                }
                store_tile(Ypart + sp1 * RP * kLd, tile1, acc0 + acc1, 0xFFFFu);
            }
        } else {
            for (int u = wave; u < MT1 * nsplit; u += nwaves) {
                const int tile = u % MT1, sp = u / MT1;
                const int k0 = (KQa * sp) / nsplit, k1 = (KQa * (sp + 1)) / nsplit;
                f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
                const f32x4* ap = reinterpret_cast<const f32x4*>(F1) + ((size_t)tile * KQ1) * 64 + lane;
                quads(ap, 0, k0, k1, acc0, acc1);
                if (full) quads(ap + (size_t)KQa * 64, KQa, k0, k1, acc0, acc1);
                store_tile(Ypart + sp * RP * kLd, tile, acc0 + acc1, 0xFFFFu);
            }
        }
    };

    // replicated per-trajectory scalar state
    float loss = 0.f, lsg = P.lsg0, ljl = P.ljl0, lr = 0.f, gnorm = 1.f, anorm = 0.f;
    float cfac = 1.f, step = 0.f;
    int phase = tvalid ? PH_OUTER_START : PH_DONE, outer = 0, inner = 0, trial = 0;
    bool needs_dir = false;
    irm_stats st{};
    st.series_len = rec ? 1 : 0;
    const unsigned tmask = (1u << D) - 1u;
    const unsigned fullmask = (ntb >= 32) ? 0xFFFFFFFFu : ((1u << ntb) - 1u);
    __syncthreads();
    IRM_STAMP(14);

    for (int round = 0;; ++round) {
        const int par = round & 1;
        const unsigned dirmask = flagw[par];
        const unsigned rmask = flagw[3 + par];
        const bool dense = flagw[5 + par] != 0u;  // b' has rows beyond the endpoints: full stage 1
        IRM_STAMP(4);
        if (tid == 0) {  // next round's masks (set in this round's flag section)
            flagw[par ^ 1] = 0u;
            flagw[3 + (par ^ 1)] = 0u;
            flagw[5 + (par ^ 1)] = 0u;
        }
        // ------------------------------------------------ direction (stage 1+2)
        if (dirmask) {
            // the two endpoint velocity rows of the trajectory's gradient inputs (sparse stage 1), read
            // before stage 1 (the waits move to the first use after the stage-1 barrier)
            float e0[D], e1[D];
#pragma unroll
            for (int k = 0; k < D; ++k) {
                e0[k] = X[NK * kLd + t * D + k];
                e1[k] = X[(NK + N - 1) * kLd + t * D + k];
            }
            IRM_STAMP(1);
            IRM_COUNT(13, dense);
            stage1(dense);
            if constexpr (!BLS) {
                // GD: z = V_Rᵀ·e' (the last accepted step's rounding residual, e' = −e·J/lr, rows of dP)
                // into Ymix, one unit per r-tile over all k-quads, operator from L2 — added to y' for
                // stage 2's F tiles, i.e. [T; V] += L·e·J one step late (k_lean's scheme)
                const float* xl = dP + (lane >> 4) * kLd + (lane & 15);
                // V_R = I (dense operator): z is e' itself (the MFMA's 1·e' plus exact zeros, from +0)
                if (P.v_ident) {
                    for (int u = nwaves - 1 - wave; u < MT1; u += nwaves) {
                        const float* er = dP + (u * 16 + 4 * (lane >> 4)) * kLd + (lane & 15);
                        f32x4 c0;
#pragma unroll
                        for (int i = 0; i < 4; ++i) c0[i] = 0.f + er[i * kLd];
                        store_tile(Ymix, u, c0, 0xFFFFu);
                    }
                } else
                for (int u = nwaves - 1 - wave; u < MT1; u += nwaves) {
                    const f32x4* ap = reinterpret_cast<const f32x4*>(P.VTs) + (size_t)u * KQa * 64 + lane;
                    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
                    for (int kq = 0; kq < KQa; ++kq) {
                        const f32x4 a = ap[(size_t)kq * 64];
                        const float* xb = xl + kq * 16 * kLd;
                        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], xb[0], acc0, 0, 0, 0);
                        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], xb[4 * kLd], acc1, 0, 0, 0);
                        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], xb[8 * kLd], acc0, 0, 0, 0);
                        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], xb[12 * kLd], acc1, 0, 0, 0);
                    }
                    store_tile(Ymix, u, acc0 + acc1, 0xFFFFu);
                }
            }
            IRM_STAMP(5);
            __syncthreads();
            IRM_STAMP(0);
            // BLS norms from y' rows (lane n = row r):
            //   ‖G‖² = Σ_r y'(JᵀJ)⁻¹y'ᵀ,  alpha_norm·‖G‖ = Σ_r (y'·w)², w = (JᵀJ)⁻¹Jᵀ1
            if (bls && needs_dir) {
                float g2 = 0.f, al = 0.f;
                if (yrow) {
                    float y[D];
#pragma unroll
                    for (int d = 0; d < D; ++d) y[d] = fmaf(fb0, e0[d], fb1 * e1[d]);
                    for (int sp = 0; sp < nsplit; ++sp) {
#pragma unroll
                        for (int d = 0; d < D; ++d) y[d] += Ypart[(sp * RP + n) * kLd + t * D + d];
                    }
#pragma unroll
                    for (int k = 0; k < D; ++k) {
                        float m = 0.f;
#pragma unroll
                        for (int d = 0; d < D; ++d) m = fmaf(y[d], cold[C_MINV + d * D + k], m);
                        g2 = fmaf(y[k], m, g2);
                        al = fmaf(cold[C_WAL + k], y[k], al);
                    }
                    al = al * al;
                }
                g2 = wred_sum(g2);
                al = wred_sum(al);
                if (lane == 0) {
                    wp[wave * 2] = g2;
                    wp[wave * 2 + 1] = al;
                }
            }
            IRM_STAMP(2);
            // stage 2: G tiles; GD also dP = F(MP × RP)·Σ_s Ypart[s], only the direction columns
            {
                constexpr int kTG = REGOPS ? 1 : 4;  // L2-operand tiles per pass (dense / large-N operators)
                const float* xl = Ypart + (lane >> 4) * kLd + (lane & 15);
                // y' rows (+ GD: z, the folded rounding residual, for the F tiles)
                auto bload = [&](int i, float& b0, float& b1, float& b2, float& b3, bool withz = true) {
                    b0 = b1 = b2 = b3 = 0.f;
                    for (int sp = 0; sp < nsplit; ++sp) {
                        const float* xb = xl + (sp * RP + i * 16) * kLd;
                        b0 += xb[0];
                        b1 += xb[4 * kLd];
                        b2 += xb[8 * kLd];
                        b3 += xb[12 * kLd];
                    }
                    if (withz) {
                        const float* zb = Ymix + (i * 16 + (lane >> 4)) * kLd + (lane & 15);
                        b0 += zb[0];
                        b1 += zb[4 * kLd];
                        b2 += zb[8 * kLd];
                        b3 += zb[12 * kLd];
                    }
                };
                {
                    // G tiles: (V_R·y')[waypoint] into X's position rows (X was consumed by stage 1;
                    // only the direction columns are written; every evaluation round rewrites X), from the
                    // top wave down
                    // dense operator (V_R = I): tile u of V_R·y' is y' rows u·16.. themselves — the MFMA's
                    // 1·y + exact zeros, i.e. the partial sums from +0 (bload's order): no operator loads
                    if (P.v_ident) {
                        for (int u = nwaves - 1 - wave; u < KQa; u += nwaves) {
                            const float* yr = Ypart + (u * 16 + 4 * (lane >> 4)) * kLd + (lane & 15);
                            f32x4 c0 = {0.f, 0.f, 0.f, 0.f};
                            for (int sp = 0; sp < nsplit; ++sp) {
#pragma unroll
                                for (int i = 0; i < 4; ++i) c0[i] += yr[(sp * RP + i) * kLd];
                            }
                            store_tile(X, u, c0, dirmask);
                        }
                    } else
                    // up to kTG tiles per pass over the k-quads: one B read shared by the pass's tiles and
                    // their A fragments in flight together (each tile's accumulation order unchanged)
                    for (int u0 = nwaves - 1 - wave; u0 < KQa; u0 += kTG * nwaves) {
                        f32x4 c[kTG];
#pragma unroll
                        for (int g = 0; g < kTG; ++g) c[g] = f32x4{0.f, 0.f, 0.f, 0.f};
                        for (int i = 0; i < KQ2; ++i) {
                            float b0, b1, b2, b3;
                            bload(i, b0, b1, b2, b3, false);
                            f32x4 a[kTG];
#pragma unroll
                            for (int g = 0; g < kTG; ++g) {
                                const int u = u0 + g * nwaves;
                                a[g] = u < KQa ? reinterpret_cast<const f32x4*>(P.VNs)[((size_t)u * KQ2 + i) * 64 + lane]
                                               : f32x4{0.f, 0.f, 0.f, 0.f};
                            }
#pragma unroll
                            for (int g = 0; g < kTG; ++g) {
                                if (u0 + g * nwaves < KQa) {
                                    c[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[g][0], b0, c[g], 0, 0, 0);
                                    c[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[g][1], b1, c[g], 0, 0, 0);
                                    c[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[g][2], b2, c[g], 0, 0, 0);
                                    c[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[g][3], b3, c[g], 0, 0, 0);
                                }
                            }
                        }
#pragma unroll
                        for (int g = 0; g < kTG; ++g)
                            if (u0 + g * nwaves < KQa) store_tile(X, u0 + g * nwaves, c[g], dirmask);
                    }
                }
                if constexpr (BLS) {
                    // BLS: no F tiles (the trial trajectories are evaluated exactly)
                } else if (REGOPS) {
                    f32x4 acc[S2T];
#pragma unroll
                    for (int j = 0; j < S2T; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
                    float bv[2][4];
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        if (i < KQ2) bload(i, bv[i][0], bv[i][1], bv[i][2], bv[i][3]);
                    }
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        if (i < KQ2) {
#pragma unroll
                            for (int j = 0; j < S2T; ++j) {
                                if (wave + j * nwaves < MT2) {
                                    acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a2[j * 2 + i][0], bv[i][0], acc[j], 0, 0, 0);
                                    acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a2[j * 2 + i][1], bv[i][1], acc[j], 0, 0, 0);
                                    acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a2[j * 2 + i][2], bv[i][2], acc[j], 0, 0, 0);
                                    acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a2[j * 2 + i][3], bv[i][3], acc[j], 0, 0, 0);
                                }
                            }
                        }
                    }
#pragma unroll
                    for (int j = 0; j < S2T; ++j)
                        if (wave + j * nwaves < MT2) store_tile(dP, wave + j * nwaves, acc[j], dirmask);
                } else {
                    for (int t0 = wave; t0 < MT2; t0 += kTG * nwaves) {  // kTG tiles per pass, as above
                        f32x4 c[kTG];
#pragma unroll
                        for (int g = 0; g < kTG; ++g) c[g] = f32x4{0.f, 0.f, 0.f, 0.f};
                        for (int i = 0; i < KQ2; ++i) {
                            float b0, b1, b2, b3;
                            bload(i, b0, b1, b2, b3);
                            f32x4 a[kTG];
#pragma unroll
                            for (int g = 0; g < kTG; ++g) {
                                const int tile = t0 + g * nwaves;
                                a[g] = tile < MT2 ? reinterpret_cast<const f32x4*>(F2)[((size_t)tile * KQ2 + i) * 64 + lane]
                                                  : f32x4{0.f, 0.f, 0.f, 0.f};
                            }
#pragma unroll
                            for (int g = 0; g < kTG; ++g) {
                                if (t0 + g * nwaves < MT2) {
                                    c[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[g][0], b0, c[g], 0, 0, 0);
                                    c[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[g][1], b1, c[g], 0, 0, 0);
                                    c[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[g][2], b2, c[g], 0, 0, 0);
                                    c[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[g][3], b3, c[g], 0, 0, 0);
                                }
                            }
                        }
#pragma unroll
                        for (int g = 0; g < kTG; ++g)
                            if (t0 + g * nwaves < MT2) store_tile(dP, t0 + g * nwaves, c[g], dirmask);
                    }
                }
            }
            __syncthreads();
            IRM_STAMP(3);
            if (needs_dir) {
                // GD: latch this lane's direction rows (+ the endpoint-velocity columns)
                if constexpr (!BLS) {
#pragma unroll
                    for (int k = 0; k < D; ++k) {
                        float ut = dP[n * kLd + t * D + k], uv = dP[(NK + n) * kLd + t * D + k];
                        // endpoint velocity rows: their operator columns in every round (stage 1's
                        // operator has zero columns there)
                        ut = fmaf(h0T, e0[k], fmaf(h1T, e1[k], ut));
                        uv = fmaf(h0V, e0[k], fmaf(h1V, e1[k], uv));
                        dT[k] = ut;
                        dV[k] = uv;
                    }
                }
                IRM_STAMP(16);
                // G = (V_R·y')·J⁻¹ + its endpoint velocity columns (y' = y·JᵀJ, G = V_R·y·Jᵀ)
                {
                    float gr[D];
#pragma unroll
                    for (int k = 0; k < D; ++k)
                        gr[k] = valid ? fmaf(hv0, e0[k], fmaf(hv1, e1[k], X[n * kLd + t * D + k])) : 0.f;
#pragma unroll
                    for (int k = 0; k < D; ++k) {
                        float gk = 0.f;
#pragma unroll
                        for (int l = 0; l < D; ++l) gk = fmaf(gr[l], cold[C_JINV + l * D + k], gk);
                        Gl[k] = gk;
                    }
                }
                if (bls) {
                    float tg = 0.f, ta = 0.f;
                    for (int ww = 0; ww < WPT; ++ww) {
                        tg += wp[(t * WPT + ww) * 2];
                        ta += wp[(t * WPT + ww) * 2 + 1];
                    }
                    gnorm = sqrtf(tg);
                    anorm = ta / gnorm;
                    st.grad_evals++;  // inner-loop head: cost + grad at α (optimizer_BLS.py:163-164)
                    st.cost_evals++;
                    phase = PH_BLS_TRIAL;
                    trial = 0;
                } else {
                    cfac = P.gd_c[outer];  // fp32(1 − λ_reg·lr) (optimizer_GD.py:185)
                    step = lr;
                }
                needs_dir = false;
            }
        }
        if (phase == PH_BLS_TRIAL) cfac = unfused(1.f - unfused(P.lreg * lr));  // (1 − λ_reg·bls_lr) in fp32 (optimizer_BLS.py:139)
        // ------------------------------------------------------- resync
        // Trajectories whose inner loop ended last round: [T; V] = eval_exact(α) (α is the reference's
        // fp32 iterate), so the constraint check below and the caller's evaluate(α_out) see the same
        // waypoints bit for bit; GD's pending residual is absorbed.
        if (rmask) {  // block-uniform; α is carried explicitly in fp32 (both optimisers)
            const bool rs = tvalid && ((rmask >> t) & 1u);  // wave-uniform
            if (rs && valid) {
#pragma unroll
                for (int k = 0; k < D; ++k) {
                    X[n * kLd + t * D + k] = ab[k];
                    dP[n * kLd + t * D + k] = 0.f;  // the pending residual is in the exact trajectory
                }
            }
            __syncthreads();
            if (rs && valid) {
                eval_exact<D>(P, X + t * D, n, q, v, cold_ptr(2), cold_ptr(3));
                if (rec && st.series_len > 0) {
                    float* ser = cold_ptr(0);
                    const int ms = cold_int(C_MAXSER);
#pragma unroll
                    for (int k = 0; k < D; ++k) ser[((b * ms) + st.series_len - 1) * N * D + n * D + k] = q[k];
                }
            }
        }
        IRM_STAMP(17);
        // ------------------------------------------------------- update
        float q2[D], v2[D], aj[BLS ? D : 1];
        // (K / dK rows per pipelined batch of the trial's exact evaluation: 8, as the resync's)
#ifndef IRM_X_TRIAL_U
        constexpr int kTrialU = 8;
#else
        constexpr int kTrialU = IRM_X_TRIAL_U;
#endif
        if constexpr (BLS) {
            // the trial's α_j = fl(fl(c_j·α) − fl(lr_j·ĝ)), ĝ = G/‖G‖ (optimizer_BLS.py:139, 165), through
            // X's position rows (consumed by this round's stage 1 and latch; rewritten by the gradient
            // inputs after the evaluation barrier), [T; V] = eval_exact(α_j)
            const bool trl = (phase == PH_BLS_TRIAL);  // wave-uniform
            if (trl && valid) {
#pragma unroll
                for (int k = 0; k < D; ++k) {
                    aj[k] = unfused(unfused(cfac * ab[k]) - unfused(lr * (Gl[k] / gnorm)));
                    X[n * kLd + t * D + k] = aj[k];
                }
            }
            __syncthreads();
            if (trl && valid) {
                eval_exact<D, kTrialU>(P, X + t * D, n, q2, v2, cold_ptr(2), cold_ptr(3));
            } else {
#pragma unroll
                for (int k = 0; k < D; ++k) {
                    q2[k] = q[k];
                    v2[k] = v[k];
                }
            }
        } else if (phase == PH_GD_INNER) {
#pragma unroll
            for (int k = 0; k < D; ++k) {
                q2[k] = fmaf(cfac, q[k], -(step * dT[k]));
                v2[k] = fmaf(cfac, v[k], -(step * dV[k]));
            }
        } else {
#pragma unroll
            for (int k = 0; k < D; ++k) {
                q2[k] = q[k];
                v2[k] = v[k];
            }
        }
        // ------------------------------------------------------- evaluate
        IRM_STAMP(6);
        const bool ev = (phase != PH_DONE);  // wave-uniform
        WP<D> w;
        if (ev) {
            if (valid) {
                if constexpr (S::kVariants) {
                    if (P.whole_robot) eval_waypoint<D, true, true, true>(P, q2, v2, obs, w);
                    else eval_waypoint<D, false, true, true>(P, q2, v2, obs, w);
                } else {
                    eval_waypoint<D, false, true, true>(P, q2, v2, obs, w);
                }
            }
            IRM_STAMP(8);
            const LeanW cw = lean_weights(P, ljl);
            const float us = fmaf(cw.c_mean, w.cv, cw.c_pen * (w.jp + w.jv));
            ered_store(valid, w.cv, us, w.tx, w.tn, w.va, phase == PH_RESYNC, n0, red, wave);
            if (valid && (n == 0 || n == N - 1)) {  // trajectory.py:183-204 rows 0 and N−1
                float a = 0.f, bb = 0.f;
#pragma unroll
                for (int d = 0; d < D; ++d) {
                    const float e = q2[d] - (n == 0 ? s[d] : g[d]);
                    a = fmaf(e, e, a);
                    bb = fmaf(v2[d], v2[d], bb);
                }
                sg[t * 4 + (n == 0 ? 0 : 2)] = a;
                sg[t * 4 + (n == 0 ? 1 : 3)] = bb;
            }
        }
        IRM_STAMP(9);
        __syncthreads();
        IRM_STAMP(7);
        if (ev) {
            // combine the trajectory's wave partials (fixed order)
            const float* r0 = red + (t * WPT) * 8;
            float cmax = r0[0];
            int cidx = __float_as_int(r0[1]);
            float usum = r0[2], tx = r0[3], tn = r0[4], va = r0[5];
            for (int ww = 1; ww < WPT; ++ww) {
                const float* rw = red + (t * WPT + ww) * 8;
                amax_step(cmax, cidx, rw[0], __float_as_int(rw[1]));
                usum += rw[2];
                tx = fmaxf(tx, rw[3]);
                tn = fminf(tn, rw[4]);
                va = fmaxf(va, rw[5]);
            }
            const float e_a0 = sg[t * 4 + 0], e_b0 = sg[t * 4 + 1], e_a1 = sg[t * 4 + 2], e_b1 = sg[t * 4 + 3];
            IRM_STAMP(18);
            const float sgpc = fmaf(0.5f, e_a0, 0.5f * e_a1);                   // trajectory.py:187
            const float sgvc = fmaf(0.5f, e_b0, 0.5f * e_b1);                   // trajectory.py:203
            // trajectory.py:85-87 + 281 (mean and joint-limit terms pre-summed in usum)
            const float nl = fmaf(lsg, sgpc + sgvc, fmaf(P.lam_max, cmax, usum));
            const float lsg_e = lsg, ljl_e = ljl;
            // --------------------------------------------------- decide
            int accept = 0;
            bool snap = false, to_end = false;
            if (phase == PH_OUTER_START) {  // optimizer_GD.py:209-211 / optimizer_BLS.py:193
                loss = nl;
                if (!bls) st.cost_evals++;
                accept = 2;
                lr = bls ? cold[C_BLR0] : cold[outer];
                needs_dir = true;
                if (!bls) phase = PH_GD_INNER;
                // BLS with max_outer_iteration <= 0: the reference's outer while_loop never runs and
                // optimize() returns α0 (optimizer_BLS.py:184-186, 210-213) — straight to the resync
                // (α materialised, constraints reported), no outer iteration counted
                if (P.max_inner <= 0 || (bls && cold_int(C_MAXOUT) <= 0)) to_end = true;
            } else if (phase == PH_BLS_REEVAL) {  // gradient at the unchanged α after a fully rejected search
                needs_dir = true;
            } else if (phase == PH_RESYNC) {
                // constraintsFulfilled(α) (trajectory.py:129-137, robot.py:90-113) on the
                // materialised α; optimizer_GD.py:214-224 / optimizer_BLS.py:201-211
                const float eps_p = cold[C_EPSP], eps_v = cold[C_EPSV];
                const bool ok = sqrtf(e_a0) < eps_p && sqrtf(e_a1) < eps_p && sqrtf(e_b0) < eps_v &&
                                sqrtf(e_b1) < eps_v && tx <= cold[C_PMAX] && tn >= cold[C_PMIN] && va <= cold[C_VMAX];
                if (!bls || cold_int(C_MAXOUT) > 0) st.outer_iterations++;
                st.constraints_ok = ok ? 1 : 0;
                if (ok) {
                    phase = PH_DONE;
                } else {
                    outer++;
                    lsg = lsg * cold[C_LCI];
                    ljl = ljl * cold[C_LCI];
                    inner = 0;
                    phase = (outer >= cold_int(C_MAXOUT)) ? PH_DONE : PH_OUTER_START;
                }
            } else if (phase == PH_GD_INNER) {  // optimizer_GD.py:180-195
                st.grad_evals++;
                st.cost_evals++;
                if (loss - nl < P.llr) {
                    to_end = true;  // minimized: the step is discarded
                } else {
                    accept = 1;
                    loss = nl;
                    inner++;
                    st.inner_iterations++;
                    snap = true;
                    if (inner >= P.max_inner) to_end = true;
                    else needs_dir = true;
                }
            } else {  // PH_BLS_TRIAL: optimizer_BLS.py:136-150, 172-178
                st.cost_evals++;
                st.bls_trials++;
                const float required = loss - cold[C_BA] * lr * anorm;
                // line-search log of problem 0 (diagnostics; the reference's per-trial values,
                // optimizer_BLS.py:139-149, 163-166)
                if (b == 0 && n == 0 && st.bls_trials - 1 < cold_int(C_TRCAP)) {
                    float* r = cold_ptr(4) + (size_t)(st.bls_trials - 1) * kTraceW;
                    r[0] = (float)outer;
                    r[1] = (float)inner;
                    r[2] = (float)trial;
                    r[3] = lr;
                    r[4] = nl;
                    r[5] = required;
                    r[6] = (nl > required) ? 0.f : 1.f;
                    r[7] = loss;
                    r[8] = gnorm;
                    r[9] = anorm;
                }
                bool inner_end = false, rejected_all = false;
                float improve = 0.f;
                if (nl > required) {
                    lr = lr * cold[C_BM];
                    trial++;
                    if (trial >= cold_int(C_MAXBLS)) inner_end = rejected_all = true;  // new_loss = loss
                } else {
                    accept = 1;
                    lr = lr * cold[C_BP];
                    improve = loss - nl;
                    loss = nl;
                    inner_end = true;
                }
                if (inner_end) {
                    if (improve < P.llr) {
                        to_end = true;
                    } else {
                        inner++;
                        st.inner_iterations++;
                        snap = true;
                        if (inner >= P.max_inner) {
                            to_end = true;
                        } else if (rejected_all) {
                            phase = PH_BLS_REEVAL;
                        } else {
                            needs_dir = true;
                        }
                    }
                }
            }
            if (to_end) {  // inner loop over: materialise α next round, then check constraints
                st.final_loss = loss;
                needs_dir = false;
                phase = PH_RESYNC;
            }
            IRM_STAMP(10);
            // ------------------------- gradient inputs at T2, mixed by JᵀJ (→ y' = y·JᵀJ)
            bool bfar = false;
            if (valid) {
                float a[D], bb[D], tg[D];
                const bool endrow = (n == 0 || n == N - 1);
#pragma unroll
                for (int k = 0; k < D; ++k) tg[k] = (n == N - 1) ? g[k] : s[k];
                grad_waypoint_lean<D>(P, w, q2, v2, n == cidx, endrow ? lsg_e : 0.f, lean_weights(P, ljl_e), tg, a, bb);
#pragma unroll
                for (int k = 0; k < D; ++k) {
                    float ma = 0.f, mb = 0.f;
#pragma unroll
                    for (int d = 0; d < D; ++d) {
                        ma = fmaf(a[d], P.JtJ[d * D + k], ma);
                        mb = fmaf(bb[d], P.JtJ[d * D + k], mb);
                    }
                    X[n * kLd + t * D + k] = ma;
                    X[(NK + n) * kLd + t * D + k] = mb;
                    bfar |= (!endrow && bb[k] != 0.f);
                }
            }
            if (__ballot(bfar) && lane == 0) atomicOr(&flagw[5 + (par ^ 1)], 1u);
            IRM_STAMP(12);
            // --------------------------------------------------- accept
            if (accept == 1) {
                if constexpr (BLS) {
                    // the trial's α_j and its exactly evaluated [T; V]
#pragma unroll
                    for (int k = 0; k < D; ++k) {
                        ab[k] = aj[k];
                        q[k] = q2[k];
                        v[k] = v2[k];
                    }
                } else {
                    // α' = fl(fl(c·α) − fl(lr·G)) (optimizer_GD.py:81, 185) and its residual e' = −e·J/lr
                    // for the next stage 1 (dP rows of this lane: stage 2 has been read)
                    float er[D];
#pragma unroll
                    for (int k = 0; k < D; ++k) {
                        ab[k] = alpha_step(ab[k], cfac, lr, Gl[k], step, Gl[k], er[k]);
                        q[k] = q2[k];
                        v[k] = v2[k];
                    }
                    if (valid) {
                        const float ne = -1.f / fmaxf(lr, kMinRefStep);
#pragma unroll
                        for (int k = 0; k < D; ++k) {
                            float z = 0.f;
#pragma unroll
                            for (int l = 0; l < D; ++l) z = fmaf(er[l], cold[C_J + l * D + k], z);
                            dP[n * kLd + t * D + k] = ne * z;
                        }
                    }
                }
            }
            // extended-vis snapshot after every non-breaking inner iteration
            // (optimizer_GD.py:153-154, optimizer_BLS.py:106-107)
            if (rec && snap && st.series_len < cold_int(C_MAXSER)) {
                if (valid) {
                    float* ser = cold_ptr(0);
                    const int ms = cold_int(C_MAXSER);
#pragma unroll
                    for (int k = 0; k < D; ++k) ser[((b * ms) + st.series_len) * N * D + n * D + k] = q[k];
                }
                st.series_len++;
            }
            if (n == 0) {
                if (needs_dir) atomicOr(&flagw[par ^ 1], tmask << (t * D));
                if (phase == PH_DONE) atomicOr(&flagw[2], 1u << t);
                if (phase == PH_RESYNC) atomicOr(&flagw[3 + (par ^ 1)], 1u << t);
            }
        }
        IRM_STAMP(15);
        __syncthreads();
        IRM_STAMP(11);
        if (flagw[2] == fullmask) break;
    }

    // ----------------------------------------------------------- epilogue
    // Every trajectory ended through PH_RESYNC: α = ab and T = eval_exact(α) exactly.
    if (valid) {
#pragma unroll
        for (int k = 0; k < D; ++k) {
            if (P.traj_out) P.traj_out[(b * N + n) * D + k] = q[k];
            if (P.alpha_out) P.alpha_out[(b * N + n) * D + k] = ab[k];
        }
    }
    if (P.stats && tvalid && n == 0) P.stats[b] = st;
    if (tid == 0) prof.flush(P.prof);
}

// ------------------------------------------- GD single loop, lean optimiser
// optimizer_GD.py jit_optimize (max_outer_iteration == 1, dualOptimization false;
// optimizer_GD.py:68-97): G = ∇L(α); α' = (1 − λ_reg·lr)·α − lr·G; accept iff
// L − L(α') ≥ loop_loss_reduction, else stop keeping α; at most max_inner steps; then
// constraintsFulfilled(α) decides constraints_ok.  Without the general state machine: every
// trajectory is either stepping or done, so a round needs no phase logic, no direction / resync
// masks; one parity flag word per round (bit per wave still stepping, bit 31 = dense stage 1) is
// OR-ed by the wave leaders and read by every wave after the end barrier.  Shape-specialised,
// F operators register-resident.
//
// α is carried in fp32 with the reference's rounding.  The reference iterates α (|α| ≈ 1e3, ulp
// ≈ 6e-5, singular K) in fp32: α' = fl(fl(c·α) − fl(lr·G)) — and the rounding of c·α is biased
// (c = 1 − 1.8e-7 moves α by 1.5–3 ulp per step), so its iterate drifts from the same iteration in
// exact arithmetic by ~1e-2 in waypoint space over 200 steps, 10× its own ±1-ulp sensitivity
// (tests/test_reference_bench.py).  Each lane therefore keeps its waypoint's α row
// and applies exactly that update.  The gradient inputs are mixed by Jᵀ when written ([a'; b'] =
// [a; b]·Jᵀ), so stage 1 gives y'' = Fᵀ[a; b]·Jᵀ and G = Lᵀ[a; b]·Jᵀ = V_R·y'' comes from a
// stage-2 tile set (G's endpoint velocity columns through hV) with no mix; the waypoint state
// [T; V] = L·α·J follows the exact part c·[T; V] − lr·(F·y'')·J as before, and the rounding
// residual e = α' − (c·α − lr·G) (error-free transformations: fma residuals and TwoSum) enters
// one round later through stage 1: z = V_Rᵀ·e', e' = −e/lr, is added to y'' on the way into stage
// 2's F tiles, i.e. [T; V] += L·e·J (rank R: the discarded part is below σ_R / σ_0 ≈ 1e-6 of it).
// Only J enters the per-lane mixes (D² scalars: at D = 7 three D×D matrices spilled SGPRs).  The
// evaluation point of a round therefore lags the exact L·α·J by one residual (≤ 1e-4 in
// waypoints, the size of the reference's own fp32 K@α noise); α itself is bit-for-bit the
// reference's update of the G the kernel computes, and the epilogue returns it with
// traj_out = K·α_out·J correctly rounded.
// LDS is column-major here — X / dP as [column][row] (stride MP + 8), the stage-1 partials as
// [split][column][r] (stride RP + 8), e' and G as [column][waypoint] (stride NK + 8) — with the
// k-permuted operator fragments (F1p / F2p / VTp / VNp, frag_index_kp): a lane's four B values of
// a k-group are then one ds_read_b128 and an MFMA result tile one ds_write_b128 per lane (strides
// ≡ 8 mod 16 keep both conflict-free).
// WPL waypoints per lane (lane li of a trajectory owns waypoints li + j·NW/WPL): WPL = 2 lets
// N = 256 trajectories run four to a 512-thread workgroup (C4) without exceeding 256 VGPRs.
template <int WPL>
__device__ __forceinline__ void ered_store_wpl(const bool (&live)[WPL], const float (&cv)[WPL], float us,
                                               float tx, float tn, float va, bool ext, int n0, int nwl,
                                               float* red, int wave) {
    if constexpr (WPL == 1) {
        ered_store(live[0], cv[0], us, tx, tn, va, ext, n0, red, wave);
    } else {
        // this lane's best waypoint (first index on ties: j = 0 is the smaller index)
        float best = live[0] ? cv[0] : -INFINITY;
        int jb = 0;
#pragma unroll
        for (int j = 1; j < WPL; ++j) {
            const float c = live[j] ? cv[j] : -INFINITY;
            if (c > best) {
                best = c;
                jb = j;
            }
        }
        const bool any = live[0];
        float m = best, s = any ? us : 0.f;  // best ≥ +0 or −inf: maxpos (see ered_store)
        m = maxpos(m, dppf<0xB1>(m));
        s += dppf<0xB1>(s);
        m = maxpos(m, dppf<0x4E>(m));
        s += dppf<0x4E>(s);
        m = maxpos(m, dppf<0x141>(m));
        s += dppf<0x141>(s);
        m = maxpos(m, dppf<0x140>(m));
        s += dppf<0x140>(s);
        auto pm = __builtin_amdgcn_permlane16_swap(__float_as_uint(m), __float_as_uint(m), false, false);
        auto ps = __builtin_amdgcn_permlane16_swap(__float_as_uint(s), __float_as_uint(s), false, false);
        const float m2 = maxpos(__uint_as_float(pm[0]), __uint_as_float(pm[1]));
        const float s2 = __uint_as_float(ps[0]) + __uint_as_float(ps[1]);
        auto qm = __builtin_amdgcn_permlane32_swap(__float_as_uint(m2), __float_as_uint(m2), false, false);
        auto qs = __builtin_amdgcn_permlane32_swap(__float_as_uint(s2), __float_as_uint(s2), false, false);
        const float wm = maxpos(__uint_as_float(qm[0]), __uint_as_float(qm[1]));
        const float ws = __uint_as_float(qs[0]) + __uint_as_float(qs[1]);
        int idx = 0x7fffffff;
#pragma unroll
        for (int j = WPL - 1; j >= 0; --j) {  // the smallest j with a hit holds the first index
            const unsigned long long hit = __ballot(best == wm && jb == j && live[j]);
            if (hit) idx = n0 + j * nwl + __builtin_ctzll(hit);
        }
        float ox = 0.f, on = 0.f, oa = 0.f;
        if (ext) {
            ox = wred_max(any ? tx : -INFINITY);
            on = wred_min(any ? tn : INFINITY);
            oa = wred_max(any ? va : 0.f);
        }
        if ((threadIdx.x & 63) == 0) {
            float* q = red + wave * 8;
            q[0] = wm;
            q[1] = __int_as_float(idx);
            q[2] = ws;
            q[3] = ox;
            q[4] = on;
            q[5] = oa;
        }
    }
}

// Control flows of the lean kernel: the GD single loop (optimizer_GD.py:68-97, the bench path), the
// GD dual loop (optimizer_GD.py:173-232) and the BLS dual loop (optimizer_BLS.py:127-213).
enum LeanFlow : int { LF_GD1 = 0, LF_GD2 = 1, LF_BLS = 2 };
// Per-trajectory phase (LF_GD2 / LF_BLS): a GD step or BLS trial this round, the end of an inner
// loop (α's exact trajectory, constraintsFulfilled, λ escalation), done.
enum LeanPhase : int { LP_STEP = 0, LP_RESYNC = 1, LP_DONE = 2 };
// BLS line-search helpers (k_lean): when one trajectory of a workgroup is left, the first done slot
// evaluates its next trial (lr·β₋) in the same round.  D ≤ 3, one waypoint per lane, N ≤ 128 in
// 512-thread workgroups (or N ≤ 64): where the exchange regions fit the LDS at full occupancy.
template <class S, int MAXT, int WPL, bool FULL, int FLOW>
constexpr bool lean_help() {
    return FLOW == LF_BLS && S::D <= 3 && WPL == 1 && FULL && S::kNW > 0 && (S::NK <= 64 || (S::NK <= 128 && MAXT > 256));
}

// FULL: the launch has exactly MAXT threads, so the stage-2 tiles per wave are known exactly
// (otherwise kS2T(MAXT) bounds them for smaller launches): C7's 256-thread variant then holds 4
// tiles of operator fragments instead of 8 (32 VGPRs) and does not spill.
template <class S, int MAXT, int WPL, bool FULL = false, int FLOW = LF_GD1>
__global__ __launch_bounds__(MAXT, (MAXT <= 256 && WPL == 1) ? 2 : 1) void k_lean(KParams P) {
    constexpr bool GD1 = FLOW == LF_GD1, BLS = FLOW == LF_BLS;
    constexpr int D = S::D;
    constexpr int S1Q = kS1Q(MAXT);
    // stage-2 tiles per wave: all of this shape's tiles over the workgroup's waves (N = 256: 4)
    constexpr int S2X = (S::MP / 16 + MAXT / 64 - 1) / (MAXT / 64);
    constexpr int S2T = (FULL || S2X > kS2T(MAXT)) ? S2X : kS2T(MAXT);
    // velocity half of stage 1 register-resident too — except in the dual-loop / BLS flows beyond C3's
    // shape, whose extra state leaves no room (read from L2 in the dense rounds there)
    constexpr bool RV = (MAXT > 256 || WPL > 1) && (GD1 || (D == 3 && S::NK <= 128));
    constexpr int NWL = S::NW / WPL;  // lanes per trajectory
    constexpr int WPTL = NWL / 64;    // waves per trajectory
    constexpr bool VL = lean_vlds(S::NK, D, MAXT);  // V_R fragments staged in LDS (else read from L2)
    static_assert(NWL % 64 == 0, "whole waves per trajectory");
    static_assert(WPL == 1 || (WPL == 2 && S::kNW > 0 && S::kNW == S::NK),
                  "two waypoints per lane: every lane's waypoints exist (N a multiple of 64)");
    // the dense operator (DenseShape: R = N, F = L, V_R = I) runs the GD single loop with its own stages
    constexpr bool DENSE = S::kDense;
    static_assert(S::RP == 32 || (DENSE && GD1 && WPL == 1 && FULL),
                  "k_lean runs at operator rank 32 (stage 2's kR24 slot skip), or the dense operator's GD loop");
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const S sh(P);
    const Head H = plan_head(sh.MP, sh.RP, sh.NSPLIT, true, true);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nwaves = FULL ? MAXT / 64 : P.BT >> 6;
    if constexpr (FULL) __builtin_assume(wave >= 0 && wave < MAXT / 64);  // tile guards fold
    const int N = sh.N, TB = P.TB, RP = sh.RP, MP = sh.MP, NK = sh.NK;
    const int t = wave / WPTL;
    const int li = tid - t * NWL;               // this lane within its trajectory
    const int n0 = (wave - t * WPTL) * 64;     // li of this wave's lane 0
    const int tb0 = blockIdx.x * TB;
    const int ntb = min(TB, P.B - tb0);
    if (ntb <= 0) return;
    const bool tvalid = t < ntb;
    int nn[WPL];
    bool vl[WPL];
#pragma unroll
    for (int j = 0; j < WPL; ++j) {
        nn[j] = li + j * NWL;
        vl[j] = tvalid && nn[j] < N;
    }
    // every lane of a valid trajectory holds waypoints when N fills whole waves: wherever only valid
    // trajectories run (evaluation, gradient inputs, the α update), the waypoint guards fold away
    constexpr bool kAllLive = S::kNW > 0 && S::kNW == S::N;
    bool wl[WPL];  // vl[j] where the trajectory is known to be valid
#pragma unroll
    for (int j = 0; j < WPL; ++j) wl[j] = kAllLive || nn[j] < N;
    const size_t b = (size_t)(tb0 + (tvalid ? t : 0));
    const bool rec = !GD1 && P.record_series && P.series;
    Prof prof;
    if (tid == 0) prof.init();

    float* X = smem + H.X;
    float* dP = smem + H.dP;
    float* Ypart = smem + H.Ypart;
    float* red = smem + H.red;
    float* sg = smem + H.sg;
    float* wp = smem + H.wp;
    unsigned* fw = reinterpret_cast<unsigned*>(smem + H.flags);
    float* obsL = smem + H.obs;
    const int nsplit = sh.NSPLIT, zsplit = lean_zsplit(sh.NSPLIT, VL);
    constexpr bool kHelp = lean_help<S, MAXT, WPL, FULL, FLOW>();
    // helpers read t*'s α, T, V from SS: t* publishes them at the top of each helper round rather than
    // after every accepted trial of every trajectory (C3-BLS −1 %, its faithful line −0.6 %; bit-identical)
    constexpr bool kSSLazy = kHelp;
    const LeanX LX = lean_extra(plan_lds(P, false, true, true).total, MP, NK, RP, nsplit, VL, D, kHelp ? MAXT : 0, BLS, DENSE);
    float* Eb = smem + LX.eb;  // e' rows [column][waypoint]
    float* Zp = smem + LX.zp;  // stage-1 partials of V_Rᵀ·e'
    float* Gb = smem + LX.gb;  // (V_R·y'')[waypoint] rows [column][waypoint]
    // b'[0], b'[N−1] of this trajectory (a copy of X's endpoint velocity rows, written with them): the B
    // operand of stage 1's endpoint MFMA (below)
    float* EPt = smem + LX.ep + t * 2 * kEpS;
    static_assert(D <= kEpS, "endpoint rows fit their slots");
    const float* VT = VL ? smem + LX.vt : P.VTp;
    const float* VN = VL ? smem + LX.vn : P.VNp;
    // V_R fragment quad q (VT: V_Rᵀ for z, VN: V_R for G): from LDS when staged there, else from L2 through a
    // buffer descriptor — the lane's offset in one VGPR, the wave-uniform quad offset in an SGPR, so a wave's
    // batch of fragment loads holds no 64-bit address per load (at N = 256 those spilled)
    const unsigned vbytes = (unsigned)(frag_floats(RP, NK) * 4);
    const __amdgpu_buffer_rsrc_t rVT = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(P.VTp), 0, (int)vbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rVN = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(P.VNp), 0, (int)vbytes, 0x00020000);
    auto vt_frag = [&](int q) -> f32x4 {
        if constexpr (VL) return reinterpret_cast<const f32x4*>(VT)[(size_t)q * 64 + lane];
        else return ld_frag(rVT, lane * 16, q * 1024);
    };
    auto vn_frag = [&](int q) -> f32x4 {
        if constexpr (VL) return reinterpret_cast<const f32x4*>(VN)[(size_t)q * 64 + lane];
        else return ld_frag(rVN, lane * 16, q * 1024);
    };

    const int KQ1 = MP / 16, KQa = NK / 16, MT1 = RP / 16, KQ2 = RP / 16, MT2 = MP / 16, MTG = NK / 16;
    const int ldx = MP + 8, ldy = lean_ldy(RP), lde = lean_ld(NK);  // column strides, all ≡ 8 mod 64
    const int cl = lane & 15, r4 = 4 * (lane >> 4);  // MFMA column / first of 4 rows of this lane
    // Bank swizzle of every [column][row] buffer: row r of column c lives at r ^ (c & 4) (the 4-row
    // quads of a 16-row group swap pairwise in columns 4-7 / 12-15).  With column strides ≡ 8 mod 64
    // the MFMA tiles' ds_read_b128 (16-lane groups, 64 banks) and ds_write_b128 (8-lane groups, 32
    // banks) are then both conflict-free; per-row accesses stay so (a column's rows only permute).
    const int r4x = r4 ^ (cl & 4);
    auto swz = [](int r, int c) { return r ^ (c & 4); };
    // 7-DoF shapes: a lane index laundered at a rare path's use, so that the path's per-lane addresses are
    // formed there instead of being held across the round loop (the 7-DoF dual-loop / BLS variants spilled
    // them); the 3-joint shapes have the registers, and measured 3 % slower on C3-BLS with it
    auto lnd = [](int x) {
        if constexpr (D > 3) asm volatile("" : "+v"(x));
        return x;
    };
    int ycl = cl;     // stage 2's Ypart column for this lane's B column (a helper round: the helper's read t*'s)
    int r4y = r4x;    // its first row under the row swizzle of column ycl
    const bool has1 = wave < MT1 * nsplit;
    const int tile1 = wave % MT1, sp1 = wave / MT1;
    const int kq0 = (KQa * sp1) / nsplit, kq1 = (KQa * (sp1 + 1)) / nsplit;

    // ----------------------------------------------------------- prologue
    f32x4 a1[S1Q], a1v[RV ? S1Q : 1], a2[S2T * 2];
    auto load_ops = [&]() {
        if constexpr (!VL) {  // (the shapes whose operands are read from L2: N = 256, 7-DoF, 256-thread)
            // buffer loads (the lane's offset in one VGPR): this also runs after each 7-DoF resync
            // (kReloadOps), where per-load 64-bit addresses held across the round loop were spilled
            const __amdgpu_buffer_rsrc_t r1 = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<float*>(P.F1p), 0, (int)(frag_floats(RP, MP) * 4), 0x00020000);
            const __amdgpu_buffer_rsrc_t r2 = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<float*>(P.F2p), 0, (int)(frag_floats(MP, RP) * 4), 0x00020000);
            const int vo = lane * 16;
#pragma unroll
            for (int i = 0; i < S1Q; ++i) {
                a1[i] = f32x4{0.f, 0.f, 0.f, 0.f};
                if (has1 && kq0 + i < kq1) a1[i] = ld_frag(r1, vo, ((tile1 * KQ1 + kq0 + i) * 64) * 16);
                if constexpr (RV) {
                    a1v[i] = f32x4{0.f, 0.f, 0.f, 0.f};
                    if (has1 && kq0 + i < kq1) a1v[i] = ld_frag(r1, vo, ((tile1 * KQ1 + KQa + kq0 + i) * 64) * 16);
                }
            }
#pragma unroll
            for (int j = 0; j < S2T; ++j)
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    a2[j * 2 + i] = f32x4{0.f, 0.f, 0.f, 0.f};
                    const int tile = wave + j * nwaves;
                    if (tile < MT2 && i < KQ2) a2[j * 2 + i] = ld_frag(r2, vo, ((tile * KQ2 + i) * 64) * 16);
                }
        } else {
            const f32x4* g1 = reinterpret_cast<const f32x4*>(P.F1p);
            const f32x4* g2 = reinterpret_cast<const f32x4*>(P.F2p);
#pragma unroll
            for (int i = 0; i < S1Q; ++i) {
                a1[i] = f32x4{0.f, 0.f, 0.f, 0.f};
                if (has1 && kq0 + i < kq1) a1[i] = g1[((size_t)tile1 * KQ1 + kq0 + i) * 64 + lane];
                if constexpr (RV) {
                    a1v[i] = f32x4{0.f, 0.f, 0.f, 0.f};
                    if (has1 && kq0 + i < kq1) a1v[i] = g1[((size_t)tile1 * KQ1 + KQa + kq0 + i) * 64 + lane];
                }
            }
#pragma unroll
            for (int j = 0; j < S2T; ++j)
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    a2[j * 2 + i] = f32x4{0.f, 0.f, 0.f, 0.f};
                    const int tile = wave + j * nwaves;
                    if (tile < MT2 && i < KQ2) a2[j * 2 + i] = g2[((size_t)tile * KQ2 + i) * 64 + lane];
                }
        }
    };
    if constexpr (!DENSE) load_ops();  // (DENSE: every operator fragment streamed from L2 in its stage)
    // The endpoint velocity rows b'[0], b'[N−1] (stage 1's operator Fᵀ has zero columns there, so that a
    // sparse round can skip the velocity half) enter y'' through one more MFMA per stage-1 row tile, on
    // the split-0 units: k = 0 ↔ b'[0], k = 1 ↔ b'[N−1], k = 2, 3 zero.  A = the operator's endpoint
    // columns Fᵀ[r][NK], Fᵀ[r][NK + N − 1] (F_bot rows 0 and N − 1), held in one VGPR for the launch;
    // B = the trajectory's compact copy of the two rows (EPt, column cl = t·D + k).  Stage 2 then sees
    // them in y'' like every other row: the direction F·(y'' + z), G = V_R·y'' and the BLS norms need no
    // endpoint terms of their own.
    const bool hasep = has1 && sp1 == 0;  // wave-uniform
    float aep = 0.f;
    if (hasep && (lane >> 4) < 2) aep = P.Fbot[(size_t)((lane >> 4) ? N - 1 : 0) * RP + tile1 * 16 + (lane & 15)];
    // this lane's B address: column cl of trajectory cl / D, row k = lane >> 4 (a zero slot for k ≥ 2)
    const int epoff = (lane >> 4) < 2 ? LX.ep + (cl / D) * 2 * kEpS + (lane >> 4) * kEpS + cl % D : LX.ep0;
    // the 7-DoF BLS flow forms it again at its use (held across the round loop it was spilled)
    auto ep_at = [&]() {
        if constexpr (BLS && D > 3 && MAXT > 256) {
            int l = lane;
            asm volatile("" : "+v"(l));
            const int c = l & 15;
            return (l >> 4) < 2 ? LX.ep + (c / D) * 2 * kEpS + (l >> 4) * kEpS + c % D : LX.ep0;
        } else {
            return epoff;
        }
    };
    if constexpr (VL) {
        const int nv = (int)frag_floats(RP, NK) / 4;  // = frag_floats(NK, RP) / 4
        const f32x4* gt = reinterpret_cast<const f32x4*>(P.VTp);
        const f32x4* gn = reinterpret_cast<const f32x4*>(P.VNp);
        f32x4* lt = reinterpret_cast<f32x4*>(smem + LX.vt);
        f32x4* ln = reinterpret_cast<f32x4*>(smem + LX.vn);
        for (int e = tid; e < nv; e += P.BT) {
            lt[e] = gt[e];
            ln[e] = gn[e];
        }
    }
    for (int e = tid; e < 16 * lde; e += P.BT) Eb[e] = 0.f;  // no pending residual; rows ≥ N stay 0 (BLS: α rows)
    if constexpr (BLS)
        for (int e = tid; e < kMaxTraj * kTsW; e += P.BT) smem[LX.ts + e] = 0.f;  // no slot in a line search yet
    for (int e = tid; e < kMaxTraj * 2 * kEpS + 4; e += P.BT) smem[LX.ep + e] = 0.f;  // + the zero word
    stage_obstacles(P, tb0, ntb, obsL);
    stage_alpha<D>(P, tb0, ntb, X, NK);
    if (tid < 2) fw[tid] = 0u;
    // J for the resyncs' exact evaluations (eval_exact's Jm), in the head's parameter block
    float* Jl = smem + H.cold + C_J;
    if (tid < D * D) Jl[tid] = P.J[tid];
    __syncthreads();
    // the reference's α (fp32, this lane's waypoint rows) and T0 = (K·α0)·J, V0 = (dK·α0)·J
    float q[WPL][D], v[WPL][D], al[WPL][D];
    float s[D], g[D];
#pragma unroll
    for (int k = 0; k < D; ++k) {
        s[k] = tvalid ? P.start[b * D + k] : 0.f;
        g[k] = tvalid ? P.goal[b * D + k] : 0.f;
    }
    float epf[WPL], tg[WPL][D];  // start/goal rows of the gradient inputs, per lane
    unsigned long long endm[WPL];  // the wave's endpoint-row lanes
#pragma unroll
    for (int j = 0; j < WPL; ++j) {
        epf[j] = (nn[j] == 0 || nn[j] == N - 1) ? 1.f : 0.f;
        // opaque to the compiler: tests of epf stay one compare (it otherwise re-derives the nested
        // n == 0 / n == N − 1 tests from the select, an exec-mask cascade of ≈ 20 scalar instructions)
        asm volatile("" : "+v"(epf[j]));
        endm[j] = __ballot(epf[j] != 0.f);
#pragma unroll
        for (int k = 0; k < D; ++k) tg[j][k] = (nn[j] == N - 1) ? g[k] : s[k];
    }
#pragma unroll
    for (int j = 0; j < WPL; ++j) {
#pragma unroll
        for (int k = 0; k < D; ++k) {
            q[j][k] = v[j][k] = 0.f;
            al[j][k] = vl[j] ? X[nn[j] * kLd + t * D + k] : 0.f;
            // BLS: the α rows the trial stages read (written with every accepted trial)
            if (BLS && vl[j]) Eb[(t * D + k) * lde + swz(nn[j], t * D + k)] = al[j][k];
        }
        if (vl[j]) {
            eval_exact<D>(P, X + t * D, nn[j], q[j], v[j]);
            if (rec) {  // series frame 0: the initial trajectory
#pragma unroll
                for (int k = 0; k < D; ++k) P.series[(b * P.max_series) * N * D + nn[j] * D + k] = q[j][k];
            }
        }
    }
    __syncthreads();
    for (int e = tid; e < MP * kLd; e += P.BT) X[e] = 0.f;
    const float* obs = obsL + (P.obs_stride ? t * obs_pitch(P.O) : 0);  // (a helper round: t*'s)
    // 9-12 obstacles (the reference's 11): the padded table in VGPRs for the whole launch (24 floats),
    // so the per-round evaluation does not wait on its LDS reads
    // (and the 3-joint GD dual loop: C3 faithful 3.70 -> 3.60 ms; the BLS flow with it measured C3-BLS
    // −0.5 % but C2 +2.7 %, not used; the 7-DoF dual loop spills with it)
#if defined(IRM_X_OREG_ALL)
    constexpr bool OREG = true;
#else
    constexpr bool OREG = GD1 || (D <= 3 && !BLS);
#endif
    f32x4 oreg[OREG ? 6 : 1];
    const bool obs_reg = ((P.O + 3) >> 2) == 3;
#pragma unroll
    for (int i = 0; i < (OREG ? 6 : 1); ++i) oreg[i] = obs_reg ? reinterpret_cast<const f32x4*>(obs)[i] : f32x4{0.f, 0.f, 0.f, 0.f};
    // replicated per-trajectory state
    float lsg = P.lsg0, ljl = P.ljl0;
    float lr = BLS ? P.bls_lr0 : P.gd_lr[0];
    float cfac = P.gd_c[0];  // GD: fp32(1 − λ_reg·lr) of the outer iteration
    float gnorm = 1.f, anorm = 0.f;  // BLS: ‖G‖ and alpha_norm of the current direction
    int outer = 0, inner = 0, trial = 0;
    int phase = tvalid ? LP_STEP : LP_DONE;
    bool needs_dir = false, xdense = false;
    const float nilr = -1.f / fmaxf(lr, kMinRefStep);  // GD single loop: e' = −e/lr (the dual loop recomputes per outer)

    // evaluation of (q2, v2) with this trajectory's waves: wave partials + endpoint rows
    auto evaluate = [&](const float (&q2)[WPL][D], const float (&v2)[WPL][D], bool ext, float ljl_e,
                        WP<D> (&w)[WPL]) {
        float cvs[WPL], us = 0.f, tx = -INFINITY, tn = INFINITY, va = 0.f;
        const LeanW cw = lean_weights(P, ljl_e);
        // every lane of an evaluating trajectory holds waypoints when N fills whole waves (only valid
        // trajectories evaluate): the liveness selects of the reductions fold away
        bool lv[WPL];
#pragma unroll
        for (int j = 0; j < WPL; ++j) lv[j] = kAllLive || vl[j];
        if constexpr (WPL == 2) {  // both waypoints' obstacle terms in one pass (vl[0] = vl[1] = tvalid here)
            if (tvalid) {
                eval_waypoint<D, false, false, true>(P, q2[0], v2[0], obs, w[0]);
                eval_waypoint<D, false, false, true>(P, q2[1], v2[1], obs, w[1]);
                potential_pair<D>(P, obs, w[0], w[1]);
            }
        }
#pragma unroll
        for (int j = 0; j < WPL; ++j) {
            if (WPL == 1 && lv[j]) eval_waypoint<D, false, true, true>(P, q2[j], v2[j], obs, w[j], OREG ? oreg : nullptr);  // oreg: read only when nq == 3
            cvs[j] = w[j].cv;
            const float u = fmaf(cw.c_mean, w[j].cv, cw.c_pen * (w[j].jp + w[j].jv));
            if (j == 0) {
                us = u;
                tx = w[j].tx;
                tn = w[j].tn;
                va = w[j].va;
            } else if (vl[j]) {
                us += u;
                tx = fmaxf(tx, w[j].tx);
                tn = fminf(tn, w[j].tn);
                va = fmaxf(va, w[j].va);
            }
        }
        IRM_STAMP(6);
        ered_store_wpl<WPL>(lv, cvs, us, tx, tn, va, ext, n0, NWL, red, wave);
#pragma unroll
        for (int j = 0; j < WPL; ++j) {
            const int n = nn[j];
            if (lv[j] && epf[j] != 0.f) {  // trajectory.py:183-204 rows 0 and N−1 (epf: one compare, no cascade)
                float a = 0.f, bb = 0.f;
#pragma unroll
                for (int d = 0; d < D; ++d) {
                    const float e = q2[j][d] - tg[j][d];  // tg: s on row 0, g on row N − 1
                    a = fmaf(e, e, a);
                    bb = fmaf(v2[j][d], v2[j][d], bb);
                }
                sg[t * 4 + (n == 0 ? 0 : 2)] = a;
                sg[t * 4 + (n == 0 ? 1 : 3)] = bb;
            }
        }
    };
    struct Fin {
        float nl, tx, tn, va, a0, b0, a1, b1;
        int idx;
    };
    // Latency-hiding load batches (finalize's records and start/goal terms, stage 2's split-K partial
    // sums, the z unit's operands) hold more values live at once: stage 2's and the z unit's only for
    // N <= 128, where they fit without spills; at N = 256 (four splits, eight z ranges) they pushed the
    // spill-free GD single-loop variants into scratch (C5: 14 spilled VGPRs)
    // finalize's batch: fixed shapes with one waypoint per lane (C4's two-waypoints-per-lane kernel, one
    // wave record per trajectory, measured 2 % slower with it; C5 / C7 1.5-2 % faster)
    constexpr bool kLatF = S::kNW > 0 && WPL == 1;
    constexpr bool kLatS = S::kNW > 0 && S::NK <= 128;   // stage 2's and the z unit's: N <= 128
    auto finalize = [&](float lsg_e, int ft) {  // ft: the trajectory slot whose records are read
        if constexpr (!kLatF) {
            const float* r0 = red + (ft * WPTL) * 8;
            float cmax = r0[0];
            int cidx = __float_as_int(r0[1]);
            float usum = r0[2], tx = r0[3], tn = r0[4], va = r0[5];
            for (int ww = 1; ww < WPTL; ++ww) {
                const float* rw = red + (ft * WPTL + ww) * 8;
                amax_step(cmax, cidx, rw[0], __float_as_int(rw[1]));
                usum += rw[2];
                tx = fmaxf(tx, rw[3]);
                tn = fminf(tn, rw[4]);
                va = fmaxf(va, rw[5]);
            }
            Fin f;
            f.a0 = sg[ft * 4 + 0];
            f.b0 = sg[ft * 4 + 1];
            f.a1 = sg[ft * 4 + 2];
            f.b1 = sg[ft * 4 + 3];
            const float sgpc = fmaf(0.5f, f.a0, 0.5f * f.a1);  // trajectory.py:187
            const float sgvc = fmaf(0.5f, f.b0, 0.5f * f.b1);  // trajectory.py:203
            f.nl = fmaf(lsg_e, sgpc + sgvc, fmaf(P.lam_max, cmax, usum));
            f.idx = cidx;
            f.tx = tx;
            f.tn = tn;
            f.va = va;
            return f;
        }
        // every wave record and the start/goal terms are read before the first use (one LDS round trip;
        // the argmax merge as selects, so no read is sunk into a branch)
        float rr[WPTL][6], sgr[4];
#pragma unroll
        for (int ww = 0; ww < WPTL; ++ww)
#pragma unroll
            for (int e = 0; e < 6; ++e) rr[ww][e] = red[(ft * WPTL + ww) * 8 + e];
#pragma unroll
        for (int e = 0; e < 4; ++e) sgr[e] = sg[ft * 4 + e];
        __builtin_amdgcn_sched_barrier(0);
        float cmax = rr[0][0];
        int cidx = __float_as_int(rr[0][1]);
        float usum = rr[0][2], tx = rr[0][3], tn = rr[0][4], va = rr[0][5];
#pragma unroll
        for (int ww = 1; ww < WPTL; ++ww) {
            const float ov = rr[ww][0];
            const int oi = __float_as_int(rr[ww][1]);
            const bool take = (ov > cmax) | ((ov == cmax) & (oi < cidx));  // amax_step (no short-circuit branch)
            cmax = take ? ov : cmax;
            cidx = take ? oi : cidx;
            usum += rr[ww][2];
            tx = fmaxf(tx, rr[ww][3]);
            tn = fminf(tn, rr[ww][4]);
            va = fmaxf(va, rr[ww][5]);
        }
        Fin f;
        f.a0 = sgr[0];
        f.b0 = sgr[1];
        f.a1 = sgr[2];
        f.b1 = sgr[3];
        const float sgpc = fmaf(0.5f, f.a0, 0.5f * f.a1);  // trajectory.py:187
        const float sgvc = fmaf(0.5f, f.b0, 0.5f * f.b1);  // trajectory.py:203
        // the same value in every lane (LDS broadcasts): as a scalar, the loss and the step decisions
        // built on it are wave-uniform to the compiler too (scalar branches, the loss in an SGPR)
        f.nl = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(
                                             __builtin_bit_cast(int, fmaf(lsg_e, sgpc + sgvc, fmaf(P.lam_max, cmax, usum)))));
        f.idx = cidx;
        f.tx = tx;
        f.tn = tn;
        f.va = va;
        return f;
    };
    // gradient inputs at (q2, v2), mixed by Jᵀ, into X; returns "b' non-zero away from the endpoints"
    auto grad_inputs = [&](const WP<D> (&w)[WPL], const float (&q2)[WPL][D], const float (&v2)[WPL][D], int cidx,
                           float lsg_e, float ljl_e, int gt) {  // gt: the trajectory slot whose X columns are written
        float* EPg = EPt + (gt - t) * 2 * kEpS;
        unsigned long long bfar = 0ull;  // lanes with b' ≠ 0 (as ballots of the compares: no boolean in a VGPR)
        const LeanW cw = lean_weights(P, ljl_e);
#pragma unroll
        for (int j = 0; j < WPL; ++j) {
            const int n = nn[j];
            if (wl[j]) {  // (valid trajectories only)
                float a[D], bb[D], ep[D];
                grad_waypoint_lean<D>(P, w[j], q2[j], v2[j], n == cidx, epf[j] * lsg_e, cw, tg[j], a, bb);
                const bool endrow = epf[j] != 0.f;
#pragma unroll
                for (int k = 0; k < D; ++k) {
                    float ma = 0.f, mb = 0.f;
#pragma unroll
                    for (int d = 0; d < D; ++d) {
                        ma = fmaf(a[d], P.J[k * D + d], ma);
                        mb = fmaf(bb[d], P.J[k * D + d], mb);
                    }
                    X[(gt * D + k) * ldx + swz(n, gt * D + k)] = ma;
                    X[(gt * D + k) * ldx + NK + swz(n, gt * D + k)] = mb;
                    bfar |= __ballot(bb[k] != 0.f) & ~endm[j];
                    ep[k] = mb;
                }
                if (endrow) {  // the compact copy of the endpoint rows (read at the next round's top)
                    // (one region with a per-lane address: the nested n == 0 / n == N − 1 tests compiled to
                    // an exec-mask cascade of ≈ 20 scalar instructions on every wave)
                    const int n2 = lnd(n);  // (7-DoF: the offset formed here, not held across the round loop)
                    float* e = EPg + (n2 == 0 ? 0 : kEpS);
#pragma unroll
                    for (int k = 0; k < D; ++k) e[k] = ep[k];
                }
            }
        }
        return bfar != 0ull;
    };
    // GD single loop, fixed-shape launches: stage 1's B operand (both halves; the velocity half is used
    // in dense rounds only) is read at the top of the round, before the flag word (X was written before
    // the previous barrier), so the flag and operand LDS round trips overlap; same values, same MFMA
    // order (bit-identical, tools/sched_check.py).  C3 0.769 -> 0.759 ms; the position half alone: no gain.
    constexpr bool kFix1 = S::KQU > 0 && S::KQU <= S1Q;
    constexpr int KQU1 = kFix1 ? S::KQU : S1Q;
    // (the GD dual loop with the same prefetch: 4.33 -> 4.47 ms, 242 VGPRs there; not used)
    constexpr bool kPre1 = GD1 && FULL && kFix1;
    constexpr bool kPreW = kPre1 && RV;
    auto stage1_load = [&](f32x4 (&bv)[KQU1], f32x4 (&bw)[KQU1], float& bep) {
        const float* xl = X + cl * ldx + r4x;
        if (has1) {  // wave-uniform
#pragma unroll
            for (int i = 0; i < KQU1; ++i) {
                bv[i] = *reinterpret_cast<const f32x4*>(xl + (kq0 + i) * 16);
                if constexpr (kPreW) bw[i] = *reinterpret_cast<const f32x4*>(xl + (KQa + kq0 + i) * 16);
            }
            bep = smem[epoff];  // (a valid word on every stage-1 wave; used on the endpoint waves)
        }
    };
    // Ypart[sp] = Fᵀ·[a'; b'] over this wave's unit (+ the endpoint rows' MFMA on the split-0 units)
    auto stage1 = [&](bool full, const f32x4 (&pre)[KQU1], const f32x4 (&prew)[KQU1], float prep) {
        if (!has1) return;
        const float* xl = X + cl * ldx + r4x;
        constexpr bool kFix = kFix1;
        constexpr int KQU = KQU1;
        auto in = [&](int i) { return kFix ? i < KQU : kq0 + i < kq1; };
        const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
        f32x4 bv[KQU], bw[RV ? KQU : 1];
#pragma unroll
        for (int i = 0; i < KQU; ++i) {
            if constexpr (kPre1) bv[i] = pre[i];
            else bv[i] = in(i) ? *reinterpret_cast<const f32x4*>(xl + (kq0 + i) * 16) : z4;
        }
        if constexpr (RV) {
            if (full) {
#pragma unroll
                for (int i = 0; i < KQU; ++i) {
                    if constexpr (kPreW) bw[i] = prew[i];
                    else bw[i] = in(i) ? *reinterpret_cast<const f32x4*>(xl + (KQa + kq0 + i) * 16) : z4;
                }
            }
        }
        f32x4 acc0 = z4, acc1 = z4;
        // fixed shapes: the second chain's first product is the endpoint MFMA's successor or starts from
        // zero itself (one MFMA result either way: no zeroed accumulator on the non-endpoint waves)
        if constexpr (kFix) {
            if (hasep) {
                acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(aep, kPre1 ? prep : smem[ep_at()], z4, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[0][1], bv[0][1], acc1, 0, 0, 0);
            } else {
                acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[0][1], bv[0][1], z4, 0, 0, 0);
            }
        } else if (hasep) {
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(aep, kPre1 ? prep : smem[ep_at()], acc1, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < KQU; ++i) {
            if (in(i)) {
                acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[i][0], bv[i][0], acc0, 0, 0, 0);
                if (!kFix || i > 0) acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[i][1], bv[i][1], acc1, 0, 0, 0);
                acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[i][2], bv[i][2], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[i][3], bv[i][3], acc1, 0, 0, 0);
            }
        }
        if (full) {
            if constexpr (RV) {
#pragma unroll
                for (int i = 0; i < KQU; ++i) {
                    if (in(i)) {
                        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1v[i][0], bw[i][0], acc0, 0, 0, 0);
                        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1v[i][1], bw[i][1], acc1, 0, 0, 0);
                        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1v[i][2], bw[i][2], acc0, 0, 0, 0);
                        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1v[i][3], bw[i][3], acc1, 0, 0, 0);
                    }
                }
            } else if constexpr (!VL) {
                // (buffer loads: the lane's offset in one VGPR, no 64-bit address held across the round loop)
                const __amdgpu_buffer_rsrc_t r1 = __builtin_amdgcn_make_buffer_rsrc(
                    const_cast<float*>(P.F1p), 0, (int)(frag_floats(RP, MP) * 4), 0x00020000);
                for (int kq = kq0; kq < kq1; ++kq) {
                    const f32x4 a = ld_frag(r1, lane * 16, ((tile1 * KQ1 + KQa + kq) * 64) * 16);
                    const f32x4 bb = *reinterpret_cast<const f32x4*>(xl + (KQa + kq) * 16);
                    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], bb[0], acc0, 0, 0, 0);
                    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], bb[1], acc1, 0, 0, 0);
                    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], bb[2], acc0, 0, 0, 0);
                    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], bb[3], acc1, 0, 0, 0);
                }
            } else {
                const f32x4* ap = reinterpret_cast<const f32x4*>(P.F1p) + ((size_t)tile1 * KQ1 + KQa) * 64 + lane;
                for (int kq = kq0; kq < kq1; ++kq) {
                    const f32x4 a = ap[(size_t)kq * 64];
                    const f32x4 bb = *reinterpret_cast<const f32x4*>(xl + (KQa + kq) * 16);
                    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], bb[0], acc0, 0, 0, 0);
                    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], bb[1], acc1, 0, 0, 0);
                    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], bb[2], acc0, 0, 0, 0);
                    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], bb[3], acc1, 0, 0, 0);
                }
            }
        }
        *reinterpret_cast<f32x4*>(Ypart + (sp1 * 16 + cl) * ldy + tile1 * 16 + r4x) = acc0 + acc1;
    };
    // z = V_Rᵀ·e' (the last accepted step's rounding residual) at rank 16: the residual's components
    // along singular directions 16-31 of [K; dK] are below σ_16/σ_0 ≈ 4e-4 of |L·e| ≈ 1e-4, i.e. under
    // 1e-7 per step, so only V_R's first row tile is applied (half the MFMAs of rank 32; Zp rows 16-31
    // stay zero).  zsplit k-ranges over the waves from the top down (C3: waves 4-7, idle in the Fᵀ
    // stage), operator from LDS / L2.
    // FULL launches of a fixed shape with an even split: the unit's operator and e' loads are issued
    // up front (one wait), then the MFMAs — the same accumulation order as the loop below
    constexpr int kZS = lean_zsplit(S::NSPLIT, VL), kKQa = S::NK / 16;
    constexpr bool kZFix = FULL && S::kNW > 0 && kKQa % kZS == 0 && kZS <= MAXT / 64;
    constexpr int kKQZ = kZFix ? kKQa / kZS : 1;
    constexpr int kMTG = S::NK / 16, kGT = (kMTG + MAXT / 64 - 1) / (MAXT / 64);
    constexpr bool kS2Fix = FULL && S::kNW > 0;
    // GD flows of the fixed shapes: the z unit's V_Rᵀ fragments and the G tiles' V_R fragments are the same
    // every round — held in VGPRs for the launch instead of re-read from LDS / L2 each round
    // (C3 faithful 3.93 -> 3.75 ms, C3 even; from L2 too: C7 1.33 -> 1.27 ms, C7 faithful 7.52 -> 7.30 ms,
    // C5 1.405 -> 1.326 ms, C4 even; bit-identical.  Not the 7-DoF N = 256 dual loop / 256-thread
    // variants, which spill with them)
    constexpr bool kVReg = !BLS && !DENSE && kZFix && kS2Fix && (VL || !(D > 3 && S::NK > 128) || (GD1 && MAXT > 256));
    // otherwise (C5's dual loop) the z unit's V_Rᵀ fragments are loaded at the round's top, so their L2
    // latency passes under stage 1 instead of holding the z waves at the stage-1 barrier
    // (C5 faithful −1.4 %, C4 even; bit-identical)
    constexpr bool kZPre = !BLS && !DENSE && kZFix && !kVReg;
    f32x4 vtR[kVReg ? kKQZ : 1], vnR[kVReg ? kGT : 1][2];
    if constexpr (kVReg) {
        const int sp = nwaves - 1 - wave;
#pragma unroll
        for (int i = 0; i < kKQZ; ++i) vtR[i] = sp < kZS ? vt_frag(sp * kKQZ + i) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int g = 0; g < kGT; ++g) {
            const int u = nwaves - 1 - wave + g * nwaves;
            vnR[g][0] = vnR[g][1] = f32x4{0.f, 0.f, 0.f, 0.f};
            if (u < kMTG) {
                vnR[g][0] = vn_frag(u * KQ2);
                vnR[g][1] = vn_frag(u * KQ2 + 1);
            }
        }
    }
    auto zpre_load = [&](f32x4 (&zp)[kZPre ? kKQZ : 1]) {
        if constexpr (kZPre) {
            const int sp = nwaves - 1 - wave;
            if (sp < kZS) {
#pragma unroll
                for (int i = 0; i < kKQZ; ++i) zp[i] = vt_frag(sp * kKQZ + i);
            }
        }
    };
    auto stage1z = [&](const f32x4 (&zp)[kZPre ? kKQZ : 1]) {
        const float* el = Eb + cl * lde + r4x;
        if constexpr (kZFix) {
            constexpr int KQZ = kKQZ;
            const int sp = nwaves - 1 - wave;
            if (sp >= kZS) return;
            f32x4 a[KQZ], bb[KQZ];
#pragma unroll
            for (int i = 0; i < KQZ; ++i) {
                if constexpr (kZPre) a[i] = zp[i];
                else a[i] = kVReg ? vtR[i] : vt_frag(sp * KQZ + i);
                bb[i] = *reinterpret_cast<const f32x4*>(el + (sp * KQZ + i) * 16);
            }
            if constexpr (kLatS) __builtin_amdgcn_sched_barrier(0);  // all loads in flight before the first MFMA
            f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int i = 0; i < KQZ; ++i) {
                acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][0], bb[i][0], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][1], bb[i][1], acc1, 0, 0, 0);
                acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][2], bb[i][2], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][3], bb[i][3], acc1, 0, 0, 0);
            }
            *reinterpret_cast<f32x4*>(Zp + (sp * 16 + cl) * ldy + r4x) = acc0 + acc1;
            return;
        }
        for (int sp = nwaves - 1 - wave; sp < zsplit; sp += nwaves) {
            const int k0 = (KQa * sp) / zsplit, k1 = (KQa * (sp + 1)) / zsplit;
            f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
            for (int kq = k0; kq < k1; ++kq) {
                const f32x4 a = vt_frag(kq);
                const f32x4 bb = *reinterpret_cast<const f32x4*>(el + kq * 16);
                acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], bb[0], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], bb[1], acc1, 0, 0, 0);
                acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], bb[2], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], bb[3], acc1, 0, 0, 0);
            }
            *reinterpret_cast<f32x4*>(Zp + (sp * 16 + cl) * ldy + r4x) = acc0 + acc1;
        }
    };
    // stage 2: dP = F·(Σ_s Ypart[s] + Σ_s Zp[s]) (the pending residual folded in) at rank 16 (kR16F),
    // Gb = V_R·Σ_s Ypart[s] at rank 24 (kR24): the host puts the singular components 24-31 (σ/σ_0 ≈
    // 3e-8, fp32 noise of the rank-32 factorisation) into the rank slots that MFMAs 2-3 of the second
    // k-quad read, and those MFMAs are skipped (irm_host.cpp, slot()); k_lean always runs at RP = 32.
    // The α iterate uses G (rank 24, the reference's gradient to fp32 resolution); the waypoint state
    // follows the rank-16 direction, off L·α·J by ≲ 1.5e-7 of a step per step (the one-residual lag
    // below is 1e-4), and every inner-loop end replaces it by eval_exact(α).
    // FULL launches of a fixed shape: the G tiles of a wave are known at compile time; their operator
    // fragments are loaded with the partial sums and their MFMAs interleave with the F tiles' (same
    // accumulation order per tile as the general form below)
    constexpr bool kS2Batch = kS2Fix && kLatS;  // stage 2's partial sums read in one batch
    // WF: the F tiles (dP, with the residual z folded in), WG: the G tiles (Gb).  The GD flows run both in
    // one pass; the BLS flow runs G in the rounds with a new gradient input and F in every trial round
    // (its trial's own residual folded in, so the direction is the trial iterate's)
    // the GD single loop's G tiles issued after the stage-2 barrier (their MFMAs under the update and
    // evaluation; C3 -2.0 %, bit-identical)
#ifdef IRM_X_GLATE_ALL
    constexpr bool kGLate = !BLS && !DENSE && kS2Fix && kS2Batch;
#else
    // (WPTL > 1 only: glate_tiles' waves write G rows of trajectories they do not own, and with one wave per
    // trajectory — N ≤ 64 — only a wave barrier would sit between that write and the owner's read)
    constexpr bool kGLate = GD1 && D <= 3 && kS2Fix && kS2Batch && WPTL > 1;
#endif
    f32x4 glY0 = f32x4{0.f, 0.f, 0.f, 0.f}, glY1 = f32x4{0.f, 0.f, 0.f, 0.f};
    // (kGLate) the G tiles, issued right after the stage-2 barrier: their MFMAs under the update /
    // evaluation's VALU work; Gb is read after the evaluation's barrier (the decision).  Issued after the
    // update instead, C3 measured +5.7 %
    auto glate_tiles = [&]() {
#pragma unroll
        for (int g = 0; g < kGT; ++g) {
            const int u = nwaves - 1 - wave + g * nwaves;
            if (u < kMTG) {
                const f32x4 g0 = kVReg ? vnR[g][0] : vn_frag(u * KQ2);
                const f32x4 g1 = kVReg ? vnR[g][1] : vn_frag(u * KQ2 + 1);
                f32x4 ag = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int m = 0; m < 4; ++m) ag = __builtin_amdgcn_mfma_f32_16x16x4f32(g0[m], glY0[m], ag, 0, 0, 0);
#pragma unroll
                for (int m = 0; m < 2; ++m) ag = __builtin_amdgcn_mfma_f32_16x16x4f32(g1[m], glY1[m], ag, 0, 0, 0);
                *reinterpret_cast<f32x4*>(Gb + cl * lde + u * 16 + r4x) = ag;
            }
        }
    };
    auto stage2f = [&](auto WFc, auto WGc) {
        constexpr bool WF = decltype(WFc)::value, WG = decltype(WGc)::value;
        f32x4 acc[S2T];
#pragma unroll
        for (int j = 0; j < S2T; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
        f32x4 ga[kS2Fix ? kGT : 1][2];
        if constexpr (kS2Fix && WG) {
#pragma unroll
            for (int g = 0; g < kGT; ++g) {
                const int u = nwaves - 1 - wave + g * nwaves;
                ga[g][0] = ga[g][1] = f32x4{0.f, 0.f, 0.f, 0.f};
                if (u < kMTG) {
                    ga[g][0] = kVReg ? vnR[g][0] : vn_frag(u * KQ2);
                    ga[g][1] = kVReg ? vnR[g][1] : vn_frag(u * KQ2 + 1);
                }
            }
        }
        f32x4 by[2], bt[2];
        if constexpr (kS2Batch) {
            // every split-K partial of y'' and z is read before the first sum (one LDS round trip; the
            // machine scheduler otherwise reuses one register quad for the reads and waits after each,
            // seven round trips per round); same sums in the same order as the general form below
            // (the second k-quad feeds only the G tiles' MFMAs 0-1 (kR24): its rows 0-1 of each quad)
            // (read as whole quads: the swizzled layout is conflict-free for ds_read_b128, not for the
            // b64 reads the compiler narrows these to — SQ_LDS_BANK_CONFLICT 0.8 M -> 4.1 M cycles)
            constexpr int NS = S::NSPLIT;
            f32x4 yp[NS], zq[kZS], yq[NS];
#pragma unroll
            for (int sp = 0; sp < NS; ++sp) {
                yp[sp] = *reinterpret_cast<const f32x4*>(Ypart + (sp * 16 + ycl) * ldy + r4y);
                yq[sp] = *reinterpret_cast<const f32x4*>(Ypart + (sp * 16 + ycl) * ldy + 16 + r4y);
            }
#pragma unroll
            for (int sp = 0; sp < (WF ? kZS : 0); ++sp) zq[sp] = *reinterpret_cast<const f32x4*>(Zp + (sp * 16 + cl) * ldy + r4x);
            // every quad stays whole (no narrowing, no register reuse of its unused half while in flight)
#pragma unroll
            for (int sp = 0; sp < NS; ++sp) asm volatile("" ::"v"(yq[sp]));
#pragma unroll
            for (int g = 0; g < (WG ? kGT : 0); ++g) asm volatile("" ::"v"(ga[g][1]));
            __builtin_amdgcn_sched_barrier(0);
            // the sums start from the first partial (not from +0: four adds fewer per quad; a partial
            // of −0 stays −0, which changes no MFMA product sum that is not exactly zero)
            f32x2 b1 = {yq[0].x, yq[0].y};
            by[0] = yp[0];
#pragma unroll
            for (int sp = 1; sp < NS; ++sp) {
                by[0] += yp[sp];
                b1 += f32x2{yq[sp].x, yq[sp].y};
            }
            if constexpr (kS2Fix && WF && WG) {
                // the G tiles first, on y'' alone (read first), while the z partials are still in flight;
                // then the F tiles on y'' + z — each tile's MFMA chain unchanged (bit-identical; C3 −0.4 %,
                // C3 faithful −1 %)
                const f32x4 by1 = f32x4{b1.x, b1.y, 0.f, 0.f};
                f32x4 ag[kGT];
                if constexpr (kGLate) {
                    glY0 = by[0];
                    glY1 = by1;
                }
#pragma unroll
                for (int g = 0; g < kGT; ++g) {
                    ag[g] = f32x4{0.f, 0.f, 0.f, 0.f};
                    if (!kGLate && nwaves - 1 - wave + g * nwaves < kMTG) {
#pragma unroll
                        for (int m = 0; m < 4; ++m) ag[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(ga[g][0][m], by[0][m], ag[g], 0, 0, 0);
#pragma unroll
                        for (int m = 0; m < 2; ++m) ag[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(ga[g][1][m], by1[m], ag[g], 0, 0, 0);
                    }
                }
                __builtin_amdgcn_sched_barrier(0);  // (the z sums after the G chain: it must not wait for them)
                f32x4 bz = zq[0];
#pragma unroll
                for (int sp = 1; sp < kZS; ++sp) bz += zq[sp];
                const f32x4 b0 = by[0] + bz;
#pragma unroll
                for (int m = 0; m < 4; ++m)
#pragma unroll
                    for (int j = 0; j < S2T; ++j)
                        if (wave + j * nwaves < MT2)
                            acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a2[j * 2][m], b0[m], acc[j], 0, 0, 0);
#pragma unroll
                for (int j = 0; j < S2T; ++j)
                    if (wave + j * nwaves < MT2)
                        *reinterpret_cast<f32x4*>(dP + cl * ldx + (wave + j * nwaves) * 16 + r4x) = acc[j];
#pragma unroll
                for (int g = 0; g < kGT; ++g) {
                    const int u = nwaves - 1 - wave + g * nwaves;
                    if (!kGLate && u < kMTG) *reinterpret_cast<f32x4*>(Gb + cl * lde + u * 16 + r4x) = ag[g];
                }
                return;
            }
            if constexpr (WF) {
                f32x4 bz = zq[0];
#pragma unroll
                for (int sp = 1; sp < kZS; ++sp) bz += zq[sp];
                bt[0] = by[0] + bz;
            } else {
                bt[0] = by[0];
            }
            by[1] = bt[1] = f32x4{b1.x, b1.y, 0.f, 0.f};
        }
#pragma unroll
        for (int i = 0; i < (kS2Batch ? 0 : 2); ++i) {
            by[i] = bt[i] = f32x4{0.f, 0.f, 0.f, 0.f};
            if (i < KQ2) {
                f32x4 bz = {0.f, 0.f, 0.f, 0.f};
                for (int sp = 0; sp < nsplit; ++sp)
                    by[i] += *reinterpret_cast<const f32x4*>(Ypart + (sp * 16 + ycl) * ldy + i * 16 + r4y);
                if (i == 0 && WF) {  // z has rank 16: rows 0-15 only
                    for (int sp = 0; sp < zsplit; ++sp)
                        bz += *reinterpret_cast<const f32x4*>(Zp + (sp * 16 + cl) * ldy + r4x);
                }
                bt[i] = by[i] + bz;
            }
        }
        // the waypoint direction F·(y'' + z) at rank 16: F_r·y''_r ∝ σ_r², (σ_16/σ_0)² ≈ 1.5e-7 (N = 128),
        // i.e. the fp32 rounding level of the direction itself (kR16F)
        if constexpr (kS2Fix) {
            f32x4 ag[kGT];
#pragma unroll
            for (int g = 0; g < kGT; ++g) ag[g] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int m = 0; m < 4; ++m) {
#pragma unroll
                for (int j = 0; j < (WF ? S2T : 0); ++j)
                    if (wave + j * nwaves < MT2)
                        acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a2[j * 2][m], bt[0][m], acc[j], 0, 0, 0);
#pragma unroll
                for (int g = 0; g < (WG ? kGT : 0); ++g)
                    if (nwaves - 1 - wave + g * nwaves < kMTG)
                        ag[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(ga[g][0][m], by[0][m], ag[g], 0, 0, 0);
            }
#pragma unroll
            for (int m = 0; m < 2; ++m)  // kR24
#pragma unroll
                for (int g = 0; g < (WG ? kGT : 0); ++g)
                    if (nwaves - 1 - wave + g * nwaves < kMTG)
                        ag[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(ga[g][1][m], by[1][m], ag[g], 0, 0, 0);
#pragma unroll
            for (int j = 0; j < (WF ? S2T : 0); ++j)
                if (wave + j * nwaves < MT2)
                    *reinterpret_cast<f32x4*>(dP + cl * ldx + (wave + j * nwaves) * 16 + r4x) = acc[j];
#pragma unroll
            for (int g = 0; g < (WG ? kGT : 0); ++g) {
                const int u = nwaves - 1 - wave + g * nwaves;
                if (u < kMTG) *reinterpret_cast<f32x4*>(Gb + cl * lde + u * 16 + r4x) = ag[g];
            }
            return;
        }
#pragma unroll
        for (int j = 0; j < (WF ? S2T : 0); ++j) {
            if (wave + j * nwaves < MT2) {
#pragma unroll
                for (int m = 0; m < 4; ++m)
                    acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a2[j * 2][m], bt[0][m], acc[j], 0, 0, 0);
            }
        }
#pragma unroll
        for (int j = 0; j < (WF ? S2T : 0); ++j) {
            if (wave + j * nwaves < MT2)
                *reinterpret_cast<f32x4*>(dP + cl * ldx + (wave + j * nwaves) * 16 + r4x) = acc[j];
        }
        // G tiles (waypoint rows of V_R·y''), from the top wave down
        for (int u = nwaves - 1 - wave; WG && u < MTG; u += nwaves) {
            f32x4 ag = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                if (i < KQ2) {
                    const f32x4 a = vn_frag(u * KQ2 + i);
#pragma unroll
                    for (int m = 0; m < (i == 1 ? 2 : 4); ++m)  // kR24
                        ag = __builtin_amdgcn_mfma_f32_16x16x4f32(a[m], by[i][m], ag, 0, 0, 0);
                }
            }
            *reinterpret_cast<f32x4*>(Gb + cl * lde + u * 16 + r4x) = ag;
        }
    };
    // ---- BLS trial stages.  A trial j of a line search is evaluated at its own fp32 iterate
    // α_j = fl(fl(c_j·α) − fl(lr_j·ĝ)) (optimizer_BLS.py:139-140): its trajectory is c_j·[T; V] − s_j·F·(y'' + z_j)·J
    // with z_j = V_Rᵀ·e'_j, e'_j = −(α_j − (c_j·α − s_j·G))/s_j the iterate's rounding residual.
    // The G-tile waves form e'_j themselves, element by element of their G tiles (the MFMA result layout
    // of a tile is the k-permuted B layout of the z MFMAs over the same 16 waypoints), and accumulate their
    // tiles' share of z_j in the same pass: no per-lane residual rows, no barrier between G, the residual
    // and z.  A round with a new direction: stage 1 → barrier → G tiles + ‖G‖ + α_j + z partials →
    // barrier → F tiles → barrier; a round that continues a line search: α_j + z partials from the stored
    // G / α rows → barrier → F tiles → barrier.  Every column's trial is its trajectory's current one (lr
    // from TS); a helper's columns take t*'s next (lr·β₋): ycl is the column whose y'', G and α the
    // lane's column reads.
    constexpr int kNZP = lean_bls_nzp(S::kNW > 0 ? S::NK : 256);
    const int nzp = min(nwaves, MTG);  // z partials (one per G-tile wave)
    // (fixed shapes up to N = 128: at N = 256 the batch's per-tile operands — four tiles per wave at 256
    // threads — pushed the BLS variants into scratch; those take the per-tile loop, same sums in the same order)
    constexpr bool kBFix = FULL && S::kNW > 0 && S::NK <= 128;
    constexpr int kNZc = kBFix ? (MAXT / 64 < S::NK / 16 ? MAXT / 64 : S::NK / 16) : 1;
    static_assert(!BLS || !kBFix || kNZc <= kNZP, "z partials fit their region");
    float* Ab = smem + LX.eb;    // BLS: α rows [column][waypoint] (Eb's place)
    float* Ajb = smem + LX.aj;   // BLS: the round's trial iterate α_j, rows [column][waypoint]
    float* Zq = smem + LX.zp;    // BLS: z partials, quad-major
    float* TS = smem + LX.ts;    // BLS: per-slot lr, ‖G‖, in-a-line-search flag
    // V_R staged in LDS: the G-tile waves' V_R / V_Rᵀ fragments held in VGPRs for the launch (as kVReg)
    constexpr int kTB = kBFix ? (S::NK / 16 + MAXT / 64 - 1) / (MAXT / 64) : 1;  // tiles per wave
    // (C3-BLS faithful 7.21 -> 7.17 ms, C3-BLS 1.426 -> 1.419 ms; bit-identical)
    constexpr bool kVRegB = BLS && VL && kBFix;
    f32x4 bvt[kVRegB ? kTB : 1], bvn[kVRegB ? kTB : 1][2];
    if constexpr (kVRegB) {
#pragma unroll
        for (int g = 0; g < kTB; ++g) {
            const int u = nwaves - 1 - wave + g * (MAXT / 64);
            bvt[g] = bvn[g][0] = bvn[g][1] = f32x4{0.f, 0.f, 0.f, 0.f};
            if (u < S::NK / 16) {
                bvt[g] = vt_frag(u);
                bvn[g][0] = vn_frag(u * KQ2);
                bvn[g][1] = vn_frag(u * KQ2 + 1);
            }
        }
    }
    auto bls_gz = [&](auto freshc, bool hmr, int hsr) {  // fresh (a new direction this round): G from y''
        constexpr bool fresh = decltype(freshc)::value;
        const int pz = nwaves - 1 - wave;  // this wave's z partial; its G tiles are u = pz + g·nwaves
        if (pz >= MTG) return;             // (wave-uniform)
        const int sc = ycl / D;            // the trial's trajectory slot (t* for a helper's columns)
        // the slot's trial scalars, read with the round's first LDS batch
        const float lrs = TS[sc * kTsW + 0];
        const bool act = TS[sc * kTsW + 2] != 0.f;  // (other slots: no residual)
        constexpr int kT = kBFix ? (S::NK / 16 + MAXT / 64 - 1) / (MAXT / 64) : 1;  // tiles per wave (fixed)
        const int ntl = kBFix ? kT : (MTG - pz + nwaves - 1) / nwaves;
        f32x4 Gt[kBFix ? kT : 1];
        // fixed shapes: every tile's α rows and V_Rᵀ fragment (and, continuing a search, its stored G) read
        // in the round's first LDS batch
        f32x4 Ap[kBFix ? kT : 1], Vp[kBFix ? kT : 1];
        if constexpr (kBFix) {
#pragma unroll
            for (int g = 0; g < kT; ++g) {
                const int u = pz + g * (MAXT / 64);
                Ap[g] = Vp[g] = Gt[g] = f32x4{0.f, 0.f, 0.f, 0.f};
                if (u < S::NK / 16) {
                    Ap[g] = *reinterpret_cast<const f32x4*>(Ab + ycl * lde + u * 16 + r4y);
                    Vp[g] = kVRegB ? bvt[g] : vt_frag(u);
                    if constexpr (!fresh) Gt[g] = *reinterpret_cast<const f32x4*>(Gb + ycl * lde + u * 16 + r4y);
                }
            }
        }
        float gn;
        if constexpr (fresh) {
            // y'' of column ycl, ranks r4..r4+3 and 16+r4..19+r4, summed over the stage-1 splits in order
            f32x4 y0, y1;
            if constexpr (kBFix) {
                f32x4 yp[S::NSPLIT], yq[S::NSPLIT], gv[kT][2];
#pragma unroll
                for (int sp = 0; sp < S::NSPLIT; ++sp) {
                    yp[sp] = *reinterpret_cast<const f32x4*>(Ypart + (sp * 16 + ycl) * ldy + r4y);
                    yq[sp] = *reinterpret_cast<const f32x4*>(Ypart + (sp * 16 + ycl) * ldy + 16 + r4y);
                }
#pragma unroll
                for (int g = 0; g < kT; ++g) {
                    const int u = pz + g * (MAXT / 64);
                    gv[g][0] = gv[g][1] = f32x4{0.f, 0.f, 0.f, 0.f};
                    if (u < S::NK / 16) {
                        gv[g][0] = kVRegB ? bvn[g][0] : vn_frag(u * KQ2);
                        gv[g][1] = kVRegB ? bvn[g][1] : vn_frag(u * KQ2 + 1);
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
                y0 = yp[0];
                y1 = yq[0];
#pragma unroll
                for (int sp = 1; sp < S::NSPLIT; ++sp) {
                    y0 += yp[sp];
                    y1 += yq[sp];
                }
                // G = V_R·y'' at rank 24 (kR24, the order of stage2f), issued before the norm's VALU work
#pragma unroll
                for (int g = 0; g < kT; ++g) {
                    Gt[g] = f32x4{0.f, 0.f, 0.f, 0.f};
                    if (pz + g * (MAXT / 64) < S::NK / 16) {
#pragma unroll
                        for (int m = 0; m < 4; ++m) Gt[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(gv[g][0][m], y0[m], Gt[g], 0, 0, 0);
#pragma unroll
                        for (int m = 0; m < 2; ++m) Gt[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(gv[g][1][m], y1[m], Gt[g], 0, 0, 0);
                    }
                }
            } else {
                y0 = *reinterpret_cast<const f32x4*>(Ypart + ycl * ldy + r4y);
                y1 = *reinterpret_cast<const f32x4*>(Ypart + ycl * ldy + 16 + r4y);
                for (int sp = 1; sp < nsplit; ++sp) {
                    y0 += *reinterpret_cast<const f32x4*>(Ypart + (sp * 16 + ycl) * ldy + r4y);
                    y1 += *reinterpret_cast<const f32x4*>(Ypart + (sp * 16 + ycl) * ldy + 16 + r4y);
                }
            }
            // ‖G‖² = ‖y''‖² (V_R orthonormal) per trajectory (optimizer_BLS.py:165): the lane's 8 squares, the
            // column over its four lane rows (permlane swaps: the same sums in the same order in every lane),
            // then the slot's D columns in column order (lanes sc·D + a of row 0); every G-tile wave forms
            // the same values
            float sq = 0.f;
#pragma unroll
            for (int i = 0; i < 4; ++i) sq = fmaf(y0[i], y0[i], sq);
#pragma unroll
            for (int i = 0; i < 4; ++i) sq = fmaf(y1[i], y1[i], sq);
            const auto p16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(sq), __float_as_uint(sq), false, false);
            const float s2 = __uint_as_float(p16[0]) + __uint_as_float(p16[1]);
            const auto p32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(s2), __float_as_uint(s2), false, false);
            const int cs = __float_as_int(__uint_as_float(p32[0]) + __uint_as_float(p32[1]));
            float g2;
            if constexpr (D <= 3) {
                // the slot's D column sums by in-row shifts (the slot's columns sit in this lane's row; a
                // helper's own columns hold t*'s sums, from the same y'' columns): same adds in the same order
                // as the gather below, without its LDS round trips
                const int o = cl % D;
                const float c0 = __int_as_float(cs);
                const float r1 = __int_as_float(__builtin_amdgcn_mov_dpp(cs, 0x111, 0xF, 0xF, true));  // row_shr:1
                const float l1 = __int_as_float(__builtin_amdgcn_mov_dpp(cs, 0x101, 0xF, 0xF, true));  // row_shl:1
                if constexpr (D == 1) {
                    g2 = c0;
                } else if constexpr (D == 2) {
                    g2 = (o == 0 ? c0 : r1) + (o == 0 ? l1 : c0);
                } else {
                    const float r2 = __int_as_float(__builtin_amdgcn_mov_dpp(cs, 0x112, 0xF, 0xF, true));  // row_shr:2
                    const float l2 = __int_as_float(__builtin_amdgcn_mov_dpp(cs, 0x102, 0xF, 0xF, true));  // row_shl:2
                    const float a0 = o == 0 ? c0 : (o == 1 ? r1 : r2);
                    const float a1 = o == 0 ? l1 : (o == 1 ? c0 : r1);
                    const float a2 = o == 0 ? l2 : (o == 1 ? l1 : c0);
                    g2 = (a0 + a1) + a2;
                }
            } else {
                g2 = __int_as_float(__builtin_amdgcn_ds_bpermute((sc * D) << 2, cs));
#pragma unroll
                for (int a = 1; a < D; ++a) g2 += __int_as_float(__builtin_amdgcn_ds_bpermute((sc * D + a) << 2, cs));
            }
            gn = __builtin_amdgcn_sqrtf(g2);  // v_sqrt_f32 (≤ 1 ulp): every user reads this value (TS)
            if (pz == 0 && lane < kCols && ycl == cl && cl % D == 0) TS[(cl / D) * kTsW + 1] = gn;  // for the trajectories and the later rounds
            if constexpr (!kBFix) {
                const f32x4 g0 = vn_frag(pz * KQ2), g1 = vn_frag(pz * KQ2 + 1);
                Gt[0] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int m = 0; m < 4; ++m) Gt[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(g0[m], y0[m], Gt[0], 0, 0, 0);
#pragma unroll
                for (int m = 0; m < 2; ++m) Gt[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(g1[m], y1[m], Gt[0], 0, 0, 0);
                (void)ntl;
            }
        } else {
            gn = TS[sc * kTsW + 1];
        }
        const float lrx = (hmr && cl / D == hsr) ? lrs * P.bls_bm : lrs;  // a helper: t*'s next trial (:147)
        const float cjx = unfused(1.f - unfused(P.lreg * lrx));            // optimizer_BLS.py:139
        // ĝ = G/‖G‖ (optimizer_BLS.py:165): the IEEE quotient through the correctly rounded reciprocal (div_rcp
        // with rcp_rn_of); the waypoint-space step s = lr/‖G‖ (not reference arithmetic: the residual e'
        // absorbs its rounding) through the refined one, as the trajectory lanes form it
        const float rr = rcp_refined(gn), rg = rcp_rn_of(gn, rr);
        const float sx = div_rcp(lrx, gn, rr);  // the trajectory lanes' step (the same expression there)
        const float ne = -rcp_refined(fmaxf(sx, kMinRefStep));
        f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
        auto tile = [&](int u, f32x4 G, bool store_g, f32x4 A, f32x4 a) {  // α rows, V_Rᵀ fragment (rank tile 0)
            if (store_g) *reinterpret_cast<f32x4*>(Gb + cl * lde + u * 16 + r4x) = G;  // for the later rounds
            f32x4 AJ, E;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float gh = div_rcp(G[i], gn, rg);
#ifdef IRM_DIV_CHECK
                if (act && pz < MTG) {  // diagnostics: ĝ against the IEEE division, and round 5's refined-rcp form
                    const unsigned mis = __fdiv_rn(G[i], gn) != gh ? 1u : 0u;
                    const unsigned mis5 = __fdiv_rn(G[i], gn) != div_rcp(G[i], gn, rcp_refined(gn)) ? 1u : 0u;
                    atomicAdd(&P.prof[(size_t)blockIdx.x * kProfPhases + 0], (unsigned long long)mis);
                    atomicAdd(&P.prof[(size_t)blockIdx.x * kProfPhases + 1], (unsigned long long)mis5);
                    atomicAdd(&P.prof[(size_t)blockIdx.x * kProfPhases + 2], 1ull);
                }
#endif
                // α_j = fl(fl(c·α) − fl(lr·ĝ)) (optimizer_BLS.py:139) and its scaled residual e' = (c·α − α_j)/s − G,
                // u = fl(c·α − α_j) in one rounding (alpha_step_gd2's form: e' to 2^-24 of |G|)
                const float p1 = unfused(cjx * A[i]), p2 = unfused(lrx * gh);
                AJ[i] = unfused(p1 - p2);
                const float uu = fmaf(cjx, A[i], -AJ[i]);
                E[i] = act ? fmaf(-uu, ne, -G[i]) : 0.f;
            }
            *reinterpret_cast<f32x4*>(Ajb + cl * lde + u * 16 + r4x) = AJ;
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], E[0], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], E[1], acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], E[2], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], E[3], acc1, 0, 0, 0);
        };
        if constexpr (kBFix) {
#pragma unroll
            for (int g = 0; g < kT; ++g) {
                const int u = pz + g * (MAXT / 64);
                if (u < S::NK / 16) tile(u, Gt[g], fresh, Ap[g], Vp[g]);
            }
        } else {
            for (int u = pz; u < MTG; u += nwaves) {
                f32x4 G;
                if (fresh && u == pz) {
                    G = Gt[0];
                } else if (fresh) {  // further tiles of the wave (general launches)
                    const f32x4 g0 = vn_frag(u * KQ2), g1 = vn_frag(u * KQ2 + 1);
                    f32x4 y0 = *reinterpret_cast<const f32x4*>(Ypart + ycl * ldy + r4y);
                    f32x4 y1 = *reinterpret_cast<const f32x4*>(Ypart + ycl * ldy + 16 + r4y);
                    for (int sp = 1; sp < nsplit; ++sp) {
                        y0 += *reinterpret_cast<const f32x4*>(Ypart + (sp * 16 + ycl) * ldy + r4y);
                        y1 += *reinterpret_cast<const f32x4*>(Ypart + (sp * 16 + ycl) * ldy + 16 + r4y);
                    }
                    G = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int m = 0; m < 4; ++m) G = __builtin_amdgcn_mfma_f32_16x16x4f32(g0[m], y0[m], G, 0, 0, 0);
#pragma unroll
                    for (int m = 0; m < 2; ++m) G = __builtin_amdgcn_mfma_f32_16x16x4f32(g1[m], y1[m], G, 0, 0, 0);
                } else {
                    G = *reinterpret_cast<const f32x4*>(Gb + ycl * lde + u * 16 + r4y);
                }
                tile(u, G, fresh, *reinterpret_cast<const f32x4*>(Ab + ycl * lde + u * 16 + r4y),
                     vt_frag(u));
            }
        }
        *reinterpret_cast<f32x4*>(Zq + pz * 256 + (r4 >> 2) * 64 + cl * 4) = acc0 + acc1;
    };
    // the F tiles of every column's trial: dP = F·(y'' + Σ_w z partial w) at rank 16 (kR16F)
    auto bls_f = [&]() {
        const float* zq = Zq + (r4 >> 2) * 64 + cl * 4;
        f32x4 by0, bz;
        if constexpr (kBFix) {  // every partial read before the first sum (one LDS round trip)
            f32x4 yp[S::NSPLIT], zz[kNZc];
#pragma unroll
            for (int sp = 0; sp < S::NSPLIT; ++sp) yp[sp] = *reinterpret_cast<const f32x4*>(Ypart + (sp * 16 + ycl) * ldy + r4y);
#pragma unroll
            for (int w = 0; w < kNZc; ++w) zz[w] = *reinterpret_cast<const f32x4*>(zq + w * 256);
            __builtin_amdgcn_sched_barrier(0);
            by0 = yp[0];
#pragma unroll
            for (int sp = 1; sp < S::NSPLIT; ++sp) by0 += yp[sp];
            bz = zz[0];
#pragma unroll
            for (int w = 1; w < kNZc; ++w) bz += zz[w];
        } else {
            by0 = *reinterpret_cast<const f32x4*>(Ypart + ycl * ldy + r4y);
            for (int sp = 1; sp < nsplit; ++sp) by0 += *reinterpret_cast<const f32x4*>(Ypart + (sp * 16 + ycl) * ldy + r4y);
            bz = *reinterpret_cast<const f32x4*>(zq);
            for (int w = 1; w < nzp; ++w) bz += *reinterpret_cast<const f32x4*>(zq + w * 256);
        }
        const f32x4 bt = by0 + bz;
        f32x4 acc[S2T];
#pragma unroll
        for (int j = 0; j < S2T; ++j) {
            acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
            if (wave + j * nwaves < MT2) {
#pragma unroll
                for (int m = 0; m < 4; ++m) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a2[j * 2][m], bt[m], acc[j], 0, 0, 0);
            }
        }
#pragma unroll
        for (int j = 0; j < S2T; ++j)
            if (wave + j * nwaves < MT2) *reinterpret_cast<f32x4*>(dP + cl * ldx + (wave + j * nwaves) * 16 + r4x) = acc[j];
    };
    // ---- the dense operator (DENSE: DenseShape, F = L = [K; dK], V_R = I — G is y'' and z is e').
    // Stage 1, y'' = Fᵀ·[a'; b']: the N/16 row tiles of y'' over the waves, each over the whole k range
    // (the position half; the velocity half in dense rounds) plus the endpoint velocity rows' MFMA (as the
    // rank-32 kernel's split-0 units).  Stage 2, dP = F·(y'' + e'): the MP/16 row tiles of [T; V] over the
    // waves, the B operand one quad of y'' + e' per k-quad from LDS.  Every operator fragment (Fᵀ, F:
    // 512 KB each at N = 256) is streamed from L2 kDPF k-quads ahead of its MFMAs; a sched_barrier per
    // k-quad keeps the compiler from hoisting the whole stream (its registers) up front.
    constexpr int kDW = MAXT / 64;
    constexpr int kD1 = DENSE ? (S::RP / 16 + kDW - 1) / kDW : 1;  // stage-1 row tiles per wave
    constexpr int kD2 = DENSE ? (S::MP / 16 + kDW - 1) / kDW : 1;  // stage-2 row tiles per wave
    constexpr int kDQ = DENSE ? S::NK / 16 : 1;                    // k-quads per half
    constexpr int kDPF = 2;  // prefetch depth (k-quads; 3 and 4 measured the same: the stages are MFMA-bound)
    float aepd[kD1];  // F_bot rows 0 / N−1 of the wave's stage-1 row tiles (the endpoint MFMA's A)
#pragma unroll
    for (int j = 0; j < kD1; ++j) {
        const int tl = wave + j * kDW;
        aepd[j] = 0.f;
        if (DENSE && tl < RP / 16 && (lane >> 4) < 2) aepd[j] = P.Fbot[(size_t)((lane >> 4) ? N - 1 : 0) * RP + tl * 16 + (lane & 15)];
    }
    auto dense_stage1 = [&](bool full) {
        const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
        constexpr int KQ1c = S::MP / 16;
        const __amdgpu_buffer_rsrc_t r1 = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float*>(P.F1p), 0, (int)(frag_floats(S::RP, S::MP) * 4), 0x00020000);
        const int vo = lane * 16;
        auto g1ld = [&](int tl, int kq) { return ld_frag(r1, vo, ((tl * KQ1c + kq) * 64) * 16); };
        const float* xl = X + cl * ldx + r4x;
        const float bep = smem[epoff];
        f32x4 acc[kD1];
#pragma unroll
        for (int j = 0; j < kD1; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(aepd[j], bep, z4, 0, 0, 0);
        auto half = [&](int kb) {  // k-quads kb … kb + kDQ − 1 of Fᵀ's MP columns
            f32x4 a[kDPF][kD1], b[kDPF];
#pragma unroll
            for (int p = 0; p < kDPF; ++p) {
#pragma unroll
                for (int j = 0; j < kD1; ++j) a[p][j] = g1ld(wave + j * kDW, kb + p);
                b[p] = *reinterpret_cast<const f32x4*>(xl + (kb + p) * 16);
            }
#pragma unroll
            for (int kq = 0; kq < kDQ; ++kq) {
                const int sl = kq % kDPF;
                f32x4 ac[kD1];
#pragma unroll
                for (int j = 0; j < kD1; ++j) ac[j] = a[sl][j];
                const f32x4 bc = b[sl];
                if (kq + kDPF < kDQ) {
#pragma unroll
                    for (int j = 0; j < kD1; ++j) a[sl][j] = g1ld(wave + j * kDW, kb + kq + kDPF);
                    b[sl] = *reinterpret_cast<const f32x4*>(xl + (kb + kq + kDPF) * 16);
                }
#pragma unroll
                for (int m = 0; m < 4; ++m)
#pragma unroll
                    for (int j = 0; j < kD1; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(ac[j][m], bc[m], acc[j], 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
            }
        };
        half(0);
        if (full) half(kDQ);
#pragma unroll
        for (int j = 0; j < kD1; ++j)
            *reinterpret_cast<f32x4*>(Ypart + cl * ldy + (wave + j * kDW) * 16 + r4x) = acc[j];
    };
    auto dense_stage2 = [&]() {
        constexpr int KQ2c = S::RP / 16;
        const __amdgpu_buffer_rsrc_t r2 = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float*>(P.F2p), 0, (int)(frag_floats(S::MP, S::RP) * 4), 0x00020000);
        const int vo = lane * 16;
        auto g2ld = [&](int tl, int kq) { return ld_frag(r2, vo, ((tl * KQ2c + kq) * 64) * 16); };
        const float* yl = Ypart + cl * ldy + r4x;
        const float* el = Eb + cl * lde + r4x;
        f32x4 acc[kD2], a[kDPF][kD2], by[kDPF], be[kDPF];
#pragma unroll
        for (int j = 0; j < kD2; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int p = 0; p < kDPF; ++p) {
#pragma unroll
            for (int j = 0; j < kD2; ++j) a[p][j] = g2ld(wave + j * kDW, p);
            by[p] = *reinterpret_cast<const f32x4*>(yl + p * 16);
            be[p] = *reinterpret_cast<const f32x4*>(el + p * 16);
        }
#pragma unroll
        for (int kq = 0; kq < kDQ; ++kq) {
            const int sl = kq % kDPF;
            f32x4 ac[kD2];
#pragma unroll
            for (int j = 0; j < kD2; ++j) ac[j] = a[sl][j];
            const f32x4 bt = by[sl] + be[sl];  // y'' + e' (z = V_Rᵀ·e' = e')
            if (kq + kDPF < kDQ) {
#pragma unroll
                for (int j = 0; j < kD2; ++j) a[sl][j] = g2ld(wave + j * kDW, kq + kDPF);
                by[sl] = *reinterpret_cast<const f32x4*>(yl + (kq + kDPF) * 16);
                be[sl] = *reinterpret_cast<const f32x4*>(el + (kq + kDPF) * 16);
            }
#pragma unroll
            for (int m = 0; m < 4; ++m)
#pragma unroll
                for (int j = 0; j < kD2; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(ac[j][m], bt[m], acc[j], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int j = 0; j < kD2; ++j)
            *reinterpret_cast<f32x4*>(dP + cl * ldx + (wave + j * kDW) * 16 + r4x) = acc[j];
    };
    // this lane's direction rows Δ = (F·y'')·J for waypoint j (the endpoint velocity rows are in y'')
    auto direction = [&](int j, float (&dt)[D], float (&dv)[D]) {
        float ut[D], uv[D];
#pragma unroll
        for (int k = 0; k < D; ++k) {
            ut[k] = dP[(t * D + k) * ldx + swz(nn[j], t * D + k)];
            uv[k] = dP[(t * D + k) * ldx + NK + swz(nn[j], t * D + k)];
        }
#pragma unroll
        for (int k = 0; k < D; ++k) {
            float a = ut[0] * P.J[k], c = uv[0] * P.J[k];
#pragma unroll
            for (int l = 1; l < D; ++l) {
                a = fmaf(ut[l], P.J[l * D + k], a);
                c = fmaf(uv[l], P.J[l * D + k], c);
            }
            dt[k] = a;
            dv[k] = c;
        }
    };
    // G[n] = (V_R·y'')[n] (no mix: [a'; b'] carry Jᵀ; the endpoint velocity rows are in y'')
    auto grad_alpha = [&](int j, float (&G)[D], int gt) {  // gt: the trajectory slot whose G is read
        const int r = wl[j] ? nn[j] : 0;  // (valid trajectories only)
#pragma unroll
        for (int k = 0; k < D; ++k) {
            if constexpr (DENSE) G[k] = Ypart[(gt * D + k) * ldy + swz(r, gt * D + k)];  // V_R = I: G = y''
            else G[k] = Gb[(gt * D + k) * lde + swz(r, gt * D + k)];
        }
    };
    // a lane's row offset in a series frame, formed where it is used (a value held across the round loop
    // is a per-lane 64-bit address the 7-DoF dual loop spilled)
    auto ser_row = [&](int j) {
        int r = nn[j] * D;
        if constexpr (D > 3) asm volatile("" : "+v"(r));
        return r;
    };
    auto snapshot = [&](irm_stats& st) {  // extended-vis frame after a non-breaking inner iteration
        if (rec && st.series_len < P.max_series) {
#pragma unroll
            for (int j = 0; j < WPL; ++j) {
                if (vl[j]) {
#pragma unroll
                    for (int k = 0; k < D; ++k)
                        P.series[((b * P.max_series) + st.series_len) * N * D + ser_row(j) + k] = q[j][k];
                }
            }
            st.series_len++;
        }
    };

    // ---- BLS line-search helpers (kHelp, lean_help): when one trajectory t* of the workgroup is left in a
    // line search, the first done slot evaluates its next trial (lr·β₋, optimizer_BLS.py:143-147) in the
    // same round: a rejected trial changes nothing but lr, so the sequential search's decisions, counters
    // and log are unchanged — only rounds are saved.  The helper reads t*'s α, T, V rows (ss, written by
    // t* whenever they change) and scalars (hp, every round); its trial's direction folds its own residual
    // into t*'s y'' (stage 2 reads t*'s Ypart columns for the helper's columns); every wave of both slots
    // replays the decision; if the helper's trial is the accepted one, the helper writes t*'s gradient
    // inputs and α, T, V, which t* adopts at the next round's start.
    float* SS = smem + LX.ss;  // [3·D][MAXT]: α, T, V of the thread's waypoint
    float* HP = smem + LX.hp;  // [slot][kHpW]: lr, ljl, lsg, loss, trial, inner, bfar (per wave of the slot)
    constexpr int kSlots = (MAXT / 64) / WPTL;
    auto ss_write = [&](int tt, const float (&a)[WPL][D], const float (&qq)[WPL][D], const float (&vv)[WPL][D]) {
        const int th = tt * NWL + li;
#pragma unroll
        for (int k = 0; k < D; ++k) {
            SS[k * MAXT + th] = a[0][k];
            SS[(D + k) * MAXT + th] = qq[0][k];
            SS[(2 * D + k) * MAXT + th] = vv[0][k];
        }
    };
    auto ss_read = [&](int tt) {
        const int th = tt * NWL + li;
#pragma unroll
        for (int k = 0; k < D; ++k) {
            al[0][k] = SS[k * MAXT + th];
            q[0][k] = SS[(D + k) * MAXT + th];
            v[0][k] = SS[(2 * D + k) * MAXT + th];
        }
    };
    bool adopt = false;  // t*: the helper's trial was accepted — take its α, T, V at the next round's start
    // BLS: this trajectory's trial scalars for the trial stages (lr of its next trial, in a line search)
    auto ts_write = [&]() {
        if (n0 == 0 && lane == 0) {
            TS[t * kTsW + 0] = lr;
            TS[t * kTsW + 2] = phase == LP_STEP ? 1.f : 0.f;
        }
    };
    int n_rounds = 0, n_hm = 0;  // diagnostics (trace_b bit 29): kernel rounds / helper rounds until this trajectory ended

    // round 0 (optimizer_GD.py:93 / :210: the loss at α0) and the first gradient inputs
    irm_stats st{};
    st.series_len = rec ? 1 : 0;
    // BLS: the per-trajectory counters in VGPRs (the compiler would keep these wave-uniform values in SGPRs,
    // and the BLS flow's scalar state spills SGPRs to VGPR lanes — readlane / writelane on the round's path):
    // C3-BLS −0.9 %, its faithful line −0.4 %, C2 −0.7 %; the GD dual loop 1-1.6 % slower with it, not used
    if constexpr (BLS && D <= 3) {  // (the 7-DoF BLS variants have no VGPRs to spare)
        asm volatile("" : "+v"(st.inner_iterations), "+v"(st.outer_iterations), "+v"(st.grad_evals), "+v"(st.cost_evals),
                     "+v"(st.bls_trials), "+v"(st.series_len), "+v"(n_rounds), "+v"(n_hm));
    }
    auto write_out = [&]() {  // this trajectory's outputs: T, α, counters
#pragma unroll
        for (int j = 0; j < WPL; ++j) {
            if (vl[j]) {
#pragma unroll
                for (int k = 0; k < D; ++k) {
                    if (P.traj_out) P.traj_out[(b * N + nn[j]) * D + k] = q[j][k];
                    if (P.alpha_out) P.alpha_out[(b * N + nn[j]) * D + k] = al[j][k];
                }
            }
        }
        if (P.stats && li == 0) P.stats[b] = st;
    };

    float loss;
    bool done = !tvalid;
    {
        WP<D> w[WPL];
        evaluate(q, v, false, ljl, w);
        __syncthreads();
        const Fin f = finalize(lsg, t);
        loss = f.nl;
        if constexpr (!BLS) st.cost_evals = 1;
        bool to_end = P.max_inner <= 0;
        // BLS with max_outer_iteration <= 0: the outer while_loop never runs and α0 is returned
        // (optimizer_BLS.py:184-186, 210-213): straight to the constraint check
        if constexpr (BLS) to_end = to_end || P.max_outer <= 0;
        bool bfar = false;
        if constexpr (GD1) {
            if (to_end) done = true;
        } else if (to_end) {
            phase = LP_RESYNC;
            st.final_loss = loss;
        } else {
            needs_dir = true;
        }
        if (!done && !to_end) {
            bfar = grad_inputs(w, q, v, f.idx, lsg, ljl, t);
            xdense = bfar;
        }
        if constexpr (BLS) {
            if (tvalid) ts_write();
        }
        if constexpr (kHelp) {
            if (tvalid) {
                if constexpr (!kSSLazy) ss_write(t, al, q, v);
                if (n0 == 0 && lane == 0) {
                    HP[t * kHpW + 0] = lr;
                    HP[t * kHpW + 1] = ljl;
                    HP[t * kHpW + 2] = lsg;
                    HP[t * kHpW + 3] = loss;
                    HP[t * kHpW + 4] = __int_as_float(0);
                    HP[t * kHpW + 5] = __int_as_float(0);
                }
            }
        }
        if constexpr (GD1) {
            if (lane == 0 && (!done || bfar)) atomicOr(&fw[0], (done ? 0u : 1u << wave) | (bfar ? 1u << 31 : 0u));
        } else {
            if (lane == 0 && tvalid)
                atomicOr(&fw[0], (1u << wave) | (needs_dir ? 1u << 28 : 0u) | (phase == LP_RESYNC ? 1u << 29 : 0u) |
                                     (phase == LP_STEP ? 1u << 30 : 0u) |
                                     ((BLS ? xdense && phase == LP_STEP : bfar) ? 1u << 31 : 0u));
        }
    }
    __syncthreads();

    IRM_STAMP(14);
    // K / dK rows per software-pipelined batch of the resync's eval_exact: the loads are latency-bound
    // (one L2 round trip per batch), so D = 3 with one waypoint per lane takes 8 rows per batch — no extra
    // spills there (C3 faithful 4.57 -> 4.42 ms, C3 BLS faithful 5.68 -> 5.60, C2 0.706 -> 0.689, same
    // box, same sums in the same order); the D = 7 / two-waypoint variants keep 2 (register peak)
    constexpr bool kReloadOps = D > 3 && MAXT > 256;
#ifndef IRM_X_RESYNC_U
    constexpr int kResyncU = (D <= 3 && WPL == 1) ? 8 : 2;
#else
    constexpr int kResyncU = (D <= 3 && WPL == 1) ? IRM_X_RESYNC_U : 2;
#endif
    // ---------------------------------------------------------- rounds
    // The second half of the waves (4-7: the younger partner on each SIMD) loses VALU arbitration to
    // the older one in every phase; static priority for that half (MI355X_MICROARCH.md, two waves per
    // SIMD, item 4): C3 +1.7 %.  Priority only reorders issue: results are unchanged.
    if (wave >= 4) __builtin_amdgcn_s_setprio(1);
#ifdef IRM_X_PRIO_RESTORE
    bool hm_prev = false;  // (kHelp) the previous round was a helper round: its priorities are still set
#endif
    for (int par = 0;; par ^= 1) {
        f32x4 pre1[KQU1], pre1w[KQU1];
        f32x4 zpre[kZPre ? kKQZ : 1];
        zpre_load(zpre);
        float pre1e = 0.f;  // read only on the endpoint waves (hasep)
        // (the flag word read before the operand batch, so the branch need not wait for the batch: C3 even
        // to 2 % slower, not kept)
        if constexpr (kPre1) stage1_load(pre1, pre1w, pre1e);
        const unsigned fl = fw[par];
        if constexpr (GD1) {
            if ((fl & 0x7FFFFFFFu) == 0u) break;  // every trajectory of the block is done
        } else {
            if ((fl & 0xFFFFu) == 0u) break;
        }
        const bool dense = (fl >> 31) != 0u;
        const bool dirr = GD1 || ((fl >> 28) & 1u);  // some trajectory needs a direction this round
        const bool rsy = !GD1 && ((fl >> 29) & 1u);  // some trajectory ends an inner loop this round
        if (tid == 0) fw[par ^ 1] = 0u;
        bool hm = false, helper = false;  // helper round (block-uniform) / this wave helps
        int ts = 0, hs = 0;               // t*, the helper slot
        float h_lr0 = 0.f, h_lr = 0.f, h_ljl = 0.f, h_lsg = 0.f, h_loss = 0.f, h_gn = 1.f, h_an = 0.f;
        int h_trial = 0, h_inner = 0;
        if constexpr (kHelp) {
            n_rounds++;
            if (adopt) {  // t*: the previous round accepted the helper's trial
                ss_read(t);
                xdense = HP[t * kHpW + 6 + (wave - t * WPTL)] != 0.f;
                adopt = false;
            }
            if (!rec && !P.lean_nohelp && ((fl >> 30) & 1u) && kSlots > 1) {
                unsigned live = 0u;
#pragma unroll
                for (int s2 = 0; s2 < kSlots; ++s2)
                    if ((fl >> (s2 * WPTL)) & ((1u << WPTL) - 1u)) live |= 1u << s2;
                if (__builtin_popcount(live) == 1) {
                    hm = true;
                    n_hm++;
                    ts = __builtin_ctz(live);
                    // the neighbouring slot: the other SIMD pair (slot s = waves 2s, 2s+1 → SIMDs 2s mod 4,
                    // 2s+1 mod 4 at two waves per slot), so the helper's VALU does not share t*'s SIMDs
                    hs = ts ^ 1;
                    // the helper's MFMA columns must exist: with five 3-joint trajectories per workgroup
                    // (N ≤ 64, traj_per_block = 5) slot 5 would own columns 15-17 — take the slot below t*
                    // then (ts ≥ 2 there, and slot ts − 1's columns end below t*'s)
                    if ((hs + 1) * D > kCols) hs = ts - 1;
                    helper = t == hs;
                }
            }
            ycl = (hm && cl / D == hs) ? ts * D + cl % D : cl;
            r4y = r4 ^ (ycl & 4);
            // a helper round: t*'s waves (the launch's critical path) ahead of every other wave of their SIMDs
            // (C2 0.516 -> 0.498 ms, C3-BLS faithful even; priority only reorders issue)
            if (hm) {
                if (t == ts) __builtin_amdgcn_s_setprio(3);
                else __builtin_amdgcn_s_setprio(0);
            }
            // (the helper priorities stay set in the rounds after a helper round — a lone trajectory's resync
            // rounds: t* keeps the issue lead there.  Restoring the launch's split once the helper rounds end,
            // IRM_X_PRIO_RESTORE, measured C3-BLS faithful +0.8 %, C2 even; priority only reorders issue)
#ifdef IRM_X_PRIO_RESTORE
            else if (hm_prev) {  // back to the launch's split (waves 4-7 at 1)
                if (wave >= 4) __builtin_amdgcn_s_setprio(1);
                else __builtin_amdgcn_s_setprio(0);
            }
            hm_prev = hm;
#endif
            // t* publishes its α, T, V for the helper at the top of each helper round (the helper reads them
            // after this round's G-tile barrier), instead of after every accepted trial of every trajectory
            if constexpr (kSSLazy) {
                if (hm && t == ts) ss_write(t, al, q, v);
            }
            if (helper) {  // wave-uniform: t*'s state and scalars (its own trajectory is done and written out)
                if constexpr (!kSSLazy) ss_read(ts);
                const size_t bs = (size_t)(tb0 + ts);
#pragma unroll
                for (int k = 0; k < D; ++k) tg[0][k] = (nn[0] == N - 1) ? P.goal[bs * D + k] : P.start[bs * D + k];
                vl[0] = wl[0];
                obs = obsL + (P.obs_stride ? ts * obs_pitch(P.O) : 0);  // t*'s obstacles (per-problem sets)
                if constexpr (OREG) {  // (the register copy of the table too)
                    if (P.obs_stride && obs_reg) {
#pragma unroll
                        for (int i = 0; i < 6; ++i) oreg[i] = reinterpret_cast<const f32x4*>(obs)[i];
                    }
                }
                h_lr0 = HP[ts * kHpW + 0];
                h_lr = h_lr0 * P.bls_bm;
                h_ljl = HP[ts * kHpW + 1];
                h_lsg = HP[ts * kHpW + 2];
                h_loss = HP[ts * kHpW + 3];
                // (a direction round of t* — the only live trajectory, so dirr is its own — resets its trial
                // count at the inner-loop head, after HP was written)
                h_trial = dirr ? 0 : __float_as_int(HP[ts * kHpW + 4]);
                h_inner = __float_as_int(HP[ts * kHpW + 5]);
            }
        }
        IRM_STAMP(0);
        if constexpr (!BLS) {
            if (dirr) {  // block-uniform
                IRM_COUNT(13, dense);
                if constexpr (DENSE) {
                    dense_stage1(dense);
                } else {
                    stage1(dense, pre1, pre1w, pre1e);
                    stage1z(zpre);
                }
                IRM_STAMP(1);
                __syncthreads();
                IRM_STAMP(2);
                if constexpr (DENSE) dense_stage2();
                else stage2f(std::true_type{}, std::true_type{});
                IRM_STAMP(3);
                __syncthreads();
                IRM_STAMP(4);
                if constexpr (kGLate) glate_tiles();
            }
        } else if ((fl >> 30) & 1u) {  // block-uniform: some trajectory has a line-search trial this round
            // (a round with a new direction: stage 1 first; the trial stages of bls_gz / bls_f, above)
            if (dirr) {
                IRM_COUNT(13, dense);
                stage1(dense, pre1, pre1w, pre1e);
                IRM_STAMP(1);
                __syncthreads();
                IRM_STAMP(2);
            }
            if (dirr) bls_gz(std::true_type{}, hm, hs);
            else bls_gz(std::false_type{}, hm, hs);
            if (dirr) {
                // alpha_norm·‖G‖ = Σ_r (y''_r·1)² with G = V_R·y'' (optimizer_BLS.py:166 without forming G; the
                // endpoint velocity rows are in y''), rows r = li < RP of the trajectory's first wave (‖G‖:
                // the G-tile waves, bls_gz)
                if (needs_dir && n0 == 0) {  // wave-uniform
                    float s1 = 0.f;
                    if (tvalid && li < RP) {
                        float sa = 0.f;
                        const int lr = lnd(li);
#pragma unroll
                        for (int a = 0; a < D; ++a) {
                            float y = Ypart[(t * D + a) * ldy + swz(lr, t * D + a)];
                            for (int sp = 1; sp < nsplit; ++sp) y += Ypart[(sp * 16 + t * D + a) * ldy + swz(lr, t * D + a)];
                            sa += y;
                        }
                        s1 = sa * sa;
                    }
                    s1 = wred_sum(s1);
                    if (lane == 0) wp[t * 2 + 1] = s1;
                }
            }
            IRM_STAMP(3);
            __syncthreads();
            IRM_STAMP(4);
            if constexpr (kSSLazy) {
                if (helper) ss_read(ts);  // (t* wrote them at this round's top)
            }
            bls_f();
            __syncthreads();
        }
        // ------------------------------------------------ BLS: a new direction (the inner-loop head)
        if constexpr (BLS) {
            if (needs_dir) {  // wave-uniform; optimizer_BLS.py:163-166
                gnorm = TS[t * kTsW + 1];  // ‖G‖ as the trial stages used it (bls_gz)
                anorm = wp[t * 2 + 1] / gnorm;
                st.grad_evals++;  // cost + grad at α (optimizer_BLS.py:163-164)
                st.cost_evals++;
                trial = 0;
                needs_dir = false;
            }
        }
        // this round's step (BLS: the trial's; a helper's: t*'s next trial, lr·β₋)
        float cj = cfac, stepj = lr, lrj = lr, gnj = gnorm;
        if constexpr (BLS) {
            if (helper) {
                h_gn = TS[ts * kTsW + 1];  // t*'s ‖G‖ and alpha_norm, the same values as t*'s latch
                h_an = wp[ts * 2 + 1] / h_gn;
                lrj = h_lr;
                gnj = h_gn;
            }
            cj = unfused(1.f - unfused(P.lreg * lrj));  // (1 − λ_reg·bls_lr) in fp32 (optimizer_BLS.py:139)
            stepj = div_rcp(lrj, gnj, rcp_refined(gnj));  // bls_gz's step, bit for bit
        }
        // ------------------------------------------------ end of an inner loop: α's exact trajectory
        if (rsy) {  // block-uniform
            const bool rs = phase == LP_RESYNC;  // wave-uniform
            if (rs) {
#pragma unroll
                for (int j = 0; j < WPL; ++j) {
                    if (vl[j]) {
#pragma unroll
                        for (int k = 0; k < D; ++k) {
                            X[(t * D + k) * ldx + lnd(nn[j])] = al[j][k];
                            if constexpr (!BLS) Eb[(t * D + k) * lde + swz(nn[j], t * D + k)] = 0.f;  // absorbed by the exact trajectory
                        }
                    }
                }
            }
            __syncthreads();
            if (rs) {
#pragma unroll
                for (int j = 0; j < WPL; ++j) {
                    if (vl[j]) {
                        if constexpr (D <= 3) eval_exact<D, kResyncU, true>(P, X + (t * D) * ldx, nn[j], q[j], v[j], nullptr, nullptr, 1, ldx, Jl);
                        else eval_exact_loop<D, 4>(P, X + (t * D) * ldx, ldx, nn[j], N, Jl, q[j], v[j]);
                        // the last extended-vis frame shows the exact trajectory of the returned α
                        if (rec && st.series_len > 0) {
#pragma unroll
                            for (int k = 0; k < D; ++k)
                                P.series[((b * P.max_series) + st.series_len - 1) * N * D + ser_row(j) + k] = q[j][k];
                        }
                    }
                }
            }
            // the operator fragments again (from L2): so they are not live across the resync's exact
            // evaluation, whose register peak spilled them (the 7-DoF dual-loop / BLS kernels)
            if constexpr (kReloadOps) {
                asm volatile("" ::: "memory");
                load_ops();
            }
            __syncthreads();  // X is rewritten by this round's gradient inputs
        }
        // ------------------------------------------------ update + evaluate
        float q2[WPL][D], v2[WPL][D];
        WP<D> w[WPL];
        // the GD single loop's G rows of the α update read with the direction (stage 2 wrote both), so their
        // LDS round trip is off the decision's path: C3 −1.3 %; the dual loop, C5 and C7 measured 0.8-1 %
        // slower with it (bit-identical either way)
#ifdef IRM_X_GPRE
        constexpr bool kGPre = !BLS;
#else
        constexpr bool kGPre = GD1 && D <= 3 && !kGLate;
#endif
        float Gp[kGPre ? WPL : 1][D];
        // BLS: this slot's trial iterate α_j read with the direction (bls_gz wrote it), off the accept's path
        constexpr bool kAjPre = BLS;
        float Ajp[kAjPre ? WPL : 1][D];
        const bool stepping = GD1 ? !done : (phase == LP_STEP || helper);  // wave-uniform
        const bool ev = GD1 ? !done : (phase != LP_DONE || helper);
        if (ev) {
#pragma unroll
            for (int j = 0; j < WPL; ++j) {
                if (stepping) {
                    float dt[D], dv[D];
                    {
                        direction(j, dt, dv);
                        if constexpr (kGPre) grad_alpha(j, Gp[j], t);
                        if constexpr (kAjPre) {
#pragma unroll
                            for (int k = 0; k < D; ++k) Ajp[j][k] = Ajb[(t * D + k) * lde + swz(wl[j] ? lnd(nn[j]) : 0, t * D + k)];
                        }
#pragma unroll
                        for (int k = 0; k < D; ++k) {
                            const float tq = -(stepj * dt[k]), tv = -(stepj * dv[k]);
                            q2[j][k] = fmaf(cj, q[j][k], tq);
                            v2[j][k] = fmaf(cj, v[j][k], tv);
                            // the products stay live past the FMAs: three-address FMAs, whose results
                            // can take the waypoint state's own registers (no copies at the round's end)
                            if constexpr (GD1) asm volatile("" ::"v"(tq), "v"(tv), "v"(q2[j][k]), "v"(v2[j][k]));
                        }
                    }
                } else {
#pragma unroll
                    for (int k = 0; k < D; ++k) {
                        q2[j][k] = q[j][k];
                        v2[j][k] = v[j][k];
                    }
                }
            }
            IRM_STAMP(5);
            if constexpr (GD1) {
                // the GD single loop's waypoint state moves to the trial point unconditionally: a
                // rejected step ends the trajectory, whose q / v are not read again (the epilogue
                // evaluates α exactly) — no copies on the accept path
#pragma unroll
                for (int j = 0; j < WPL; ++j)
#pragma unroll
                    for (int k = 0; k < D; ++k) {
                        q[j][k] = q2[j][k];
                        v[j][k] = v2[j][k];
                    }
            }
            // an inner loop's end is evaluated with the next outer iteration's λ (its loss and gradient
            // start that iteration; the constraint terms do not depend on λ)
            const bool rs = !GD1 && phase == LP_RESYNC;
            evaluate(q2, v2, rs, helper ? h_ljl : rs ? ljl * P.lci : ljl, w);
        }
        IRM_STAMP(7);
        if constexpr (WPTL > 1) {
            __syncthreads();  // the trajectory's wave partials come from several waves
        } else if (hm) {      // block-uniform: t* reads the helper's records
            __syncthreads();
        } else {              // one wave per trajectory: its own LDS writes, in order
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
        }
        IRM_STAMP(8);
        if constexpr (kHelp) {
            if (helper) {  // replay t*'s decision up to this trial: is it the accepted one?
                const Fin f0 = finalize(h_lsg, ts);
                if (f0.nl > h_loss - P.bls_a * h_lr0 * h_an && h_trial + 1 < P.max_bls) {
                    const Fin f1 = finalize(h_lsg, t);
                    if (!(f1.nl > h_loss - P.bls_a * h_lr * h_an)) {
                        // t*'s α_j (the trial stages' iterate of this slot's columns), T, V — adopted at the next
                        // round's start; α_j also into t*'s α rows for the next trial stages
                        float ajh[WPL][D];
#pragma unroll
                        for (int k = 0; k < D; ++k) {
                            ajh[0][k] = kAjPre ? Ajp[0][k] : Ajb[(t * D + k) * lde + swz(nn[0], t * D + k)];
                            if (wl[0]) Ab[(ts * D + k) * lde + swz(nn[0], ts * D + k)] = ajh[0][k];
                        }
                        ss_write(ts, ajh, q2, v2);
                        if (!(h_loss - f1.nl < P.llr) && h_inner + 1 < P.max_inner) {
                            const bool bf = grad_inputs(w, q2, v2, f1.idx, h_lsg, h_ljl, ts);  // t*'s columns
                            if (lane == 0) {
                                HP[ts * kHpW + 6 + (wave - t * WPTL)] = bf ? 1.f : 0.f;
                                if (bf) atomicOr(&fw[par ^ 1], 1u << 31);
                            }
                        }
                    }
                }
            }
        }
        if (ev && !helper) {
            const bool rs = !GD1 && phase == LP_RESYNC;
            const float lsg_e = rs ? lsg * P.lci : lsg;
            const Fin f = finalize(lsg_e, t);
            IRM_STAMP(9);
            bool bfar = false, to_end = false, accept = false, snap = false, more = false;
            if constexpr (!BLS) needs_dir = false;  // GD: every step consumes its direction
            if constexpr (GD1) {
                st.grad_evals++;
                st.cost_evals++;
                if (loss - f.nl < P.llr) {
                    done = true;  // minimized: the step is discarded (optimizer_GD.py:87-90)
                } else {
                    accept = true;
                    loss = f.nl;
                    inner++;
                    st.inner_iterations++;
                    if (inner >= P.max_inner) done = true;
                    else more = true;
                }
            } else if (rs) {
                // constraintsFulfilled(α) (trajectory.py:129-137, robot.py:90-113) on α's exact
                // trajectory; optimizer_GD.py:214-224 / optimizer_BLS.py:196-208
                const bool ok = sqrtf(f.a0) < P.eps_p && sqrtf(f.a1) < P.eps_p && sqrtf(f.b0) < P.eps_v &&
                                sqrtf(f.b1) < P.eps_v && f.tx <= P.pmax && f.tn >= P.pmin && f.va <= P.vmax;
                if (!BLS || P.max_outer > 0) st.outer_iterations++;
                st.constraints_ok = ok ? 1 : 0;
                outer++;
                if (ok || outer >= P.max_outer) {
                    phase = LP_DONE;
                } else {  // next outer iteration: λ escalated, lr reset, loss at α (optimizer_GD.py:210)
                    lsg = lsg_e;
                    ljl = ljl * P.lci;
                    loss = f.nl;
                    inner = 0;
                    if constexpr (BLS) {
                        lr = P.bls_lr0;
                    } else {
                        lr = P.gd_lr[outer];
                        cfac = P.gd_c[outer];
                        st.cost_evals++;
                    }
                    if (P.max_inner <= 0) {
                        st.final_loss = loss;  // phase stays LP_RESYNC: the empty inner loop ends at once
                    } else {
                        phase = LP_STEP;
                        more = true;
                    }
                }
            } else if constexpr (!BLS) {  // GD dual loop inner step (optimizer_GD.py:180-195)
                st.grad_evals++;
                st.cost_evals++;
                if (loss - f.nl < P.llr) {
                    to_end = true;  // minimized: the step is discarded
                } else {
                    accept = true;
                    snap = true;
                    loss = f.nl;
                    inner++;
                    st.inner_iterations++;
                    if (inner >= P.max_inner) to_end = true;
                    else more = true;
                }
            } else {  // BLS trial (optimizer_BLS.py:136-150, 172-178)
                bool inner_end = false, rejected_all = false;
                float improve = 0.f;
                // this round's trials in the sequential order: t*'s own, then (helper round) the helper's
#pragma unroll
                for (int kk = 0; kk < (kHelp ? 2 : 1); ++kk) {
                    if (kk == 1 && (!hm || accept || inner_end)) break;  // (the helper's trial was not reached)
                    const Fin fk = kk == 0 ? f : finalize(lsg_e, hs);
                    st.cost_evals++;
                    st.bls_trials++;
                    const float required = loss - P.bls_a * lr * anorm;
                    if (P.trace && b == (size_t)(P.trace_b & 0xFFFFFF) && li == 0 && st.bls_trials - 1 < P.trace_cap) {  // line-search log
                        float* r = P.trace + (size_t)(st.bls_trials - 1) * kTraceW;
                        r[0] = (float)outer;
                        r[1] = (float)inner;
                        r[2] = (float)trial;
                        r[3] = lr;
                        r[4] = fk.nl;
                        r[5] = required;
                        r[6] = (fk.nl > required) ? 0.f : 1.f;
                        r[7] = loss;
                        r[8] = gnorm;
                        r[9] = anorm;
                        if (P.trace_b >> 30) {  // diagnostics: helper round (outer + 100), helper's trial (trial + 1000)
                            if (hm) r[0] += 100.f;
                            if (kk == 1) r[2] += 1000.f;
                        }
                    }
                    if (fk.nl > required) {
                        lr = lr * P.bls_bm;
                        trial++;
                        if (trial >= P.max_bls) inner_end = rejected_all = true;  // new_loss = loss
                    } else {
                        if (kk == 0) accept = true;
                        else adopt = true;  // the helper's α_j and trajectory, next round
                        lr = lr * P.bls_bp;
                        improve = loss - fk.nl;
                        loss = fk.nl;
                        inner_end = true;
                    }
                }
                if (inner_end) {
                    if (improve < P.llr) {
                        to_end = true;
                    } else {
                        inner++;
                        st.inner_iterations++;
                        snap = true;
                        if (inner >= P.max_inner) {
                            to_end = true;
                        } else if (rejected_all) {
                            needs_dir = true;  // the same α: X still holds its gradient inputs
                            bfar = xdense;
                        } else {
                            more = true;
                        }
                    }
                }
            }
            if (accept && BLS) {
                // the trial's iterate α_j (formed by the trial stages, bls_gz) and its trajectory
                // (optimizer_BLS.py:149); α_j into the α rows for the next trial stages
#pragma unroll
                for (int j = 0; j < WPL; ++j)
#pragma unroll
                    for (int k = 0; k < D; ++k) {
                        const int o = (t * D + k) * lde + swz(wl[j] ? lnd(nn[j]) : 0, t * D + k);
                        if (wl[j]) {
                            al[j][k] = kAjPre ? Ajp[j][k] : Ajb[o];
                            Ab[o] = al[j][k];
                        }
                        q[j][k] = q2[j][k];
                        v[j][k] = v2[j][k];
                    }
            } else if (accept) {
                // α' = fl(fl(c·α) − fl(lr·G)) (optimizer_GD.py:81) and its residual for the next direction
                // (−e/lr folded into stage 2's y'')
                const float ne = GD1 ? nilr : -1.f / fmaxf(stepj, kMinRefStep);
#pragma unroll
                for (int j = 0; j < WPL; ++j) {
                    float G[D];
                    if constexpr (kGPre) {
#pragma unroll
                        for (int k = 0; k < D; ++k) G[k] = Gp[j][k];
                    } else {
                        grad_alpha(j, G, t);
                    }
                    // the D element chains first (one basic block, interleaved), then the residual stores
                    float eo[D];
#pragma unroll
                    for (int k = 0; k < D; ++k) {
                        al[j][k] = alpha_step_gd2(al[j][k], cj, stepj, G[k], ne, eo[k]);
                        if constexpr (!GD1) {
                            q[j][k] = q2[j][k];
                            v[j][k] = v2[j][k];
                        }
                    }
                    if (wl[j]) {
#pragma unroll
                        for (int k = 0; k < D; ++k) Eb[(t * D + k) * lde + swz(nn[j], t * D + k)] = eo[k];
                    }
                }
            }
            if (snap) snapshot(st);
            if (to_end) {  // inner loop over: α's exact trajectory and the constraint check next round
                st.final_loss = loss;
                phase = LP_RESYNC;
            }
            if constexpr (GD1) {
                if (more) bfar = grad_inputs(w, q2, v2, f.idx, lsg, ljl, t);
                if (lane == 0 && (!done || bfar))
                    atomicOr(&fw[par ^ 1], (done ? 0u : 1u << wave) | (bfar ? 1u << 31 : 0u));
            } else {
                if (more) {
                    if (!(kHelp && adopt)) {  // (adopted: the helper wrote the gradient inputs)
                        bfar = grad_inputs(w, q2, v2, f.idx, lsg, ljl, t);
                        xdense = bfar;
                    }
                    needs_dir = true;
                }
                if constexpr (BLS) ts_write();  // the next round's trial stages read lr and the phase
                if constexpr (kHelp) {
                    // publish this trajectory's state for a helper: α, T, V when they changed (an accepted
                    // trial of its own, a new outer iteration's exact trajectory), the scalars every round
                    if (!kSSLazy && phase == LP_STEP && (accept || rs)) ss_write(t, al, q, v);
                    if (phase != LP_DONE && n0 == 0 && lane == 0) {
                        HP[t * kHpW + 0] = lr;
                        HP[t * kHpW + 1] = ljl;
                        HP[t * kHpW + 2] = lsg;
                        HP[t * kHpW + 3] = loss;
                        HP[t * kHpW + 4] = __int_as_float(trial);
                        HP[t * kHpW + 5] = __int_as_float(inner);
                    }
                    // done: the outputs now (this slot's registers may serve as a helper from here on)
                    if (phase == LP_DONE && tvalid) {
                        if ((P.trace_b >> 29) & 1) st.series_len = n_rounds | (n_hm << 16);  // diagnostics
                        write_out();
                    }
                }
                if (lane == 0 && phase != LP_DONE)
                    atomicOr(&fw[par ^ 1], (1u << wave) | (needs_dir ? 1u << 28 : 0u) |
                                               (phase == LP_RESYNC ? 1u << 29 : 0u) | (phase == LP_STEP ? 1u << 30 : 0u) |
                                               // BLS: every trajectory in a line search keeps the velocity
                                               // half on while its inputs have one (its Ypart / Gb columns
                                               // are recomputed by other trajectories' direction rounds)
                                               ((BLS ? xdense && phase == LP_STEP : bfar) ? 1u << 31 : 0u));
            }
        }
        IRM_STAMP(11);
        __syncthreads();
        IRM_STAMP(12);
    }

    // ---------------------------------------------------------- epilogue
    if constexpr (GD1) {
        // T = eval_exact(α) (correctly rounded K·α·J), constraintsFulfilled(α) (trajectory.py:129-137,
        // robot.py:90-113) on it.  Every wave has left the loop after its last barrier: X is free.
        st.final_loss = loss;
#pragma unroll
        for (int j = 0; j < WPL; ++j) {
            if (vl[j]) {
#pragma unroll
                for (int k = 0; k < D; ++k) X[nn[j] * kLd + t * D + k] = al[j][k];
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < WPL; ++j)
            if (vl[j]) eval_exact<D>(P, X + t * D, nn[j], q[j], v[j]);
        {
            WP<D> w[WPL];
            evaluate(q, v, true, ljl, w);
        }
        __syncthreads();
        if (tvalid) {
            const Fin f = finalize(lsg, t);
            const bool ok = sqrtf(f.a0) < P.eps_p && sqrtf(f.a1) < P.eps_p && sqrtf(f.b0) < P.eps_v &&
                            sqrtf(f.b1) < P.eps_v && f.tx <= P.pmax && f.tn >= P.pmin && f.va <= P.vmax;
            st.outer_iterations = 1;
            st.constraints_ok = ok ? 1 : 0;
        }
    }
    // (LF_GD2 / LF_BLS: every trajectory ended through LP_RESYNC — q, v are α's exact trajectory;
    // kHelp: written when the trajectory finished)
    if (!kHelp && tvalid) write_out();
    if (tid == 0) prof.flush(P.prof);
}

// --------------------------------------------------- α-space eval kernels
// mode 0: evaluate (K or dK)·α·J; 1: cost; 2: cost + grad; 3: constraints.
// trajectory.py:63-65, 271-297, 129-180; same lane mapping as k_optimize.
template <int D, int MAXT>
__global__ __launch_bounds__(MAXT) void k_forward(KParams P, int mode) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const Plan L = plan_lds(P, false, false);
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int N = P.N, NW = P.NW, TB = P.TB, MP = P.MP;
    const int WPT = NW >> 6;
    const int t = wave / WPT;
    const int n = tid - t * NW;
    const int tb0 = blockIdx.x * TB;
    const int ntb = min(TB, P.B - tb0);
    if (ntb <= 0) return;
    const bool tvalid = t < ntb;
    const bool valid = tvalid && n < N;
    const size_t b = (size_t)(tb0 + (tvalid ? t : 0));
    float* XG = smem + L.X;
    float* red = smem + L.red;
    float* sg = smem + L.sg;
    float* obsL = smem + L.obs;

    stage_obstacles(P, tb0, ntb, obsL);
    stage_alpha<D>(P, tb0, ntb, XG, MP);
    __syncthreads();
    float q[D], v[D], s[D], g[D];
#pragma unroll
    for (int k = 0; k < D; ++k) {
        q[k] = v[k] = 0.f;
        s[k] = tvalid ? P.start[b * D + k] : 0.f;
        g[k] = tvalid ? P.goal[b * D + k] : 0.f;
    }
    if (valid) eval_exact<D>(P, XG + t * D, n, q, v);
    __syncthreads();
    if (mode == 0) {
        if (valid) {
#pragma unroll
            for (int k = 0; k < D; ++k) P.out0[(b * N + n) * D + k] = P.which ? v[k] : q[k];
        }
        return;
    }
    WP<D> w;
    if (tvalid) {
        if (valid) eval_waypoint_rt<D>(P, q, v, obsL, w);
        eval_partials<D>(P, valid, w, n, wave, q, v, s, g, red, sg, t);
    }
    __syncthreads();
    EvalOut E{};
    if (tvalid) E = eval_finalize(P, red, sg, t, t * WPT, WPT, P.lam_sg, P.lam_jl);
    if (tvalid && n == 0) {
        if (mode == 1 || mode == 2) {
            if (P.out0) P.out0[b] = E.loss;
        } else if (mode == 3) {
            const bool f0 = E.ds < P.eps_p && E.dg < P.eps_p;
            const bool f1 = E.vs < P.eps_v && E.vg < P.eps_v;
            const bool f2 = E.tmax <= P.pmax && E.tmin >= P.pmin;
            const bool f3 = E.vabs <= P.vmax;
            if (P.out_ok) P.out_ok[b] = (f0 && f1 && f2 && f3) ? 1 : 0;
            if (P.out0) {
                float* r = P.out0 + b * 11;
                r[0] = E.ds; r[1] = E.dg; r[2] = E.vs; r[3] = E.vg;
                r[4] = E.tmax; r[5] = E.tmin; r[6] = E.vabs;
                r[7] = f0; r[8] = f1; r[9] = f2; r[10] = f3;
            }
        }
    }
    if (mode != 2) return;
    if (valid) {
        float a[D], bb[D];
        grad_waypoint<D>(P, w, q, v, n, E.idx, P.lam_sg, P.lam_jl, s, g, a, bb);
#pragma unroll
        for (int k = 0; k < D; ++k) {
            XG[n * kLd + t * D + k] = a[k];
            XG[(N + n) * kLd + t * D + k] = bb[k];
        }
    }
    __syncthreads();
    // G = (Kᵀa + dKᵀb)·Jᵀ  (trajectory.py:295)
    if (valid) {
        float G[D];
        grad_exact<D>(P, XG + t * D, n, G);
#pragma unroll
        for (int k = 0; k < D; ++k) P.out1[(b * N + n) * D + k] = G[k];
    }
}

// ------------------------------------------------------------- launchers
template <class Fn>
inline hipError_t dispatch_d(int D, Fn&& fn) {
    switch (D) {
        case 1: return fn(std::integral_constant<int, 1>{});
        case 2: return fn(std::integral_constant<int, 2>{});
        case 3: return fn(std::integral_constant<int, 3>{});
        case 4: return fn(std::integral_constant<int, 4>{});
        case 5: return fn(std::integral_constant<int, 5>{});
        case 6: return fn(std::integral_constant<int, 6>{});
        case 7: return fn(std::integral_constant<int, 7>{});
        case 8: return fn(std::integral_constant<int, 8>{});
        default: return hipErrorInvalidValue;
    }
}

template <class Fn>
inline hipError_t dispatch_t(int BT, Fn&& fn) {
    if (BT <= 256) return fn(std::integral_constant<int, 256>{});
    if (BT <= 512) return fn(std::integral_constant<int, 512>{});
    if (BT <= 1024) return fn(std::integral_constant<int, 1024>{});
    return hipErrorInvalidValue;
}

template <class K, class... Args>
inline hipError_t launch_lds(K kernel, int grid, int threads, size_t lds, hipStream_t s, Args... args) {
    hipError_t e = hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kernel, dim3(grid), dim3(threads), lds, s, args...);
    return hipGetLastError();
}

template <class T>
struct type_tag {
    using type = T;
};

// LDS of k_lean: the optimiser head + obstacles, no staged F fragments, the lean regions.
inline size_t lean_lds(const KParams& p, bool help = false, bool bls = false, bool dense = false) {
    KParams q = p;
    q.regops = 1;
    return (size_t)lean_extra(plan_lds(q, false, true, true).total, p.MP, p.NK, p.RP, p.nsplit, lean_vlds(p.NK, p.D, p.BT),
                              p.D, help ? p.BT : 0, bls, dense).total * 4;
}

// The lean kernel's control flow for a launch (-1: the general kernel serves it): the GD single
// loop (dualOptimization = max_outer_iteration > 1, optimizer_GD.py:18) without extended-vis
// snapshots is the bench flow; GD with snapshots or a dual loop, and BLS, the full flows.
inline int lean_flow(const KParams& p) {
    if (!p.lean_ok) return -1;
    if (p.optimizer == IRM_OPT_BLS) return LF_BLS;
    return (p.max_outer <= 1 && !p.record_series) ? LF_GD1 : LF_GD2;
}
// help: the launch's instantiation carries the BLS line-search helpers' exchange regions (lean_help), so
// the check sees the LDS the launch will request (per-problem obstacle tables grow the base with TB·O)
inline bool lean_fits(const KParams& p, bool help = false, bool bls = false) {
    return (p.RP / 16) * p.nsplit <= p.BT / 64 && p.NK / 16 <= 4 * p.nsplit && lean_lds(p, help, bls) <= 160 * 1024;
}

// k_optimize<Shape> with the MAXT / operator-placement / optimiser variants (one shape per
// instantiation unit, irm_opt_inst.hip).
template <class Sh>
hipError_t launch_general_shape(const KParams& p, hipStream_t s, LaunchDesc* desc);

template <class Sh>
inline int shape_name(char* buf, size_t n) {
    if constexpr (Sh::kDense) return snprintf(buf, n, "DenseShape<%d,%d>", Sh::D, Sh::N);
    else if constexpr (Sh::kNW > 0) return snprintf(buf, n, "FixShape<%d,%d,%d>", Sh::D, Sh::N, Sh::RP);
    else return snprintf(buf, n, "DynShape<%d>", Sh::D);
}
inline const char* flow_name(int flow) { return flow == LF_GD1 ? "GD1" : flow == LF_GD2 ? "GD2" : "BLS"; }
// the optimiser's control flow in LeanFlow terms (k_optimize runs every flow in one instantiation)
inline int optimizer_flow(const KParams& p) {
    if (p.optimizer == IRM_OPT_BLS) return LF_BLS;
    return (p.max_outer <= 1 && !p.record_series) ? LF_GD1 : LF_GD2;
}

// The one place an optimiser kernel is launched: records what runs in `desc` (irm_optimize_plan) and
// launches unless desc->describe_only.
template <class K>
inline hipError_t run_optimizer(LaunchDesc* desc, K kernel, int grid, int threads, size_t lds, hipStream_t s,
                                const KParams& p) {
    if (desc) {
        desc->grid = grid;
        desc->threads = threads;
        desc->lds_bytes = (int)lds;
        desc->traj_per_block = p.TB;
        if (desc->describe_only) return hipSuccess;
    }
    return launch_lds(kernel, grid, threads, lds, s, p);
}

template <class Sh, int TT, int WPL, bool FULL, int FLOW>
hipError_t launch_lean_one(const KParams& p, int grid, hipStream_t s, LaunchDesc* desc) {
    if (desc) {
        char sn[48];
        shape_name<Sh>(sn, sizeof(sn));
        snprintf(desc->kernel, sizeof(desc->kernel), "k_lean<%s,%d,%d,%s,%s>", sn, TT, WPL, FULL ? "FULL" : "PART",
                 flow_name(FLOW));
        desc->lean = 1;
        desc->flow = FLOW;
        desc->wpl = WPL;
        desc->rank_z = desc->rank_dir = 16;  // k_lean's per-stage ranks at RP = 32
        desc->rank_g = 24;
        if constexpr (Sh::kDense) {  // V_R = I: G is y'' and z is e' (no MFMAs), the direction at rank N
            desc->rank_z = desc->rank_g = 0;
            desc->rank_dir = Sh::RP;
        }
    }
    return run_optimizer(desc, k_lean<Sh, TT, WPL, FULL, FLOW>, grid, p.BT,
                         lean_lds(p, lean_help<Sh, TT, WPL, FULL, FLOW>(), FLOW == LF_BLS, Sh::kDense), s, p);
}

template <class Sh, int TT, int WPL, bool FULL>
hipError_t launch_lean_flow(const KParams& p, int flow, int grid, hipStream_t s, LaunchDesc* desc) {
    switch (flow) {
        case LF_GD1: return launch_lean_one<Sh, TT, WPL, FULL, LF_GD1>(p, grid, s, desc);
        case LF_GD2: return launch_lean_one<Sh, TT, WPL, FULL, LF_GD2>(p, grid, s, desc);
        default: return launch_lean_one<Sh, TT, WPL, FULL, LF_BLS>(p, grid, s, desc);
    }
}

template <class Sh>
hipError_t launch_optimize_shape(const KParams& p, hipStream_t s, LaunchDesc* desc) {
    const int grid = (p.B + p.TB - 1) / p.TB;
    if (grid <= 0) return hipSuccess;
    return dispatch_t(p.BT, [&](auto tc) {
        constexpr int TT = decltype(tc)::value;
        const int flow = lean_flow(p);
        if constexpr (!Sh::kVariants && TT == 512) {
            if constexpr (Sh::kNW == 128) {
                // diagnostic (IRM_LEAN_WPL=2): one wave per trajectory, two waypoints per lane
                KParams q = p;
                q.BT = p.BT / 2;
                q.NW = p.NW / 2;
                if (p.lean_wpl == 2 && flow == LF_GD1 && lean_fits(q))  // (GD only)
                    return launch_lean_one<Sh, 256, 2, false, LF_GD1>(q, grid, s, desc);
            }
        }
        if constexpr (!Sh::kVariants && TT <= 512) {  // the lean kernel (F operators register-resident:
            // one stage-1 unit per wave; workgroups are padded to TT threads by choose_shape)
            const bool help = flow == LF_BLS && lean_help<Sh, TT, 1, true, LF_BLS>();
            if (flow >= 0 && p.BT == TT && lean_fits(p, help, flow == LF_BLS))
                return launch_lean_flow<Sh, TT, 1, true>(p, flow, grid, s, desc);
        }
        if constexpr (!Sh::kVariants && TT == 1024) {
            if constexpr (Sh::kNW == 256 && Sh::D * 3 <= kCols) {  // ≥ 3 trajectories fit the MFMA columns
                // N = 256 with more than two trajectories per workgroup: two waypoints per lane
                KParams q = p;
                q.BT = p.BT / 2;
                q.NW = p.NW / 2;
                if (flow >= 0 && lean_fits(q, false, flow == LF_BLS)) return launch_lean_flow<Sh, 512, 2, false>(q, flow, grid, s, desc);
            }
        }
        return launch_general_shape<Sh>(p, s, desc);
    });
}

// The general optimiser k_optimize<Shape, …> (every optimiser / control flow).  Instantiated in its
// own unit (irm_opt_inst.hip, IRM_INST_GEN_*) so that build.py can compile it with the
// iterative-ILP machine scheduler, which measured 10 % faster on it (faithful C3) while the lean
// kernels keep the default scheduler.
// The dense operator's k_lean (DenseShape, GD single loop, one 512-thread workgroup of TB trajectories):
// *served = false leaves the launch to the general kernel (another workgroup size, LDS).
template <class Sh>
hipError_t launch_dense_shape(const KParams& p, hipStream_t s, LaunchDesc* desc, bool* served) {
    *served = false;
    if (p.BT != 512 || p.TB * Sh::D > kCols || lean_flow(p) != LF_GD1) return hipSuccess;
    KParams q = p;
    q.nsplit = 1;  // one split: every wave's stage-1 row tiles over the whole k range
    if (lean_lds(q, false, false, true) > 160 * 1024) return hipSuccess;
    *served = true;
    const int grid = (p.B + p.TB - 1) / p.TB;
    if (grid <= 0) return hipSuccess;
    return launch_lean_one<Sh, 512, 1, true, LF_GD1>(q, grid, s, desc);
}

template <class Sh>
hipError_t launch_general_shape(const KParams& p, hipStream_t s, LaunchDesc* desc) {
    const bool stage = p.ops_in_lds != 0;
    const Plan L = plan_lds(p, stage, true);
    const size_t lds = (size_t)L.total * 4;
    const int grid = (p.B + p.TB - 1) / p.TB;
    if (grid <= 0) return hipSuccess;
    return dispatch_t(p.BT, [&](auto tc) {
        constexpr int TT = decltype(tc)::value;
        auto name = [&](bool ops_lds, bool regops, bool bls, bool full) {
            if (!desc) return;
            char sn[48];
            shape_name<Sh>(sn, sizeof(sn));
            snprintf(desc->kernel, sizeof(desc->kernel), "k_optimize<%s,%d,%s,%s,%s%s>", sn, TT,
                     ops_lds ? "OPS_LDS" : "OPS_L2", regops ? "REGOPS" : "-", bls ? "BLS" : "GD", full ? ",FULL" : "");
            desc->lean = 0;
            desc->flow = optimizer_flow(p);
            desc->wpl = 1;
            desc->rank_z = desc->rank_dir = desc->rank_g = p.RP;
            if (p.v_ident) desc->rank_g = desc->rank_z = 0;  // V_R = I: G is y'', z is e' (no MFMAs)
        };
        auto go = [&](auto bc) {
            constexpr bool BB = decltype(bc)::value;
            if constexpr (TT <= 512) {
                if constexpr (!Sh::kVariants) {
                    if (p.regops && p.BT == TT) {
                        name(true, true, BB, true);
                        return run_optimizer(desc, k_optimize<Sh, TT, true, true, BB, true>, grid, p.BT, lds, s, p);
                    }
                }
                if (p.regops) {
                    name(true, true, BB, false);
                    return run_optimizer(desc, k_optimize<Sh, TT, true, true, BB>, grid, p.BT, lds, s, p);
                }
            }
            name(stage, false, BB, false);
            return stage ? run_optimizer(desc, k_optimize<Sh, TT, true, false, BB>, grid, p.BT, lds, s, p)
                         : run_optimizer(desc, k_optimize<Sh, TT, false, false, BB>, grid, p.BT, lds, s, p);
        };
        return p.optimizer == IRM_OPT_BLS ? go(std::integral_constant<bool, true>{})
                                          : go(std::integral_constant<bool, false>{});
    });
}

template <int D>
hipError_t launch_forward_dim(const KParams& p, int mode, hipStream_t s) {
    const Plan L = plan_lds(p, false, false);
    const size_t lds = (size_t)L.total * 4;
    const int grid = (p.B + p.TB - 1) / p.TB;
    if (grid <= 0) return hipSuccess;
    return dispatch_t(p.BT, [&](auto tc) {
        constexpr int TT = decltype(tc)::value;
        return launch_lds(k_forward<D, TT>, grid, p.BT, lds, s, p, mode);
    });
}

// Instantiated in irm_opt_inst.hip (IRM_INST_* macros); irm_kernels.hip only dispatches.
#define IRM_FIX_SHAPES(X) X(3, 50) X(3, 64) X(3, 128) X(3, 256) X(7, 128) X(7, 256)
#define IRM_EXTERN_FIX(D_, N_) \
    extern template hipError_t launch_optimize_shape<FixShape<D_, N_, 32>>(const KParams&, hipStream_t, LaunchDesc*);
#define IRM_EXTERN_DENSE(D_, N_) \
    extern template hipError_t launch_dense_shape<DenseShape<D_, N_>>(const KParams&, hipStream_t, LaunchDesc*, bool*);
#define IRM_EXTERN_DYN(D_)                                                                                      \
    extern template hipError_t launch_optimize_shape<DynShape<D_>>(const KParams&, hipStream_t, LaunchDesc*); \
    extern template hipError_t launch_forward_dim<D_>(const KParams&, int, hipStream_t);

}  // namespace irm
