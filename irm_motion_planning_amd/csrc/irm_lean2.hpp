// irm_lean2.hpp — k_lean2: the GD single loop (optimizer_GD.py:68-97, the bench flow) with TWO LANES PER
// WAYPOINT.  Included by irm_kernels_impl.hpp after k_lean, whose helpers and LDS layout it shares.
//
// Why: k_lean's round is an MFMA phase (≈3 k cycles) and a per-waypoint VALU phase (≈5 k cycles) run by
// one lane per waypoint, two waves per SIMD, and that VALU phase is latency-bound (a wave issues on ≈37 %
// of its cycles).  Here the 128 waypoints of a trajectory take 256 lanes (4 waves), lane
// pair (l, l ^ 32) of one wave owning waypoint n: the low lane ("position half", h = 0) carries the
// position row T[n] of the state, the high lane (h = 1) the velocity row V[n], and every per-waypoint
// step is split data-parallel between the two — the same instructions on different data, so a wave
// does half of each step instead of all of it:
//   * direction and update: each lane its own row of Δ[T; V] (its half of the 2N rows of [K; dK]);
//   * FK: the joint angles split ⌈D/2⌉ / ⌊D/2⌋, the link sums combined across the pair;
//   * obstacle potential: each lane half of the obstacle table, the sums combined across the pair;
//   * joint-limit penalties: positions in the low lane, velocities in the high lane;
//   * α update: the joints split ⌈D/2⌉ / ⌊D/2⌋;
//   * gradient inputs: a (positions: obstacle, start/goal, position limits) in the low lane, b
//     (velocities: start/goal velocity, velocity limits) in the high lane — row n or NK + n of [a'; b'].
// A workgroup is 1024 threads = 16 waves = four waves per SIMD for the same four trajectories as k_lean's
// 512-thread workgroup (BASELINE configs[2]: 1024 problems = one workgroup per CU).  The MFMA stages are
// k_lean's (same operators, fragments, LDS layout, split-K and rank cuts) spread over 16 waves.
//
// Arithmetic: the same expressions in the same order as k_lean per quantity, except the sums that now
// combine two lanes' partials — the obstacle potential (two halves of the table, then added), the cost
// sum (penalties per half) — which round differently; the fp32 α iteration with the reference's rounding
// is unchanged (alpha_step_gd).  Parity: tests/test_gpu_parity.py (oracle band, reference fixtures,
// batch-neighbour independence) as for k_lean.
// (included inside namespace irm)
#pragma once

// Lane-pair exchange (v_permlane32_swap): in every lane, the value of the pair's low lane (h = 0) and
// of its high lane (h = 1).
__device__ __forceinline__ void pair_vals(float x, float& lo, float& hi) {
    const auto pm = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    lo = __uint_as_float(pm[0]);
    hi = __uint_as_float(pm[1]);
}
__device__ __forceinline__ float pair_lo(float x) {
    float lo, hi;
    pair_vals(x, lo, hi);
    return lo;
}
__device__ __forceinline__ float pair_hi(float x) {
    float lo, hi;
    pair_vals(x, lo, hi);
    return hi;
}
__device__ __forceinline__ float pair_sum(float x) {  // (low lane's x) + (high lane's x), in both lanes
    float lo, hi;
    pair_vals(x, lo, hi);
    return lo + hi;
}

// LDS of k_lean2: k_lean's layout at the same shape (head, obstacles, lean regions with V_R staged) plus
// stage 1's operator fragments, both halves (k_lean keeps them in VGPRs, which the 128-VGPR budget of
// four waves per SIMD does not allow), and the endpoint operator columns.
struct Lean2X {
    LeanX lx;
    int f1v, total;
};
inline __host__ __device__ Lean2X lean2_extra(int base, int MP, int NK, int RP, int nsplit) {
    Lean2X e{};
    e.lx = lean_extra(base, MP, NK, RP, nsplit, true);
    e.f1v = e.lx.total;
    e.total = e.f1v + al4(2 * (RP / 16) * (NK / 16) * 64 * 4);  // 2 halves × MT1 × KQa fragments of 64 lanes × 4
    return e;
}

template <class S>
__global__ __launch_bounds__(1024, 1) void k_lean2(KParams P) {
    constexpr int D = S::D, N = S::N, NK = S::NK, MP = S::MP, RP = S::RP;
    constexpr int NWV = 16;                // waves per workgroup
    constexpr int WPT2 = N / 32;           // waves per trajectory (32 waypoints × 2 lanes per wave)
    constexpr int JA = (D + 1) / 2;        // joints of the low lane (angles, α); the high lane: D − JA
    constexpr int NSPLIT = S::NSPLIT, KQa = NK / 16, KQ1 = MP / 16, MT1 = RP / 16, KQ2 = RP / 16;
    constexpr int MT2 = MP / 16, MTG = NK / 16;
    constexpr int KQU = KQa / NSPLIT;      // stage-1 k-quads per unit
    constexpr int kZS = lean_zsplit(NSPLIT, true), KQZ = KQa / kZS;
    static_assert(N % 32 == 0 && NK == N && RP == 32 && D <= 8, "k_lean2: N a multiple of 32, rank 32");
    static_assert(MT2 == NWV, "one stage-2 F tile per wave");
    static_assert(MT1 * NSPLIT <= NWV && kZS <= NWV && MTG <= NWV && KQa % NSPLIT == 0 && KQa % kZS == 0, "units");
    static_assert(4 * WPT2 * 64 <= 1024, "four trajectories per workgroup");
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const Head H = plan_head(MP, RP, NSPLIT, true, true);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    __builtin_assume(wave >= 0 && wave < NWV);
    const int t = wave / WPT2, v = wave - t * WPT2;
    const int h = lane >> 5;                 // 0: position half, 1: velocity half
    const int n = v * 32 + (lane & 31);      // this lane's waypoint
    const int r = h ? NK + n : n;            // this lane's row of [a; b] / [T; V] / Δ
    const int tb0 = blockIdx.x * P.TB;
    const int ntb = min(P.TB, P.B - tb0);
    if (ntb <= 0) return;
    const bool tvalid = t < ntb;
    const size_t b = (size_t)(tb0 + (tvalid ? t : 0));
    Prof prof;
    if (tid == 0) prof.init();

    float* X = smem + H.X;
    float* dP = smem + H.dP;
    float* Ypart = smem + H.Ypart;
    float* red = smem + H.red;
    float* sg = smem + H.sg;
    unsigned* fw = reinterpret_cast<unsigned*>(smem + H.flags);
    float* obsL = smem + H.obs;
    const Lean2X L2 = lean2_extra(plan_lds(P, false, true, true).total, MP, NK, RP, NSPLIT);
    const LeanX& LX = L2.lx;
    float* Eb = smem + LX.eb;
    float* Zp = smem + LX.zp;
    float* Gb = smem + LX.gb;
    const float* VT = smem + LX.vt;
    const float* VN = smem + LX.vn;
    const f32x4* F1v = reinterpret_cast<const f32x4*>(smem + L2.f1v);

    const int ldx = MP + 8, ldy = lean_ldy(RP), lde = lean_ld(NK);
    const int cl = lane & 15, r4 = 4 * (lane >> 4);
    const int r4x = r4 ^ (cl & 4);
    auto swz = [](int rr, int c) { return rr ^ (c & 4); };
    const bool has1 = wave < MT1 * NSPLIT;
    const int tile1 = wave % MT1, sp1 = wave / MT1;
    const int kq0 = KQU * sp1;

    // ----------------------------------------------------------- prologue
    f32x4 a2;
    {
        const f32x4* g1 = reinterpret_cast<const f32x4*>(P.F1p);
        const f32x4* g2 = reinterpret_cast<const f32x4*>(P.F2p);
        a2 = g2[((size_t)wave * KQ2) * 64 + lane];  // F tile `wave`, k-quad 0 (the direction's rank 16)
        // every stage-1 unit's fragments, [half][unit][k-quad][lane], into LDS
        f32x4* l1v = reinterpret_cast<f32x4*>(smem + L2.f1v);
        constexpr int NU = MT1 * NSPLIT * KQU * 64;
        for (int e = tid; e < 2 * NU; e += 1024) {
            const int hf = e / NU, e2 = e - hf * NU;
            const int u = e2 / (KQU * 64), i = (e2 / 64) % KQU, ln = e2 % 64;
            l1v[e] = g1[((size_t)(u % MT1) * KQ1 + hf * KQa + KQU * (u / MT1) + i) * 64 + ln];
        }
        const int nv = (int)frag_floats(RP, NK) / 4;
        const f32x4* gt = reinterpret_cast<const f32x4*>(P.VTp);
        const f32x4* gn = reinterpret_cast<const f32x4*>(P.VNp);
        f32x4* lt = reinterpret_cast<f32x4*>(smem + LX.vt);
        f32x4* ln4 = reinterpret_cast<f32x4*>(smem + LX.vn);
        for (int e = tid; e < nv; e += 1024) {
            lt[e] = gt[e];
            ln4[e] = gn[e];
        }
    }
    // endpoint operator columns (Δ rows: hL, G rows: hVL), read from LDS where used
    float* hL = smem + LX.hl;
    float* hVL = smem + LX.hv;
    for (int e = tid; e < 2 * MP; e += 1024) hL[e] = P.Hend[e];
    for (int e = tid; e < 2 * NK; e += 1024) hVL[e] = P.HV[e];
    for (int e = tid; e < 16 * lde; e += 1024) Eb[e] = 0.f;
    stage_obstacles(P, tb0, ntb, obsL);
    stage_alpha<D>(P, tb0, ntb, X, NK);
    if (tid < 2) fw[tid] = 0u;
    __syncthreads();
    // per-lane constants of the half: penalty centre / scales / thresholds, start-goal targets, link lengths
    const float ctr = h ? 0.f : P.mean_pos, scl = h ? P.inv_vmax : P.inv_std_pos;
    const float scl2 = h ? P.inv_vmax2 : P.inv_std2;
    const float thh = h ? P.thr_v : P.thr_hi, thl = h ? -P.thr_v : P.thr_lo;
    const float epf = (n == 0 || n == N - 1) ? 1.f : 0.f;
    float tgt[D], lk[JA];
#pragma unroll
    for (int k = 0; k < D; ++k) {
        const float sk = tvalid ? P.start[b * D + k] : 0.f, gk = tvalid ? P.goal[b * D + k] : 0.f;
        tgt[k] = h ? 0.f : (n == N - 1 ? gk : sk);
    }
#pragma unroll
    for (int i = 0; i < JA; ++i) lk[i] = h ? (JA + i < D ? P.link[JA + i < D ? JA + i : 0] : 0.f) : P.link[i];
    // the state row (T or V of K·α0·J, correctly rounded) and this lane's joints of α
    float x[D], al[JA];
    {
        float q0[D], v0[D];
#pragma unroll
        for (int k = 0; k < D; ++k) q0[k] = v0[k] = 0.f;
        if (tvalid) eval_exact<D>(P, X + t * D, n, q0, v0);
#pragma unroll
        for (int k = 0; k < D; ++k) x[k] = h ? v0[k] : q0[k];
#pragma unroll
        for (int i = 0; i < JA; ++i) {
            const int k = h ? JA + i : i;
            al[i] = (tvalid && k < D) ? X[n * kLd + t * D + k] : 0.f;
        }
    }
    __syncthreads();
    for (int e = tid; e < MP * kLd; e += 1024) X[e] = 0.f;
    const float* obs = obsL + (P.obs_stride ? t * obs_pitch(P.O) : 0);
    const int nq = (P.O + 3) >> 2;  // obstacle quads; each half takes nq of the 2·nq f32x4 pairs
    f32x4 oreg[3];
    const bool obs_reg = nq == 3;
#pragma unroll
    for (int i = 0; i < 3; ++i)
        oreg[i] = obs_reg ? reinterpret_cast<const f32x4*>(obs)[h * 3 + i] : f32x4{0.f, 0.f, 0.f, 0.f};
    float lsg = P.lsg0, ljl = P.ljl0;
    const float lr = P.gd_lr[0], cfac = P.gd_c[0];
    const float nilr = -1.f / fmaxf(lr, kMinRefStep);
    int inner = 0;

    // ------------------------------------------- evaluation of the state rows xx (both halves)
    struct E2 {
        float jx[D], jy[D], gx, gy;
    };
    auto evaluate = [&](const float (&xx)[D], bool ext, float ljl_e, E2& w) {
        float q[D], cum[D];
#pragma unroll
        for (int k = 0; k < D; ++k) q[k] = pair_lo(xx[k]);  // the positions in both lanes
#pragma unroll
        for (int k = 0; k < D; ++k) cum[k] = (k ? cum[k - 1] : 0.f) + q[k];
        float sn[JA], cs[JA];
        bool big = false;
#pragma unroll
        for (int i = 0; i < JA; ++i) {
            const float a = h ? cum[JA + i < D ? JA + i : D - 1] : cum[i];
            big |= fabsf(a) > 1.0e4f;
            sn[i] = a;
        }
        if (__builtin_expect(__ballot(big) != 0ull, 0)) {
#pragma unroll
            for (int i = 0; i < JA; ++i) sincos_fast(sn[i], sn[i], cs[i]);
        } else {
#pragma unroll
            for (int i = 0; i < JA; ++i) sincos_poly(sn[i], sn[i], cs[i]);
        }
        // FK (robot.py:29-36): the half's link sums, then low + high (= the sequential joint order)
        float fxp = 0.f, fyp = 0.f;
#pragma unroll
        for (int i = 0; i < JA; ++i) {
            fxp += lk[i] * cs[i];
            fyp += lk[i] * sn[i];
        }
        const float fx = pair_sum(fxp), fy = pair_sum(fyp);
        // Jacobian (robot.py:75-87), meaningful in the low lane (the high half's angles exchanged)
        float Sx = 0.f, Sy = 0.f, xs[D], ys[D];
#pragma unroll
        for (int k = 0; k < D; ++k) {
            const float s_ = k < JA ? sn[k] : pair_hi(sn[k - JA]);
            const float c_ = k < JA ? cs[k] : pair_hi(cs[k - JA]);
            xs[k] = -(P.link[k] * s_);
            ys[k] = P.link[k] * c_;
            Sx += xs[k];
            Sy += ys[k];
        }
        float Cx = 0.f, Cy = 0.f;
#pragma unroll
        for (int k = 0; k < D; ++k) {
            Cx += xs[k];
            Cy += ys[k];
            w.jx[k] = (xs[k] + Sx) - Cx;
            w.jy[k] = (ys[k] + Sy) - Cy;
        }
        // obstacle potential (environment.py:46-58): this lane's half of the padded pair table
        const f32x2 fx2 = {fx, fx}, fy2 = {fy, fy}, one = {1.f, 1.f};
        f32x2 cv2 = {0.f, 0.f}, ax2 = {0.f, 0.f}, ay2 = {0.f, 0.f};
        const f32x4* o4 = reinterpret_cast<const f32x4*>(obs) + h * nq;
        if (obs_reg) {
            f32x2 dx[3], dy[3], u[3];
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                dx[i] = fx2 - oreg[i].xy;
                dy[i] = fy2 - oreg[i].zw;
                const f32x2 e = dy[i] * dy[i] + (dx[i] * dx[i] + one);
                u[i] = f32x2{__builtin_amdgcn_rcpf(e.x), __builtin_amdgcn_rcpf(e.y)};
            }
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                cv2 += u[i];
                const f32x2 u2 = u[i] * u[i];
                ax2 += dx[i] * u2;
                ay2 += dy[i] * u2;
            }
        } else {
            for (int c = 0; c < nq; ++c) {
                const f32x4 p = o4[c];
                const f32x2 dx = fx2 - p.xy, dy = fy2 - p.zw;
                const f32x2 e = dy * dy + (dx * dx + one);
                const f32x2 u = {__builtin_amdgcn_rcpf(e.x), __builtin_amdgcn_rcpf(e.y)};
                cv2 += u;
                const f32x2 u2 = u * u;
                ax2 += dx * u2;
                ay2 += dy * u2;
            }
        }
        const float cv = 1.6f * pair_sum(cv2.x + cv2.y);
        w.gx = -3.2f * pair_sum(ax2.x + ax2.y);
        w.gy = -3.2f * pair_sum(ay2.x + ay2.y);
        // joint-limit penalty of the half (trajectory.py:215-227 / 245-255) and the constraint extrema
        float pen = 0.f, e1 = -INFINITY, e2 = INFINITY;
#pragma unroll
        for (int k = 0; k < D; ++k) {
            const float z = (xx[k] - ctr) * scl;
            const bool m = (xx[k] > thh) || (xx[k] < thl);
            pen += (P.cvdl && !m) ? 0.f : 0.5f * (z * z);
            e1 = fmaxf(e1, h ? fabsf(xx[k]) : xx[k]);
            e2 = fminf(e2, xx[k]);
        }
        const float us = (h ? 0.f : P.one_m_lmax * (cv * P.invN)) + ljl_e * (pen * P.invN);
        IRM_STAMP(6);
        // wave records: max / first-index argmax of the potential (low lanes), Σ us, extrema
        {
            const bool lo = tvalid && !h;
            float m = lo ? cv : -INFINITY, s = tvalid ? us : 0.f;
            m = maxpos(m, dppf<0xB1>(m));
            s += dppf<0xB1>(s);
            m = maxpos(m, dppf<0x4E>(m));
            s += dppf<0x4E>(s);
            m = maxpos(m, dppf<0x141>(m));
            s += dppf<0x141>(s);
            m = maxpos(m, dppf<0x140>(m));
            s += dppf<0x140>(s);
            float wm, ws;
            {
                auto pm = __builtin_amdgcn_permlane16_swap(__float_as_uint(m), __float_as_uint(m), false, false);
                auto ps = __builtin_amdgcn_permlane16_swap(__float_as_uint(s), __float_as_uint(s), false, false);
                const float m2 = maxpos(__uint_as_float(pm[0]), __uint_as_float(pm[1]));
                const float s2 = __uint_as_float(ps[0]) + __uint_as_float(ps[1]);
                auto qm = __builtin_amdgcn_permlane32_swap(__float_as_uint(m2), __float_as_uint(m2), false, false);
                auto qs = __builtin_amdgcn_permlane32_swap(__float_as_uint(s2), __float_as_uint(s2), false, false);
                wm = maxpos(__uint_as_float(qm[0]), __uint_as_float(qm[1]));
                ws = __uint_as_float(qs[0]) + __uint_as_float(qs[1]);
            }
            const unsigned long long hit = __ballot(lo && cv == wm);
            const int idx = hit ? v * 32 + __builtin_ctzll(hit) : 0x7fffffff;
            float ox = 0.f, on = 0.f, oa = 0.f;
            if (ext) {
                ox = wred_max(lo ? e1 : -INFINITY);
                on = wred_min(lo ? e2 : INFINITY);
                oa = wred_max((tvalid && h) ? e1 : 0.f);
            }
            if (lane == 0) {
                float* q4 = red + wave * 8;
                q4[0] = wm;
                q4[1] = __int_as_float(idx);
                q4[2] = ws;
                q4[3] = ox;
                q4[4] = on;
                q4[5] = oa;
            }
        }
        if (tvalid && (n == 0 || n == N - 1)) {  // trajectory.py:183-204 rows 0 and N−1 (positions: h = 0)
            float a = 0.f;
#pragma unroll
            for (int k = 0; k < D; ++k) {
                const float e = xx[k] - tgt[k];
                a += e * e;
            }
            sg[t * 4 + (n == 0 ? 0 : 2) + h] = a;
        }
    };
    struct Fin {
        float nl, tx, tn, va, a0, b0, a1, b1;
        int idx;
    };
    auto finalize = [&](float lsg_e) {
        const float* r0 = red + (t * WPT2) * 8;
        float cmax = r0[0];
        int cidx = __float_as_int(r0[1]);
        float usum = r0[2], tx = r0[3], tn = r0[4], va = r0[5];
#pragma unroll
        for (int ww = 1; ww < WPT2; ++ww) {
            const float* rw = red + (t * WPT2 + ww) * 8;
            amax_step(cmax, cidx, rw[0], __float_as_int(rw[1]));
            usum += rw[2];
            tx = fmaxf(tx, rw[3]);
            tn = fminf(tn, rw[4]);
            va = fmaxf(va, rw[5]);
        }
        Fin f;
        f.a0 = sg[t * 4 + 0];
        f.b0 = sg[t * 4 + 1];
        f.a1 = sg[t * 4 + 2];
        f.b1 = sg[t * 4 + 3];
        const float sgpc = 0.5f * f.a0 + 0.5f * f.a1;  // trajectory.py:187
        const float sgvc = 0.5f * f.b0 + 0.5f * f.b1;  // trajectory.py:203
        f.nl = (P.lam_max * cmax + usum) + lsg_e * (sgpc + sgvc);
        f.idx = cidx;
        f.tx = tx;
        f.tn = tn;
        f.va = va;
        return f;
    };
    // gradient inputs of this lane's row (a: positions, b: velocities), mixed by Jᵀ, into X; returns
    // "b' non-zero away from the endpoints" for the wave
    auto grad_inputs = [&](const E2& w, const float (&xx)[D], int cidx, float lsg_e, float ljl_e) {
        bool bfar = false;
        if (tvalid) {
            const float wt = (n == cidx ? P.lam_max : 0.f) + P.one_m_lmax * P.invN;
            const float wx = wt * w.gx, wy = wt * w.gy;
            float gv[D];
#pragma unroll
            for (int d = 0; d < D; ++d) {
                const float sgk = epf * (xx[d] - tgt[d]);
                float jl = 0.f;
                const bool m = (xx[d] > thh) || (xx[d] < thl);
                if (!P.cvdl || m) jl = ((xx[d] - ctr) * scl2) * P.invN;
                const float ob = h ? 0.f : (wx * w.jx[d] + wy * w.jy[d]);
                gv[d] = (ob + lsg_e * sgk) + ljl_e * jl;
                bfar |= (h != 0) & (gv[d] != 0.f) & (epf == 0.f);
            }
#pragma unroll
            for (int k = 0; k < D; ++k) {
                float mk = 0.f;
#pragma unroll
                for (int d = 0; d < D; ++d) mk += gv[d] * P.J[k * D + d];
                X[(t * D + k) * ldx + swz(r, t * D + k)] = mk;
            }
        }
        return __ballot(bfar) != 0ull;
    };

    // round 0: the loss at α0 (optimizer_GD.py:93) and the first gradient inputs
    irm_stats st{};
    float loss;
    bool done = !tvalid;
    {
        E2 w;
        evaluate(x, false, ljl, w);
        __syncthreads();
        const Fin f = finalize(lsg);
        loss = f.nl;
        st.cost_evals = 1;
        if (P.max_inner <= 0) done = true;
        bool bfar = false;
        if (!done) bfar = grad_inputs(w, x, f.idx, lsg, ljl);
        if (lane == 0 && (!done || bfar)) atomicOr(&fw[0], (done ? 0u : 1u << wave) | (bfar ? 1u << 31 : 0u));
    }
    __syncthreads();
    if (wave >= NWV / 2) __builtin_amdgcn_s_setprio(1);

    const float* xl = X + cl * ldx + r4x;
    for (int par = 0;; par ^= 1) {
        f32x4 pre1[KQU];
        if (has1) {
#pragma unroll
            for (int i = 0; i < KQU; ++i) pre1[i] = *reinterpret_cast<const f32x4*>(xl + (kq0 + i) * 16);
        }
        const unsigned fl = fw[par];
        if ((fl & 0x7FFFFFFFu) == 0u) break;
        const bool dense = (fl >> 31) != 0u;
        if (tid == 0) fw[par ^ 1] = 0u;
        float e0[D], e1[D];
#pragma unroll
        for (int k = 0; k < D; ++k) {
            const float* xc = X + (t * D + k) * ldx;
            e0[k] = xc[NK + swz(0, t * D + k)];
            e1[k] = xc[NK + swz(N - 1, t * D + k)];
        }
        IRM_STAMP(0);
        // ---- stage 1: Ypart = Fᵀ·[a'; b'] (waves 0..MT1·NSPLIT−1), z = V_Rᵀ·e' at rank 16 (top waves)
        if (has1) {
            f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0, a1[KQU];
#pragma unroll
            for (int i = 0; i < KQU; ++i) a1[i] = F1v[(wave * KQU + i) * 64 + lane];
#pragma unroll
            for (int i = 0; i < KQU; ++i) {
                acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[i][0], pre1[i][0], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[i][1], pre1[i][1], acc1, 0, 0, 0);
                acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[i][2], pre1[i][2], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[i][3], pre1[i][3], acc1, 0, 0, 0);
            }
            if (dense) {
                f32x4 av[KQU], bw[KQU];
#pragma unroll
                for (int i = 0; i < KQU; ++i) {
                    av[i] = F1v[(MT1 * NSPLIT + wave) * KQU * 64 + i * 64 + lane];
                    bw[i] = *reinterpret_cast<const f32x4*>(xl + (KQa + kq0 + i) * 16);
                }
#pragma unroll
                for (int i = 0; i < KQU; ++i) {
                    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i][0], bw[i][0], acc0, 0, 0, 0);
                    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i][1], bw[i][1], acc1, 0, 0, 0);
                    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i][2], bw[i][2], acc0, 0, 0, 0);
                    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i][3], bw[i][3], acc1, 0, 0, 0);
                }
            }
            *reinterpret_cast<f32x4*>(Ypart + (sp1 * 16 + cl) * ldy + tile1 * 16 + r4x) = acc0 + acc1;
        }
        {
            const int sp = NWV - 1 - wave;
            if (sp < kZS) {
                const float* el = Eb + cl * lde + r4x;
                const f32x4* ap = reinterpret_cast<const f32x4*>(VT) + lane + (size_t)(sp * KQZ) * 64;
                f32x4 a[KQZ], bb[KQZ];
#pragma unroll
                for (int i = 0; i < KQZ; ++i) {
                    a[i] = ap[(size_t)i * 64];
                    bb[i] = *reinterpret_cast<const f32x4*>(el + (sp * KQZ + i) * 16);
                }
                f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
#pragma unroll
                for (int i = 0; i < KQZ; ++i) {
                    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][0], bb[i][0], acc0, 0, 0, 0);
                    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][1], bb[i][1], acc1, 0, 0, 0);
                    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][2], bb[i][2], acc0, 0, 0, 0);
                    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][3], bb[i][3], acc1, 0, 0, 0);
                }
                *reinterpret_cast<f32x4*>(Zp + (sp * 16 + cl) * ldy + r4x) = acc0 + acc1;
            }
        }
        IRM_STAMP(1);
        __syncthreads();
        IRM_STAMP(2);
        // ---- stage 2: dP tile `wave` = F·(y'' + z) at rank 16; G tile (top waves) = V_R·y'' at rank 24
        {
            const int u = NWV - 1 - wave;
            const bool hasg = u < MTG;
            f32x4 ga0 = {0.f, 0.f, 0.f, 0.f}, ga1 = ga0;
            if (hasg) {
                const f32x4* ap = reinterpret_cast<const f32x4*>(VN) + (size_t)u * KQ2 * 64 + lane;
                ga0 = ap[0];
                ga1 = ap[64];
            }
            f32x4 by0 = {0.f, 0.f, 0.f, 0.f}, by1 = by0, bz = by0;
#pragma unroll
            for (int sp = 0; sp < NSPLIT; ++sp) {
                by0 += *reinterpret_cast<const f32x4*>(Ypart + (sp * 16 + cl) * ldy + r4x);
                if (hasg) by1 += *reinterpret_cast<const f32x4*>(Ypart + (sp * 16 + cl) * ldy + 16 + r4x);
            }
#pragma unroll
            for (int sp = 0; sp < kZS; ++sp) bz += *reinterpret_cast<const f32x4*>(Zp + (sp * 16 + cl) * ldy + r4x);
            const f32x4 bt = by0 + bz;
            f32x4 acc = {0.f, 0.f, 0.f, 0.f}, ag = acc;
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a2[m], bt[m], acc, 0, 0, 0);
                if (hasg) ag = __builtin_amdgcn_mfma_f32_16x16x4f32(ga0[m], by0[m], ag, 0, 0, 0);
            }
            if (hasg) {
#pragma unroll
                for (int m = 0; m < 2; ++m)  // kR24
                    ag = __builtin_amdgcn_mfma_f32_16x16x4f32(ga1[m], by1[m], ag, 0, 0, 0);
            }
            *reinterpret_cast<f32x4*>(dP + cl * ldx + wave * 16 + r4x) = acc;
            if (hasg) *reinterpret_cast<f32x4*>(Gb + cl * lde + u * 16 + r4x) = ag;
        }
        IRM_STAMP(3);
        __syncthreads();
        IRM_STAMP(4);
        // ---- update (this lane's row) and evaluation
        float x2[D];
        E2 w;
        if (!done) {
            float u[D];
            const float hE0 = hL[r], hE1 = hL[MP + r];
#pragma unroll
            for (int k = 0; k < D; ++k) {
                u[k] = dP[(t * D + k) * ldx + swz(r, t * D + k)];
                u[k] = fmaf(hE0, e0[k], fmaf(hE1, e1[k], u[k]));
            }
#pragma unroll
            for (int k = 0; k < D; ++k) {
                float a = 0.f;
#pragma unroll
                for (int l = 0; l < D; ++l) a = fmaf(u[l], P.J[l * D + k], a);
                x2[k] = cfac * x[k] - lr * a;
            }
            IRM_STAMP(5);
            evaluate(x2, false, ljl, w);
        }
        IRM_STAMP(7);
        __syncthreads();  // the trajectory's wave records come from four waves
        IRM_STAMP(8);
        if (!done) {
            const Fin f = finalize(lsg);
            IRM_STAMP(9);
            bool more = false, accept = false;
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
            if (accept) {
                // α' = fl(fl(c·α) − fl(lr·G)) for this lane's joints (optimizer_GD.py:81) and the residual
                // e' = −e/lr for the next round's z
                const float hv0 = hVL[n], hv1 = hVL[NK + n];
#pragma unroll
                for (int i = 0; i < JA; ++i) {
                    const int k = h ? JA + i : i;
                    if (k < D) {  // (the high lane's last joint slot is empty when D is odd)
                        const int kh = JA + i < D ? JA + i : 0;  // (static after unrolling: no dynamic register indexing)
                        const float e0k = h ? e0[kh] : e0[i], e1k = h ? e1[kh] : e1[i];
                        const float G = fmaf(hv0, e0k, fmaf(hv1, e1k, Gb[(t * D + k) * lde + swz(n, t * D + k)]));
                        float er;
                        al[i] = alpha_step_gd(al[i], cfac, lr, G, er);
                        Eb[(t * D + k) * lde + swz(n, t * D + k)] = er * nilr;
                    }
                }
#pragma unroll
                for (int k = 0; k < D; ++k) x[k] = x2[k];
            }
            bool bfar = false;
            if (more) bfar = grad_inputs(w, x2, f.idx, lsg, ljl);
            if (lane == 0 && (!done || bfar)) atomicOr(&fw[par ^ 1], (done ? 0u : 1u << wave) | (bfar ? 1u << 31 : 0u));
        }
        IRM_STAMP(11);
        __syncthreads();
        IRM_STAMP(12);
    }

    // ---------------------------------------------------------- epilogue
    // T = eval_exact(α) (correctly rounded K·α·J), constraintsFulfilled(α) on it (trajectory.py:129-137)
    st.final_loss = loss;
    if (tvalid) {
#pragma unroll
        for (int i = 0; i < JA; ++i) {
            const int k = h ? JA + i : i;
            if (k < D) X[n * kLd + t * D + k] = al[i];
        }
    }
    __syncthreads();
    float qf[D], vf[D];
#pragma unroll
    for (int k = 0; k < D; ++k) qf[k] = vf[k] = 0.f;
    if (tvalid) eval_exact<D>(P, X + t * D, n, qf, vf);
#pragma unroll
    for (int k = 0; k < D; ++k) x[k] = h ? vf[k] : qf[k];
    {
        E2 w;
        evaluate(x, true, ljl, w);
    }
    __syncthreads();
    if (tvalid) {
        const Fin f = finalize(lsg);
        const bool ok = sqrtf(f.a0) < P.eps_p && sqrtf(f.a1) < P.eps_p && sqrtf(f.b0) < P.eps_v &&
                        sqrtf(f.b1) < P.eps_v && f.tx <= P.pmax && f.tn >= P.pmin && f.va <= P.vmax;
        st.outer_iterations = 1;
        st.constraints_ok = ok ? 1 : 0;
        if (!h) {
#pragma unroll
            for (int k = 0; k < D; ++k)
                if (P.traj_out) P.traj_out[(b * N + n) * D + k] = qf[k];
        }
#pragma unroll
        for (int i = 0; i < JA; ++i) {
            const int k = h ? JA + i : i;
            if (k < D && P.alpha_out) P.alpha_out[(b * N + n) * D + k] = al[i];
        }
        if (P.stats && n == 0 && !h) P.stats[b] = st;
    }
    if (tid == 0) prof.flush(P.prof);
}

// LDS bytes of a k_lean2 launch (q: the launch's parameters, BT = 1024)
inline size_t lean2_lds(const KParams& p) {
    KParams q = p;
    q.regops = 1;
    return (size_t)lean2_extra(plan_lds(q, false, true, true).total, p.MP, p.NK, p.RP, p.nsplit).total * 4;
}
