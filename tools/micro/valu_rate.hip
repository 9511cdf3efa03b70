// Micro-benchmark: cycles per wave-instruction of the VALU forms the optimiser's VALU phase uses
// (v_fma_f32, v_pk_fma_f32, v_rcp_f32, v_cndmask_b32, DPP v_mov), at 1 / 2 / 4 waves per SIMD.
// Each lane runs 8 independent chains (no dependency stall), 64 instructions per loop trip.
//   hipcc -O3 --offload-arch=gfx950 -o valu_rate valu_rate.hip && ./valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kTrips = 2000;

template <int OP>
__global__ void k_rate(float* out, unsigned long long* cyc) {
    float a0 = threadIdx.x * 1e-3f, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
          a7 = a0 + 7;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}, p4 = {a1, a0}, p5 = {a3, a2}, p6 = {a5, a4},
       p7 = {a7, a6};
    const float m = 0.999f, c = 1e-4f;
    const f2 pm = {m, m}, pc = {c, c};
    __syncthreads();
    unsigned long long t0;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    for (int it = 0; it < kTrips; ++it) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            if constexpr (OP == 0) {  // v_fma_f32
                asm volatile(
                    "v_fma_f32 %0, %0, %8, %9\n\tv_fma_f32 %1, %1, %8, %9\n\tv_fma_f32 %2, %2, %8, %9\n\t"
                    "v_fma_f32 %3, %3, %8, %9\n\tv_fma_f32 %4, %4, %8, %9\n\tv_fma_f32 %5, %5, %8, %9\n\t"
                    "v_fma_f32 %6, %6, %8, %9\n\tv_fma_f32 %7, %7, %8, %9"
                    : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                    : "v"(m), "v"(c));
            } else if constexpr (OP == 1) {  // v_pk_fma_f32 (two fp32 FMAs per lane)
                asm volatile(
                    "v_pk_fma_f32 %0, %0, %8, %9\n\tv_pk_fma_f32 %1, %1, %8, %9\n\tv_pk_fma_f32 %2, %2, %8, %9\n\t"
                    "v_pk_fma_f32 %3, %3, %8, %9\n\tv_pk_fma_f32 %4, %4, %8, %9\n\tv_pk_fma_f32 %5, %5, %8, %9\n\t"
                    "v_pk_fma_f32 %6, %6, %8, %9\n\tv_pk_fma_f32 %7, %7, %8, %9"
                    : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3), "+v"(p4), "+v"(p5), "+v"(p6), "+v"(p7)
                    : "v"(pm), "v"(pc));
            } else if constexpr (OP == 2) {  // v_rcp_f32 (transcendental unit)
                asm volatile(
                    "v_rcp_f32 %0, %0\n\tv_rcp_f32 %1, %1\n\tv_rcp_f32 %2, %2\n\tv_rcp_f32 %3, %3\n\t"
                    "v_rcp_f32 %4, %4\n\tv_rcp_f32 %5, %5\n\tv_rcp_f32 %6, %6\n\tv_rcp_f32 %7, %7"
                    : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
            } else if constexpr (OP == 3) {  // v_mov_b32 with DPP row_shr:1
                asm volatile(
                    "v_mov_b32_dpp %0, %1 row_shr:1\n\tv_mov_b32_dpp %1, %2 row_shr:1\n\t"
                    "v_mov_b32_dpp %2, %3 row_shr:1\n\tv_mov_b32_dpp %3, %4 row_shr:1\n\t"
                    "v_mov_b32_dpp %4, %5 row_shr:1\n\tv_mov_b32_dpp %5, %6 row_shr:1\n\t"
                    "v_mov_b32_dpp %6, %7 row_shr:1\n\tv_mov_b32_dpp %7, %0 row_shr:1"
                    : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
            } else if constexpr (OP == 4) {  // dependent v_fma_f32 chain (latency)
                asm volatile(
                    "v_fma_f32 %0, %0, %1, %2\n\tv_fma_f32 %0, %0, %1, %2\n\tv_fma_f32 %0, %0, %1, %2\n\t"
                    "v_fma_f32 %0, %0, %1, %2\n\tv_fma_f32 %0, %0, %1, %2\n\tv_fma_f32 %0, %0, %1, %2\n\t"
                    "v_fma_f32 %0, %0, %1, %2\n\tv_fma_f32 %0, %0, %1, %2"
                    : "+v"(a0)
                    : "v"(m), "v"(c));
            } else if constexpr (OP == 5) {  // dependent v_pk_fma_f32 chain (latency)
                asm volatile(
                    "v_pk_fma_f32 %0, %0, %1, %2\n\tv_pk_fma_f32 %0, %0, %1, %2\n\tv_pk_fma_f32 %0, %0, %1, %2\n\t"
                    "v_pk_fma_f32 %0, %0, %1, %2\n\tv_pk_fma_f32 %0, %0, %1, %2\n\tv_pk_fma_f32 %0, %0, %1, %2\n\t"
                    "v_pk_fma_f32 %0, %0, %1, %2\n\tv_pk_fma_f32 %0, %0, %1, %2"
                    : "+v"(p0)
                    : "v"(pm), "v"(pc));
            } else if constexpr (OP == 6) {  // v_add_f32 (VOP2)
                asm volatile(
                    "v_add_f32 %0, %0, %8\n\tv_add_f32 %1, %1, %8\n\tv_add_f32 %2, %2, %8\n\t"
                    "v_add_f32 %3, %3, %8\n\tv_add_f32 %4, %4, %8\n\tv_add_f32 %5, %5, %8\n\t"
                    "v_add_f32 %6, %6, %8\n\tv_add_f32 %7, %7, %8"
                    : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                    : "v"(c));
            }
        }
    }
    unsigned long long t1;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    const float s = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + p0.x + p1.x + p2.x + p3.x + p4.y + p5.y + p6.y + p7.y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int OP>
void run(const char* name, int wps) {
    const int blocks = 256, threads = 256 * wps;  // one workgroup per CU, wps waves per SIMD
    float* out;
    unsigned long long* cyc;
    hipMalloc(&out, sizeof(float) * blocks * threads);
    hipMalloc(&cyc, sizeof(unsigned long long) * blocks * threads / 64);
    k_rate<OP><<<blocks, threads>>>(out, cyc);  // warm-up
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    k_rate<OP><<<blocks, threads>>>(out, cyc);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const int nw = blocks * threads / 64;
    unsigned long long* h = new unsigned long long[nw];
    hipMemcpy(h, cyc, sizeof(unsigned long long) * nw, hipMemcpyDeviceToHost);
    double avg = 0;
    for (int i = 0; i < nw; ++i) avg += (double)h[i];
    avg /= nw;
    const double ninst = (double)kTrips * 64;
    // s_memtime ticks at the shader clock; also report wall-derived cycles at 2.4 GHz
    printf("%-22s waves/SIMD %d: %6.2f memtime-ticks per wave-instr, wall %.3f ms = %6.2f cyc/instr/wave @2.4GHz\n",
           name, wps, avg / ninst, ms, ms * 2.4e6 / ninst);
    delete[] h;
    hipFree(out);
    hipFree(cyc);
}

int main() {
    for (int w : {1, 2, 4}) {
        run<0>("v_fma_f32 (indep)", w);
        run<1>("v_pk_fma_f32 (indep)", w);
        run<6>("v_add_f32 (indep)", w);
        run<2>("v_rcp_f32 (indep)", w);
        run<3>("v_mov_dpp (chain)", w);
        run<4>("v_fma_f32 (dep)", w);
        run<5>("v_pk_fma_f32 (dep)", w);
    }
    return 0;
}
