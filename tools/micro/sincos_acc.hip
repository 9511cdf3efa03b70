// Developer micro-benchmark: accuracy of sin/cos variants on gfx950 vs double precision.
// hipcc --offload-arch=gfx950 -O3 -o sincos_acc sincos_acc.hip && ./sincos_acc
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

__device__ __forceinline__ void sc_poly(float x, float& sn, float& cs) {  // = irm sincos_fast
    const float kf = rintf(x * 0.636619772f);
    float r = fmaf(kf, -1.57079637050628662109375f, x);
    r = fmaf(kf, 4.371138828673793e-08f, r);
    r = fmaf(kf, 1.7151245100058819e-15f, r);
    const float z = r * r;
    const float sp = fmaf(r * z, fmaf(z, fmaf(z, -1.9515295891e-4f, 8.3321608736e-3f), -1.6666654611e-1f), r);
    const float cp = fmaf(z * z, fmaf(z, fmaf(z, 2.443315711809948e-5f, -1.388731625493765e-3f), 4.166664568298827e-2f),
                          fmaf(-0.5f, z, 1.0f));
    const int q = (int)kf & 3;
    const float s0 = (q & 1) ? cp : sp, c0 = (q & 1) ? sp : cp;
    sn = (q & 2) ? -s0 : s0;
    cs = ((q + 1) & 2) ? -c0 : c0;
}
__device__ __forceinline__ void sc_hyb(float x, float& sn, float& cs) {  // reduction + hardware sin/cos
    const float kf = rintf(x * 0.636619772f);
    float r = fmaf(kf, -1.57079637050628662109375f, x);
    r = fmaf(kf, 4.371138828673793e-08f, r);
    r = fmaf(kf, 1.7151245100058819e-15f, r);
    const float rv = r * 0.15915494309189535f;
    const float sp = __builtin_amdgcn_sinf(rv), cp = __builtin_amdgcn_cosf(rv);
    const int q = (int)kf & 3;
    const float s0 = (q & 1) ? cp : sp, c0 = (q & 1) ? sp : cp;
    sn = (q & 2) ? -s0 : s0;
    cs = ((q + 1) & 2) ? -c0 : c0;
}
__global__ void k(const float* x, float* o, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float a, b, c, d;
    sc_poly(x[i], a, b);
    sc_hyb(x[i], c, d);
    o[4 * i] = a; o[4 * i + 1] = b; o[4 * i + 2] = c; o[4 * i + 3] = d;
}
static double ulp(float v) { return nextafterf(fabsf(v), INFINITY) - fabsf(v); }
int main() {
    const int n = 1 << 22;
    float* hx = (float*)malloc(n * 4); float* ho = (float*)malloc(n * 16);
    for (int i = 0; i < n; ++i) hx[i] = -12.f + 24.f * (float)i / n;
    float *dx, *dout;
    hipMalloc(&dx, n * 4); hipMalloc(&dout, n * 16);
    hipMemcpy(dx, hx, n * 4, hipMemcpyHostToDevice);
    k<<<(n + 255) / 256, 256>>>(dx, dout, n);
    hipMemcpy(ho, dout, n * 16, hipMemcpyDeviceToHost);
    double e[4] = {0, 0, 0, 0}, ea[4] = {0, 0, 0, 0};
    for (int i = 0; i < n; ++i) {
        double s = sin((double)hx[i]), c = cos((double)hx[i]);
        double ref[4] = {s, c, s, c};
        for (int j = 0; j < 4; ++j) {
            double err = fabs(ho[4 * i + j] - ref[j]);
            double u = ulp((float)ref[j]);
            if (fabs(ref[j]) > 1e-3 && err / u > e[j]) e[j] = err / u;
            if (err > ea[j]) ea[j] = err;
        }
    }
    printf("max ulp (|ref|>1e-3): poly sin %.2f cos %.2f | hw sin %.2f cos %.2f\n", e[0], e[1], e[2], e[3]);
    printf("max abs: poly sin %.3g cos %.3g | hw sin %.3g cos %.3g\n", ea[0], ea[1], ea[2], ea[3]);
    return 0;
}
