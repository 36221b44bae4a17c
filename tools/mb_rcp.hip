// Accuracy of v_rcp_f64 alone and after one / two Newton steps against the correctly rounded 1/x (ulps), over
// 2^24 log-uniform x in [2^-30, 2^30] (the ToA fits' model values lie well inside).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <cstdlib>
__global__ void k(const double* x, double* out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double v = x[i];
    double r0 = __builtin_amdgcn_rcp(v);
    double r1 = fma(fma(-v, r0, 1.0), r0, r0);
    double r2 = fma(fma(-v, r1, 1.0), r1, r1);
    out[4 * i] = r0;
    out[4 * i + 1] = r1;
    out[4 * i + 2] = r2;
    out[4 * i + 3] = 1.0 / v;
}
static double ulps(double a, double b) {
    int64_t ia, ib;
    memcpy(&ia, &a, 8);
    memcpy(&ib, &b, 8);
    return fabs((double)(ia - ib));
}
int main() {
    const int n = 1 << 24;
    double *hx = (double*)malloc(n * 8), *ho = (double*)malloc(4 * (size_t)n * 8);
    uint64_t s = 88172645463325252ull;
    for (int i = 0; i < n; ++i) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        const double u = (double)(s >> 11) / 9007199254740992.0;
        hx[i] = ldexp(1.0 + u, (int)(u * 1e6) % 61 - 30);
    }
    double *dx, *dout;
    hipMalloc(&dx, n * 8);
    hipMalloc(&dout, 4 * (size_t)n * 8);
    hipMemcpy(dx, hx, n * 8, hipMemcpyHostToDevice);
    k<<<(n + 255) / 256, 256>>>(dx, dout, n);
    hipMemcpy(ho, dout, 4 * (size_t)n * 8, hipMemcpyDeviceToHost);
    double m0 = 0, m1 = 0, m2 = 0, md = 0;
    for (int i = 0; i < n; ++i) {
        const double ref = 1.0 / hx[i];
        m0 = fmax(m0, ulps(ho[4 * i], ref));
        m1 = fmax(m1, ulps(ho[4 * i + 1], ref));
        m2 = fmax(m2, ulps(ho[4 * i + 2], ref));
        md = fmax(md, ulps(ho[4 * i + 3], ref));
    }
    printf("max ulps vs 1/x: v_rcp_f64 %.0f, +1 Newton %.0f, +2 Newton %.0f, device 1/x %.0f\n", m0, m1, m2, md);
    return 0;
}
