// Developer check: qsp::rcp (hardware reciprocal + two Newton steps) against the same two steps from the
// IEEE 1/x on the host, for negative and positive arguments over the whole exponent range, and near
// powers of two.  Prints the count of differing results and the first few.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../uclv_qs_pushing_matlab_amd/csrc/qsp_fp.hpp"

__global__ void rcp_kernel(const double* x, double* r, double* w, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        r[i] = qsp::rcp(x[i]);
        w[i] = 1.0 / x[i];
    }
}
static uint64_t sm(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
int main() {
    const int n = 1 << 22;
    std::vector<double> x(n), r(n), w(n);
    uint64_t s = 7;
    for (int i = 0; i < n; ++i) {
        const int e = -1022 + (int)(sm(s) % 2045);
        double m = 1.0 + (double)(sm(s) >> 11) * 0x1.0p-53;
        if (i % 8 == 1) m = 1.0 + (double)(sm(s) % 64) * 0x1.0p-52;          // just above a power of two
        if (i % 8 == 2) m = 2.0 - (double)(1 + sm(s) % 64) * 0x1.0p-52;      // just below
        x[i] = ldexp(m, e) * ((sm(s) & 1) ? -1.0 : 1.0);
    }
    double *dx, *dr, *dw;
    if (hipMalloc(&dx, n * 8) != hipSuccess || hipMalloc(&dr, n * 8) != hipSuccess || hipMalloc(&dw, n * 8) != hipSuccess) return 1;
    if (hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice) != hipSuccess) return 1;
    hipLaunchKernelGGL(rcp_kernel, dim3(n / 256), dim3(256), 0, 0, dx, dr, dw, n);
    if (hipMemcpy(r.data(), dr, n * 8, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    if (hipMemcpy(w.data(), dw, n * 8, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    long bad = 0, badneg = 0, badw = 0, badw_normal = 0, bycls[3] = {0, 0, 0};
    long byexp[64] = {0}, cnt[64] = {0};
    for (int i = 0; i < n; ++i) {
        const double h = qsp::rcp_host(x[i]);
        int e = 0;
        frexp(x[i], &e);
        const int bucket = (e + 1024) / 32;
        cnt[bucket]++;
        if (memcmp(&h, &r[i], 8) != 0) {
            if (bad < 4) printf("x %.17g  device %.17g  host %.17g\n", x[i], r[i], h);
            ++bad;
            badneg += x[i] < 0;
            bycls[(i % 8 == 1) ? 1 : ((i % 8 == 2) ? 2 : 0)]++;
            byexp[bucket]++;
        }
        if (memcmp(&h, &w[i], 8) != 0) {
            ++badw;
            badw_normal += fabs(h) >= 2.2250738585072014e-308;
        }
    }
    printf("rcp: %ld of %d differ (%ld negative)\n", bad, n, badneg);
    printf("rcp by binary exponent (bucket of 32): ");
    for (int b = 0; b < 64; ++b)
        if (byexp[b]) printf("[%d,%d): %ld/%ld  ", b * 32 - 1024, b * 32 - 992, byexp[b], cnt[b]);
    printf("\nrcp differing by sample class: random mantissa %ld of %d, just above a power of two %ld of %d, "
           "just below %ld of %d\n", bycls[0], n * 6 / 8, bycls[1], n / 8, bycls[2], n / 8);
    printf("IEEE 1/x on the device: %ld differ from the host's rcp (%ld where 1/x is a normal number)\n", badw, badw_normal);
    return 0;
}
