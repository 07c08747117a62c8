// Operand-layout probe (developer tool) for v_mfma_f64_4x4x4_4b_f64: for every lane l0,
// B is one-hot at l0 and A holds 1000 + lane, so the nonzero outputs show which A lanes
// feed which C lanes through B's (k, j) at l0.  Prints "l0: lane=value ..." lines.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void probe(double* out) {
    const int l = threadIdx.x;
    for (int l0 = 0; l0 < 64; ++l0) {
        const double a = 1000.0 + l;
        const double b = (l == l0) ? 1.0 : 0.0;
        out[l0 * 64 + l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
    }
}

int main() {
    double* d;
    if (hipMalloc(&d, 64 * 64 * 8) != hipSuccess) return 1;
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    std::vector<double> h(64 * 64);
    if (hipMemcpy(h.data(), d, 64 * 64 * 8, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    for (int l0 = 0; l0 < 64; ++l0) {
        printf("%d:", l0);
        for (int l = 0; l < 64; ++l)
            if (h[l0 * 64 + l] != 0.0) printf(" %d=%g", l, h[l0 * 64 + l]);
        printf("\n");
    }
    return 0;
}
