// Microbenchmark (developer tool): which FP64 operations give the same bits on gfx950 as on
// the host CPU.  The bit-exact oracle twin relies on it: IEEE division, sqrt,
// fmod, floor, rint and fma must be correctly rounded (or exact) on the device, the
// hardware-reciprocal refinement rcp() must equal the same refinement started from the
// correctly rounded 1/x, and the library's own sincos (qsp_fp.hpp) must give the same bits on
// both sides.  ocml's sin/cos against glibc is reported for information.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I uclv_qs_pushing_matlab_amd/csrc \
//         scripts/ubench/fp_exact.hip -o scripts/ubench/fp_exact
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "qsp_fp.hpp"

enum Op { OP_SQRT, OP_DIV, OP_RCP, OP_FMOD, OP_FLOOR, OP_FMA, OP_SINCOS, OP_OCML, OP_COUNT };
static const char* kName[OP_COUNT] = {"sqrt", "a/b", "rcp (hw + 2 Newton) vs 1/x + 2 Newton", "fmod",
                                      "floor(a/b)", "fma", "qsp_sincos (device vs host)", "ocml sincos vs glibc"};

__global__ void run_ops(int op, const double* a, const double* b, const double* c, double* o1, double* o2, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double x = a[i], y = b[i], z = c[i];
    double r1 = 0.0, r2 = 0.0;
    switch (op) {
        case OP_SQRT: r1 = sqrt(x); break;
        case OP_DIV: r1 = x / y; break;
        case OP_RCP: r1 = qsp::rcp(x); break;
        case OP_FMOD: r1 = fmod(x, y); break;
        case OP_FLOOR: r1 = floor(x / y); break;
        case OP_FMA: r1 = fma(x, y, z); break;
        case OP_SINCOS: qsp::sin_cos(x, &r1, &r2); break;
        case OP_OCML: sincos(x, &r1, &r2); break;
    }
    o1[i] = r1;
    o2[i] = r2;
}

static uint64_t sm(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static double uni(uint64_t& s) { return (double)(sm(s) >> 11) * 0x1.0p-53; }
// random double with exponent uniform in [e0, e1] and a random mantissa
static double wide(uint64_t& s, int e0, int e1) {
    const int e = e0 + (int)(sm(s) % (uint64_t)(e1 - e0 + 1));
    return ldexp(1.0 + uni(s), e);
}
static uint64_t bits(double v) { uint64_t u; memcpy(&u, &v, 8); return u; }
static bool same(double p, double q) { return bits(p) == bits(q) || (std::isnan(p) && std::isnan(q)); }
static double ulps(double p, double q) {
    if (same(p, q)) return 0.0;
    const double d = fabs(p - q), u = nextafter(fabs(q), INFINITY) - fabs(q);
    return d / u;
}

#define CK(x) do { if ((x) != hipSuccess) { printf("HIP error line %d\n", __LINE__); return 1; } } while (0)

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : (1 << 22);
    std::vector<double> a(n), b(n), c(n), o1(n), o2(n);
    double *da, *db, *dc, *d1, *d2;
    CK(hipMalloc(&da, n * 8)); CK(hipMalloc(&db, n * 8)); CK(hipMalloc(&dc, n * 8));
    CK(hipMalloc(&d1, n * 8)); CK(hipMalloc(&d2, n * 8));
    uint64_t seed = 20260303;
    int fails = 0;
    for (int op = 0; op < OP_COUNT; ++op) {
        for (int i = 0; i < n; ++i) {
            const int part = i % 4;   // wide ranges and the path's own ranges
            switch (op) {
                case OP_SQRT: a[i] = part == 0 ? wide(seed, -1000, 1000) : (part == 1 ? uni(seed) * 1e-2 : wide(seed, -60, 10)); break;
                case OP_DIV: a[i] = (uni(seed) - 0.5) * wide(seed, -300, 300); b[i] = (uni(seed) - 0.5) * wide(seed, -300, 300); break;
                case OP_RCP: a[i] = part == 0 ? wide(seed, -1000, 1000) : (part == 1 ? wide(seed, -50, 4) : (part == 2 ? wide(seed, -14, 2) : uni(seed) * 100.0)); break;
                case OP_FMOD: a[i] = (uni(seed) - 0.5) * (part == 0 ? 4.0 : 1e4); b[i] = 0.2 + 0.5 * uni(seed); break;
                case OP_FLOOR: a[i] = (uni(seed) - 0.5) * 4.0; b[i] = 0.2 + 0.5 * uni(seed); break;
                case OP_FMA: a[i] = (uni(seed) - 0.5) * wide(seed, -200, 200); b[i] = (uni(seed) - 0.5) * wide(seed, -200, 200); c[i] = (uni(seed) - 0.5) * wide(seed, -400, 400); break;
                default: a[i] = part == 0 ? (uni(seed) - 0.5) * 8.0 : (part == 1 ? (uni(seed) - 0.5) * 1e3 : (part == 2 ? (uni(seed) - 0.5) * 1e-6 : (uni(seed) - 0.5) * 1e6)); break;
            }
        }
        if (op == OP_SQRT) { a[0] = 0.0; a[1] = -0.0; a[2] = INFINITY; a[3] = 4.9406564584124654e-324; }
        if (op == OP_RCP) { a[0] = 0.0; a[1] = INFINITY; a[2] = 2.2250738585072014e-308; a[3] = 1e-300; }
        CK(hipMemcpy(da, a.data(), n * 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(db, b.data(), n * 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(dc, c.data(), n * 8, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(run_ops, (n + 255) / 256, 256, 0, 0, op, da, db, dc, d1, d2, n);
        CK(hipGetLastError());
        CK(hipMemcpy(o1.data(), d1, n * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(o2.data(), d2, n * 8, hipMemcpyDeviceToHost));
        long bad = 0;
        double maxulp = 0.0;
        int first = -1;
        for (int i = 0; i < n; ++i) {
            double h1 = 0.0, h2 = 0.0;
            switch (op) {
                case OP_SQRT: h1 = sqrt(a[i]); break;
                case OP_DIV: h1 = a[i] / b[i]; break;
                case OP_RCP: h1 = qsp::rcp_host(a[i]); break;
                case OP_FMOD: h1 = fmod(a[i], b[i]); break;
                case OP_FLOOR: h1 = floor(a[i] / b[i]); break;
                case OP_FMA: h1 = fma(a[i], b[i], c[i]); break;
                case OP_SINCOS: qsp::sin_cos(a[i], &h1, &h2); break;
                case OP_OCML: h1 = sin(a[i]); h2 = cos(a[i]); break;
            }
            const bool ok = same(o1[i], h1) && (op < OP_SINCOS || same(o2[i], h2));
            if (!ok) {
                ++bad;
                if (first < 0) first = i;
                maxulp = fmax(maxulp, fmax(ulps(o1[i], h1), ulps(o2[i], h2)));
            }
        }
        // the library sincos against glibc (accuracy, not identity)
        double acc = 0.0;
        if (op == OP_SINCOS)
            for (int i = 0; i < n; ++i)
                if (fabs(a[i]) < 1e5) acc = fmax(acc, fmax(ulps(o1[i], sin(a[i])), ulps(o2[i], cos(a[i]))));
        printf("%-40s %9d samples: %8ld differ (max %.2f ulp)", kName[op], n, bad, maxulp);
        if (op == OP_SINCOS) printf("; vs glibc max %.2f ulp (|x| < 1e5)", acc);
        if (first >= 0) printf("; first a=%.17g b=%.17g dev=%.17g", a[first], b[first], o1[first]);
        printf("\n");
        if (bad && op != OP_OCML) fails++;
    }
    printf("%s\n", fails ? "FP EXACTNESS: FAIL" : "FP EXACTNESS: OK");
    return fails ? 2 : 0;
}
