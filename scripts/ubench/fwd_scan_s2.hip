// Microbenchmark (developer tool): the forward walk of the QP kernel's two-stages-per-lane layout
// (qsp_solver.hip riccati_solve<2, ...>: per lane step, each slot forms du = kk + K dx and steps the
// affine dynamics, then dx moves to the next lane by DPP) against an associative (prefix) scan of
// the closed-loop affine maps dx_{k+1} = F_k dx_k + c_k, F = A + B K, c = B kk + b: each lane composes
// its two slots' maps, a Hillis-Steele prefix scan over the group's lanes composes the lanes before
// it (partner lane j - 2^d through ds_bpermute), and every slot then applies its own map input.
// Layout: N = 50 (configs[4]), L = ceil((N+1)/2) = 26 lanes per instance, two instances per wave,
// one-wave workgroups padded with dynamic LDS to one wave per SIMD (the kernel's occupancy at S = 2).
// Usage: fwd_scan_s2 [N] [instances] [reps] [lds KB]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

struct St {   // one stage: A's free entries, B, defect, K, kk
    double a[6], B[8], bb[4], K[8], kk[2];
};
constexpr int NIN = 28;

__device__ __forceinline__ double shfl_d(double v, int src) {
    const int lo = __shfl(__double2loint(v), src), hi = __shfl(__double2hiint(v), src);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double from_prev(double old, double v) {   // lane i <- lane i-1 (DPP wave shift)
    const int lo = __builtin_amdgcn_update_dpp(__double2loint(old), __double2loint(v), 0x138, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(__double2hiint(old), __double2hiint(v), 0x138, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ void load(const double* in, St& s) {
    double* d = &s.a[0];
#pragma unroll
    for (int q = 0; q < NIN; ++q) d[q] = in[q];
}
// the production dyn_step (A = [[1,0,a0,a1],[0,1,a2,a3],[0,0,1,a4],[0,0,0,a5]])
__device__ __forceinline__ void dyn_step(const St& s, const double du[2], double dx[4]) {
    const double n0 = fma(s.B[1], du[1], fma(s.B[0], du[0], fma(s.a[1], dx[3], fma(s.a[0], dx[2], s.bb[0] + dx[0]))));
    const double n1 = fma(s.B[3], du[1], fma(s.B[2], du[0], fma(s.a[3], dx[3], fma(s.a[2], dx[2], s.bb[1] + dx[1]))));
    const double n2 = fma(s.B[5], du[1], fma(s.B[4], du[0], fma(s.a[4], dx[3], s.bb[2] + dx[2])));
    const double n3 = fma(s.B[7], du[1], fma(s.B[6], du[0], fma(s.a[5], dx[3], s.bb[3])));
    dx[0] = n0; dx[1] = n1; dx[2] = n2; dx[3] = n3;
}
__device__ __forceinline__ void control(const St& s, const double dx[4], double du[2]) {
    du[0] = fma(s.K[3], dx[3], fma(s.K[2], dx[2], fma(s.K[1], dx[1], fma(s.K[0], dx[0], s.kk[0]))));
    du[1] = fma(s.K[7], dx[3], fma(s.K[6], dx[2], fma(s.K[5], dx[1], fma(s.K[4], dx[0], s.kk[1]))));
}

__global__ void __launch_bounds__(64) walk_kernel(const double* in, const double* x0, double* out, int N, int nI,
                                                  int reps) {
    extern __shared__ double pad[];
    const int lane = threadIdx.x & 63, L = (N + 2) / 2, G = 64 / L;
    const int grp = lane / L, lig = lane - grp * L;
    const int inst = blockIdx.x * G + grp;
    const bool real = grp < G && inst < nI;
    St s[2];
#pragma unroll
    for (int ls = 0; ls < 2; ++ls) {
        const int k = 2 * lig + ls;
        load(in + ((size_t)(real ? inst : 0) * N + (k < N ? k : N - 1)) * NIN, s[ls]);
    }
    if (threadIdx.x == 1000) pad[0] = 0.0;
    double o[2][3] = {{0, 0, 0}, {0, 0, 0}};
    const int lsN = N - 2 * (L - 1);
    for (int r = 0; r < reps; ++r) {
        double dx[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) dx[q] = x0[(size_t)(real ? inst : 0) * 4 + q] + 1e-300 * o[0][0];
        for (int j = 0; j < L; ++j) {
            const bool act = lig == j;
#pragma unroll
            for (int ls = 0; ls < 2; ++ls) {
                if (j == L - 1 && ls >= lsN) continue;
                double du[2];
                control(s[ls], dx, du);
                if (act) { o[ls][0] = dx[3]; o[ls][1] = du[0]; o[ls][2] = du[1]; }
                dyn_step(s[ls], du, dx);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) dx[q] = from_prev(dx[q], dx[q]);
        }
    }
    if (real)
        for (int ls = 0; ls < 2; ++ls) {
            const int k = 2 * lig + ls;
            if (k < N)
                for (int q = 0; q < 3; ++q) out[((size_t)inst * N + k) * 3 + q] = o[ls][q];
        }
}

struct Aff { double F[16], c[4]; };   // x -> F x + c
// closed-loop map of one stage: F = A + B K, c = B kk + b
__device__ __forceinline__ void make_aff(const St& s, Aff& m) {
    const double A[4][4] = {{1.0, 0.0, s.a[0], s.a[1]}, {0.0, 1.0, s.a[2], s.a[3]}, {0.0, 0.0, 1.0, s.a[4]},
                            {0.0, 0.0, 0.0, s.a[5]}};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int q = 0; q < 4; ++q) m.F[4 * i + q] = fma(s.B[2 * i + 1], s.K[4 + q], fma(s.B[2 * i], s.K[q], A[i][q]));
        m.c[i] = fma(s.B[2 * i + 1], s.kk[1], fma(s.B[2 * i], s.kk[0], s.bb[i]));
    }
}
// g <- g o f  (first f, then g)
__device__ __forceinline__ void compose(Aff& g, const Aff& f) {
    Aff r;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
            r.F[4 * i + j] = fma(g.F[4 * i + 3], f.F[12 + j], fma(g.F[4 * i + 2], f.F[8 + j], fma(g.F[4 * i + 1], f.F[4 + j], g.F[4 * i] * f.F[j])));
        r.c[i] = fma(g.F[4 * i + 3], f.c[3], fma(g.F[4 * i + 2], f.c[2], fma(g.F[4 * i + 1], f.c[1], fma(g.F[4 * i], f.c[0], g.c[i]))));
    }
    g = r;
}

__global__ void __launch_bounds__(64) scan_kernel(const double* in, const double* x0, double* out, int N, int nI,
                                                  int reps) {
    extern __shared__ double pad[];
    const int lane = threadIdx.x & 63, L = (N + 2) / 2, G = 64 / L;
    const int grp = lane / L, lig = lane - grp * L;
    const int inst = blockIdx.x * G + grp;
    const bool real = grp < G && inst < nI;
    St s[2];
#pragma unroll
    for (int ls = 0; ls < 2; ++ls) {
        const int k = 2 * lig + ls;
        load(in + ((size_t)(real ? inst : 0) * N + (k < N ? k : N - 1)) * NIN, s[ls]);
    }
    if (threadIdx.x == 1000) pad[0] = 0.0;
    double o[2][3] = {{0, 0, 0}, {0, 0, 0}};
    for (int r = 0; r < reps; ++r) {
        Aff m0, m1;
        make_aff(s[0], m0);
        make_aff(s[1], m1);
        Aff e = m1;
        compose(e, m0);   // the lane's two stages: m1 o m0
        if (2 * lig + 1 >= N) e = m0;   // a lane with one stage (or none: unused)
        // inclusive prefix over the lanes: lane j <- E_j o ... o E_0
        for (int off = 1; off < L; off <<= 1) {
            const bool take = lig >= off;
            const int src = take ? lane - off : lane;
            Aff f;
            double* fd = &f.F[0];
            const double* ed = &e.F[0];
#pragma unroll
            for (int q = 0; q < 20; ++q) fd[q] = shfl_d(ed[q], src);
            if (take) compose(e, f);
        }
        // the state entering this lane: the previous lane's prefix applied to dx0
        Aff f;
        {
            double* fd = &f.F[0];
            const double* ed = &e.F[0];
            const int src = lig >= 1 ? lane - 1 : lane;
#pragma unroll
            for (int q = 0; q < 20; ++q) fd[q] = shfl_d(ed[q], src);
        }
        double d0[4], dx[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) d0[q] = x0[(size_t)(real ? inst : 0) * 4 + q] + 1e-300 * o[0][0];
#pragma unroll
        for (int i = 0; i < 4; ++i)
            dx[i] = lig == 0 ? d0[i] : fma(f.F[4 * i + 3], d0[3], fma(f.F[4 * i + 2], d0[2], fma(f.F[4 * i + 1], d0[1], fma(f.F[4 * i], d0[0], f.c[i]))));
#pragma unroll
        for (int ls = 0; ls < 2; ++ls) {
            double du[2];
            control(s[ls], dx, du);
            o[ls][0] = dx[3]; o[ls][1] = du[0]; o[ls][2] = du[1];
            if (ls == 0) dyn_step(s[0], du, dx);
        }
    }
    if (real)
        for (int ls = 0; ls < 2; ++ls) {
            const int k = 2 * lig + ls;
            if (k < N)
                for (int q = 0; q < 3; ++q) out[((size_t)inst * N + k) * 3 + q] = o[ls][q];
        }
}


// closed-loop walk on the lanes' composite maps (E = m1 o m0 per lane, built as the scan builds it):
// dx entering lane j+1 = E_j dx entering lane j, one 4x4 affine step per lane under the lane mask
__global__ void __launch_bounds__(64) cwalk_kernel(const double* in, const double* x0, double* out, int N, int nI,
                                                   int reps) {
    extern __shared__ double pad[];
    const int lane = threadIdx.x & 63, L = (N + 2) / 2, G = 64 / L;
    const int grp = lane / L, lig = lane - grp * L;
    const int inst = blockIdx.x * G + grp;
    const bool real = grp < G && inst < nI;
    St s[2];
#pragma unroll
    for (int ls = 0; ls < 2; ++ls) {
        const int k = 2 * lig + ls;
        load(in + ((size_t)(real ? inst : 0) * N + (k < N ? k : N - 1)) * NIN, s[ls]);
    }
    if (threadIdx.x == 1000) pad[0] = 0.0;
    double o[2][3] = {{0, 0, 0}, {0, 0, 0}};
    for (int r = 0; r < reps; ++r) {
        Aff m0, e;
        make_aff(s[0], m0);
        make_aff(s[1], e);
        compose(e, m0);
        double dx[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) dx[q] = x0[(size_t)(real ? inst : 0) * 4 + q] + 1e-300 * o[0][0];
        for (int j = 0; j < L - 1; ++j) {
            if (lig >= j && lig < L - 1) {
                double n[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) n[i] = fma(e.F[4 * i + 3], dx[3], fma(e.F[4 * i + 2], dx[2], fma(e.F[4 * i + 1], dx[1], fma(e.F[4 * i], dx[0], e.c[i]))));
#pragma unroll
                for (int i = 0; i < 4; ++i) dx[i] = from_prev(dx[i], n[i]);
            }
        }
#pragma unroll
        for (int ls = 0; ls < 2; ++ls) {
            double du[2];
            control(s[ls], dx, du);
            o[ls][0] = dx[3]; o[ls][1] = du[0]; o[ls][2] = du[1];
            if (ls == 0) dyn_step(s[0], du, dx);
        }
    }
    if (real)
        for (int ls = 0; ls < 2; ++ls) {
            const int k = 2 * lig + ls;
            if (k < N)
                for (int q = 0; q < 3; ++q) out[((size_t)inst * N + k) * 3 + q] = o[ls][q];
        }
}

int main(int argc, char** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 50;
    const int nI = argc > 2 ? atoi(argv[2]) : 16384;
    const int reps = argc > 3 ? atoi(argv[3]) : 10;
    const int ldsKB = argc > 4 ? atoi(argv[4]) : 36;
    const int L = (N + 2) / 2, G = 64 / L;
    if (L > 64 || N < 2) { printf("2 <= N, N + 1 <= 128\n"); return 1; }
    std::vector<double> h((size_t)nI * N * NIN), hx((size_t)nI * 4);
    srand(11);
    auto rnd = [] { return (double)rand() / RAND_MAX - 0.5; };
    for (size_t i = 0; i < (size_t)nI * N; ++i) {
        double* d = &h[i * NIN];
        for (int q = 0; q < 6; ++q) d[q] = 0.05 * rnd();
        d[5] += 1.0;
        for (int q = 0; q < 8; ++q) d[6 + q] = 0.05 * rnd();
        for (int q = 0; q < 4; ++q) d[14 + q] = 1e-3 * rnd();
        for (int q = 0; q < 8; ++q) d[18 + q] = 2.0 * rnd();     // K: a stabilising-size feedback
        for (int q = 0; q < 2; ++q) d[26 + q] = 1e-3 * rnd();
    }
    for (auto& v : hx) v = 1e-2 * rnd();
    double *din, *dx0, *dw, *ds;
    const size_t nout = (size_t)nI * N * 3;
    CK(hipMalloc(&din, h.size() * 8));
    CK(hipMalloc(&dx0, hx.size() * 8));
    CK(hipMalloc(&dw, nout * 8));
    CK(hipMalloc(&ds, nout * 8));
    CK(hipMemcpy(din, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dx0, hx.data(), hx.size() * 8, hipMemcpyHostToDevice));
    const int blocks = (nI + G - 1) / G;
    const size_t lds = (size_t)ldsKB * 1024;
    CK(hipFuncSetAttribute((const void*)walk_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    CK(hipFuncSetAttribute((const void*)scan_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    CK(hipFuncSetAttribute((const void*)cwalk_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    double* dc;
    CK(hipMalloc(&dc, nout * 8));
    float tc = 0;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float tw = 0, ts = 0;
    for (int pass = 0; pass < 2; ++pass) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(walk_kernel, dim3(blocks), dim3(64), lds, 0, din, dx0, dw, N, nI, reps);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&tw, e0, e1));
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(scan_kernel, dim3(blocks), dim3(64), lds, 0, din, dx0, ds, N, nI, reps);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ts, e0, e1));
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(cwalk_kernel, dim3(blocks), dim3(64), lds, 0, din, dx0, dc, N, nI, reps);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&tc, e0, e1));
    }
    CK(hipGetLastError());
    std::vector<double> ow(nout), os(nout);
    CK(hipMemcpy(ow.data(), dw, nout * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(os.data(), ds, nout * 8, hipMemcpyDeviceToHost));
    double maxrel = 0.0, scale = 0.0;
    for (size_t q = 0; q < nout; ++q) scale = fmax(scale, fabs(ow[q]));
    for (size_t q = 0; q < nout; ++q) maxrel = fmax(maxrel, fabs(ow[q] - os[q]) / (scale + 1e-300));
    std::vector<double> oc(nout);
    CK(hipMemcpy(oc.data(), dc, nout * 8, hipMemcpyDeviceToHost));
    double maxc = 0.0;
    for (size_t q = 0; q < nout; ++q) maxc = fmax(maxc, fabs(ow[q] - oc[q]) / (scale + 1e-300));
    printf("S=2 forward walk N=%d L=%d instances=%d reps=%d lds=%dKB: walk %.3f ms, scan %.3f ms (scan/walk %.2f), "
           "closed-loop lane walk %.3f ms (%.2f); max |walk - scan| / max|walk| = %.2e, closed-loop %.2e\n", N, L, nI, reps,
           ldsKB, tw / reps, ts / reps, ts / tw, tc / reps, tc / tw, maxrel, maxc);
    return 0;
}
