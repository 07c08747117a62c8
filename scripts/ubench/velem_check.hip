// Developer check: the S = 2 factorisation scan's element arithmetic (qsp_solver.hip velem_stage,
// velem_terminal, velem_combine) on the device, for comparison with the twin's tw_velem_check
// (scripts/velem_check.py).  Reads n cases of 68 doubles from argv[1], writes n x 88 doubles to argv[2].
#include "../../uclv_qs_pushing_matlab_amd/csrc/qsp_solver.hip"

#include <cstdio>
#include <vector>

__global__ void velem_check_kernel(int n, const double* in, double* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double* c = in + (size_t)i * 68;
    qsp::VElem e, e1, t;
    qsp::velem_stage(c, c + 6, c + 14, c + 18, c + 22, c + 24, c + 28, e);
    qsp::velem_stage(c + 30, c + 36, c + 44, c + 48, c + 52, c + 54, c + 58, e1);
    qsp::velem_combine(e, e1);
    const double* ed = &e.A[0];
    for (int q = 0; q < 44; ++q) out[(size_t)i * 88 + q] = ed[q];
    const double g6[6] = {c[64], c[65], c[66], c[67], 0.0, 0.0};
    if (c[60] > 0.0) {
        qsp::velem_terminal(c + 60, g6, t);
    } else {
        qsp::VElem u;
        qsp::velem_stage(c + 30, c + 36, c + 44, c + 48, c + 52, c + 54, c + 58, t);
        qsp::velem_stage(c, c + 6, c + 14, c + 18, c + 22, c + 24, c + 28, u);
        qsp::velem_combine(t, u);
    }
    qsp::velem_combine(e, t);
    for (int q = 0; q < 44; ++q) out[(size_t)i * 88 + 44 + q] = ed[q];
}

int main(int argc, char** argv) {
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 1;
    std::vector<double> h;
    double buf[68];
    while (fread(buf, 8, 68, f) == 68) h.insert(h.end(), buf, buf + 68);
    fclose(f);
    const int n = (int)(h.size() / 68);
    double *din, *dout;
    if (hipMalloc(&din, h.size() * 8) != hipSuccess || hipMalloc(&dout, (size_t)n * 88 * 8) != hipSuccess) return 2;
    hipMemcpy(din, h.data(), h.size() * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(velem_check_kernel, dim3((n + 63) / 64), dim3(64), 0, 0, n, din, dout);
    std::vector<double> o((size_t)n * 88);
    if (hipMemcpy(o.data(), dout, o.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return 3;
    FILE* g = fopen(argv[2], "wb");
    fwrite(o.data(), 8, o.size(), g);
    fclose(g);
    printf("velem_check: %d cases\n", n);
    return 0;
}
