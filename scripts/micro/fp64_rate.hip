// Microbenchmark: sustained FP64 VALU issue rate on this GPU (FMA and RCP), to calibrate the roofline of
// the FP64-bound shooting kernel.  Build: hipcc --offload-arch=gfx950 -O3 fp64_rate.hip -o fp64_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>

template <int CHAINS, bool RCP>
__global__ void __launch_bounds__(256) k(double* out, int iters, double a) {
    double x[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) x[c] = 1.0 + 1e-3 * (threadIdx.x + c);
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) {
            if (RCP) x[c] = __builtin_amdgcn_rcp(x[c]) + a;
            else x[c] = fma(x[c], a, 1e-9);
        }
    }
    double s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int CHAINS, bool RCP>
void run(const char* name, int blocks) {
    double* out;
    (void)hipMalloc(&out, sizeof(double) * blocks * 256);
    const int iters = 4096;
    hipLaunchKernelGGL((k<CHAINS, RCP>), dim3(blocks), dim3(256), 0, 0, out, iters, 0.999999);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((k<CHAINS, RCP>), dim3(blocks), dim3(256), 0, 0, out, iters, 0.999999);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double waveinst = 5.0 * blocks * 4.0 * iters * CHAINS * (RCP ? 2 : 1);
    printf("%-12s chains=%d blocks=%d: %.3f ms, %.3e wave-instr/s, %.2f wave-instr/clk/CU @2.4GHz\n", name, CHAINS,
           blocks, ms / 5, waveinst / (ms * 1e-3), waveinst / (ms * 1e-3) / 256 / 2.4e9);
    (void)hipFree(out);
}

// accuracy of v_rcp_f64 alone and with one / two Newton steps, over x in [1e-3, 1e3]
__global__ void k_acc(double* err, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double x = exp(-6.9 + 13.8 * (i + 0.5) / n) * (1.0 + 1e-7 * (i % 977));
    const double ref = 1.0 / x;
    double y = __builtin_amdgcn_rcp(x);
    err[3 * i] = fabs(y - ref) / ref;
    double e = fma(-x, y, 1.0);
    y = fma(y, e, y);
    err[3 * i + 1] = fabs(y - ref) / ref;
    e = fma(-x, y, 1.0);
    y = fma(y, e, y);
    err[3 * i + 2] = fabs(y - ref) / ref;
}

int main() {
    {
        const int n = 1 << 22;
        double* d;
        (void)hipMalloc(&d, sizeof(double) * 3 * n);
        hipLaunchKernelGGL(k_acc, dim3(n / 256), dim3(256), 0, 0, d, n);
        double* h = (double*)malloc(sizeof(double) * 3 * n);
        (void)hipMemcpy(h, d, sizeof(double) * 3 * n, hipMemcpyDeviceToHost);
        double m[3] = {0, 0, 0};
        for (int i = 0; i < n; ++i)
            for (int k = 0; k < 3; ++k) m[k] = h[3 * i + k] > m[k] ? h[3 * i + k] : m[k];
        printf("v_rcp_f64 max rel err: raw %.3e, 1 NR %.3e, 2 NR %.3e (eps %.3e)\n", m[0], m[1], m[2], 2.22e-16);
        free(h);
        (void)hipFree(d);
    }
    run<1, false>("fma", 8192);
    run<4, false>("fma", 8192);
    run<8, false>("fma", 8192);
    run<8, false>("fma", 2048);
    run<8, false>("fma", 1024);
    run<1, true>("rcp+add", 8192);
    run<8, true>("rcp+add", 8192);
    return 0;
}
