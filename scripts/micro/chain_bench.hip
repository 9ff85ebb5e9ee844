// Micro-benchmark of the stage-chain factorisation (cocofest_amd/csrc/cfx_chain.hip) on a random block-tridiagonal
// system of the reaching task's shape (M nodes of sp unknowns): per-level kernel times with HIP events, and the
// Gauss-Jordan pivot block alone (one workgroup, no neighbours).  Bounds: every buffer is sized from M and sp below.
// build: hipcc -O3 --offload-arch=gfx950 -I../../include chain_bench.hip -o bin/chain_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>
thread_local std::string g_create_error;
#include "../../cocofest_amd/csrc/cfx_chain.hip"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

int main(int argc, char** argv) {
    const int M = argc > 1 ? atoi(argv[1]) : 1501;
    constexpr int SP = 80;
    const size_t nb = (size_t)M * SP * SP;
    std::vector<double> h(3 * nb);
    srand(1);
    for (size_t e = 0; e < 3 * nb; ++e) h[e] = (rand() / (double)RAND_MAX - 0.5) * (e < nb ? 1.0 : 0.1);
    for (int k = 0; k < M; ++k)
        for (int r = 0; r < SP; ++r) h[(size_t)k * SP * SP + r * SP + (r * 7 + 3) % SP] += 20.0;  // needs pivoting
    double *d, *w;
    int32_t* info;
    CK(hipMalloc(&d, 3 * nb * sizeof(double)));
    CK(hipMalloc(&w, 2 * nb * sizeof(double)));
    CK(hipMalloc(&info, sizeof(int32_t)));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const cfx_chain::Chain C{d, d + nb, d + 2 * nb, w, w + nb, 0, 0, M};
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&cfx_chain::k_chain_upd<SP, true>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)cfx_chain::chain_upd_lds<SP, true>()));
    for (int rep = 0; rep < 3; ++rep) {
        CK(hipMemcpy(d, h.data(), 3 * nb * sizeof(double), hipMemcpyHostToDevice));
        float tot = 0;
        for (int l = 0; (1 << l) < M; ++l) {
            const int hh = 1 << l, ne = (M - hh + 2 * hh - 1) / (2 * hh), ns = (M + 2 * hh - 1) / (2 * hh);
            float te, tu;
            CK(hipEventRecord(a));
            hipLaunchKernelGGL(cfx_chain::k_chain_elim<SP>, dim3(ne, 1), dim3(256), 0, 0, C, hh, 2 * hh, hh, info);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            CK(hipEventElapsedTime(&te, a, b));
            CK(hipEventRecord(a));
            if (ns < cfx_chain::kUpdGlobalB)
                cfx_chain::k_chain_upd<SP, true><<<dim3(ns, 1, 3), dim3(256), cfx_chain::chain_upd_lds<SP, true>(), 0>>>(C, hh);
            else
                cfx_chain::k_chain_upd<SP, false><<<dim3(ns, 1, 3), dim3(256), cfx_chain::chain_upd_lds<SP, false>(), 0>>>(C, hh);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            CK(hipEventElapsedTime(&tu, a, b));
            if (rep == 2) printf("level %2d: %4d elim %8.1f us, %4d upd %8.1f us\n", l, ne, te * 1e3, ns, tu * 1e3);
            tot += te + tu;
        }
        if (rep == 2) printf("total %.3f ms\n", tot);
    }
    // one solve with one right-hand side (after the last factorisation above)
    {
        double *rr, *tt;
        CK(hipMalloc(&rr, (size_t)M * SP * sizeof(double)));
        CK(hipMalloc(&tt, (size_t)M * SP * sizeof(double)));
        std::vector<double> hr((size_t)M * SP, 1.0);
        CK(hipMemcpy(rr, hr.data(), hr.size() * sizeof(double), hipMemcpyHostToDevice));
        const cfx_chain::Rhs X{rr, 0, 0, tt, 0, 0};
        float ts = 0;
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipEventRecord(a));
            CK(cfx_chain::solve_sp<SP>(C, 1, X, 1, 0));
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            CK(hipEventElapsedTime(&ts, a, b));
        }
        printf("one solve (1 rhs): %.1f us\n", ts * 1e3);
    }
    // the pivot block alone: one workgroup, no neighbours (h = M)
    float t1;
    CK(hipEventRecord(a));
    for (int r = 0; r < 20; ++r)
        hipLaunchKernelGGL(cfx_chain::k_chain_elim<SP>, dim3(1, 1), dim3(256), 0, 0, C, 0, 1, M, info);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&t1, a, b));
    printf("single Gauss-Jordan block: %.1f us\n", t1 * 1e3 / 20);
    return 0;
}
