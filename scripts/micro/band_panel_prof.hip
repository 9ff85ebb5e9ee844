// Phase clocks of the panel band LU (k_band_lu_panel, cocofest_amd/csrc/cfx_band.hip built with CFX_BAND_PROF):
// one factorisation of a random single band (n, kl, ku), thread 0's wall clock (s_memrealtime, 100 MHz) summed
// per phase over the panels (look-ahead kernel: write-back, own trailing columns, the next panel's factorisation,
// barrier wait), for wavefront 0 and wavefront 1.  Prints one JSON line with the per-panel microseconds of each phase.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 scripts/micro/band_panel_prof.hip -o scripts/micro/bin/band_panel_prof
//   scripts/micro/bin/band_panel_prof [n kl ku reps]
#define CFX_BAND_PROF 1
#include "../../cocofest_amd/csrc/cfx_band.hip"

#include <cstdio>
#include <random>
#include <vector>

thread_local std::string g_create_error;

#define CK(x)                                                                                    \
    do {                                                                                         \
        hipError_t e_ = (x);                                                                     \
        if (e_ != hipSuccess) {                                                                  \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                         \
            std::exit(1);                                                                        \
        }                                                                                        \
    } while (0)

int main(int argc, char** argv) {
    const int n = argc > 1 ? std::atoi(argv[1]) : 119640, kl = argc > 2 ? std::atoi(argv[2]) : 108,
              ku = argc > 3 ? std::atoi(argv[3]) : 108, reps = argc > 4 ? std::atoi(argv[4]) : 3;
    const int ldab = 2 * kl + ku + 1, kv = kl + ku;
    std::vector<double> h((size_t)n * ldab, 0.0);
    std::mt19937_64 rng(7);
    std::normal_distribution<double> nd;
    for (int j = 0; j < n; ++j)
        for (int i = std::max(0, j - ku); i <= std::min(n - 1, j + kl); ++i)
            h[(size_t)j * ldab + kv + i - j] = nd(rng) + (i == j ? 4.0 * kv : 0.0);
    double* ab;
    int32_t *ipiv, *info;
    CK(hipMalloc(&ab, h.size() * sizeof(double)));
    CK(hipMalloc(&ipiv, (size_t)n * sizeof(int32_t)));
    CK(hipMalloc(&info, sizeof(int32_t)));
    setenv("CFX_BAND_PLACEMENT", "5", 1);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int r = 0; r < reps; ++r) {
        CK(hipMemcpy(ab, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice));
        CK(hipEventRecord(a));
        if (cfx_band_lu(n, kl, ku, 1, ab, ipiv, info, 0, nullptr, nullptr) != 0) {
            std::fprintf(stderr, "cfx_band_lu: %s\n", g_create_error.c_str());
            return 1;
        }
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        unsigned long long p[16];
        CK(hipMemcpyFromSymbol(p, HIP_SYMBOL(cfx::g_panel_prof), sizeof(p)));
        const int nb = cfx::kPanelNB, panels = (n + nb - 1) / nb;
        // per panel: [2] reach / first zero pivot, [3] write-back + blocked multipliers + LDS barrier, [4] own trailing
        // columns, [5] (wavefront 0) fill rows + next panel re-read + its factorisation, [6] wait at the closing barrier
        const char* names[8] = {"reach", "writeback_lt", "trail", "lookahead_rest", "barrier_wait", "panel_fence_load",
                                "panel_steps", "panel_store"};
        const int ids[8] = {2, 3, 4, 5, 6, 0, 1, 7};
        std::printf("{\"n\": %d, \"kl\": %d, \"ku\": %d, \"nb\": %d, \"ms\": %.3f, \"us_per_panel\": %.3f", n, kl, ku,
                    nb, ms, 1e3 * ms / panels);
        double tot = 0;
        for (int w = 0; w < 2; ++w)
            for (int i = 0; i < 8; ++i) {
                std::printf(", \"w%d_%s\": %.3f", w, names[i], p[8 * w + ids[i]] * 0.01 / panels);  // 100 MHz ticks
                if (w == 0) tot += p[ids[i]] * 0.01 / panels;
            }
        std::printf(", \"sum_us\": %.3f}\n", tot);
    }
    return 0;
}
