// Pattern ceilings of the secondary callback shapes: the shooting kernels' HBM traffic pattern —
// per instance and interval read x_k, u_k (x_{k+1} carried to the next interval), write the NX continuity values and
// the NJ structural J_g values — with no arithmetic beyond a copy-like update, in the launch shape the library uses:
// 64-instance tiles, two adjacent instances per lane (16-byte accesses), KPT consecutive intervals per thread with the
// interval chunks as the fast grid index, non-temporal stores.
//   cfg3: BASELINE configs[2] (Ding2007 pulse width, N = 100): NX 2, NU 1, NJ 6 -> 8,816 B per instance, KPT 5
//   msk : BASELINE configs[4] (arm26 + 2 Ding2007-with-fatigue muscles, N = 10): NX 14, NU 2, NJ 208 -> 19,152 B
// Bounds: element e of instance b lives at ((b / 64) E + e) 64 + b % 64 with e < E (E = EV, EG or EJ, the per-instance
// lengths the buffers are allocated with) and b < B, B a multiple of 64 (checked below).
// build: hipcc -O3 --offload-arch=gfx950 shape_bw.hip -o bin/shape_bw ; run: bin/shape_bw [B] [reps]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                              \
    do {                                                                      \
        hipError_t e_ = (x);                                                  \
        if (e_ != hipSuccess) {                                               \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));      \
            std::exit(1);                                                     \
        }                                                                     \
    } while (0)

__device__ __forceinline__ int64_t tix(int E, int e, int64_t b) { return ((b >> 6) * E + e) * 64 + (b & 63); }

__device__ __forceinline__ void st2(double* p, double a, double b) {
    __builtin_nontemporal_store(a, p);
    __builtin_nontemporal_store(b, p + 1);
}

template <int N, int NX, int NU, int NJ, int KPT>
__global__ void __launch_bounds__(256) k_shape(const double* __restrict__ V, double* __restrict__ G,
                                               double* __restrict__ J, int64_t B) {
    constexpr int NZ = NX + NU, EV = N * NZ + NX, EG = N * NX, EJ = N * NJ;
    const int chunk = blockIdx.x;  // interval chunks fast
    const int64_t b = ((int64_t)blockIdx.y * 256 + threadIdx.x) * 2;
    if (b >= B) return;
    const int k0 = chunk * KPT, k1 = min(N, k0 + KPT);
    double2 x[NX];
#pragma unroll
    for (int r = 0; r < NX; ++r) x[r] = *reinterpret_cast<const double2*>(V + tix(EV, k0 * NZ + r, b));
    for (int k = k0; k < k1; ++k) {
        double2 u[NU > 0 ? NU : 1], n[NX];
#pragma unroll
        for (int r = 0; r < NU; ++r) u[r] = *reinterpret_cast<const double2*>(V + tix(EV, k * NZ + NX + r, b));
#pragma unroll
        for (int r = 0; r < NX; ++r) n[r] = *reinterpret_cast<const double2*>(V + tix(EV, (k + 1) * NZ + r, b));
#pragma unroll
        for (int r = 0; r < NX; ++r) st2(G + tix(EG, k * NX + r, b), x[r].x - n[r].x, x[r].y - n[r].y);
        const double2 c = NU > 0 ? u[0] : x[0];
#pragma unroll
        for (int q = 0; q < NJ; ++q) st2(J + tix(EJ, k * NJ + q, b), x[q % NX].x * q + c.x, x[q % NX].y * q + c.y);
#pragma unroll
        for (int r = 0; r < NX; ++r) x[r] = n[r];
    }
}

template <int N, int NX, int NU, int NJ, int KPT>
static void run(const char* name, int64_t B, int reps) {
    constexpr int NZ = NX + NU, EV = N * NZ + NX, EG = N * NX, EJ = N * NJ;
    double *V, *G, *J;
    CHECK(hipMalloc(&V, sizeof(double) * EV * B));
    CHECK(hipMalloc(&G, sizeof(double) * EG * B));
    CHECK(hipMalloc(&J, sizeof(double) * EJ * B));
    CHECK(hipMemset(V, 0, sizeof(double) * EV * B));
    const dim3 grid((N + KPT - 1) / KPT, (unsigned)((B / 2 + 255) / 256));
    for (int w = 0; w < 5; ++w) hipLaunchKernelGGL((k_shape<N, NX, NU, NJ, KPT>), grid, dim3(256), 0, 0, V, G, J, B);
    hipEvent_t a, e;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&e));
    CHECK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k_shape<N, NX, NU, NJ, KPT>), grid, dim3(256), 0, 0, V, G, J, B);
    CHECK(hipEventRecord(e));
    CHECK(hipEventSynchronize(e));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, e));
    ms /= reps;
    const double bytes = 8.0 * (EV + EG + EJ) * (double)B;
    std::printf("{\"shape\": \"%s\", \"batch\": %lld, \"bytes_per_instance\": %d, \"ms\": %.4f, \"TBps\": %.3f, "
                "\"frac_8TBps\": %.3f}\n",
                name, (long long)B, 8 * (EV + EG + EJ), ms, bytes / (ms * 1e-3) / 1e12, bytes / (ms * 1e-3) / 8e12);
    CHECK(hipFree(V));
    CHECK(hipFree(G));
    CHECK(hipFree(J));
}

int main(int argc, char** argv) {
    const int64_t B3 = argc > 1 ? std::atoll(argv[1]) : (1 << 18);
    const int reps = argc > 2 ? std::atoi(argv[2]) : 100;
    if (B3 < 64 || B3 % 64 != 0) {
        std::printf("batch must be a positive multiple of 64\n");
        return 1;
    }
    run<100, 2, 1, 6, 5>("cfg3 (N 100, nx 2, nu 1, 6 J_g values per interval; KPT 5)", B3, reps);
    run<10, 14, 2, 208, 1>("msk cfg5 (N 10, nx 14, nu 2, 208 J_g values per interval; KPT 1)", 1 << 16, reps);
    return 0;
}
