// Microbenchmark: the HBM ceiling of the collocation g + J_g kernel's traffic pattern (bench `collocation`: cfg 2 by
// Legendre degree 4, N = 20, nx = 2, B = 2^18) with no arithmetic beyond a copy-like combination of the inputs.
// Per instance and interval: read the d = 4 collocation states x^1..x^4 and x_{k+1}^0 (x^0 carried from the previous
// interval), write 10 g rows and 56 J_g values — 1,616 B read and 10,560 B written per instance, the kernel's
// algorithmic bytes.  Same grid as k_colloc's default shape (thread = 2 adjacent instances x 1 interval, interval
// chunks on grid.x), SoA or 64-instance tiles, non-temporal or plain 16-byte stores; plus a pure write stream and a
// pure read stream over the J_g buffer.  Prints one line per variant: ms per launch and TB/s of the algorithmic
// bytes (12,176 B per instance).
//   hipcc -O3 --offload-arch=gfx950 scripts/micro/colloc_bw.hip -o /tmp/colloc_bw && /tmp/colloc_bw
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr int N = 20, NX = 2, DEG = 4, NZ = (DEG + 1) * NX, EV = N * NZ + NX, EG = N * (DEG + 1) * NX, NJK = 56,
              EJ = N * NJK;

template <bool TILED>
__device__ __forceinline__ int64_t idx(int64_t B, int E, int e, int64_t b) {
    if (TILED) return ((b >> 6) * E + e) * 64 + (b & 63);
    return (int64_t)e * B + b;
}

template <bool NT>
__device__ __forceinline__ void st2(double* p, double a, double b) {
    typedef double d2 __attribute__((ext_vector_type(2)));
    if (NT)
        __builtin_nontemporal_store(d2{a, b}, reinterpret_cast<d2*>(p));
    else
        *reinterpret_cast<double2*>(p) = make_double2(a, b);
}

template <bool TILED, bool NT>
__global__ void __launch_bounds__(256) k_pattern(const double* __restrict__ V, double* __restrict__ G,
                                                 double* __restrict__ J, int64_t B) {
    const int k = blockIdx.x;  // interval fast
    const int64_t b = ((int64_t)blockIdx.y * 256 + threadIdx.x) * 2;
    if (b >= B) return;
    double xs[DEG + 2][NX][2];
#pragma unroll
    for (int i = 0; i <= DEG; ++i)
#pragma unroll
        for (int r = 0; r < NX; ++r) {
            const double2 t = *reinterpret_cast<const double2*>(V + idx<TILED>(B, EV, k * NZ + i * NX + r, b));
            xs[i][r][0] = t.x;
            xs[i][r][1] = t.y;
        }
#pragma unroll
    for (int r = 0; r < NX; ++r) {
        const double2 t = *reinterpret_cast<const double2*>(V + idx<TILED>(B, EV, (k + 1) * NZ + r, b));
        xs[DEG + 1][r][0] = t.x;
        xs[DEG + 1][r][1] = t.y;
    }
#pragma unroll
    for (int e = 0; e < (DEG + 1) * NX; ++e) {
        const int i = e % (DEG + 2), r = e % NX;
        st2<NT>(G + idx<TILED>(B, EG, k * (DEG + 1) * NX + e, b), xs[i][r][0] - xs[DEG + 1][r][0],
                xs[i][r][1] - xs[DEG + 1][r][1]);
    }
#pragma unroll
    for (int e = 0; e < NJK; ++e) {
        const int i = e % (DEG + 2), r = (e / 3) % NX;
        st2<NT>(J + idx<TILED>(B, EJ, k * NJK + e, b), xs[i][r][0] * e + xs[0][1][0], xs[i][r][1] * e + xs[0][1][1]);
    }
}

template <bool NT>
__global__ void __launch_bounds__(256) k_wstream(double* __restrict__ W, int64_t n2, double v) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n2; i += (int64_t)gridDim.x * 256)
        st2<NT>(W + 2 * i, v + i, v - i);
}

__global__ void __launch_bounds__(256) k_rstream(const double* __restrict__ R, int64_t n2, double* __restrict__ out) {
    double s = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n2; i += (int64_t)gridDim.x * 256) {
        const double2 t = *reinterpret_cast<const double2*>(R + 2 * i);
        s += t.x + t.y;
    }
    if (s == 1.2345) out[0] = s;
}

#define CHECK(x)                                                              \
    do {                                                                      \
        hipError_t e_ = (x);                                                  \
        if (e_ != hipSuccess) {                                               \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));      \
            std::exit(1);                                                     \
        }                                                                     \
    } while (0)

template <class F>
static double timed(F f, int reps) {
    for (int i = 0; i < 5; ++i) f();
    CHECK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    CHECK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) f();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main(int argc, char** argv) {
    const int64_t B = argc > 1 ? std::atoll(argv[1]) : (1 << 18);
    const int reps = argc > 2 ? std::atoi(argv[2]) : 200;
    // bounds (round 4's fault: a write stream sized (EG + EJ) B over the EJ B buffer): the pattern kernels write
    // instance pairs b, b + 1 < B of every element row, the streams 16-byte pairs below w2
    if (B < 2 || B % 2 != 0) {
        std::printf("batch must be even and >= 2\n");
        return 1;
    }
    double *V, *G, *J, *out;
    CHECK(hipMalloc(&V, sizeof(double) * EV * B));
    CHECK(hipMalloc(&G, sizeof(double) * EG * B));
    CHECK(hipMalloc(&J, sizeof(double) * EJ * B));
    CHECK(hipMalloc(&out, sizeof(double)));
    CHECK(hipMemset(V, 0, sizeof(double) * EV * B));
    const double bytes = 8.0 * (EV + EG + EJ) * (double)B;
    const dim3 grid(N, (unsigned)((B / 2 + 255) / 256));
    auto report = [&](const char* name, double ms, double nbytes) {
        std::printf("{\"variant\": \"%s\", \"batch\": %lld, \"ms\": %.4f, \"TBps\": %.3f, \"frac_8TBps\": %.3f}\n", name,
                    (long long)B, ms, nbytes / (ms * 1e-3) / 1e12, nbytes / (ms * 1e-3) / 8e12);
    };
    report("soa_nt", timed([&] { hipLaunchKernelGGL((k_pattern<false, true>), grid, dim3(256), 0, 0, V, G, J, B); }, reps),
           bytes);
    report("soa_plain",
           timed([&] { hipLaunchKernelGGL((k_pattern<false, false>), grid, dim3(256), 0, 0, V, G, J, B); }, reps), bytes);
    report("tiled_nt", timed([&] { hipLaunchKernelGGL((k_pattern<true, true>), grid, dim3(256), 0, 0, V, G, J, B); }, reps),
           bytes);
    report("tiled_plain",
           timed([&] { hipLaunchKernelGGL((k_pattern<true, false>), grid, dim3(256), 0, 0, V, G, J, B); }, reps), bytes);
    // pure streams over the J buffer alone (its EJ * B doubles: the bulk of the written bytes)
    const int64_t w2 = (int64_t)EJ * B / 2;
    const double jbytes = 8.0 * EJ * (double)B;
    if (2 * w2 > (int64_t)EJ * B) {  // every stream element pair inside the J allocation
        std::printf("stream bounds: %lld doubles over a %lld-double buffer\n", (long long)(2 * w2), (long long)EJ * B);
        return 1;
    }
    report("wstream_nt (J bytes)",
           timed([&] { hipLaunchKernelGGL((k_wstream<true>), dim3(4096), dim3(256), 0, 0, J, w2, 1.0); }, reps), jbytes);
    report("wstream_plain (J bytes)",
           timed([&] { hipLaunchKernelGGL((k_wstream<false>), dim3(4096), dim3(256), 0, 0, J, w2, 1.0); }, reps), jbytes);
    report("rstream (J bytes)",
           timed([&] { hipLaunchKernelGGL(k_rstream, dim3(4096), dim3(256), 0, 0, J, w2, out); }, reps), jbytes);
    CHECK(hipFree(V));
    CHECK(hipFree(G));
    CHECK(hipFree(J));
    CHECK(hipFree(out));
    return 0;
}
