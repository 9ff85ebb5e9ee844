// Microbenchmark: achievable HBM bandwidth for the shooting kernel's traffic pattern (per instance: read
// 42 doubles, write 40 + 100 doubles, in 20 interval steps), with no arithmetic beyond a copy-like update:
//   soa    : element e of instance b at e*B + b, 8 B per lane
//   tiled  : 64-instance tiles ((b/64)*E + e)*64 + b%64, 8 B per lane
//   soa2   : SoA, 2 adjacent instances per lane (16 B per lane)
//   soa2nt : soa2 with nontemporal stores
//   tiled2nt<KPT>: 64-instance tiles, 2 adjacent instances per lane, nontemporal stores, KPT intervals per thread
//            with the interval chunks as the fast grid index (the round-2 launch shape of k_shooting)
//   wstream/rstream: pure write / read streaming of the same byte count (reference ceilings); wstreamnt: 16-B
//            nontemporal stores
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int N = 20, NX = 2, NZ = 2, EV = N * NZ + NX, EG = N * NX, EJ = N * 5;

template <bool TILED>
__device__ __forceinline__ int64_t idx(int64_t B, int E, int e, int64_t b) {
    if (TILED) return ((b >> 6) * E + e) * 64 + (b & 63);
    return (int64_t)e * B + b;
}

template <bool TILED>
__global__ void __launch_bounds__(256) k1(const double* __restrict__ V, double* __restrict__ G, double* __restrict__ J,
                                          int64_t B) {
    const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (b >= B) return;
    double x0 = V[idx<TILED>(B, EV, 0, b)], x1 = V[idx<TILED>(B, EV, 1, b)];
    for (int kk = 0; kk < N; ++kk) {
        const double n0 = V[idx<TILED>(B, EV, (kk + 1) * NZ, b)], n1 = V[idx<TILED>(B, EV, (kk + 1) * NZ + 1, b)];
        G[idx<TILED>(B, EG, kk * 2, b)] = x0 - n0;
        G[idx<TILED>(B, EG, kk * 2 + 1, b)] = x1 - n1;
#pragma unroll
        for (int q = 0; q < 5; ++q) J[idx<TILED>(B, EJ, kk * 5 + q, b)] = x0 * q + x1;
        x0 = n0;
        x1 = n1;
    }
}

template <bool NT>
__device__ __forceinline__ void st2(double* p, double a, double b) {
    if (NT) {
        __builtin_nontemporal_store(a, p);
        __builtin_nontemporal_store(b, p + 1);
    } else {
        *reinterpret_cast<double2*>(p) = make_double2(a, b);
    }
}

template <bool NT>
__global__ void __launch_bounds__(256) k2(const double* __restrict__ V, double* __restrict__ G, double* __restrict__ J,
                                          int64_t B) {
    const int64_t b = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 2;
    if (b >= B) return;
    double2 x0 = *reinterpret_cast<const double2*>(V + b), x1 = *reinterpret_cast<const double2*>(V + B + b);
    for (int kk = 0; kk < N; ++kk) {
        const double2 n0 = *reinterpret_cast<const double2*>(V + (int64_t)((kk + 1) * NZ) * B + b);
        const double2 n1 = *reinterpret_cast<const double2*>(V + (int64_t)((kk + 1) * NZ + 1) * B + b);
        st2<NT>(G + (int64_t)(kk * 2) * B + b, x0.x - n0.x, x0.y - n0.y);
        st2<NT>(G + (int64_t)(kk * 2 + 1) * B + b, x1.x - n1.x, x1.y - n1.y);
#pragma unroll
        for (int q = 0; q < 5; ++q) st2<NT>(J + (int64_t)(kk * 5 + q) * B + b, x0.x * q + x1.x, x0.y * q + x1.y);
        x0 = n0;
        x1 = n1;
    }
}

template <int KPT>
__global__ void __launch_bounds__(256) k3(const double* __restrict__ V, double* __restrict__ G, double* __restrict__ J,
                                          int64_t B) {
    const int64_t b = ((int64_t)blockIdx.y * 256 + threadIdx.x) * 2;
    if (b >= B) return;
    const int k0 = blockIdx.x * KPT;
    typedef double nt2 __attribute__((ext_vector_type(2)));
    auto ld = [&](int E, int e) { return *reinterpret_cast<const nt2*>(V + idx<true>(B, E, e, b)); };
    auto st = [&](double* P, int E, int e, nt2 v) {
        __builtin_nontemporal_store(v, reinterpret_cast<nt2*>(P + idx<true>(B, E, e, b)));
    };
    nt2 x0 = ld(EV, k0 * NZ), x1 = ld(EV, k0 * NZ + 1);
    for (int kk = k0; kk < k0 + KPT; ++kk) {
        const nt2 n0 = ld(EV, (kk + 1) * NZ), n1 = ld(EV, (kk + 1) * NZ + 1);
        st(G, EG, kk * 2, x0 - n0);
        st(G, EG, kk * 2 + 1, x1 - n1);
#pragma unroll
        for (int q = 0; q < 5; ++q) st(J, EJ, kk * 5 + q, x0 * (double)q + x1);
        x0 = n0;
        x1 = n1;
    }
}

__global__ void kw(double4* __restrict__ out, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
        out[i] = make_double4(1.0, 2.0, 3.0, (double)i);
}
__global__ void kwnt(double* __restrict__ out, int64_t n) {
    typedef double nt2 __attribute__((ext_vector_type(2)));
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
        __builtin_nontemporal_store(nt2{1.0, (double)i}, reinterpret_cast<nt2*>(out) + i);
}
__global__ void kr(const double2* __restrict__ in, double* out, int64_t n) {
    double s = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) s += in[i].x + in[i].y;
    if (s == 1.2345) out[0] = s;
}

template <class F>
void timeit(const char* name, double bytes, F launch) {
    launch();
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    const int reps = 200;
    for (int r = 0; r < reps; ++r) launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= reps;
    printf("%-8s %.4f ms  %.0f GB/s\n", name, ms, bytes / (ms * 1e-3) / 1e9);
}

int main() {
    const int64_t B = 1 << 20;
    double *V, *G, *J;
    (void)hipMalloc(&V, 8 * B * EV);
    (void)hipMalloc(&G, 8 * B * EG);
    (void)hipMalloc(&J, 8 * B * EJ);
    (void)hipMemset(V, 0, 8 * B * EV);
    double* S;  // stream buffer sized for the write/read stream tests (never index G/J past their size)
    const double sbytes = 8.0 * B * (EG + EJ);
    (void)hipMalloc(&S, (size_t)sbytes);
    const double bytes = 8.0 * B * (EV + EG + EJ);
    for (int r = 0; r < 2; ++r) {
        timeit("soa", bytes, [&] { hipLaunchKernelGGL((k1<false>), dim3(B / 256), dim3(256), 0, 0, V, G, J, B); });
        timeit("tiled", bytes, [&] { hipLaunchKernelGGL((k1<true>), dim3(B / 256), dim3(256), 0, 0, V, G, J, B); });
        timeit("soa2", bytes, [&] { hipLaunchKernelGGL((k2<false>), dim3(B / 512), dim3(256), 0, 0, V, G, J, B); });
        timeit("soa2nt", bytes, [&] { hipLaunchKernelGGL((k2<true>), dim3(B / 512), dim3(256), 0, 0, V, G, J, B); });
        timeit("t2nt k4", bytes, [&] { hipLaunchKernelGGL((k3<4>), dim3(N / 4, B / 512), dim3(256), 0, 0, V, G, J, B); });
        timeit("t2nt k20", bytes, [&] { hipLaunchKernelGGL((k3<20>), dim3(1, B / 512), dim3(256), 0, 0, V, G, J, B); });
        timeit("wstrnt", sbytes, [&] { hipLaunchKernelGGL(kwnt, dim3(8192), dim3(256), 0, 0, S, (int64_t)(sbytes / 16)); });
        timeit("wstream", sbytes, [&] { hipLaunchKernelGGL(kw, dim3(8192), dim3(256), 0, 0, (double4*)S, (int64_t)(sbytes / 32)); });
        timeit("rstream", sbytes, [&] { hipLaunchKernelGGL(kr, dim3(8192), dim3(256), 0, 0, (const double2*)S, G, (int64_t)(sbytes / 16)); });
    }
    return 0;
}
