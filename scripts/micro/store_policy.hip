// Microbenchmark: cache policy of a write stream and the cost it leaves at the kernel boundary.  1.2 GB written per
// launch with 16-byte stores (65,536 blocks of 256, one store per lane per iteration, grid-stride), four policies:
//   plain  global_store_dwordx4                 (line kept in the XCD's L2)
//   nt     global_store_dwordx4 ... nt          (what the shooting kernel uses)
//   sc1    buffer_store_dwordx4 ... sc1         (write-through, line dropped)
//   sc1nt  buffer_store_dwordx4 ... nt sc1
// and a copy-like variant per policy (16 B read + 16 B written per lane; read share 1/2).  For each: the average over 30
// back-to-back launches (HIP events around the loop: kernel + boundary) and the average of 30 launches timed one by one
// with the queue drained in between (the kernel alone).  Build: hipcc -O3 --offload-arch=gfx950 store_policy.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef double nt2 __attribute__((ext_vector_type(2)));

template <int POL>
__device__ __forceinline__ void st16(double* base, __amdgpu_buffer_rsrc_t r, int64_t i, double a, double b) {
    if constexpr (POL == 0) {
        *reinterpret_cast<double2*>(base + i) = make_double2(a, b);
    } else if constexpr (POL == 1) {
        __builtin_nontemporal_store(nt2{a, b}, reinterpret_cast<nt2*>(base + i));
    } else {
        double2 v = make_double2(a, b);
        __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<v4i*>(&v), r, (int)(i * 8), 0, POL == 2 ? 16 : 18);
    }
}

template <int POL, bool COPY>
__global__ void __launch_bounds__(256) k_write(double* __restrict__ out, const double* __restrict__ in, int64_t n) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0x7fffffff, 0x00020000);
    const int64_t stride = (int64_t)gridDim.x * 256 * 2;
    for (int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 2; i < n; i += stride) {
        double a = (double)i, b = 1.0;
        if (COPY) {
            const double2 t = *reinterpret_cast<const double2*>(in + i);
            a = t.x * 2.0;
            b = t.y + 1.0;
        }
        st16<POL>(out, r, i, a, b);
    }
}

template <class F>
void timeit(const char* name, double bytes, F launch) {
    for (int r = 0; r < 10; ++r) launch();
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int reps = 30;
    (void)hipEventRecord(e0);
    for (int r = 0; r < reps; ++r) launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms_b2b;
    (void)hipEventElapsedTime(&ms_b2b, e0, e1);
    ms_b2b /= reps;
    double single = 0.0;
    for (int r = 0; r < reps; ++r) {
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(e0);
        launch();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        single += ms;
    }
    single /= reps;
    printf("%-12s back-to-back %.4f ms (%.0f GB/s)   one-by-one %.4f ms (%.0f GB/s)\n", name, ms_b2b,
           bytes / (ms_b2b * 1e-3) / 1e9, single, bytes / (single * 1e-3) / 1e9);
}

int main() {
    const int64_t n = (int64_t)150 << 20;  // 157M doubles = 1.26 GB
    double *out, *in;
    if (hipMalloc(&out, n * 8) != hipSuccess || hipMalloc(&in, n * 8) != hipSuccess) return 1;
    (void)hipMemset(in, 0, n * 8);
    const dim3 g(65536), b(256);
    for (int r = 0; r < 100; ++r) hipLaunchKernelGGL((k_write<1, false>), g, b, 0, 0, out, in, n);
    (void)hipDeviceSynchronize();
    for (int round = 0; round < 2; ++round) {
        timeit("w plain", 8.0 * n, [&] { hipLaunchKernelGGL((k_write<0, false>), g, b, 0, 0, out, in, n); });
        timeit("w nt", 8.0 * n, [&] { hipLaunchKernelGGL((k_write<1, false>), g, b, 0, 0, out, in, n); });
        timeit("w sc1", 8.0 * n, [&] { hipLaunchKernelGGL((k_write<2, false>), g, b, 0, 0, out, in, n); });
        timeit("w sc1nt", 8.0 * n, [&] { hipLaunchKernelGGL((k_write<3, false>), g, b, 0, 0, out, in, n); });
        timeit("copy plain", 16.0 * n, [&] { hipLaunchKernelGGL((k_write<0, true>), g, b, 0, 0, out, in, n); });
        timeit("copy nt", 16.0 * n, [&] { hipLaunchKernelGGL((k_write<1, true>), g, b, 0, 0, out, in, n); });
        timeit("copy sc1", 16.0 * n, [&] { hipLaunchKernelGGL((k_write<2, true>), g, b, 0, 0, out, in, n); });
        timeit("copy sc1nt", 16.0 * n, [&] { hipLaunchKernelGGL((k_write<3, true>), g, b, 0, 0, out, in, n); });
    }
    return 0;
}
