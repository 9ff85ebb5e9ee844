// Microbenchmark: achievable HBM write bandwidth on MI355X for store shapes the shooting kernel could use.
// 1.2 GB written per launch (the cfg-2 g + J_g output volume at B = 2^20), 30 launches per shape, after warm-up.
//   d2_gs    : 16 B per lane (dwordx4), grid-stride, 8192 blocks of 256
//   d4_gs    : 32 B per lane (2 x dwordx4), grid-stride, 8192 blocks
//   d1_gs    : 8 B per lane (dwordx2), grid-stride
//   f1_gs    : 4 B per lane (dword), grid-stride
//   chunkK   : each wave writes its own contiguous chunk of K KiB with consecutive 1 KiB instructions
//   d2_nt    : d2_gs with nontemporal stores
//   d2_g2k/16k: d2_gs with 2048 / 16384 blocks
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double d2 __attribute__((ext_vector_type(2)));

template <int W, bool NT>
__global__ void __launch_bounds__(256) k_gs(double* __restrict__ out, int64_t n_elems) {
    // W doubles per lane per iteration
    const int64_t stride = (int64_t)gridDim.x * 256 * W;
    for (int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * W; i < n_elems; i += stride) {
        if constexpr (W == 1) {
            if (NT) __builtin_nontemporal_store((double)i, out + i);
            else out[i] = (double)i;
        } else {
#pragma unroll
            for (int w = 0; w < W; w += 2) {
                d2 v = {(double)i, (double)w};
                if (NT) __builtin_nontemporal_store(v, reinterpret_cast<d2*>(out + i + w));
                else *reinterpret_cast<d2*>(out + i + w) = v;
            }
        }
    }
}

__global__ void __launch_bounds__(256) k_f1(float* __restrict__ out, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) out[i] = (float)i;
}

// each wave owns a contiguous chunk of `chunk_d2` 16-B elements (64 per instruction)
__global__ void __launch_bounds__(256) k_chunk(double* __restrict__ out, int64_t n_d2, int64_t chunk_d2) {
    const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    const int64_t nwaves = (int64_t)gridDim.x * 4;
    for (int64_t c = wave; c * chunk_d2 < n_d2; c += nwaves) {
        d2* p = reinterpret_cast<d2*>(out) + c * chunk_d2;
        for (int64_t j = lane; j < chunk_d2; j += 64) p[j] = d2{(double)j, (double)c};
    }
}

template <class F>
void timeit(const char* name, double bytes, F launch) {
    for (int r = 0; r < 5; ++r) launch();
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int reps = 30;
    (void)hipEventRecord(e0);
    for (int r = 0; r < reps; ++r) launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= reps;
    printf("%-10s %.4f ms  %.0f GB/s\n", name, ms, bytes / (ms * 1e-3) / 1e9);
}

int main() {
    const int64_t n = (int64_t)1 << 20 << 7;  // 2^27 doubles = 1.07 GB (+ room)
    double* out;
    if (hipMalloc(&out, n * 8) != hipSuccess) return 1;
    const double bytes = 8.0 * n;
    // settle
    for (int r = 0; r < 200; ++r) hipLaunchKernelGGL((k_gs<2, false>), dim3(8192), dim3(256), 0, 0, out, n);
    (void)hipDeviceSynchronize();
    for (int round = 0; round < 2; ++round) {
        timeit("d2_gs", bytes, [&] { hipLaunchKernelGGL((k_gs<2, false>), dim3(8192), dim3(256), 0, 0, out, n); });
        timeit("d4_gs", bytes, [&] { hipLaunchKernelGGL((k_gs<4, false>), dim3(8192), dim3(256), 0, 0, out, n); });
        timeit("d1_gs", bytes, [&] { hipLaunchKernelGGL((k_gs<1, false>), dim3(8192), dim3(256), 0, 0, out, n); });
        timeit("f1_gs", bytes, [&] { hipLaunchKernelGGL(k_f1, dim3(8192), dim3(256), 0, 0, (float*)out, 2 * n); });
        timeit("d2_nt", bytes, [&] { hipLaunchKernelGGL((k_gs<2, true>), dim3(8192), dim3(256), 0, 0, out, n); });
        timeit("d2_g2k", bytes, [&] { hipLaunchKernelGGL((k_gs<2, false>), dim3(2048), dim3(256), 0, 0, out, n); });
        timeit("d2_g16k", bytes, [&] { hipLaunchKernelGGL((k_gs<2, false>), dim3(16384), dim3(256), 0, 0, out, n); });
        timeit("d2_g64k", bytes, [&] { hipLaunchKernelGGL((k_gs<2, false>), dim3(65536), dim3(256), 0, 0, out, n); });
        for (int kib : {4, 16, 64, 256}) {
            char name[32];
            snprintf(name, sizeof name, "chunk%dK", kib);
            const int64_t cd2 = (int64_t)kib * 1024 / 16;
            timeit(name, bytes, [&] { hipLaunchKernelGGL(k_chunk, dim3(2048), dim3(256), 0, 0, out, n / 2, cd2); });
        }
    }
    return 0;
}
