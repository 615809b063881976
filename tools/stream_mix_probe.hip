// The achievable HBM rate of k_sel's traffic shape on this device: a grid-stride kernel reads
// n float4 (16 B per lane, coalesced) and writes the first m of them to a second buffer - C3's
// window read (3.8 GB) with its survivor stream (2.6 GB of points + keys + runs) - with no
// compute; also the pure read and the pure copy.  Prints GB/s per shape.
//   hipcc --offload-arch=gfx950 -O3 -o tools/stream_mix_probe tools/stream_mix_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                  \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                       \
        }                                                                       \
    } while (0)

__global__ __launch_bounds__(256) void k_mix(const float4* __restrict__ src, float4* __restrict__ dst,
                                             size_t n, size_t m, float* __restrict__ sink) {
    float acc = 0.0f;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const float4 v = src[i];
        if (i < m) dst[i] = v;
        else acc += v.x;
    }
    if (acc == 1234.5f) sink[0] = acc;  // (keeps the reads of the non-copied part)
}

int main() {
    const size_t n = 3800ull << 20 >> 4;  // 3.8 GB of float4
    float4 *src, *dst;
    float* sink;
    CHK(hipMalloc(&src, n * 16));
    CHK(hipMalloc(&dst, n * 16));
    CHK(hipMalloc(&sink, 4));
    CHK(hipMemset(src, 0, n * 16));
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    int cus = 0;
    CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const double fr[3] = {0.0, 2600.0 / 3800.0, 1.0};
    const char* name[3] = {"read 3.8 GB", "read 3.8 GB + write 2.6 GB", "copy 3.8 GB"};
    for (int s = 0; s < 3; ++s) {
        const size_t m = (size_t)(fr[s] * (double)n);
        for (int blocks_per_cu : {8, 16, 32}) {
            const int grid = cus * blocks_per_cu;
            k_mix<<<grid, 256>>>(src, dst, n, m, sink);  // warm-up
            CHK(hipEventRecord(a));
            const int reps = 5;
            for (int r = 0; r < reps; ++r) k_mix<<<grid, 256>>>(src, dst, n, m, sink);
            CHK(hipEventRecord(b));
            CHK(hipEventSynchronize(b));
            float ms = 0;
            CHK(hipEventElapsedTime(&ms, a, b));
            const double bytes = (double)n * 16 + (double)m * 16;
            std::printf("%-28s grid %5d: %.3f ms  %.0f GB/s\n", name[s], grid, ms / reps,
                        bytes / (ms / reps * 1e-3) / 1e9);
        }
    }
    return 0;
}
