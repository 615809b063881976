// stream_probe.hip — bandwidth of the access patterns the depth path uses (diagnostics):
// u16 loads / byte stores per thread, vs 16-B vector accesses, on a 3840x2160 frame.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); return 1; } } while (0)

__global__ void k_u16_u8(const uint16_t* __restrict__ d, uint8_t* __restrict__ o, uint32_t n) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) o[i] = d[i] ? 7 : 0;
}
__global__ void k_u16x8_u8x8(const uint4* __restrict__ d, uint2* __restrict__ o, uint32_t n8) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n8) {
        uint4 v = d[i];
        uint2 r;
        r.x = (v.x & 0xFFFF ? 7u : 0u) | (v.x >> 16 ? 7u << 8 : 0u) | (v.y & 0xFFFF ? 7u << 16 : 0u) | (v.y >> 16 ? 7u << 24 : 0u);
        r.y = (v.z & 0xFFFF ? 7u : 0u) | (v.z >> 16 ? 7u << 8 : 0u) | (v.w & 0xFFFF ? 7u << 16 : 0u) | (v.w >> 16 ? 7u << 24 : 0u);
        o[i] = r;
    }
}
// u16 loads, byte stores, one atomic per wave into 256-item counters
__global__ void k_u16_u8_atomic(const uint16_t* __restrict__ d, uint8_t* __restrict__ o, uint32_t* cnt, uint32_t n) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    bool v = i < n && d[i];
    if (i < n) o[i] = v ? 7 : 0;
    unsigned long long m = __ballot(v);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(&cnt[i >> 8], (uint32_t)__popcll(m));
}

template <class F>
float tm(hipStream_t s, int n, F f) {
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    for (int i = 0; i < 5; ++i) f();
    hipEventRecord(a, s);
    for (int i = 0; i < n; ++i) f();
    hipEventRecord(b, s); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b); return ms * 1e3f / n;
}

int main() {
    const uint32_t n = 3840 * 2160;
    uint16_t* d; uint8_t* o; uint32_t* c;
    CK(hipMalloc(&d, n * 2)); CK(hipMalloc(&o, n)); CK(hipMalloc(&c, (n / 256 + 1) * 4));
    CK(hipMemset(d, 1, n * 2)); CK(hipMemset(c, 0, (n / 256 + 1) * 4));
    hipStream_t s; CK(hipStreamCreate(&s));
    float t1 = tm(s, 50, [&] { hipLaunchKernelGGL(k_u16_u8, dim3((n + 255) / 256), dim3(256), 0, s, d, o, n); });
    float t2 = tm(s, 50, [&] { hipLaunchKernelGGL(k_u16x8_u8x8, dim3((n / 8 + 255) / 256), dim3(256), 0, s, (const uint4*)d, (uint2*)o, n / 8); });
    float t3 = tm(s, 50, [&] { hipLaunchKernelGGL(k_u16_u8_atomic, dim3((n + 255) / 256), dim3(256), 0, s, d, o, c, n); });
    printf("4K u16->u8 per thread     %.2f us  (%.0f GB/s)\n", t1, 3.0 * n / t1 / 1e3);
    printf("4K 8xu16->8xu8 per thread %.2f us  (%.0f GB/s)\n", t2, 3.0 * n / t2 / 1e3);
    printf("4K u16->u8 + wave atomic  %.2f us  (%.0f GB/s)\n", t3, 3.0 * n / t3 / 1e3);
    return 0;
}
