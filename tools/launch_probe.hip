// launch_probe.hip — measures the fixed cost of small kernels on this device (empty kernel,
// one global store, 3.5 KiB by-value argument, dependent load+store) and of back-to-back chains.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); return 1; } } while (0)

struct Big { float v[896]; int* out; };

__global__ void k_empty() {}
__global__ void k_store(int* p) { if (threadIdx.x == 0 && blockIdx.x == 0) p[0] = 1; }
__global__ void k_big(Big b) { if (threadIdx.x == 0 && blockIdx.x == 0) b.out[0] = (int)b.v[895]; }
__global__ void k_ldst(const int* a, int* p) { if (threadIdx.x == 0) p[blockIdx.x] = a[blockIdx.x] + 1; }
// every block reads 1 KiB of the by-value argument with vector loads (like a per-block LDS copy)
__global__ void k_bigvec(Big b) {
    __shared__ float s[256];
    s[threadIdx.x] = b.v[threadIdx.x * 3];
    __syncthreads();
    if (threadIdx.x == 0) b.out[blockIdx.x] = (int)s[(blockIdx.x * 7) & 255];
}
// the same 1 KiB read from a device buffer
__global__ void k_devvec(const float* v, int* out) {
    __shared__ float s[256];
    s[threadIdx.x] = v[threadIdx.x * 3];
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = (int)s[(blockIdx.x * 7) & 255];
}

template <class F>
float time_chain(hipStream_t s, int n, F f) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    for (int i = 0; i < 20; ++i) f();
    hipStreamSynchronize(s);
    hipEventRecord(a, s);
    for (int i = 0; i < n; ++i) f();
    hipEventRecord(b, s);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    return ms * 1e3f / n;
}

int main() {
    hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    int *p, *q; CK(hipMalloc(&p, 1 << 20)); CK(hipMalloc(&q, 1 << 20));
    CK(hipMemset(p, 0, 1 << 20)); CK(hipMemset(q, 0, 1 << 20));
    Big big{}; big.out = p;
    const int n = 2000;
    printf("empty 1x64      %.2f us/launch\n", time_chain(s, n, [&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s); }));
    printf("empty 1024x256  %.2f us/launch\n", time_chain(s, n, [&] { hipLaunchKernelGGL(k_empty, dim3(1024), dim3(256), 0, s); }));
    printf("store 1x64      %.2f us/launch\n", time_chain(s, n, [&] { hipLaunchKernelGGL(k_store, dim3(1), dim3(64), 0, s, p); }));
    printf("big-arg 1x64    %.2f us/launch\n", time_chain(s, n, [&] { hipLaunchKernelGGL(k_big, dim3(1), dim3(64), 0, s, big); }));
    float* dv; CK(hipMalloc(&dv, 4096)); CK(hipMemset(dv, 0, 4096));
    printf("bigvec 1200x256 %.2f us/launch\n", time_chain(s, n, [&] { hipLaunchKernelGGL(k_bigvec, dim3(1200), dim3(256), 0, s, big); }));
    printf("devvec 1200x256 %.2f us/launch\n", time_chain(s, n, [&] { hipLaunchKernelGGL(k_devvec, dim3(1200), dim3(256), 0, s, dv, p); }));
    printf("bigvec 32kx256  %.2f us/launch\n", time_chain(s, 200, [&] { hipLaunchKernelGGL(k_bigvec, dim3(32768), dim3(256), 0, s, big); }));
    printf("devvec 32kx256  %.2f us/launch\n", time_chain(s, 200, [&] { hipLaunchKernelGGL(k_devvec, dim3(32768), dim3(256), 0, s, dv, p); }));
    printf("ld+st 300x256   %.2f us/launch\n", time_chain(s, n, [&] { hipLaunchKernelGGL(k_ldst, dim3(300), dim3(256), 0, s, p, q); }));
    // single-launch latency: record/sync around one launch
    std::vector<float> lat;
    for (int i = 0; i < 50; ++i) {
        hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
        hipEventRecord(a, s);
        hipLaunchKernelGGL(k_ldst, dim3(300), dim3(256), 0, s, p, q);
        hipEventRecord(b, s);
        hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b); lat.push_back(ms * 1e3f);
    }
    float m = 0; for (float x : lat) m += x;
    printf("single ld+st event-bracketed %.2f us\n", m / lat.size());
    return 0;
}
