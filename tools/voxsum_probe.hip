// voxsum_probe.hip - cycles per 64-point row of the voxel sum (gdf_voxsum.hpp: one component per
// wave, R rows per attempt) on one voxel, against the sequential f32 chain it replaces; with
// -DPROBE_COUNTS also how often the general path runs (counting atomics cost time).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I ros_gpu_depthmap_fusion_amd/csrc \
//         tools/voxsum_probe.hip -o tools/voxsum_probe && tools/voxsum_probe [points] [walk]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

__device__ unsigned int g_probe[4];
#ifdef PROBE_COUNTS
#define GDF_VOXSUM_PROBE(what)                                      \
    do {                                                            \
        if ((threadIdx.x & 63) == 0) atomicAdd(&g_probe[what], 1u); \
    } while (0)
#endif
#include "gdf_voxsum.hpp"

#define CHK(x)                                                           \
    do {                                                                 \
        hipError_t e_ = (x);                                             \
        if (e_ != hipSuccess) {                                          \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
            std::exit(1);                                                \
        }                                                                \
    } while (0)

constexpr uint32_t kLds = 4096;  // points staged in LDS (the LDS modes wrap at kLds)

// 4 waves, wave w sums component w with comp_rows_sum<R>: from LDS (SoA) or global (AoS)
template <int R, bool LDS>
__global__ __launch_bounds__(256) void k_comp(const float4* __restrict__ pts, uint32_t n,
                                              float* out, unsigned long long* cyc) {
    __shared__ float s_soa[4][kLds];
    for (uint32_t i = threadIdx.x; i < n && i < kLds; i += 256) {
        const float4 p = pts[i];
        s_soa[0][i] = p.x;
        s_soa[1][i] = p.y;
        s_soa[2][i] = p.z;
        s_soa[3][i] = p.w;
    }
    __syncthreads();
    const uint32_t w = threadIdx.x >> 6;
    const float* gp = reinterpret_cast<const float*>(pts) + w;
    const unsigned long long t0 = clock64();
    float s;
    if (LDS) s = gdf::comp_stretch_sum<R>([&](uint32_t i) { return s_soa[w][i % kLds]; }, 0, n, 0.0f);
    else s = gdf::comp_stretch_sum<R>([&](uint32_t i) { return gp[4 * (size_t)i]; }, 0, n, 0.0f);
    const unsigned long long t1 = clock64();
    if ((threadIdx.x & 63) == 0) {
        out[w] = s;
        if (w == 0) *cyc = t1 - t0;
    }
}

// 4 waves, wave w sums component w in chunks of 1 K values staged as rows (rows_chunk_sum)
__global__ __launch_bounds__(256) void k_rows(const float4* __restrict__ pts, uint32_t n, float* out,
                                              unsigned long long* cyc) {
    __shared__ __attribute__((aligned(16))) float s_soa[4][16 * gdf::kRowStride];
    const uint32_t w = threadIdx.x >> 6;
    float s = 0.0f;
    gdf::ChainMode cm;
    unsigned long long t = 0;
    for (uint32_t c = 0; c < n; c += 1024) {
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < 1024 && c + i < n; i += 256) {
            const float4 p = pts[c + i];
            const uint32_t k = (i >> 6) * gdf::kRowStride + (i & 63);
            s_soa[0][k] = p.x;
            s_soa[1][k] = p.y;
            s_soa[2][k] = p.z;
            s_soa[3][k] = p.w;
        }
        __syncthreads();
        const unsigned long long t0 = clock64();
        s = gdf::rows_chunk_sum(s_soa[w], min(1024u, n - c), s, cm);
        t += clock64() - t0;
    }
    if ((threadIdx.x & 63) == 0) {
        out[w] = s;
        if (w == 0) *cyc = t;
    }
}

// the sequential chain from LDS: lanes 0..3 one component each
__global__ __launch_bounds__(64) void k_chain(const float4* __restrict__ pts, uint32_t n,
                                               float* out, unsigned long long* cyc) {
    __shared__ float4 s_pts[kLds];
    const uint32_t lane = threadIdx.x;
    for (uint32_t i = lane; i < n && i < kLds; i += 64) s_pts[i] = pts[i];
    __syncthreads();
    const unsigned long long t0 = clock64();
    float acc = 0.f;
    if (lane < 4) {
        const float* c = reinterpret_cast<const float*>(s_pts) + lane;
        for (uint32_t i = 0; i < n; ++i) acc = acc + c[4 * (i % kLds)];
    }
    const unsigned long long t1 = clock64();
    if (lane < 4) out[lane] = acc;
    if (lane == 0) *cyc = t1 - t0;
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? (uint32_t)std::atoi(argv[1]) : 4096;
    const bool walk = argc > 2 && std::strcmp(argv[2], "walk") == 0;  // z around 0 (a floor)
    std::mt19937 rng(7);
    std::uniform_real_distribution<float> ux(1.93f, 1.99f), uy(0.70f, 0.80f), uz(0.56f, 0.68f),
        uw(-0.004f, 0.004f);
    std::vector<float> h(4 * (size_t)n);
    for (uint32_t i = 0; i < n; ++i) {
        h[4 * i] = ux(rng);
        h[4 * i + 1] = uy(rng);
        h[4 * i + 2] = walk ? uw(rng) : uz(rng);
        h[4 * i + 3] = 1.0f;
    }
    float want[4] = {0, 0, 0, 0}, want_w[4] = {0, 0, 0, 0};  // the chain (wrapped at kLds)
    for (uint32_t i = 0; i < n; ++i)
        for (int c = 0; c < 4; ++c) {
            want[c] = want[c] + h[4 * i + c];
            want_w[c] = want_w[c] + h[4 * (i % kLds) + c];
        }
    float4* d;
    float* dout;
    unsigned long long* dc;
    CHK(hipMalloc(&d, h.size() * 4));
    CHK(hipMalloc(&dout, 16));
    CHK(hipMalloc(&dc, 8));
    CHK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    const char* names[7] = {"sequential chain, LDS", "wave/comp R=2, LDS", "wave/comp R=4, LDS",
                            "wave/comp R=8, LDS", "wave/comp R=4, global", "wave/comp R=8, global",
                            "rows of 1 K chunks"};
    for (int k = 0; k < 7; ++k) {
        for (int rep = 0; rep < 3; ++rep) {
            unsigned int z[4] = {0, 0, 0, 0};
            CHK(hipMemcpyToSymbol(HIP_SYMBOL(g_probe), z, sizeof(z)));
            switch (k) {
                case 0: hipLaunchKernelGGL(k_chain, dim3(1), dim3(64), 0, 0, d, n, dout, dc); break;
                case 1: hipLaunchKernelGGL((k_comp<2, true>), dim3(1), dim3(256), 0, 0, d, n, dout, dc); break;
                case 2: hipLaunchKernelGGL((k_comp<4, true>), dim3(1), dim3(256), 0, 0, d, n, dout, dc); break;
                case 3: hipLaunchKernelGGL((k_comp<8, true>), dim3(1), dim3(256), 0, 0, d, n, dout, dc); break;
                case 4: hipLaunchKernelGGL((k_comp<4, false>), dim3(1), dim3(256), 0, 0, d, n, dout, dc); break;
                case 5: hipLaunchKernelGGL((k_comp<8, false>), dim3(1), dim3(256), 0, 0, d, n, dout, dc); break;
                default: hipLaunchKernelGGL(k_rows, dim3(1), dim3(256), 0, 0, d, n, dout, dc); break;
            }
            CHK(hipGetLastError());
            CHK(hipDeviceSynchronize());
            float got[4];
            unsigned long long cyc;
            unsigned int pr[4];
            CHK(hipMemcpy(got, dout, 16, hipMemcpyDeviceToHost));
            CHK(hipMemcpy(&cyc, dc, 8, hipMemcpyDeviceToHost));
            CHK(hipMemcpyFromSymbol(pr, HIP_SYMBOL(g_probe), sizeof(pr)));
            const float* w = k >= 4 ? want : want_w;  // (k_rows: no wrap)
            const bool ok = std::memcmp(got, w, 16) == 0;
            if (rep == 2)
                std::printf("%-24s n=%u rows=%u cycles=%llu cycles/row=%.1f commits=%u fails=%u "
                            "nonfinite=%u unused=%u exact=%s\n",
                            names[k], n, (n + 63) / 64, cyc, (double)cyc / ((n + 63) / 64), pr[0],
                            pr[1], pr[2], pr[3], ok ? "yes" : "NO");
        }
    }
    return 0;
}
