// issue_probe.hip - single-wave VALU issue rates on gfx950 (what one wave alone sustains):
// independent f32 adds, one dependent add chain, DPP row-shift scans (4 / 16 interleaved), and
// v_cmp -> SGPR mask -> v_cndmask round trips.  Cycles from s_memtime around the loop.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/issue_probe.hip -o tools/issue_probe
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kIters = 4096;

template <int MODE>
__global__ __launch_bounds__(64) void k_issue(float* out, unsigned long long* cyc, float seed) {
    float v[16];
    int iv[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        v[i] = seed + i + threadIdx.x;
        iv[i] = (int)threadIdx.x + i;
    }
    const unsigned long long t0 = clock64();
#pragma unroll 1
    for (int it = 0; it < kIters; ++it) {
        if (MODE == 0) {  // 16 independent adds
#pragma unroll
            for (int i = 0; i < 16; ++i) v[i] = v[i] + 1.0f;
        } else if (MODE == 1) {  // one dependent chain of 16 adds
#pragma unroll
            for (int i = 0; i < 16; ++i) v[0] = v[0] + 1.0f;
        } else if (MODE == 2) {  // 4 interleaved DPP scans (6 steps each = 24 DPP adds)
#pragma unroll
            for (int i = 0; i < 4; ++i) iv[i] += __builtin_amdgcn_update_dpp(0, iv[i], 0x111, 0xf, 0xf, false);
#pragma unroll
            for (int i = 0; i < 4; ++i) iv[i] += __builtin_amdgcn_update_dpp(0, iv[i], 0x112, 0xf, 0xf, false);
#pragma unroll
            for (int i = 0; i < 4; ++i) iv[i] += __builtin_amdgcn_update_dpp(0, iv[i], 0x114, 0xf, 0xf, false);
#pragma unroll
            for (int i = 0; i < 4; ++i) iv[i] += __builtin_amdgcn_update_dpp(0, iv[i], 0x118, 0xf, 0xf, false);
        } else if (MODE == 3) {  // 16 interleaved DPP steps of one kind
#pragma unroll
            for (int i = 0; i < 16; ++i)
                iv[i] += __builtin_amdgcn_update_dpp(0, iv[i], 0x111, 0xf, 0xf, false);
        } else if (MODE == 4) {  // compare -> mask -> select round trips (dependent)
#pragma unroll
            for (int i = 0; i < 16; ++i) v[0] = v[0] > 0.5f ? v[0] - 1.0f : v[0] + 2.0f;
        } else if (MODE == 5) {  // 16 independent compare/select
#pragma unroll
            for (int i = 0; i < 16; ++i) v[i] = v[i] > 0.5f ? v[i] - 1.0f : v[i] + 2.0f;
        } else {  // readlane -> scalar -> VALU round trips
#pragma unroll
            for (int i = 0; i < 16; ++i)
                v[0] = v[0] + __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v[0]), 63));
        }
    }
    const unsigned long long t1 = clock64();
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc += v[i] + (float)iv[i];
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) *cyc = t1 - t0;
}

int main() {
    float* out;
    unsigned long long* cyc;
    hipMalloc(&out, 256);
    hipMalloc(&cyc, 8);
    const char* names[7] = {"16 independent v_add_f32", "dependent v_add_f32 chain",
                            "4 interleaved DPP scans", "16 independent DPP adds",
                            "dependent cmp/select", "16 independent cmp/select",
                            "dependent readlane+add"};
    for (int m = 0; m < 7; ++m) {
        unsigned long long c = 0;
        for (int rep = 0; rep < 3; ++rep) {
            switch (m) {
                case 0: hipLaunchKernelGGL(k_issue<0>, dim3(1), dim3(64), 0, 0, out, cyc, 1.f); break;
                case 1: hipLaunchKernelGGL(k_issue<1>, dim3(1), dim3(64), 0, 0, out, cyc, 1.f); break;
                case 2: hipLaunchKernelGGL(k_issue<2>, dim3(1), dim3(64), 0, 0, out, cyc, 1.f); break;
                case 3: hipLaunchKernelGGL(k_issue<3>, dim3(1), dim3(64), 0, 0, out, cyc, 1.f); break;
                case 4: hipLaunchKernelGGL(k_issue<4>, dim3(1), dim3(64), 0, 0, out, cyc, 1.f); break;
                case 5: hipLaunchKernelGGL(k_issue<5>, dim3(1), dim3(64), 0, 0, out, cyc, 1.f); break;
                default: hipLaunchKernelGGL(k_issue<6>, dim3(1), dim3(64), 0, 0, out, cyc, 1.f); break;
            }
            hipDeviceSynchronize();
            hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        }
        std::printf("%-28s %.2f cycles per op\n", names[m], (double)c / (kIters * 16.0));
    }
    return 0;
}
