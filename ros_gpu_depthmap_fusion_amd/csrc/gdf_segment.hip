// gdf_segment.hip — GPU object-segmentation front end for gfx950.
//
// The reference runs this step on the CPU with OpenCV after downloading the u8 occupancy grid
// (GPUDepthmapFusion::labelVoxels, src/gpu_depthmap_fusion.cpp:1872-2011: per z-layer
// connectedComponentsWithStats(8, CV_16U) + findContours(RETR_EXTERNAL, CHAIN_APPROX_NONE)),
// then uploads the labels again for the layer-connection shader (:2013-2241,
// shader/layers_connections.glsl:96-122).  Here the grid never leaves the device:
//
//   k_cc_local    one workgroup per 16x16 tile of 2x2 pixel blocks: block foreground bits and
//                 a union-find over the tile in LDS (8-adjacency between blocks, roots = the
//                 smallest block index, i.e. the first block in block-raster order);
//   k_cc_merge    unions across tile borders with global atomicMin (lock-free union-find);
//   k_cc_flatten  every block points at its root;
//   k_cc_rank     one workgroup per layer: roots ranked in block order -> label = rank + 1
//                 (OpenCV's BBDT order: components by their first 2x2 block);
//   k_cc_pixels   one wave per 64 columns x 8 rows: u16 labels, per-label stats accumulated per
//                 run of equal labels in a row (ballot masks: min/max/area/sum of x from the mask
//                 bits, no per-pixel atomics; background and the last foreground label cached
//                 across rows), the layer connection bytes (one store per distinct pair);
//   k_cc_finish   stats rows {LEFT, TOP, WIDTH, HEIGHT, AREA} and double centroids;
//   k_cc_contours one wave per layer: the layer (1-pixel zero border) staged in LDS as int8, the
//                 raster scan of cvFindNextContour in 64-pixel ballot steps, Suzuki-Abe border
//                 following of each external start (marks 2 / -126, 8-neighbour masks), chain
//                 codes out (expanded into points on download);
//   k_cc_l2c      labelsToContours (fusion.cpp:1941-1952), findContours order = reverse discovery.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gdf.h"
#include "gdf_segment.h"
#include "gdf_kernels.hpp"

namespace {

constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr uint32_t kTile = 16;       // blocks per tile side (k_cc_local / k_cc_merge)
constexpr uint32_t kRowsPerWave = 8;  // k_cc_pixels
constexpr uint32_t kStatWords = 6;    // minx, miny, maxx, maxy, area, first (raster index)
constexpr size_t kLdsMax = 160 * 1024;

// ---- block connectivity -------------------------------------------------------------------------
// bits of a 2x2 block: 1 = (2bx, 2by), 2 = (2bx+1, 2by), 4 = (2bx, 2by+1), 8 = (2bx+1, 2by+1)
__device__ __forceinline__ uint32_t block_bits(const uint8_t* __restrict__ lay, uint32_t W,
                                               uint32_t H, uint32_t bx, uint32_t by) {
    const uint32_t x = 2 * bx, y = 2 * by;
    const uint8_t* r0 = lay + (size_t)y * W;
    uint32_t b = r0[x] ? 1u : 0u;
    if (x + 1 < W && r0[x + 1]) b |= 2u;
    if (y + 1 < H) {
        const uint8_t* r1 = r0 + W;
        if (r1[x]) b |= 4u;
        if (x + 1 < W && r1[x + 1]) b |= 8u;
    }
    return b;
}
// 8-adjacent foreground pixels between block b and its neighbour n: 0 left, 1 up, 2 up-left,
// 3 up-right
__device__ __forceinline__ bool linked(uint32_t b, uint32_t n, int dir) {
    switch (dir) {
        case 0: return (b & 5u) && (n & 10u);
        case 1: return (b & 3u) && (n & 12u);
        case 2: return (b & 1u) && (n & 8u);
        default: return (b & 2u) && (n & 4u);
    }
}

// lock-free union-find (roots = minimum index; a parent is always smaller than its child)
template <int kScope>
__device__ __forceinline__ uint32_t uf_find(uint32_t* par, uint32_t x) {
    uint32_t p = __hip_atomic_load(par + x, __ATOMIC_RELAXED, kScope);
    while (p != x) {
        x = p;
        p = __hip_atomic_load(par + x, __ATOMIC_RELAXED, kScope);
    }
    return x;
}
template <int kScope>
__device__ __forceinline__ void uf_unite(uint32_t* par, uint32_t a, uint32_t b) {
    while (true) {
        a = uf_find<kScope>(par, a);
        b = uf_find<kScope>(par, b);
        if (a == b) return;
        if (a < b) {
            const uint32_t old = __hip_atomic_fetch_min(par + b, a, __ATOMIC_RELAXED, kScope);
            if (old == b) return;
            b = old;
        } else {
            const uint32_t old = __hip_atomic_fetch_min(par + a, b, __ATOMIC_RELAXED, kScope);
            if (old == a) return;
            a = old;
        }
    }
}

__global__ __launch_bounds__(256) void k_cc_local(const uint8_t* __restrict__ grid, uint32_t W,
                                                  uint32_t H, uint32_t BW, uint32_t BH,
                                                  uint32_t* __restrict__ par,
                                                  uint8_t* __restrict__ bits) {
    __shared__ uint32_t s_par[kTile * kTile];
    __shared__ uint8_t s_bits[kTile * kTile];
    const uint32_t l = threadIdx.x, lx = l % kTile, ly = l / kTile;
    const uint32_t bx = blockIdx.x * kTile + lx, by = blockIdx.y * kTile + ly, z = blockIdx.z;
    const bool in = bx < BW && by < BH;
    const uint32_t b = in ? block_bits(grid + (size_t)z * W * H, W, H, bx, by) : 0u;
    s_bits[l] = (uint8_t)b;
    s_par[l] = b ? l : kNone;
    __syncthreads();
    if (b) {
        if (lx > 0 && linked(b, s_bits[l - 1], 0)) uf_unite<__HIP_MEMORY_SCOPE_WORKGROUP>(s_par, l, l - 1);
        if (ly > 0) {
            if (linked(b, s_bits[l - kTile], 1)) uf_unite<__HIP_MEMORY_SCOPE_WORKGROUP>(s_par, l, l - kTile);
            if (lx > 0 && linked(b, s_bits[l - kTile - 1], 2))
                uf_unite<__HIP_MEMORY_SCOPE_WORKGROUP>(s_par, l, l - kTile - 1);
            if (lx + 1 < kTile && linked(b, s_bits[l - kTile + 1], 3))
                uf_unite<__HIP_MEMORY_SCOPE_WORKGROUP>(s_par, l, l - kTile + 1);
        }
    }
    __syncthreads();
    if (!in) return;
    const size_t nbl = (size_t)BW * BH;
    const size_t g = (size_t)z * nbl + (size_t)by * BW + bx;
    uint32_t out = kNone;
    if (b) {  // the tile root (smallest local index = smallest global index of the tile part)
        const uint32_t r = uf_find<__HIP_MEMORY_SCOPE_WORKGROUP>(s_par, l);
        out = (uint32_t)(z * nbl + (size_t)(blockIdx.y * kTile + r / kTile) * BW +
                         blockIdx.x * kTile + r % kTile);
    }
    par[g] = out;
    bits[g] = (uint8_t)b;
}

__global__ __launch_bounds__(256) void k_cc_merge(const uint8_t* __restrict__ bits, uint32_t BW,
                                                  uint32_t BH, uint32_t* par) {
    const uint32_t l = threadIdx.x, lx = l % kTile, ly = l / kTile;
    const uint32_t bx = blockIdx.x * kTile + lx, by = blockIdx.y * kTile + ly, z = blockIdx.z;
    if (bx >= BW || by >= BH) return;
    const uint32_t g = (uint32_t)(z * (size_t)BW * BH + (size_t)by * BW + bx);
    const uint32_t b = bits[g];
    if (!b) return;
    // neighbours (left, up, up-left, up-right) that lie in another tile
    if (lx == 0 && bx > 0 && linked(b, bits[g - 1], 0)) uf_unite<__HIP_MEMORY_SCOPE_AGENT>(par, g, g - 1);
    if (by == 0) return;
    if (ly == 0 && linked(b, bits[g - BW], 1)) uf_unite<__HIP_MEMORY_SCOPE_AGENT>(par, g, g - BW);
    if (bx > 0 && (lx == 0 || ly == 0) && linked(b, bits[g - BW - 1], 2))
        uf_unite<__HIP_MEMORY_SCOPE_AGENT>(par, g, g - BW - 1);
    if (bx + 1 < BW && (lx + 1 == kTile || ly == 0) && linked(b, bits[g - BW + 1], 3))
        uf_unite<__HIP_MEMORY_SCOPE_AGENT>(par, g, g - BW + 1);
}

__global__ __launch_bounds__(256) void k_cc_flatten(uint32_t* par, uint32_t nb) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= nb) return;
    if (par[i] == kNone) return;
    par[i] = uf_find<__HIP_MEMORY_SCOPE_AGENT>(par, i);
}

// one workgroup per layer: roots ranked in block order.  Wave w owns a contiguous range of the
// layer's blocks and walks it 64 blocks per step (coalesced; ballot + popcount), twice: counts,
// then - after a scan of the 16 wave totals - the labels.
__global__ __launch_bounds__(1024) void k_cc_rank(const uint32_t* __restrict__ par, uint32_t nbl,
                                                  uint32_t* __restrict__ blabel,
                                                  uint32_t* __restrict__ nlabels) {
    __shared__ uint32_t s_w[16];
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6, z = blockIdx.x;
    const uint32_t base = z * nbl;
    const uint32_t per = ((nbl + 15) / 16 + 63) / 64 * 64;  // blocks per wave, whole steps
    const uint32_t b0 = min(w * per, nbl), b1 = min(b0 + per, nbl);
    const unsigned long long ltm = (1ull << lane) - 1ull;
    uint32_t cnt = 0;
    for (uint32_t i = b0 + lane; i - lane < b1; i += 64) {  // (i - lane: wave-uniform)
        const bool root = i < b1 && par[base + i] == base + i;
        cnt += (uint32_t)__popcll(__ballot(root));
    }
    if (lane == 0) s_w[w] = cnt;
    __syncthreads();
    uint32_t r = 0, tot = 0;
    for (uint32_t k = 0; k < 16; ++k) {
        const uint32_t x = s_w[k];
        r += k < w ? x : 0u;
        tot += x;
    }
    for (uint32_t i = b0 + lane; i - lane < b1; i += 64) {
        const bool root = i < b1 && par[base + i] == base + i;
        const unsigned long long m = __ballot(root);
        if (root) blabel[base + i] = 1 + r + (uint32_t)__popcll(m & ltm);
        r += (uint32_t)__popcll(m);
    }
    if (t == 0) nlabels[z] = 1 + tot;
}

struct SegArgs {
    const uint8_t* grid;
    uint32_t W, H, L, BW, nbl;
    const uint32_t* par;
    const uint32_t* blabel;
    const uint32_t* lstart;
    const uint32_t* nlab;
    const uint64_t* cstart;
    uint16_t* labels;
    int32_t* st;      // [T][kStatWords]
    unsigned long long* sums;  // [T][2]
    uint8_t* conn;
    int do_conn;
    unsigned long long* bgpart;  // [L][waves of the layer][kBgWords]: background partials
};
constexpr uint32_t kBgWords = 5;

__device__ __forceinline__ uint32_t pixel_label(const SegArgs& a, uint32_t z, uint32_t x,
                                                uint32_t y) {
    return a.blabel[a.par[(size_t)z * a.nbl + (size_t)(y >> 1) * a.BW + (x >> 1)]];
}

// sum of the positions of the set bits of a 64-bit lane mask
__device__ __forceinline__ uint32_t bit_pos_sum(uint64_t m) {
    return (uint32_t)__popcll(m & 0xAAAAAAAAAAAAAAAAull) +
           2u * (uint32_t)__popcll(m & 0xCCCCCCCCCCCCCCCCull) +
           4u * (uint32_t)__popcll(m & 0xF0F0F0F0F0F0F0F0ull) +
           8u * (uint32_t)__popcll(m & 0xFF00FF00FF00FF00ull) +
           16u * (uint32_t)__popcll(m & 0xFFFF0000FFFF0000ull) +
           32u * (uint32_t)__popcll(m & 0xFFFFFFFF00000000ull);
}

struct StatAcc {  // wave-uniform partial stats of one label
    uint32_t label;
    int32_t minx, miny, maxx, maxy;
    uint32_t area, first;
    unsigned long long sx, sy;
};

__device__ __forceinline__ void acc_reset(StatAcc& s, uint32_t label) {
    s.label = label;
    s.minx = INT_MAX; s.miny = INT_MAX; s.maxx = INT_MIN; s.maxy = INT_MIN;
    s.area = 0; s.first = kNone; s.sx = 0; s.sy = 0;
}
__device__ __forceinline__ void acc_add(StatAcc& s, int32_t mnx, int32_t mxx, int32_t y,
                                        uint32_t cnt, uint32_t first, unsigned long long sx) {
    s.minx = min(s.minx, mnx);
    s.maxx = max(s.maxx, mxx);
    s.miny = min(s.miny, y);
    s.maxy = max(s.maxy, y);
    s.area += cnt;
    s.first = min(s.first, first);
    s.sx += sx;
    s.sy += (unsigned long long)cnt * (uint32_t)y;
}
__device__ __forceinline__ void acc_flush(const StatAcc& s, const SegArgs& a, uint32_t ls) {
    if (s.label == kNone || s.area == 0) return;
    if ((threadIdx.x & 63) != 0) return;
    int32_t* st = a.st + (size_t)(ls + s.label) * kStatWords;
    atomicMin(st + 0, s.minx);
    atomicMin(st + 1, s.miny);
    atomicMax(st + 2, s.maxx);
    atomicMax(st + 3, s.maxy);
    atomicAdd(reinterpret_cast<uint32_t*>(st + 4), s.area);
    atomicMin(reinterpret_cast<uint32_t*>(st + 5), s.first);
    atomicAdd(a.sums + 2 * (size_t)(ls + s.label), s.sx);
    atomicAdd(a.sums + 2 * (size_t)(ls + s.label) + 1, s.sy);
}

__global__ __launch_bounds__(64) void k_cc_pixels(SegArgs a) {
    const uint32_t lane = threadIdx.x, x0 = blockIdx.x * 64, x = x0 + lane;
    const uint32_t y0 = blockIdx.y * kRowsPerWave, z = blockIdx.z;
    const bool inx = x < a.W;
    const size_t LS = (size_t)a.W * a.H;
    const uint8_t* lay = a.grid + z * LS;
    const uint32_t ls = a.lstart[z];
    const bool conn = a.do_conn && z + 1 < a.L;
    const uint32_t nb = conn ? a.nlab[z + 1] : 0u;
    uint8_t* cm = conn ? a.conn + a.cstart[z] : nullptr;
    StatAcc bg, fg;
    acc_reset(bg, 0);
    acc_reset(fg, kNone);
    uint32_t lastA = kNone, lastB = kNone;
    for (uint32_t r = 0; r < kRowsPerWave; ++r) {
        const uint32_t y = y0 + r;
        if (y >= a.H) break;
        const size_t p = (size_t)y * a.W + x;
        uint32_t lab = 0;
        if (inx && lay[p]) lab = pixel_label(a, z, x, y);
        if (inx) a.labels[z * LS + p] = (uint16_t)lab;
        uint64_t act = __ballot(inx);
        while (act) {  // runs of equal labels in this row segment (wave-uniform)
            const uint32_t L0 = __shfl(lab, __ffsll((long long)act) - 1, 64);
            const uint64_t m = __ballot(inx && lab == L0);
            act &= ~m;
            const uint32_t cnt = (uint32_t)__popcll(m);
            const int32_t mnx = (int32_t)(x0 + __ffsll((long long)m) - 1);
            const int32_t mxx = (int32_t)(x0 + 63 - __clzll((long long)m));
            const unsigned long long sx = (unsigned long long)cnt * x0 + bit_pos_sum(m);
            const uint32_t first = y * a.W + (uint32_t)mnx;
            if (L0 == 0) {
                acc_add(bg, mnx, mxx, (int32_t)y, cnt, first, sx);
            } else {
                if (fg.label != L0) {
                    acc_flush(fg, a, ls);
                    acc_reset(fg, L0);
                }
                acc_add(fg, mnx, mxx, (int32_t)y, cnt, first, sx);
            }
        }
        if (conn) {  // layers_connections.glsl:96-122 (neighbors_size 0)
            uint32_t lb = 0;
            if (inx && lay[LS + p]) lb = pixel_label(a, z + 1, x, y);
            uint64_t act2 = __ballot(inx);
            while (act2) {
                const int ld = __ffsll((long long)act2) - 1;
                const uint32_t A = __shfl(lab, ld, 64), B = __shfl(lb, ld, 64);
                act2 &= ~__ballot(inx && lab == A && lb == B);
                if (A != lastA || B != lastB) {
                    if (lane == 0) cm[(size_t)A * nb + B] = 1;
                    lastA = A;
                    lastB = B;
                }
            }
        }
    }
    // the background label is in every wave: partials (no atomics), reduced per layer by
    // k_cc_bg_reduce; kBgWords u64 per wave: {minx | miny}, {maxx | maxy}, {area | first}, sx, sy
    if (lane == 0) {
        unsigned long long* bp =
            a.bgpart + kBgWords * ((size_t)(z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x);
        bp[0] = ((unsigned long long)(uint32_t)bg.minx << 32) | (uint32_t)bg.miny;
        bp[1] = ((unsigned long long)(uint32_t)bg.maxx << 32) | (uint32_t)bg.maxy;
        bp[2] = ((unsigned long long)bg.area << 32) | bg.first;
        bp[3] = bg.sx;
        bp[4] = bg.sy;
    }
    acc_flush(fg, a, ls);
}

// one workgroup per layer: the background label's stats from the k_cc_pixels partials
__global__ __launch_bounds__(256) void k_cc_bg_reduce(const unsigned long long* __restrict__ bgpart,
                                                      uint32_t waves_per_layer,
                                                      const uint32_t* __restrict__ lstart,
                                                      int32_t* __restrict__ st,
                                                      unsigned long long* __restrict__ sums) {
    __shared__ int32_t s_i[4][8];
    __shared__ uint32_t s_u[2][8];
    __shared__ unsigned long long s_s[2][8];
    const uint32_t z = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
    int32_t mnx = INT_MAX, mny = INT_MAX, mxx = INT_MIN, mxy = INT_MIN;
    uint32_t area = 0, first = kNone;
    unsigned long long sx = 0, sy = 0;
    const unsigned long long* bp = bgpart + (size_t)z * waves_per_layer * kBgWords;
    for (uint32_t i = t; i < waves_per_layer; i += 256) {
        const unsigned long long* q = bp + (size_t)i * kBgWords;
        const unsigned long long a0 = q[0], a1 = q[1], a2 = q[2];
        mnx = min(mnx, (int32_t)(a0 >> 32));
        mny = min(mny, (int32_t)(uint32_t)a0);
        mxx = max(mxx, (int32_t)(a1 >> 32));
        mxy = max(mxy, (int32_t)(uint32_t)a1);
        area += (uint32_t)(a2 >> 32);
        first = min(first, (uint32_t)a2);
        sx += q[3];
        sy += q[4];
    }
    for (int d = 32; d >= 1; d >>= 1) {
        mnx = min(mnx, __shfl_xor(mnx, d, 64));
        mny = min(mny, __shfl_xor(mny, d, 64));
        mxx = max(mxx, __shfl_xor(mxx, d, 64));
        mxy = max(mxy, __shfl_xor(mxy, d, 64));
        area += __shfl_xor(area, d, 64);
        first = min(first, (uint32_t)__shfl_xor((int)first, d, 64));
        sx += __shfl_xor(sx, d, 64);
        sy += __shfl_xor(sy, d, 64);
    }
    if (lane == 0) {
        s_i[0][w] = mnx; s_i[1][w] = mny; s_i[2][w] = mxx; s_i[3][w] = mxy;
        s_u[0][w] = area; s_u[1][w] = first;
        s_s[0][w] = sx; s_s[1][w] = sy;
    }
    __syncthreads();
    if (t != 0) return;
    for (int k = 1; k < 4; ++k) {
        mnx = min(mnx, s_i[0][k]); mny = min(mny, s_i[1][k]);
        mxx = max(mxx, s_i[2][k]); mxy = max(mxy, s_i[3][k]);
        area += s_u[0][k]; first = min(first, s_u[1][k]);
        sx += s_s[0][k]; sy += s_s[1][k];
    }
    int32_t* o = st + (size_t)lstart[z] * kStatWords;  // label 0 of layer z
    o[0] = mnx; o[1] = mny; o[2] = mxx; o[3] = mxy; o[4] = (int32_t)area; o[5] = (int32_t)first;
    sums[2 * (size_t)lstart[z]] = sx;
    sums[2 * (size_t)lstart[z] + 1] = sy;
}

__global__ __launch_bounds__(256) void k_cc_init_stats(int32_t* st, unsigned long long* sums,
                                                       uint32_t T) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= T) return;
    int32_t* s = st + (size_t)i * kStatWords;
    s[0] = INT_MAX; s[1] = INT_MAX; s[2] = INT_MIN; s[3] = INT_MIN; s[4] = 0; s[5] = -1;
    sums[2 * (size_t)i] = 0;
    sums[2 * (size_t)i + 1] = 0;
}

// CCStatsOp::finish: WIDTH = right - left + 1 (int wrap for an empty label), centroid = sum / area
__global__ __launch_bounds__(256) void k_cc_finish(const int32_t* __restrict__ st,
                                                   const unsigned long long* __restrict__ sums,
                                                   uint32_t T, int32_t* __restrict__ stats5,
                                                   double* __restrict__ cent,
                                                   int32_t* __restrict__ l2c) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= T) return;
    const int32_t* s = st + (size_t)i * kStatWords;
    int32_t* o = stats5 + 5 * (size_t)i;
    o[0] = s[0];
    o[1] = s[1];
    o[2] = (int32_t)((uint32_t)s[2] - (uint32_t)s[0] + 1u);
    o[3] = (int32_t)((uint32_t)s[3] - (uint32_t)s[1] + 1u);
    o[4] = s[4];
    const double area = (double)(uint32_t)s[4];
    cent[2 * (size_t)i] = (double)sums[2 * (size_t)i] / area;
    cent[2 * (size_t)i + 1] = (double)sums[2 * (size_t)i + 1] / area;
    l2c[i] = -1;
}

// ---- findContours(RETR_EXTERNAL, CHAIN_APPROX_NONE) per layer -------------------------------------
// chain code s: 0 (+1, 0), 1 (+1, -1), 2 (0, -1), 3 (-1, -1), 4 (-1, 0), 5 (-1, +1), 6 (0, +1),
// 7 (+1, +1) - icvCodeDeltas; dx + 1 / dy + 1 packed 2 bits per code
__device__ __forceinline__ int code_dx(int s) { return (int)((0x901Au >> (2 * s)) & 3u) - 1; }
__device__ __forceinline__ int code_dy(int s) { return (int)((0xA901u >> (2 * s)) & 3u) - 1; }

template <bool kLds>
struct Img {
    int8_t* p;
    __device__ __forceinline__ int get(int i) const {
        if (kLds) return p[i];
        return __hip_atomic_load(p + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    // 4 pixels at a 4-aligned index
    __device__ __forceinline__ uint32_t get4(int i) const {
        const uint32_t* q = reinterpret_cast<const uint32_t*>(p + i);
        if (kLds) return *q;
        return __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __device__ __forceinline__ void set(int i, int8_t v) const {
        if (kLds) {
            p[i] = v;
        } else {
            __hip_atomic_store(p + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __threadfence_block();
        }
    }
    __device__ __forceinline__ void zero4(int i) const {
        uint32_t* q = reinterpret_cast<uint32_t*>(p + i);
        if (kLds) *q = 0u;
        else __hip_atomic_store(q, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
};

__device__ __forceinline__ int rdlane(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ int byte_at(uint32_t w, int k) { return (int)(int8_t)(w >> (8 * k)); }

// The 3x3 neighbourhood of pixel i in ONE lane-parallel read: lane k < 8 reads the neighbour of
// chain code k, lane 8 the pixel itself.  Returns the non-zero mask of the 8 neighbours (bit s =
// code s; zero-ness never changes while marking) and the centre value.
template <bool kLds>
__device__ __forceinline__ uint32_t nbhd(const Img<kLds>& im, int i, int P, int lane, int& centre) {
    const int off = lane < 8 ? code_dy(lane) * P + code_dx(lane) : 0;
    const int v = lane < 9 ? im.get(i + off) : 0;
    centre = rdlane(v, 8);
    return (uint32_t)(__ballot(v != 0) & 0xFFu);
}

// icvFetchContour of an outer border (is_hole = 0, nbd = 2) from padded pixel i0 (row pitch P;
// wave-uniform control, one LDS read per step); lane 0 writes the marks and one chain code per
// written point (the last one leads back to the start).  Returns the point count.
template <bool kLds>
__device__ __forceinline__ uint32_t fetch_outer(const Img<kLds>& im, int P, int i0, int lane,
                                                uint8_t* codes, uint64_t cap, uint64_t& cpos,
                                                bool& overflow) {
    int c0;
    const uint32_t m0 = nbhd(im, i0, P, lane, c0);
    // clockwise from code 3 down to 5 (code 4, the scan's zero predecessor, ends the search):
    // cw bit k = m0 bit of code (3 - k) & 7 for k = 0..6
    const uint32_t cw = ((m0 >> 3) & 1u) | ((m0 >> 1) & 2u) | ((m0 << 1) & 4u) | ((m0 << 3) & 8u) |
                        ((m0 >> 3) & 16u) | ((m0 >> 1) & 32u) | ((m0 << 1) & 64u);
    if (cw == 0) {  // single point
        if (lane == 0) im.set(i0, (int8_t)(2 | -128));
        return 1;
    }
    int s = (3 - (int)__builtin_ctz(cw)) & 7;
    const int i1 = i0 + code_dy(s) * P + code_dx(s);
    int i3 = i0;
    uint32_t npts = 0;
    for (;;) {
        const int s_end = s;
        int c3;
        const uint32_t m = nbhd(im, i3, P, lane, c3);
        // counter-clockwise from s_end + 1: first non-zero neighbour (the previous pixel is one)
        const uint32_t rot = ((m | (m << 8)) >> (s_end + 1)) & 0xFFu;
        s = (s_end + 1 + (int)__builtin_ctz(rot)) & 7;
        const int i4 = i3 + code_dy(s) * P + code_dx(s);
        if (lane == 0) {
            if ((unsigned)(s - 1) < (unsigned)s_end) im.set(i3, (int8_t)(2 | -128));
            else if (c3 == 1) im.set(i3, 2);
        }
        ++npts;
        if (cpos >= cap) {
            overflow = true;
            return npts;
        }
        if (lane == 0) codes[cpos] = (uint8_t)s;
        ++cpos;
        if (i4 == i0 && i3 == i1) break;
        i3 = i4;
        s = (s + 4) & 7;
    }
    return npts;
}

__host__ __device__ inline int contour_pitch(uint32_t W) { return (int)((W + 2 + 3) & ~3u); }
__host__ __device__ inline size_t contour_image_bytes(uint32_t W, uint32_t H) {
    return (size_t)contour_pitch(W) * (H + 2) + (((H + 2) + 3) & ~3u);
}

// one workgroup per layer (8 waves stage the image, wave 0 scans); rec[4 * d] = {x, y, first
// code, points} of the d-th DISCOVERED contour.  Image (LDS, or the global scratch): Hp rows of
// P = roundup4(W + 2) int8 pixels (zero border), then Hp row flags (row has a non-zero pixel: an
// all-zero row holds no transition of the scan and is skipped; marking never zeroes a pixel).
constexpr int kContourThreads = 512;
template <bool kLds>
__global__ __launch_bounds__(kContourThreads) void k_cc_contours(
    const uint8_t* __restrict__ grid, uint32_t W, uint32_t H, int8_t* gscratch,
    uint8_t* __restrict__ codes, uint64_t code_cap, uint32_t* __restrict__ rec, uint32_t rec_cap,
    uint32_t* __restrict__ ncont, uint32_t* __restrict__ err, unsigned long long* tdbg) {
    extern __shared__ int8_t s_img[];
    const uint32_t z = blockIdx.x;
    const unsigned long long t_start = wall_clock64();
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int Wp = (int)W + 2, Hp = (int)H + 2, P = contour_pitch(W);
    const int total = (int)contour_image_bytes(W, H);
    const Img<kLds> im{kLds ? s_img : gscratch + (size_t)z * total};
    const int rowflag = P * Hp;
    // 1. zero image (with its border) and row flags
    for (int i = 4 * threadIdx.x; i < total; i += 4 * kContourThreads) im.zero4(i);
    __syncthreads();
    // 2. scatter the layer's non-zero cells (binarised: copyMakeBorder + threshold); most 16-byte
    //    chunks of an occupancy grid are zero and write nothing
    const uint8_t* lay = grid + (size_t)z * W * H;
    const uint32_t n = W * H;
    uint32_t done = 0;
    if ((reinterpret_cast<uintptr_t>(lay) & 15u) == 0) {
        const uint4* v4 = reinterpret_cast<const uint4*>(lay);
        const uint32_t n16 = n / 16;
        for (uint32_t c0 = threadIdx.x; c0 < n16; c0 += 4 * kContourThreads) {
            uint4 q[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t c = c0 + k * kContourThreads;
                q[k] = c < n16 ? v4[c] : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if ((q[k].x | q[k].y | q[k].z | q[k].w) == 0) continue;
                uint32_t i = (c0 + k * kContourThreads) * 16, y = i / W, x = i - y * W;
                const uint32_t w4[4] = {q[k].x, q[k].y, q[k].z, q[k].w};
                for (int b = 0; b < 16; ++b) {
                    if ((w4[b >> 2] >> (8 * (b & 3))) & 0xFFu) {
                        im.set((int)(y + 1) * P + (int)x + 1, 1);
                        im.set(rowflag + (int)y + 1, 1);
                    }
                    if (++x == W) {
                        x = 0;
                        ++y;
                    }
                }
            }
        }
        done = n16 * 16;
    }
    for (uint32_t i = done + threadIdx.x; i < n; i += kContourThreads)
        if (lay[i]) {
            const uint32_t y = i / W, x = i - y * W;
            im.set((int)(y + 1) * P + (int)x + 1, 1);
            im.set(rowflag + (int)y + 1, 1);
        }
    __syncthreads();
    if (wv != 0) return;  // the raster scan is sequential: one wave
    const unsigned long long t_staged = wall_clock64();
    uint8_t* cz = codes + (size_t)z * code_cap;
    uint32_t* rz = rec + (size_t)z * rec_cap * 4;
    uint64_t cpos = 0;
    uint32_t nc = 0;
    bool overflow = false;
    // 3. cvFindNextContour (mode RETR_EXTERNAL) over the non-empty rows, 64 flags per read; a row
    //    is read 256 pixels per step (4 per lane), its transitions walked in registers
    for (int yb = 1; yb < Hp - 1 && !overflow; yb += 64) {
        uint64_t rows = __ballot(yb + lane < Hp - 1 && im.get(rowflag + yb + lane) != 0);
        while (rows && !overflow) {
            const int y = yb + (int)__builtin_ctzll(rows);
            rows &= rows - 1;
            const int rb = y * P;
            int x = 1, lnbd = 0, lnbd_val = 0;  // lnbd: the row's last marked run start (0: border)
            for (int cb = 0; cb < Wp - 1 && !overflow; cb += 256) {
            reload:
                const int q = cb + 4 * lane;  // this lane's 4 pixels [q, q + 4)
                const uint32_t w = q < P ? im.get4(rb + q) : 0u;
                const uint32_t pw = (q >= 4 && q - 4 < P) ? im.get4(rb + q - 4) : 0u;
                // transitions of the run skip at positions [x, Wp - 2]: img[X] != img[X - 1]
                uint64_t T[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int pos = q + k;
                    const int left = k ? byte_at(w, k - 1) : byte_at(pw, 3);
                    T[k] = __ballot(pos >= x && pos <= Wp - 2 && byte_at(w, k) != left);
                }
                while (T[0] | T[1] | T[2] | T[3]) {
                    // the next transition in position order: lane-major, then byte
                    int best = 1 << 30, bk = 0;
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        if (T[k]) {
                            const int c = 4 * (int)__builtin_ctzll(T[k]) + k;
                            if (c < best) {
                                best = c;
                                bk = k;
                            }
                        }
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        if (k == bk) T[k] &= T[k] - 1;
                    const int X = cb + best, bl = best >> 2;
                    const uint32_t wl = (uint32_t)rdlane((int)w, bl);
                    const int p = byte_at(wl, bk);
                    const int prev = bk ? byte_at(wl, bk - 1) : byte_at((uint32_t)rdlane((int)pw, bl), 3);
                    if (prev == 0 && p == 1) {
                        int lv = lnbd_val;
                        if (lnbd >= cb) {
                            const int o = lnbd - cb;
                            lv = byte_at((uint32_t)rdlane((int)w, o >> 2), o & 3);
                        }
                        if (lv <= 0) {  // an external border start: trace it
                            if (nc >= rec_cap) {
                                overflow = true;
                                break;
                            }
                            const uint64_t c0 = cpos;
                            const uint32_t np = fetch_outer(im, P, rb + X, lane, cz, code_cap, cpos,
                                                            overflow);
                            if (lane == 0) {
                                rz[4 * nc + 0] = (uint32_t)(X - 1);
                                rz[4 * nc + 1] = (uint32_t)(y - 1);
                                rz[4 * nc + 2] = (uint32_t)c0;
                                rz[4 * nc + 3] = np;
                            }
                            ++nc;
                            if (overflow) break;
                            // the scan resumes at X + 1 with prev = the marked start (no lnbd
                            // update); the trace may have re-marked pixels of this row
                            if (lnbd < cb) lnbd_val = im.get(rb + lnbd);
                            x = X + 1;
                            goto reload;
                        }
                    } else if (p == 0 && prev >= 1) {  // a hole border start: skipped
                        if (prev & -2) {
                            lnbd = X - 1;
                            lnbd_val = prev;
                        }
                    }
                    if (p & -2) {  // resume: lnbd follows marked runs
                        lnbd = X;
                        lnbd_val = p;
                    }
                }
                x = max(x, cb + 256);
            }
        }
    }
    if (lane == 0) {
        ncont[z] = nc;
        if (overflow) atomicOr(err, 1u);
        if (tdbg) {  // GDF_SEG_DEBUG: phase times (100 MHz wall clock) and chain codes per layer
            tdbg[4 * z + 0] = t_staged - t_start;
            tdbg[4 * z + 1] = wall_clock64() - t_staged;
            tdbg[4 * z + 2] = cpos;
            tdbg[4 * z + 3] = nc;
        }
    }
}

// The contours of all layers packed back to back for ONE download each of records and chain
// codes: block z places layer z's records at roff[z] = the records of the layers before it and
// its codes at coff[z] (a layer's codes end where its last record's end: start + length);
// hdr = roff[0..L] then coff[0..L].
__global__ __launch_bounds__(256) void k_cc_pack_contours(
    const uint32_t* __restrict__ rec, uint32_t rec_cap, const uint8_t* __restrict__ codes,
    uint64_t code_cap, const uint32_t* __restrict__ ncont, uint32_t L,
    uint32_t* __restrict__ prec, uint8_t* __restrict__ pcodes, unsigned long long* __restrict__ hdr) {
    __shared__ unsigned long long s_r, s_c;
    const uint32_t z = blockIdx.x, t = threadIdx.x;
    if (t == 0) s_r = s_c = 0;
    __syncthreads();
    unsigned long long r = 0, c = 0;
    for (uint32_t q = t; q < z + (z + 1 == L ? 1u : 0u); q += 256) {  // (the last block: all L)
        const uint32_t n = min(ncont[q], rec_cap);  // (clamps: a capacity error is reported)
        if (q < z) r += n;
        if (q < z && n) {
            const uint32_t* last = rec + ((size_t)q * rec_cap + n - 1) * 4;
            c += min((unsigned long long)last[2] + last[3], (unsigned long long)code_cap);
        }
    }
    if (r) atomicAdd(&s_r, r);
    if (c) atomicAdd(&s_c, c);
    __syncthreads();
    const uint32_t n = min(ncont[z], rec_cap);
    const unsigned long long roff = s_r, coff = s_c;
    const uint32_t* rz = rec + (size_t)z * rec_cap * 4;
    for (uint32_t i = t; i < 4 * n; i += 256) prec[roff * 4 + i] = rz[i];
    const uint64_t used = n ? min((uint64_t)rz[4 * (n - 1) + 2] + rz[4 * (n - 1) + 3], code_cap) : 0;
    const uint8_t* cz = codes + (size_t)z * code_cap;
    for (uint64_t i = t; i < used; i += 256) pcodes[coff + i] = cz[i];
    if (t == 0) {
        hdr[z] = roff;
        hdr[L + 1 + z] = coff;
        if (z + 1 == L) {
            hdr[L] = roff + n;
            hdr[2 * L + 1] = coff + used;
        }
    }
}

// labelsToContours: contour j (findContours order) = discovered contour nc - 1 - j
__global__ __launch_bounds__(256) void k_cc_l2c(const uint32_t* __restrict__ rec, uint32_t rec_cap,
                                                const uint32_t* __restrict__ ncont,
                                                const uint16_t* __restrict__ labels, uint32_t W,
                                                uint32_t H, const uint32_t* __restrict__ lstart,
                                                int32_t* __restrict__ l2c) {
    const uint32_t z = blockIdx.x, nc = ncont[z];
    const uint32_t* rz = rec + (size_t)z * rec_cap * 4;
    for (uint32_t d = threadIdx.x; d < nc; d += 256) {
        const uint32_t x = rz[4 * d], y = rz[4 * d + 1];
        const uint32_t lab = labels[(size_t)z * W * H + (size_t)y * W + x];
        l2c[lstart[z] + lab] = (int32_t)(nc - 1 - d);
    }
}

// mergeLabelsAcrossLayers (fusion.cpp:2243-2361) on the device, one workgroup: the sequential
// global labels gl[k] = k are min-propagated bottom-up (layer i+1 takes the smallest label of the
// connected labels of layer i), then top-down, over the numA x numB connection matrices
// (background connects only with background), and numbered in UIntGrouper order: merged[k] = the
// rank of gl[k] among the distinct propagated values (gl[k] <= k, so a flag per value and one
// scan).  A pass is parallel over the labels it writes (each reads only the finished neighbour
// layer), so the result is the host loop's; passes are separated by barriers.
constexpr uint32_t kMergeThreads = 1024;
__global__ __launch_bounds__(kMergeThreads) void k_cc_merge_layers(
    const uint8_t* __restrict__ conn, const uint64_t* __restrict__ cstart,
    const uint32_t* __restrict__ nlab, const uint32_t* __restrict__ lstart, uint32_t L,
    uint32_t T, uint32_t* __restrict__ gl, uint32_t* __restrict__ flag,
    uint32_t* __restrict__ merged, uint32_t* __restrict__ nobj) {
    const uint32_t t = threadIdx.x;
    for (uint32_t k = t; k < T; k += kMergeThreads) {
        gl[k] = k;
        flag[k] = 0;
    }
    __syncthreads();
    for (uint32_t i = 0; i + 1 < L; ++i) {  // bottom-up: layer i+1 from layer i
        const uint32_t nA = nlab[i], nB = nlab[i + 1], sa = lstart[i], sb = lstart[i + 1];
        const uint8_t* m = conn + cstart[i];
        for (uint32_t b = t; b < nB; b += kMergeThreads) {
            uint32_t v = gl[sb + b];
            for (uint32_t a = b == 0 ? 0 : 1; a < (b == 0 ? 1u : nA); ++a)
                if (m[(size_t)a * nB + b]) v = min(v, gl[sa + a]);
            gl[sb + b] = v;
        }
        __syncthreads();
    }
    for (uint32_t j = 0; j + 1 < L; ++j) {  // top-down: layer i from layer i+1
        const uint32_t i = L - 2 - j;
        const uint32_t nA = nlab[i], nB = nlab[i + 1], sa = lstart[i], sb = lstart[i + 1];
        const uint8_t* m = conn + cstart[i];
        for (uint32_t a = t; a < nA; a += kMergeThreads) {
            uint32_t v = gl[sa + a];
            const uint8_t* row = m + (size_t)a * nB;
            for (uint32_t b = a == 0 ? 0 : 1; b < (a == 0 ? 1u : nB); ++b)
                if (row[b]) v = min(v, gl[sb + b]);
            gl[sa + a] = v;
        }
        __syncthreads();
    }
    for (uint32_t k = t; k < T; k += kMergeThreads) flag[gl[k]] = 1;
    __syncthreads();
    // exclusive scan of the flags in chunks of kMergeThreads (flag[v] becomes v's rank)
    __shared__ uint32_t wsum[kMergeThreads / 64];
    __shared__ uint32_t carry;
    if (t == 0) carry = 0;
    __syncthreads();
    const uint32_t lane = t & 63, w = t >> 6;
    for (uint32_t base = 0; base < T; base += kMergeThreads) {
        const uint32_t k = base + t;
        const uint32_t f = k < T ? flag[k] : 0;
        const uint64_t bal = __ballot(f != 0);
        const uint32_t below = __popcll(bal & ((1ull << lane) - 1));
        if (lane == 63) wsum[w] = below + f;
        __syncthreads();
        uint32_t pre = carry;
        for (uint32_t q = 0; q < w; ++q) pre += wsum[q];
        if (k < T) flag[k] = pre + below;
        __syncthreads();
        if (t == kMergeThreads - 1) carry = pre + below + f;
        __syncthreads();
    }
    for (uint32_t k = t; k < T; k += kMergeThreads) merged[k] = flag[gl[k]];
    if (t == 0) *nobj = carry;
}

// ---- host ------------------------------------------------------------------------------------------
struct GpuBuf {
    void* p = nullptr;
    size_t bytes = 0;
    GpuBuf() = default;
    GpuBuf(const GpuBuf&) = delete;
    GpuBuf& operator=(const GpuBuf&) = delete;
    ~GpuBuf() {
        if (p) (void)hipFree(p);
    }
    hipError_t ensure(size_t need) {
        if (need <= bytes) return hipSuccess;
        size_t nb = std::max(need, bytes + bytes / 2);
        nb = (nb + 255) & ~size_t(255);
        if (p) {
            hipError_t e = hipDeviceSynchronize();
            if (e != hipSuccess) return e;
            (void)hipFree(p);
            p = nullptr;
            bytes = 0;
        }
        hipError_t e = hipMalloc(&p, nb);
        if (e == hipSuccess) bytes = nb;
        return e;
    }
    template <class T>
    T* as() const { return static_cast<T*>(p); }
};

struct SegError {
    int code;
    std::string msg;
};
[[noreturn]] void seg_fail(int code, const std::string& m) { throw SegError{code, m}; }
#define SEGCHK(expr)                                                                          \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess)                                                                 \
            seg_fail(GDF_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));         \
    } while (0)

}  // namespace

struct gdf_segmenter {
    int device = 0;
    hipStream_t own = nullptr, user = nullptr;
    hipStream_t side = nullptr;  // the contour scan runs here, concurrently with the labelling
    hipEvent_t ev_ready = nullptr, ev_contours = nullptr;
    hipStream_t s() const { return user ? user : own; }
    uint32_t W = 0, H = 0, L = 0, flags = 0;
    bool have = false;
    GpuBuf par, bits, blabel, nlab, lstart, cstart, labels, st, sums, stats5, cent, l2c, conn;
    GpuBuf codes, rec, ncont, err, scratch, bgpart, tdbg;
    GpuBuf mgl, mflag, mout;      // label merge (k_cc_merge_layers)
    GpuBuf prec, pcodes, phdr;    // packed contours (k_cc_pack_contours)
    uint64_t code_cap = 0;
    uint32_t rec_cap = 0;
    std::vector<uint32_t> h_nlab, h_lstart;
    std::vector<uint64_t> h_cstart;
    uint32_t total = 0;
    uint64_t conn_bytes = 0;
    // contours resolved on the host (after the first query)
    bool contours_read = false;
    std::vector<uint32_t> h_ncont, h_rec;
    std::vector<uint64_t> h_roff, h_coff;  // per-layer offsets into h_rec (records) / h_codes
    std::vector<uint8_t> h_codes;
    uint64_t total_points = 0;
    uint32_t total_contours = 0;
};

namespace {

template <class F>
int seg_guarded(F&& f) {
    try {
        f();
        return GDF_OK;
    } catch (const SegError& e) {
        gdf::set_last_error(e.msg);
        return e.code;
    } catch (const std::bad_alloc&) {
        gdf::set_last_error("host allocation failed");
        return GDF_ERR_NOMEM;
    } catch (...) {
        gdf::set_last_error("unknown error");
        return GDF_ERR_HIP;
    }
}

// findContours of every layer on the segmenter's second stream, ordered after the work already
// on `s` (the grid producer); g->ev_contours marks its end
void launch_contours(gdf_segmenter* g, const uint8_t* grid, uint32_t W, uint32_t H, uint32_t L,
                     hipStream_t s) {
    const hipStream_t s2 = g->side;
    SEGCHK(hipEventRecord(g->ev_ready, s));
    SEGCHK(hipStreamWaitEvent(s2, g->ev_ready, 0));
    const uint64_t img = contour_image_bytes(W, H);  // pixels (pitch roundup4(W + 2)) + row flags
    g->rec_cap = (uint32_t)(((uint64_t)(W + 1) / 2) * H + 1);
    g->code_cap = 8ull * W * H + 64;
    SEGCHK(g->codes.ensure(g->code_cap * L));
    SEGCHK(g->rec.ensure((size_t)g->rec_cap * 16 * L));
    SEGCHK(g->ncont.ensure((size_t)L * 4));
    SEGCHK(g->err.ensure(4));
    SEGCHK(hipMemsetAsync(g->err.p, 0, 4, s2));
    unsigned long long* tdbg = nullptr;
    static const bool dbg = std::getenv("GDF_SEG_DEBUG") != nullptr;
    if (dbg) {
        SEGCHK(g->tdbg.ensure((size_t)L * 32));
        tdbg = g->tdbg.as<unsigned long long>();
    }
    bool lds = img <= kLdsMax;
    if (lds) {
        static bool attr_set = false;
        if (!attr_set) {
            lds = hipFuncSetAttribute((const void*)k_cc_contours<true>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)kLdsMax) == hipSuccess;
            attr_set = lds;
        }
    }
    if (lds) {
        hipLaunchKernelGGL(k_cc_contours<true>, dim3(L), dim3(kContourThreads), (size_t)img, s2, grid, W, H,
                           nullptr, g->codes.as<uint8_t>(), g->code_cap, g->rec.as<uint32_t>(),
                           g->rec_cap, g->ncont.as<uint32_t>(), g->err.as<uint32_t>(), tdbg);
    } else {
        SEGCHK(g->scratch.ensure(img * L));
        hipLaunchKernelGGL(k_cc_contours<false>, dim3(L), dim3(kContourThreads), 0, s2, grid, W, H,
                           g->scratch.as<int8_t>(), g->codes.as<uint8_t>(), g->code_cap,
                           g->rec.as<uint32_t>(), g->rec_cap, g->ncont.as<uint32_t>(),
                           g->err.as<uint32_t>(), tdbg);
    }
    if (dbg) {
        std::vector<unsigned long long> h((size_t)L * 4);
        SEGCHK(hipMemcpyAsync(h.data(), tdbg, h.size() * 8, hipMemcpyDeviceToHost, s2));
        SEGCHK(hipStreamSynchronize(s2));
        for (uint32_t z = 0; z < L; ++z)
            std::fprintf(stderr, "seg contours layer %u: stage %.1f us, scan+trace %.1f us, %llu codes, %llu contours\n",
                         z, h[4 * z] / 100.0, h[4 * z + 1] / 100.0, h[4 * z + 2], h[4 * z + 3]);
    }
    SEGCHK(hipGetLastError());
    SEGCHK(hipEventRecord(g->ev_contours, s2));
}

void run_label_layers(gdf_segmenter* g, const uint8_t* grid, uint32_t W, uint32_t H, uint32_t L,
                      uint32_t flags, hipStream_t s) {
    g->have = false;  // (a failed call leaves no result behind)
    g->contours_read = false;
    if (!grid || W == 0 || H == 0 || L == 0) seg_fail(GDF_ERR_ARG, "empty grid");
    if (W > 65534 || H > 65534) seg_fail(GDF_ERR_ARG, "layers wider or taller than 65534 cells");
    const uint32_t BW = (W + 1) / 2, BH = (H + 1) / 2;
    const uint64_t nbl = (uint64_t)BW * BH, nb = nbl * L;
    if (nb >= 0xFFFFFFF0ull) seg_fail(GDF_ERR_ARG, "grid too large for 32-bit block indices");
    SEGCHK(g->par.ensure(nb * 4));
    SEGCHK(g->bits.ensure(nb));
    SEGCHK(g->blabel.ensure(nb * 4));
    SEGCHK(g->nlab.ensure((size_t)L * 4));
    if (flags & GDF_SEG_CONTOURS) launch_contours(g, grid, W, H, L, s);
    const dim3 tiles((BW + kTile - 1) / kTile, (BH + kTile - 1) / kTile, L);
    hipLaunchKernelGGL(k_cc_local, tiles, dim3(256), 0, s, grid, W, H, BW, BH,
                       g->par.as<uint32_t>(), g->bits.as<uint8_t>());
    hipLaunchKernelGGL(k_cc_merge, tiles, dim3(256), 0, s, g->bits.as<const uint8_t>(), BW, BH,
                       g->par.as<uint32_t>());
    hipLaunchKernelGGL(k_cc_flatten, dim3((uint32_t)((nb + 255) / 256)), dim3(256), 0, s,
                       g->par.as<uint32_t>(), (uint32_t)nb);
    hipLaunchKernelGGL(k_cc_rank, dim3(L), dim3(1024), 0, s, g->par.as<const uint32_t>(),
                       (uint32_t)nbl, g->blabel.as<uint32_t>(), g->nlab.as<uint32_t>());
    SEGCHK(hipGetLastError());
    g->h_nlab.assign(L, 0);
    SEGCHK(hipMemcpyAsync(g->h_nlab.data(), g->nlab.p, (size_t)L * 4, hipMemcpyDeviceToHost, s));
    SEGCHK(hipStreamSynchronize(s));
    g->h_lstart.assign(L, 0);
    g->h_cstart.assign(L, 0);
    uint64_t T = 0, cb = 0;
    for (uint32_t i = 0; i < L; ++i) {
        if (g->h_nlab[i] > 65536u)
            seg_fail(GDF_ERR_CAPACITY, "more than 65535 components in a layer (CV_16U labels)");
        g->h_lstart[i] = (uint32_t)T;
        T += g->h_nlab[i];
    }
    const bool do_conn = (flags & GDF_SEG_CONNECTIONS) != 0;
    if (do_conn)
        for (uint32_t i = 0; i + 1 < L; ++i) {
            g->h_cstart[i] = cb;
            cb += (uint64_t)g->h_nlab[i] * g->h_nlab[i + 1];
        }
    if (cb > (1ull << 32)) seg_fail(GDF_ERR_CAPACITY, "layer connection matrices exceed 4 GiB");
    g->total = (uint32_t)T;
    g->conn_bytes = cb;
    SEGCHK(g->lstart.ensure((size_t)L * 4));
    SEGCHK(g->cstart.ensure((size_t)L * 8));
    SEGCHK(g->labels.ensure((size_t)W * H * L * 2));
    SEGCHK(g->st.ensure(T * kStatWords * 4));
    SEGCHK(g->sums.ensure(T * 16));
    SEGCHK(g->stats5.ensure(T * 20));
    SEGCHK(g->cent.ensure(T * 16));
    SEGCHK(g->l2c.ensure(T * 4));
    SEGCHK(g->conn.ensure(std::max<uint64_t>(cb, 1)));
    SEGCHK(hipMemcpyAsync(g->lstart.p, g->h_lstart.data(), (size_t)L * 4, hipMemcpyHostToDevice, s));
    SEGCHK(hipMemcpyAsync(g->cstart.p, g->h_cstart.data(), (size_t)L * 8, hipMemcpyHostToDevice, s));
    if (cb) SEGCHK(hipMemsetAsync(g->conn.p, 0, cb, s));  // prepareLayersConnections' clear
    const uint32_t tb = (uint32_t)((T + 255) / 256);
    hipLaunchKernelGGL(k_cc_init_stats, dim3(tb), dim3(256), 0, s, g->st.as<int32_t>(),
                       g->sums.as<unsigned long long>(), (uint32_t)T);
    SegArgs a{grid, W, H, L, BW, (uint32_t)nbl, g->par.as<const uint32_t>(),
              g->blabel.as<const uint32_t>(), g->lstart.as<const uint32_t>(),
              g->nlab.as<const uint32_t>(), g->cstart.as<const uint64_t>(),
              g->labels.as<uint16_t>(), g->st.as<int32_t>(), g->sums.as<unsigned long long>(),
              g->conn.as<uint8_t>(), do_conn ? 1 : 0, nullptr};
    const dim3 pgrid((W + 63) / 64, (H + kRowsPerWave - 1) / kRowsPerWave, L);
    const uint32_t wpl = pgrid.x * pgrid.y;
    SEGCHK(g->bgpart.ensure((size_t)wpl * L * kBgWords * 8));
    a.bgpart = g->bgpart.as<unsigned long long>();
    hipLaunchKernelGGL(k_cc_pixels, pgrid, dim3(64), 0, s, a);
    hipLaunchKernelGGL(k_cc_bg_reduce, dim3(L), dim3(256), 0, s,
                       g->bgpart.as<const unsigned long long>(), wpl,
                       g->lstart.as<const uint32_t>(), g->st.as<int32_t>(),
                       g->sums.as<unsigned long long>());
    hipLaunchKernelGGL(k_cc_finish, dim3(tb), dim3(256), 0, s, g->st.as<const int32_t>(),
                       g->sums.as<const unsigned long long>(), (uint32_t)T,
                       g->stats5.as<int32_t>(), g->cent.as<double>(), g->l2c.as<int32_t>());
    SEGCHK(hipGetLastError());
    if (flags & GDF_SEG_CONTOURS) {
        // the contour scan (one workgroup per layer, the longest kernel) ran concurrently on the
        // second stream since the start of this call
        SEGCHK(hipStreamWaitEvent(s, g->ev_contours, 0));
        hipLaunchKernelGGL(k_cc_l2c, dim3(L), dim3(256), 0, s, g->rec.as<const uint32_t>(),
                           g->rec_cap, g->ncont.as<const uint32_t>(),
                           g->labels.as<const uint16_t>(), W, H, g->lstart.as<const uint32_t>(),
                           g->l2c.as<int32_t>());
        SEGCHK(hipGetLastError());
    }
    g->W = W;
    g->H = H;
    g->L = L;
    g->flags = flags;
    g->have = true;
}

void need_result(gdf_segmenter* g) {
    if (!g->have) seg_fail(GDF_ERR_STATE, "no segmentation result (call gdf_seg_label_layers)");
}

// contour records and chain codes to the host (once per result)
void read_contours(gdf_segmenter* g) {
    need_result(g);
    if (!(g->flags & GDF_SEG_CONTOURS)) seg_fail(GDF_ERR_STATE, "contours were not requested");
    if (g->contours_read) return;
    const hipStream_t s = g->s();
    // compact host copies (k_cc_pack_contours): layer z's records at h_roff[z], its chain codes
    // at h_coff[z] - one download of each
    const uint32_t L = g->L;
    SEGCHK(g->prec.ensure(g->rec.bytes));
    SEGCHK(g->pcodes.ensure(g->codes.bytes));
    SEGCHK(g->phdr.ensure((size_t)(2 * L + 2) * 8));
    hipLaunchKernelGGL(k_cc_pack_contours, dim3(L), dim3(256), 0, s, g->rec.as<const uint32_t>(),
                       g->rec_cap, g->codes.as<const uint8_t>(), g->code_cap,
                       g->ncont.as<const uint32_t>(), L, g->prec.as<uint32_t>(),
                       g->pcodes.as<uint8_t>(), g->phdr.as<unsigned long long>());
    SEGCHK(hipGetLastError());
    std::vector<unsigned long long> hdr(2 * (size_t)L + 2);
    uint32_t err = 0;
    g->h_ncont.assign(L, 0);
    SEGCHK(hipMemcpyAsync(&err, g->err.p, 4, hipMemcpyDeviceToHost, s));
    SEGCHK(hipMemcpyAsync(g->h_ncont.data(), g->ncont.p, (size_t)L * 4, hipMemcpyDeviceToHost, s));
    SEGCHK(hipMemcpyAsync(hdr.data(), g->phdr.p, hdr.size() * 8, hipMemcpyDeviceToHost, s));
    SEGCHK(hipStreamSynchronize(s));
    if (err) seg_fail(GDF_ERR_CAPACITY, "contour capacity exceeded");
    g->h_roff.assign(hdr.begin(), hdr.begin() + L + 1);
    g->h_coff.assign(hdr.begin() + L + 1, hdr.end());
    g->h_rec.resize(g->h_roff[L] * 4);
    g->h_codes.resize(g->h_coff[L]);
    if (!g->h_rec.empty())
        SEGCHK(hipMemcpyAsync(g->h_rec.data(), g->prec.p, g->h_rec.size() * 4, hipMemcpyDeviceToHost, s));
    if (!g->h_codes.empty())
        SEGCHK(hipMemcpyAsync(g->h_codes.data(), g->pcodes.p, g->h_codes.size(), hipMemcpyDeviceToHost, s));
    SEGCHK(hipStreamSynchronize(s));
    g->total_contours = (uint32_t)g->h_roff[L];
    g->total_points = 0;
    for (size_t d = 0; d < g->h_roff[L]; ++d) g->total_points += g->h_rec[4 * d + 3];
    g->contours_read = true;
}

}  // namespace

extern "C" {

int gdf_seg_create(int device, gdf_segmenter** out) {
    if (!out) return GDF_ERR_ARG;
    return seg_guarded([&] {
        SEGCHK(hipSetDevice(device));
        auto* g = new gdf_segmenter();
        g->device = device;
        hipError_t e = hipStreamCreateWithFlags(&g->own, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&g->side, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&g->ev_ready, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&g->ev_contours, hipEventDisableTiming);
        if (e != hipSuccess) {
            delete g;
            SEGCHK(e);
        }
        *out = g;
    });
}

int gdf_seg_destroy(gdf_segmenter* g) {
    if (!g) return GDF_OK;
    (void)hipSetDevice(g->device);
    (void)hipStreamSynchronize(g->s());
    if (g->side) (void)hipStreamSynchronize(g->side);
    if (g->own) (void)hipStreamDestroy(g->own);
    if (g->side) (void)hipStreamDestroy(g->side);
    if (g->ev_ready) (void)hipEventDestroy(g->ev_ready);
    if (g->ev_contours) (void)hipEventDestroy(g->ev_contours);
    delete g;
    return GDF_OK;
}

int gdf_seg_set_stream(gdf_segmenter* g, void* stream) {
    if (!g) return GDF_ERR_ARG;
    g->user = static_cast<hipStream_t>(stream);
    return GDF_OK;
}

int gdf_seg_label_layers(gdf_segmenter* g, const uint8_t* grid, uint32_t W, uint32_t H,
                         uint32_t L, uint32_t flags) {
    if (!g) return GDF_ERR_ARG;
    return seg_guarded([&] {
        SEGCHK(hipSetDevice(g->device));
        run_label_layers(g, grid, W, H, L, flags, g->s());
    });
}

int gdf_seg_label_engine_grid(gdf_segmenter* g, gdf_engine* e, uint32_t flags) {
    if (!g || !e) return GDF_ERR_ARG;
    const uint8_t* occ = nullptr;
    uint32_t gs[3] = {0, 0, 0};
    uint64_t nc = 0;
    void* st = nullptr;
    int rc = gdf_get_device_results(e, nullptr, nullptr, nullptr, &occ);
    if (rc == GDF_OK) rc = gdf_get_grid_size(e, gs, &nc);
    if (rc == GDF_OK) rc = gdf_get_stream(e, &st);
    if (rc != GDF_OK) return rc;
    if (!occ) {
        gdf::set_last_error("the engine has no occupancy grid yet");
        return GDF_ERR_STATE;
    }
    return seg_guarded([&] {
        SEGCHK(hipSetDevice(g->device));
        run_label_layers(g, occ, gs[0], gs[1], gs[2], flags, static_cast<hipStream_t>(st));
        // later downloads on the segmenter's stream must follow the engine stream's work
        if (static_cast<hipStream_t>(st) != g->s()) SEGCHK(hipStreamSynchronize(static_cast<hipStream_t>(st)));
    });
}

int gdf_seg_get_counts(gdf_segmenter* g, gdf_seg_counts* out) {
    if (!g || !out) return GDF_ERR_ARG;
    return seg_guarded([&] {
        need_result(g);
        if (g->flags & GDF_SEG_CONTOURS) read_contours(g);
        out->width = g->W;
        out->height = g->H;
        out->layers = g->L;
        out->total_labels = g->total;
        out->total_contours = g->total_contours;
        out->total_contour_points = g->total_points;
        out->connection_bytes = g->conn_bytes;
    });
}

int gdf_seg_download_labels(gdf_segmenter* g, uint16_t* out, uint64_t cap) {
    if (!g || !out) return GDF_ERR_ARG;
    return seg_guarded([&] {
        need_result(g);
        const uint64_t n = (uint64_t)g->W * g->H * g->L;
        if (cap < n) seg_fail(GDF_ERR_CAPACITY, "labels capacity too small");
        SEGCHK(hipMemcpyAsync(out, g->labels.p, n * 2, hipMemcpyDeviceToHost, g->s()));
        SEGCHK(hipStreamSynchronize(g->s()));
    });
}

int gdf_seg_download_num_labels(gdf_segmenter* g, uint32_t* out, uint32_t cap) {
    if (!g || !out) return GDF_ERR_ARG;
    return seg_guarded([&] {
        need_result(g);
        if (cap < g->L) seg_fail(GDF_ERR_CAPACITY, "num_labels capacity too small");
        std::memcpy(out, g->h_nlab.data(), (size_t)g->L * 4);
    });
}

int gdf_seg_download_stats(gdf_segmenter* g, int32_t* stats5, double* cent, uint32_t cap) {
    if (!g) return GDF_ERR_ARG;
    return seg_guarded([&] {
        need_result(g);
        if (cap < g->total) seg_fail(GDF_ERR_CAPACITY, "stats capacity too small");
        if (stats5)
            SEGCHK(hipMemcpyAsync(stats5, g->stats5.p, (size_t)g->total * 20, hipMemcpyDeviceToHost, g->s()));
        if (cent)
            SEGCHK(hipMemcpyAsync(cent, g->cent.p, (size_t)g->total * 16, hipMemcpyDeviceToHost, g->s()));
        SEGCHK(hipStreamSynchronize(g->s()));
    });
}

int gdf_seg_download_connections(gdf_segmenter* g, uint8_t* out, uint64_t cap, uint64_t* starts,
                                 uint32_t starts_cap) {
    if (!g) return GDF_ERR_ARG;
    return seg_guarded([&] {
        need_result(g);
        if (!(g->flags & GDF_SEG_CONNECTIONS)) seg_fail(GDF_ERR_STATE, "connections were not requested");
        if (out) {
            if (cap < g->conn_bytes) seg_fail(GDF_ERR_CAPACITY, "connections capacity too small");
            if (g->conn_bytes)
                SEGCHK(hipMemcpyAsync(out, g->conn.p, g->conn_bytes, hipMemcpyDeviceToHost, g->s()));
            SEGCHK(hipStreamSynchronize(g->s()));
        }
        if (starts) {
            const uint32_t n = g->L ? g->L - 1 : 0;
            if (starts_cap < n) seg_fail(GDF_ERR_CAPACITY, "starts capacity too small");
            std::memcpy(starts, g->h_cstart.data(), (size_t)n * 8);
        }
    });
}

int gdf_seg_download_contours(gdf_segmenter* g, int32_t* l2c, uint32_t* per_layer,
                              uint32_t* sizes, int32_t* pts, uint64_t pts_cap) {
    if (!g) return GDF_ERR_ARG;
    return seg_guarded([&] {
        read_contours(g);
        if (l2c) {
            SEGCHK(hipMemcpyAsync(l2c, g->l2c.p, (size_t)g->total * 4, hipMemcpyDeviceToHost, g->s()));
            SEGCHK(hipStreamSynchronize(g->s()));
        }
        if (per_layer) std::memcpy(per_layer, g->h_ncont.data(), (size_t)g->L * 4);
        if (pts && pts_cap < g->total_points) seg_fail(GDF_ERR_CAPACITY, "points capacity too small");
        uint64_t q = 0;
        uint32_t c = 0;
        for (uint32_t z = 0; z < g->L; ++z) {
            const uint32_t n = g->h_ncont[z];
            const uint32_t* r = g->h_rec.data() + g->h_roff[z] * 4;
            const uint8_t* cz = g->h_codes.data() + g->h_coff[z];
            for (uint32_t j = 0; j < n; ++j) {  // findContours order = reverse discovery
                const uint32_t d = n - 1 - j;
                const uint32_t np = r[4 * d + 3];
                if (sizes) sizes[c] = np;
                ++c;
                if (!pts) continue;
                int32_t x = (int32_t)r[4 * d], y = (int32_t)r[4 * d + 1];
                const uint8_t* cc = cz + r[4 * d + 2];
                static const int dx[8] = {1, 1, 0, -1, -1, -1, 0, 1};
                static const int dy[8] = {0, -1, -1, -1, 0, 1, 1, 1};
                for (uint32_t k = 0; k < np; ++k) {
                    pts[2 * q] = x;
                    pts[2 * q + 1] = y;
                    ++q;
                    if (k + 1 < np) {
                        x += dx[cc[k] & 7];
                        y += dy[cc[k] & 7];
                    }
                }
            }
        }
    });
}

}  // extern "C"

namespace {

// mergeLabelsAcrossLayers (fusion.cpp:2243-2361) by k_cc_merge_layers on the segmenter's stream:
// the connection matrices stay on the device, only the merged ids (4 B per label) come back.
uint32_t merge_labels(gdf_segmenter* g, uint32_t* merged) {
    const hipStream_t s = g->s();
    const uint32_t T = g->total;
    SEGCHK(g->mgl.ensure((size_t)std::max(T, 1u) * 4));
    SEGCHK(g->mflag.ensure((size_t)std::max(T, 1u) * 4));
    SEGCHK(g->mout.ensure((size_t)std::max(T, 1u) * 4 + 4));
    uint32_t* out = g->mout.as<uint32_t>();
    hipLaunchKernelGGL(k_cc_merge_layers, dim3(1), dim3(kMergeThreads), 0, s,
                       g->conn.as<const uint8_t>(), g->cstart.as<const uint64_t>(),
                       g->nlab.as<const uint32_t>(), g->lstart.as<const uint32_t>(), g->L, T,
                       g->mgl.as<uint32_t>(), g->mflag.as<uint32_t>(), out, out + T);
    SEGCHK(hipGetLastError());
    uint32_t n = 0;
    if (T) SEGCHK(hipMemcpyAsync(merged, out, (size_t)T * 4, hipMemcpyDeviceToHost, s));
    SEGCHK(hipMemcpyAsync(&n, out + T, 4, hipMemcpyDeviceToHost, s));
    SEGCHK(hipStreamSynchronize(s));
    return n;
}

}  // namespace

extern "C" {

int gdf_seg_merge_labels(gdf_segmenter* g, uint32_t* merged, uint32_t cap, uint32_t* nobj) {
    if (!g) return GDF_ERR_ARG;
    return seg_guarded([&] {
        need_result(g);
        if (!(g->flags & GDF_SEG_CONNECTIONS)) seg_fail(GDF_ERR_STATE, "connections were not requested");
        if (merged && cap < g->total) seg_fail(GDF_ERR_CAPACITY, "merged capacity too small");
        std::vector<uint32_t> m(g->total);
        const uint32_t n = merge_labels(g, m.data());
        if (merged) std::copy(m.begin(), m.end(), merged);
        if (nobj) *nobj = n;
    });
}

int gdf_seg_create_objects(gdf_segmenter* g, const float lower[3], const float cs[3],
                           gdf_cc_object* objs, uint32_t cap, uint32_t* comps, uint32_t comps_cap,
                           uint32_t* nobj) {
    if (!g || !lower || !cs) return GDF_ERR_ARG;
    return seg_guarded([&] {
        need_result(g);
        if (!(g->flags & GDF_SEG_CONNECTIONS)) seg_fail(GDF_ERR_STATE, "connections were not requested");
        const uint32_t T = g->total;
        std::vector<uint32_t> merged(T);
        const uint32_t n = merge_labels(g, merged.data());
        if (nobj) *nobj = n;
        if (!objs && !comps) return;
        if (objs && cap < n) seg_fail(GDF_ERR_CAPACITY, "objects capacity too small");
        if (comps && comps_cap < T) seg_fail(GDF_ERR_CAPACITY, "components capacity too small");
        std::vector<int32_t> st((size_t)T * 5);
        std::vector<double> ce((size_t)T * 2);
        SEGCHK(hipMemcpyAsync(st.data(), g->stats5.p, (size_t)T * 20, hipMemcpyDeviceToHost, g->s()));
        SEGCHK(hipMemcpyAsync(ce.data(), g->cent.p, (size_t)T * 16, hipMemcpyDeviceToHost, g->s()));
        std::vector<int32_t> l2c(T, -1);
        if (g->flags & GDF_SEG_CONTOURS) {
            read_contours(g);
            SEGCHK(hipMemcpyAsync(l2c.data(), g->l2c.p, (size_t)T * 4, hipMemcpyDeviceToHost, g->s()));
        }
        SEGCHK(hipStreamSynchronize(g->s()));
        // contour sizes in findContours order, per layer
        std::vector<std::vector<uint32_t>> csize(g->L);
        if (g->flags & GDF_SEG_CONTOURS)
            for (uint32_t z = 0; z < g->L; ++z) {
                const uint32_t nc = g->h_ncont[z];
                const uint32_t* r = g->h_rec.data() + g->h_roff[z] * 4;
                for (uint32_t j = 0; j < nc; ++j) csize[z].push_back(r[4 * (nc - 1 - j) + 3]);
            }
        std::vector<uint32_t> layer(T), local(T);
        for (uint32_t z = 0, t = 0; z < g->L; ++z)
            for (uint32_t k = 0; k < g->h_nlab[z]; ++k, ++t) {
                layer[t] = z;
                local[t] = k;
            }
        // UIntGrouper over the merged ids: stable counting sort
        std::vector<uint32_t> start(n + 1, 0), order(T);
        for (uint32_t k = 0; k < T; ++k) ++start[merged[k] + 1];
        for (uint32_t i = 0; i < n; ++i) start[i + 1] += start[i];
        {
            std::vector<uint32_t> ptr(start.begin(), start.end() - 1);
            for (uint32_t k = 0; k < T; ++k) order[ptr[merged[k]]++] = k;
        }
        if (comps) std::copy(order.begin(), order.end(), comps);
        if (!objs) return;
        auto world = [&](float x, float y, float z, float* o) {  // voxelCoordToWorldCoord
            o[0] = x * cs[0] + lower[0];
            o[1] = y * cs[1] + lower[1];
            o[2] = z * cs[2] + lower[2];
        };
        for (uint32_t i = 0; i < n; ++i) {
            gdf_cc_object& ob = objs[i];
            std::memset(&ob, 0, sizeof(ob));
            const uint32_t nc = start[i + 1] - start[i];
            ob.num_components = nc;
            ob.first_component = start[i];
            ob.label = merged[order[start[i]]];
            float cx = 0.0f, cy = 0.0f;  // cv::Point2f += double / uint
            for (uint32_t k = 0; k < nc; ++k) {
                const uint32_t idx = order[start[i] + k], z = layer[idx];
                const int32_t* sr = st.data() + 5 * (size_t)idx;
                const double x = ce[2 * (size_t)idx], y = ce[2 * (size_t)idx + 1];
                const int32_t right = sr[0] + sr[2], bottom = sr[1] + sr[3];
                cx = (float)((double)cx + x / nc);
                cy = (float)((double)cy + y / nc);
                if (k == 0 || sr[0] < ob.min_voxel[0]) ob.min_voxel[0] = sr[0];
                if (k == 0 || sr[1] < ob.min_voxel[1]) ob.min_voxel[1] = sr[1];
                if (k == 0 || z < (uint32_t)ob.min_voxel[2]) ob.min_voxel[2] = (int32_t)z;
                if (k == 0 || right > ob.max_voxel[0]) ob.max_voxel[0] = right;
                if (k == 0 || bottom > ob.max_voxel[1]) ob.max_voxel[1] = bottom;
                if (k == 0 || z > (uint32_t)ob.max_voxel[2]) ob.max_voxel[2] = (int32_t)z;
                const int32_t c = l2c[idx];
                if (c >= 0) ob.num_contour_points += csize[z][(size_t)c];
            }
            ob.centroid[0] = cx;
            ob.centroid[1] = cy;
            for (int d = 0; d < 3; ++d) {
                ob.center_voxel[d] = (float)(ob.max_voxel[d] + ob.min_voxel[d]) * 0.5f;
                ob.aabb_voxel[d] = ob.max_voxel[d] - ob.min_voxel[d];
            }
            world(ob.center_voxel[0], ob.center_voxel[1], ob.center_voxel[2], ob.center_world);
            world((float)ob.min_voxel[0], (float)ob.min_voxel[1], (float)ob.min_voxel[2], ob.min_world);
            world((float)ob.max_voxel[0], (float)ob.max_voxel[1], (float)ob.max_voxel[2], ob.max_world);
            for (int d = 0; d < 3; ++d) ob.aabb_world[d] = ob.max_world[d] - ob.min_world[d];
            ob.num_layers = (uint32_t)(1 + ob.aabb_voxel[2]);
        }
    });
}

int gdf_seg_get_device_results(gdf_segmenter* g, const uint16_t** labels, const int32_t** stats5,
                               const double** cent, const uint8_t** conn) {
    if (!g) return GDF_ERR_ARG;
    if (!g->have) {
        gdf::set_last_error("no segmentation result");
        return GDF_ERR_STATE;
    }
    if (labels) *labels = g->labels.as<const uint16_t>();
    if (stats5) *stats5 = g->stats5.as<const int32_t>();
    if (cent) *cent = g->cent.as<const double>();
    if (conn) *conn = g->conn.as<const uint8_t>();
    return GDF_OK;
}

}  // extern "C"
