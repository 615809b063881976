// gdf_voxsum.hpp - the voxel sum of the GPU voxelize (device code, included by gdf_kernels.hip
// and tools/voxsum_probe.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef GDF_VOXSUM_PROBE
#define GDF_VOXSUM_PROBE(what)  // instrumentation hook (tools/voxsum_probe.hip)
#endif

namespace gdf {

// ---- the voxel sum: the sequential f32 chain, evaluated 64 terms at a time ----------------------
// The reference sums a voxel's points one after the other (inc/voxelize.h:29-35:
// s_k = fl(s_{k-1} + x_k), round-to-nearest-even), a dependent chain that cannot be reassociated in
// general.  It can, however, be evaluated EXACTLY in parallel over stretches where every rounding
// lands on one fixed grid:
//   let u be a power of two with s = m u (m integer) and y_k = x_k / u (exact scaling).  If the
//   exact value v_k = s_{k-1} + x_k lies strictly inside a binade whose ulp is u, then
//   fl(v_k) = s_{k-1} + u rint(y_k) unless y_k is a tie (fraction exactly 1/2, whose rounding
//   depends on the parity of s_{k-1}/u); if y_k is an integer and |m + sum| <= 2^24 the sum is
//   exactly representable, so fl(v_k) = v_k whatever its binade.
// With u = ulp(s) (binade exponent E = ex - 127, u = 2^(ex - 150)) a row of 64 terms becomes
// integer arithmetic: t_k = rint(y_k) (int32), an inclusive wave scan P_k = m + t_1 + ... + t_k,
// and a per-lane validity test - a rounding step needs 2^23 < |P_k| < 2^24 (then |v_k| is inside
// (2^23 u, 2^24 u) since |v_k - P_k u| < u/2; the multi-row attempts treat every step this way),
// an exact step |P_k| <= 2^24, ties and |y_k| > 2^24 (inf, NaN) fail.  The first failing lane L
// ends the stretch: the prefix [b, L) is committed as s = P_{L-1} u (exact), term L is added by
// one ordinary f32 add (the reference's own operation: a binade crossing, a tie, a NaN ...), and a
// new stretch starts at L + 1 with the new ulp.  A zero, subnormal-range or non-finite s takes
// single f32 adds until it leaves that range.  The result is bit-identical to the sequential chain
// for every input (tests/spec_sum_model.py restates it; GPU tests: tests/test_gpu_round3.py); a
// voxel sum grows monotonically for most voxels, so a stretch fails about once per doubling of
// the sum (~log2(n) extra stretches per voxel).
//
// One component per wave: a block of 4 waves sums a voxel's x, y, z, w side by side (a row fails
// only on its own component's crossings, and the voxel's latency is a quarter of one wave doing
// all four).  Measured on one gfx950 wave (tools/issue_probe.hip): an independent VALU op issues
// every 4 cycles, a DPP add every 6-7, but a v_cmp -> SGPR mask -> v_cndmask step costs ~18-22
// and so does a readlane round trip - so every lane predicate here is VALU integer arithmetic
// kept opaque to the compiler (it would turn `(b - a) >> 31` back into a compare + mask), and an
// attempt over R rows ends in ONE ballot.
__device__ __forceinline__ uint32_t opq(uint32_t x) {  // (hides x's origin from the optimizer)
    asm volatile("" : "+v"(x));
    return x;
}
__device__ __forceinline__ uint32_t u_gt(uint32_t a, uint32_t b) { return opq(b - a) >> 31; }  // a, b < 2^31
__device__ __forceinline__ float bcast_f(float v, uint32_t l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ float uniform_f(float v) {
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}
// wave64 inclusive sum scan on DPP (row shifts, then the row broadcasts of lanes 15 and 31)
__device__ __forceinline__ int dpp_iscan(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return v;
}
// N independent scans step by step (the DPP latency of one scan holds the others' steps)
template <int N>
__device__ __forceinline__ void dpp_iscan_n(int (&v)[N]) {
#pragma unroll
    for (int c = 0; c < N; ++c) v[c] += __builtin_amdgcn_update_dpp(0, v[c], 0x111, 0xf, 0xf, false);
#pragma unroll
    for (int c = 0; c < N; ++c) v[c] += __builtin_amdgcn_update_dpp(0, v[c], 0x112, 0xf, 0xf, false);
#pragma unroll
    for (int c = 0; c < N; ++c) v[c] += __builtin_amdgcn_update_dpp(0, v[c], 0x114, 0xf, 0xf, false);
#pragma unroll
    for (int c = 0; c < N; ++c) v[c] += __builtin_amdgcn_update_dpp(0, v[c], 0x118, 0xf, 0xf, false);
#pragma unroll
    for (int c = 0; c < N; ++c) v[c] += __builtin_amdgcn_update_dpp(0, v[c], 0x142, 0xa, 0xf, false);
#pragma unroll
    for (int c = 0; c < N; ++c) v[c] += __builtin_amdgcn_update_dpp(0, v[c], 0x143, 0xc, 0xf, false);
}
// One attempt of comp_stretch_sum over nv <= 64 R values (FULL: nv = 64 R, no load guards).
// Per value: y = x / u, t = rint(y) clamped to +-2^25 (a larger term leaves the binade anyway), one
// test for a tie or a NaN (|y - t| >= 1/2: equality only for ties, NaN bits above), the scan, and
// the binade test P in [lo_k, hi_k] (the bounds of |O + P| in [2^23 + 1, 2^24 - 1] moved by the
// row's offset O: no valid stretch crosses zero, so the sign of O decides).  Lanes past nv carry
// x = 0.  Returns the ballot of any failure (0: all valid) and the rows' scans.
template <int R, bool FULL, class Get>
__device__ __forceinline__ unsigned long long stretch_attempt(const Get& get, uint32_t pos,
                                                              uint32_t nv, float scale, int O0,
                                                              float (&x)[R], int (&P)[R]) {
    const uint32_t lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const uint32_t i = 64u * k + lane;
        if (FULL) x[k] = get(pos + i);
        else x[k] = i < nv ? get(pos + i) : 0.0f;
    }
    uint32_t any = 0;
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const float y = x[k] * scale;
        const float r = __builtin_amdgcn_fmed3f(__builtin_rintf(y), -33554432.0f, 33554432.0f);
        any |= u_gt(__float_as_uint(y - r) & 0x7FFFFFFFu, 0x3EFFFFFFu);
        P[k] = (int)r;
    }
    dpp_iscan_n<R>(P);
    // |O + P| in [A, B] <=> P in [A - O, B - O] (O > 0) or [-B - O, -A - O] (O < 0)
    constexpr int A = 8388609, B = 16777215;
    int O = O0;
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const int lo = O > 0 ? A - O : -B - O, hi = O > 0 ? B - O : -A - O;
        any |= opq((uint32_t)((P[k] - lo) | (hi - P[k]))) >> 31;
        O += __builtin_amdgcn_readlane(P[k], 63);
    }
    return __ballot(any != 0u);
}
// 64 values [pos, pos + 64) by the chain itself: one row loaded, then 64 dependent f32 adds of
// its lanes (the same uniform s in every lane); lanes past end add -0.0, which leaves any s as it is
template <class Get>
__device__ __forceinline__ float serial_row(const Get& get, uint32_t pos, uint32_t end, float s) {
    const uint32_t i = pos + (threadIdx.x & 63);
    const float x = i < end ? get(i) : -0.0f;
#pragma unroll
    for (int k = 0; k < 64; ++k) s = s + bcast_f(x, k);
    return s;
}
// s + x_pos + ... + x_{end-1} of one component (x_i = get(i), LDS or global memory; the values
// of [pos, end) must be readable), by stretch attempts of up to R rows (64 R values) from a cursor:
// R independent scans (row k's offset is the sum of the totals of rows < k, from lane 63), VALU
// predicates, ONE ballot per attempt.  All valid: the cursor moves on by 64 R.  A failing value j
// (first in order): the prefix before it is committed exactly, x_j is added by one f32 add (the
// reference's own operation: a binade crossing, a tie, a zero sum, ...) and the next attempt starts
// at j + 1.  A non-finite sum ends the work early (NaN stays NaN; inf changes only by a NaN or an
// opposite inf term).
// Sums that keep changing binade - a component whose running sum walks around zero (a floor at
// z ~ 0: |x| >> |s|, 1 value in ~3 fails; 4K frames hold voxels of 4 K such points) - would pay a
// whole attempt (~1.5 K cycles at R = 4) per few values: an attempt failing within its first
// 32 R values is followed by 1, 2, 4, ... 32 rows of the plain chain (serial_row, ~6 cycles per
// value; the backoff resets after any attempt that gets further), and a zero / tiny sum takes one
// chain row too.
template <int R, class Get>
__device__ __forceinline__ float comp_stretch_sum(const Get& get, uint32_t pos, uint32_t end,
                                                  float s) {
    const uint32_t lane = threadIdx.x & 63;
    uint32_t streak = 0, ser = 0;  // (wave-uniform) short attempts in a row, chain rows owed
#pragma unroll 1
    while (pos < end) {  // wave-uniform
        if (ser) {
            GDF_VOXSUM_PROBE(3);
            s = uniform_f(serial_row(get, pos, end, s));
            pos += 64u;
            --ser;
            continue;
        }
        const uint32_t nv = min(64u * R, end - pos);
        const uint32_t ex = ((uint32_t)__builtin_amdgcn_readfirstlane(__float_as_int(s)) >> 23) & 255u;
        if (ex < 24u || ex == 255u) {  // zero / tiny sum: a chain row; inf / NaN: below
            if (ex == 255u) {
                GDF_VOXSUM_PROBE(2);
                if (s != s) return s;
                // inf: only a NaN or an opposite inf term changes it (into NaN)
#pragma unroll 1
                for (; pos < end; pos += 64u) {
                    const uint32_t i = pos + lane;
                    const float t = i < end ? get(i) : 0.0f;
                    const unsigned long long b = __ballot(t != t || (__builtin_isinf(t) && t != s));
                    if (b) return uniform_f(s + bcast_f(t, (uint32_t)__builtin_ctzll(b)));
                }
                return s;
            }
            ser = 1;
            continue;
        }
        const float scale = __uint_as_float((277u - ex) << 23);  // 2^(150 - ex) = 1 / u
        const float u = __uint_as_float((ex - 23u) << 23);
        const int O0 = __builtin_amdgcn_readfirstlane((int)(s * scale));
        float x[R];
        int P[R];
        const unsigned long long bad =
            nv == 64u * R ? stretch_attempt<R, true>(get, pos, nv, scale, O0, x, P)
                          : stretch_attempt<R, false>(get, pos, nv, scale, O0, x, P);
        if (!bad) {  // the whole attempt
            GDF_VOXSUM_PROBE(0);
            int O = O0;
#pragma unroll
            for (int k = 0; k < R; ++k) O += __builtin_amdgcn_readlane(P[k], 63);
            s = (float)O * u;
            pos += nv;
            streak = 0;
            continue;
        }
        // the first failing value j = 64 k0 + L: commit [pos, pos + j), add x_j (recomputed
        // failure flags per row; rows before k0 are entirely valid)
        GDF_VOXSUM_PROBE(1);
        constexpr int A = 8388609, B = 16777215;
        int o = O0;
        uint32_t j = 0;
        float xj = 0.0f;
        bool found = false;
#pragma unroll
        for (int k = 0; k < R; ++k) {
            if (found) break;
            const float y = x[k] * scale;
            const float r = __builtin_amdgcn_fmed3f(__builtin_rintf(y), -33554432.0f, 33554432.0f);
            const int lo = o > 0 ? A - o : -B - o, hi = o > 0 ? B - o : -A - o;
            const bool f = (__builtin_fabsf(y - r) >= 0.5f) | (y != y) | (P[k] < lo) | (P[k] > hi);
            const unsigned long long b = __ballot(f);
            if (b) {
                const uint32_t L = (uint32_t)__builtin_ctzll(b);
                if (L > 0) o += __builtin_amdgcn_readlane(P[k], L - 1);
                xj = bcast_f(x[k], L);
                j = 64u * k + L;
                found = true;
            } else {
                o += __builtin_amdgcn_readlane(P[k], 63);
            }
        }
        s = uniform_f((float)o * u + xj);
        pos += j + 1;
        if (j < 32u * R) {
            ser = 1u << min(streak, 5u);
            ++streak;
        } else {
            streak = 0;
        }
    }
    return s;
}
// ---- row form: a chunk of up to 16 rows of 64 values, one row per 4 lanes -------------------------
// The stretch rule above, evaluated per ROW instead of per value: every step of a stretch is a
// rounding step inside the binade of u, i.e. every running value O + P_k (O = s / u, P_k = t_1 +
// ... + t_k, t = rint(x / u)) lies in [2^23 + 1, 2^24 - 1] (sign of O), which for a whole row holds
// iff the row's smallest and largest running prefix do.  Rows are independent given u, so:
//  1. every lane takes 16 values of one row (lanes 4r .. 4r + 3: row r), sums them loosely and
//     the wave scans the sums: s + the rows up to row r is a GUESS of s at row r's end, whose
//     binade gives the row's u (a wrong guess only costs the row its integer path);
//  2. per value y = x / u, t = rint(y) clamped to +-2^24 (any |t| >= 2^23 leaves the binade, and
//     the clamp keeps every int32 sum below 2^31), the tie flag |y - t| >= 1/2, the running
//     P with its min and max; the 4 parts of a row combine by quad DPP (offsets by a quad scan);
//  3. from the exact s: the rows' totals are scanned, a row is taken when its guessed binade is
//     s's, it has no tie / NaN and O + min P, O + max P stay in range - the ballot's first other
//     row ends the integer run: s = (O + totals before it) u exactly, that row is added by the
//     plain chain (serial_row), and phase 3 resumes after it.
// ~10 VALU ops per value spread over 64 lanes: a 1 K-value chunk costs ~1.5 K cycles instead of
// ~6 K for 4 cursor attempts, and 1 row in ~30 takes the chain on real voxels (a doubling of the
// sum, a guess at a binade edge); tests/spec_sum_model.py rows_sum restates it.
constexpr uint32_t kRowStride = 68;  // LDS floats per row of 64 (16-value reads conflict-free)

#define GDF_QPERM(v, ctrl) __builtin_amdgcn_update_dpp(0, (v), (ctrl), 0xf, 0xf, false)
__device__ __forceinline__ float dpp_iscan_f(float f) {  // inclusive wave64 sum scan (loose)
    int v = __float_as_int(f);
    v = __float_as_int(__int_as_float(v) + __int_as_float(__builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false)));
    v = __float_as_int(__int_as_float(v) + __int_as_float(__builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false)));
    v = __float_as_int(__int_as_float(v) + __int_as_float(__builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false)));
    v = __float_as_int(__int_as_float(v) + __int_as_float(__builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false)));
    v = __float_as_int(__int_as_float(v) + __int_as_float(__builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false)));
    v = __float_as_int(__int_as_float(v) + __int_as_float(__builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false)));
    return __int_as_float(v);
}

__device__ __forceinline__ float dpp_iscan16_f(float f) {  // inclusive scans of the 16-lane rows
    int v = __float_as_int(f);
    v = __float_as_int(__int_as_float(v) + __int_as_float(__builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false)));
    v = __float_as_int(__int_as_float(v) + __int_as_float(__builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false)));
    v = __float_as_int(__int_as_float(v) + __int_as_float(__builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false)));
    v = __float_as_int(__int_as_float(v) + __int_as_float(__builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false)));
    return __int_as_float(v);
}
__device__ __forceinline__ int dpp_iscan16(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);
    return v;
}

// Steps 1 and 2 for the quad of this lane (part h = lane & 3 of a row: 16 values at src, 16-byte
// aligned; vc of them valid when `partial`, the rest read as -0.0): the row's guessed binade exr,
// its total T and prefix min / max, and whether it is free of ties (rowfree, on the quad's lane 3).
// SEG: the guess scans the 16-lane DPP rows (4 independent sums of 4 rows each) instead of the wave.
struct RowInfo {
    uint32_t exr;
    int T, rmn, rmx;
    bool rowfree;
};
template <bool SEG>
__device__ __forceinline__ RowInfo row_info(const float* __restrict__ src, int vc, bool partial,
                                            float s) {
    constexpr int V = 16;
    const uint32_t h = threadIdx.x & 3;
    float x[V];
    const float4* s4 = reinterpret_cast<const float4*>(src);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const float4 v = s4[i];
        x[4 * i] = v.x;
        x[4 * i + 1] = v.y;
        x[4 * i + 2] = v.z;
        x[4 * i + 3] = v.w;
    }
    if (partial) {  // (wave-uniform)
#pragma unroll
        for (int i = 0; i < V; ++i) x[i] = i < vc ? x[i] : -0.0f;
    }
    // 1. the guess: s + the rows up to this one (loose) - the binade at the row's end, which a NaN
    // or inf term of the row or before it makes non-finite: such rows never take the integer path
    float q[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) q[i] = (x[i] + x[i + 4]) + (x[i + 8] + x[i + 12]);
    const float qs = (q[0] + q[1]) + (q[2] + q[3]);
    const float inc = SEG ? dpp_iscan16_f(qs) : dpp_iscan_f(qs);
    const float guess = s + __int_as_float(GDF_QPERM(__float_as_int(inc), 0xFF));
    RowInfo ri;
    ri.exr = (__float_as_uint(guess) >> 23) & 255u;
    const uint32_t e = min(max(ri.exr, 24u), 254u);
    const float scale = __uint_as_float((277u - e) << 23);
    // 2. integer terms, running prefix with its min / max, tie flag
    int P = 0, mn = 0x7FFFFFFF, mx = -0x7FFFFFFF - 1;
    float dmf = 0.0f;  // max |y - t|: 1/2 only for a tie (>= 1/2 for an overflow to inf; NaN:
                       // the guess above)
#pragma unroll
    for (int i = 0; i < V; ++i) {
        const float y = x[i] * scale;
        const float t = __builtin_amdgcn_fmed3f(__builtin_rintf(y), -16777216.0f, 16777216.0f);
        dmf = __builtin_fmaxf(dmf, __builtin_fabsf(y - t));
        P += (int)t;
        mn = min(mn, P);
        mx = max(mx, P);
    }
    const uint32_t m1 = 0u - (uint32_t)(h >= 1u), m2 = 0u - (uint32_t)(h >= 2u);
    int Pi = P + (int)((uint32_t)GDF_QPERM(P, 0x90) & m1);  // quad_perm [0,0,1,2]
    Pi += (int)((uint32_t)GDF_QPERM(Pi, 0x40) & m2);          // quad_perm [0,0,0,1]
    const int E = Pi - P;                                      // this part's offset in the row
    int rmn = E + mn, rmx = E + mx;
    rmn = min(rmn, GDF_QPERM(rmn, 0xB1));  // [1,0,3,2]
    rmn = min(rmn, GDF_QPERM(rmn, 0x4E));  // [2,3,0,1]
    rmx = max(rmx, GDF_QPERM(rmx, 0xB1));
    rmx = max(rmx, GDF_QPERM(rmx, 0x4E));
    uint32_t dm = __float_as_uint(dmf);  // (>= 0: ordered as unsigned)
    dm = max(dm, (uint32_t)GDF_QPERM((int)dm, 0xB1));
    dm = max(dm, (uint32_t)GDF_QPERM((int)dm, 0x4E));
    ri.T = GDF_QPERM(Pi, 0xFF);  // the row's total (lane 4r + 3's inclusive)
    ri.rmn = rmn;
    ri.rmx = rmx;
    ri.rowfree = h == 3u && dm <= 0x3EFFFFFFu;
    return ri;
}

// s + the first min(m, 64) values of a staged row by the chain itself: every lane reads the whole
// row (LDS broadcast reads, 16-byte aligned) into its registers and runs the same 64 dependent f32
// adds (s stays wave-uniform; no readlane round trip per value); values past m add -0.0, which
// leaves any s as it is.
__device__ __forceinline__ float lds_row_chain(const float* __restrict__ row, uint32_t m, float s) {
    const float4* rp = reinterpret_cast<const float4*>(row);
    float4 v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = rp[k];
    if (m < 64u) {  // (wave-uniform: a group's last, partial row)
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint32_t i = 4u * k;
            v[k].x = i < m ? v[k].x : -0.0f;
            v[k].y = i + 1u < m ? v[k].y : -0.0f;
            v[k].z = i + 2u < m ? v[k].z : -0.0f;
            v[k].w = i + 3u < m ? v[k].w : -0.0f;
        }
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        s = s + v[k].x;
        s = s + v[k].y;
        s = s + v[k].z;
        s = s + v[k].w;
    }
    return s;
}

// s + the n <= 1024 staged values by the chain alone (every lane the same adds, wave-uniform s):
// half rows of 32 values alternate between two register sets, the next one read from LDS while
// the current one is added; values past n add -0.0.
__device__ __forceinline__ float rows_chain_all(const float* __restrict__ comp, uint32_t n, float s) {
    const uint32_t nh = (n + 31u) >> 5;  // half rows
    auto load = [&](uint32_t h, float4 (&v)[8]) {
        const float4* rp = reinterpret_cast<const float4*>(comp + (h >> 1) * kRowStride + (h & 1u) * 32u);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = rp[k];
    };
    auto add = [&](uint32_t h, float4 (&v)[8]) {
        const uint32_t m = n - 32u * h;  // values of this half row (>= 1)
        if (m < 32u) {  // (wave-uniform: the chunk's last, partial half row)
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const uint32_t i = 4u * k;
                v[k].x = i < m ? v[k].x : -0.0f;
                v[k].y = i + 1u < m ? v[k].y : -0.0f;
                v[k].z = i + 2u < m ? v[k].z : -0.0f;
                v[k].w = i + 3u < m ? v[k].w : -0.0f;
            }
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            s = s + v[k].x;
            s = s + v[k].y;
            s = s + v[k].z;
            s = s + v[k].w;
        }
        asm volatile("" : "+v"(s));
    };
    float4 a[8], b[8];
    load(0, a);
    uint32_t h = 0;
#pragma unroll 1
    for (; h + 2 <= nh; h += 2) {
        load(h + 1, b);
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        add(h, a);
        if (h + 2 < nh) load(h + 2, a);
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        add(h + 1, b);
    }
    if (h < nh) add(h, a);
    return s;
}

// The stretch form; nchain counts the rows run by the chain.
__device__ __forceinline__ float rows_chunk_sum_stretch(const float* __restrict__ comp, uint32_t n,
                                                       float s, uint32_t& nchain) {
    constexpr int A = 8388609, B = 16777215;
    const uint32_t lane = threadIdx.x & 63, r = lane >> 2, h = lane & 3;
    const uint32_t nrows = (n + 63u) >> 6;
    // lanes of rows past the chunk's last read row 0 (their values are masked to -0.0 by the
    // negative count): no lane reads outside its component's rows (a k_group_runs_big<8> wave
    // owns 8 rows, not 16)
    const uint32_t rr = r < nrows ? r : 0u;
    const RowInfo ri = row_info<false>(comp + rr * kRowStride + h * 16u,
                                       (int)n - (int)(r * 64u + h * 16u), n < 64u * 16u, s);
    // 3. the rows from the exact s
    uint32_t cur = 0;
#pragma unroll 1
    while (cur < nrows) {  // wave-uniform
        const uint32_t ex = ((uint32_t)__builtin_amdgcn_readfirstlane(__float_as_int(s)) >> 23) & 255u;
        uint32_t f = cur;  // the first row off the integer path
        if (ex >= 24u && ex != 255u) {
            const float sc = __uint_as_float((277u - ex) << 23);
            const float u = __uint_as_float((ex - 23u) << 23);
            const int O0 = __builtin_amdgcn_readfirstlane((int)(s * sc));
            const bool act = h == 3u && r >= cur && r < nrows;
            const int Tm = act ? ri.T : 0;
            const int inc = dpp_iscan(Tm);
            const int Ob = O0 + inc - Tm;  // O at the row's start
            const int lo = O0 > 0 ? A : -B, hi = O0 > 0 ? B : -A;
            const bool ok = ri.rowfree && ri.exr == ex && Ob + ri.rmn >= lo && Ob + ri.rmx <= hi;
            const unsigned long long bad = __ballot(act && !ok);
            f = bad ? (uint32_t)__builtin_ctzll(bad) >> 2 : nrows;
            if (f > cur) s = (float)(O0 + __builtin_amdgcn_readlane(inc, 4u * f - 1u)) * u;
        }
        if (f >= nrows) break;
        GDF_VOXSUM_PROBE(3);
        s = lds_row_chain(comp + f * kRowStride, n - 64u * f, s);
        ++nchain;
        cur = f + 1u;
    }
    return s;
}

// Per component wave, across the chunks of a group: chunks to run by the chain alone (low byte)
// and the backoff level (next byte).  A stretch chunk that ran at least half of its rows (>= 4)
// as chain rows - a sum walking around zero, the C3 window's z - makes the next 2, 4, ... 16
// chunks plain chains (~4 cycles per value instead of a row attempt per row); a stretch chunk
// with fewer chain rows resets the backoff.  Either way the sum is the sequential chain's.
struct ChainMode {
    uint32_t left = 0, level = 0;
};

// s + the n <= 1024 values of one component staged as rows (row q at comp + q kRowStride).
__device__ __forceinline__ float rows_chunk_sum(const float* __restrict__ comp, uint32_t n, float s,
                                               ChainMode& cm) {
    if (cm.left) {  // (wave-uniform)
        --cm.left;
        return rows_chain_all(comp, n, s);
    }
    uint32_t nchain = 0;
    s = rows_chunk_sum_stretch(comp, n, s, nchain);
    const uint32_t nrows = (n + 63u) >> 6;
    if (nrows >= 4u && 2u * nchain >= nrows) {
        cm.left = 2u << min(cm.level, 3u);
        cm.level = min(cm.level + 1u, 3u);
    } else {
        cm.level = 0;
    }
    return s;
}

// ---- the 4 components side by side: a voxel of up to 256 values per chunk in ONE wave ----------
// Lanes 16 c .. 16 c + 15 (DPP row c) sum component c: quad (c, r) row r of 4, the guess scanned
// within the DPP row, step 3 for the 4 components at once (per-lane s, uniform in a DPP row; the
// ballot's 16-bit segment c gives component c's first failing row), their chain rows together
// (components without one add the wave's -0.0 row).  No barrier anywhere: a block's waves sum
// different voxels (k_group_runs).  Chunk layout (kWaveSoa floats per wave): component c's rows
// at c * kWaveCompStride, row r at + r kRowStride, row 4 all -0.0 (written once).
constexpr uint32_t kWaveCompStride = 5 * kRowStride;
constexpr uint32_t kWaveSoa = 4 * kWaveCompStride;

__device__ __forceinline__ void wave_soa_init(float* wsoa) {  // the -0.0 rows
    const uint32_t lane = threadIdx.x & 63;
#pragma unroll
    for (int c = 0; c < 4; ++c) wsoa[c * kWaveCompStride + 4 * kRowStride + lane] = -0.0f;
}

// s (this lane's component) + the chunk's n <= 256 values (rows past n hold -0.0).
__device__ __forceinline__ float rows4c_chunk(const float* __restrict__ wsoa, uint32_t n, float s) {
    constexpr int A = 8388609, B = 16777215;
    const uint32_t lane = threadIdx.x & 63, c = lane >> 4, r = (lane >> 2) & 3, h = lane & 3;
    const float* comp = wsoa + c * kWaveCompStride;
    const uint32_t nrows = (n + 63u) >> 6;
    const RowInfo ri = row_info<true>(comp + r * kRowStride + h * 16u, 0, false, s);
    uint32_t cur = 0;  // (per component)
#pragma unroll 1
    while (true) {
        const bool pending = cur < nrows;
        if (__ballot(pending) == 0) break;  // (wave-uniform)
        const uint32_t ex = (__float_as_uint(s) >> 23) & 255u;
        const bool adm = pending && ex >= 24u && ex != 255u;
        const uint32_t ec = min(max(ex, 24u), 254u);
        const float sc = __uint_as_float((277u - ec) << 23);
        const float u = __uint_as_float((ec - 23u) << 23);
        const int O0 = (int)(s * sc);
        const bool act = adm && h == 3u && r >= cur && r < nrows;
        const int Tm = act ? ri.T : 0;
        const int inc = dpp_iscan16(Tm);
        const int Ob = O0 + inc - Tm;
        const int lo = O0 > 0 ? A : -B, hi = O0 > 0 ? B : -A;
        const bool ok = ri.rowfree && ri.exr == ex && Ob + ri.rmn >= lo && Ob + ri.rmx <= hi;
        const unsigned long long bad = __ballot(act && !ok);
        const uint32_t seg = (uint32_t)(bad >> (lane & 48u)) & 0xFFFFu;
        const uint32_t f = !pending ? nrows : !adm ? cur : seg ? (uint32_t)__builtin_ctz(seg) >> 2 : nrows;
        // commit rows [cur, f): component c's inclusive total through row f - 1
        const int at = __shfl(inc, (int)((lane & 48u) + 4u * max(f, 1u) - 1u), 64);
        if (adm && f > cur) s = (float)(O0 + at) * u;
        // row f by the chain (components without one: the -0.0 row)
        const bool chain = pending && f < nrows;
        if (__ballot(chain)) {  // (wave-uniform)
            GDF_VOXSUM_PROBE(3);
            const float4* rp = reinterpret_cast<const float4*>(comp + (chain ? f : 4u) * kRowStride);
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const float4 v = rp[k];
                s = s + v.x;
                s = s + v.y;
                s = s + v.z;
                s = s + v.w;
            }
        }
        cur = chain ? f + 1u : pending ? nrows : cur;
    }
    return s;
}

// A voxel's cnt points staged in LDS (float4, AoS) summed by one wave in chunks of 256 through
// wsoa (kWaveSoa floats, wave_soa_init'ed): the lane's component (lane >> 4) of the sum.
__device__ __forceinline__ float wave_group_sum(const float4* gp, uint32_t cnt, float* wsoa) {
    const uint32_t lane = threadIdx.x & 63;
    float s = 0.0f;
#pragma unroll 1
    for (uint32_t c0 = 0; c0 < cnt; c0 += 256u) {
        const uint32_t n = min(256u, cnt - c0);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // (the previous chunk is read)
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t i = 64u * k + lane;
            const float4 v = i < n ? gp[c0 + i] : make_float4(-0.0f, -0.0f, -0.0f, -0.0f);
            wsoa[0 * kWaveCompStride + k * kRowStride + lane] = v.x;
            wsoa[1 * kWaveCompStride + k * kRowStride + lane] = v.y;
            wsoa[2 * kWaveCompStride + k * kRowStride + lane] = v.z;
            wsoa[3 * kWaveCompStride + k * kRowStride + lane] = v.w;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        s = rows4c_chunk(wsoa, n, s);
    }
    return s;
}
#undef GDF_QPERM

// the voxel output of component c (wave c of the voxel's block): x/y/z divided by the count, w
// the plain sum (inc/voxelize.h:37-45)
__device__ __forceinline__ void store_comp_mean(float* o, uint32_t c, float s, uint32_t cnt) {
    if ((threadIdx.x & 63) == 0) o[c] = c < 3 ? s / (float)cnt : s;
}

}  // namespace gdf
