// gdf_kernels.hip — gfx950 (CDNA4, wave64) kernels of the depth-fusion hot path.
//
// Reference shaders restated here (paths relative to the reference root, shader/):
//   k_mask/k_emit      convert_depthmap_to_points.glsl:83-120, filter_flying_pixels.glsl:43-165,
//                      transform_points_indirect.glsl:50-69, crop_points.glsl:38-67,
//                      apply_point_mask.glsl:42-55 (ordered: reduce-then-scan, k_scan_counts),
//                      compute_voxel_coords.glsl:34-55, voxel_grid_occupancy_of_points.glsl:30-40
//   k_ps_filter_insert filter_point_sequence.glsl:78-122 + transfer_data.glsl (rollbuffer insert)
//   k_grid_*           zero_uints / decrement_uints.glsl:31-51 / max_with_uints_times_scalar.glsl:36-46
//                      / uints_to_chars.glsl:31-50, fused into one pass over the cells
//   k_sort_*, k_group  inc/voxelize.h:74-105 + radix_grouper.h + radix_sort.h (GPU version)
#include <atomic>
#include "gdf_kernels.hpp"

// The fence-free hand-offs (publish_count / arrive_and_scan, grid_seq_enter / grid_seq_leave
// <COHERENT>) rely on gfx950's cache policy bits: cpol sc1 = agent-coherent (write-through past the
// XCD's L2), with vmcnt(0) draining the stores.  The same bits mean something else on other
// targets: device code is built for gfx950 only.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "gdf_kernels.hip targets gfx950 (CDNA4) only: its coherence hand-offs use gfx950 cache bits"
#endif
#include "gdf_voxsum.hpp"  // the voxel sum (row_sum4): exact integer stretches

#include <algorithm>

namespace gdf {

// Pointers that arrive inside structs (kernel-argument structs, LDS camera copies) are generic to
// the compiler, which then emits flat_* instructions: those count against BOTH vmcnt and lgkmcnt,
// so every LDS wait also waits for in-flight global loads (no latency hiding).  G() re-types a
// pointer as global (address space 1) so the frame kernels issue global_* instructions.
template <class T>
using gptr = __attribute__((address_space(1))) T*;
template <class T>
__device__ __forceinline__ gptr<T> G(T* p) {
    return (gptr<T>)p;
}

typedef float f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 gld4(const float4* p, uint64_t i) {
    const f4v v = ((gptr<const f4v>)p)[i];
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void gst4(float4* p, uint64_t i, const float4& w) {
    f4v v;
    v.x = w.x; v.y = w.y; v.z = w.z; v.w = w.w;
    ((gptr<f4v>)p)[i] = v;
}

// ---- small helpers ----------------------------------------------------------------------------
__device__ __forceinline__ unsigned long long lanemask_lt() {
    const int lane = threadIdx.x & 63;
    return lane ? (~0ull >> (64 - lane)) : 0ull;
}

// Tile ticket in block-arrival order (a block only ever waits on lower tickets, which are already
// running).  Exactly ntiles blocks take one; the taker of the last resets the counter, so the
// next launch on the stream starts from 0 again without a memset.
__device__ __forceinline__ uint32_t take_ticket(uint32_t* ctr, uint32_t ntiles) {
    const uint32_t t = atomicAdd(ctr, 1u);
    if (t == ntiles - 1u) atomicExch(ctr, 0u);
    return t;
}

// Ticket + look-back epoch of a launch, both device-resident (a captured frame replays with
// unchanged kernel arguments).  Every ticket taker reads the stream's epoch word E before its
// ticket; the taker of the last ticket - after every other block has read E - advances it, so
// each launch that publishes granules uses a fresh epoch E + 1 >= 1 and the next launch on the
// stream sees E + 1.  (A launch with no tiles takes no ticket, publishes nothing and leaves E.)
__device__ __forceinline__ uint32_t take_ticket_epoch(uint32_t* ctr, uint32_t ntiles,
                                                      uint32_t* epoch_word, uint32_t& epoch) {
    const uint32_t e = __hip_atomic_load(epoch_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // the read has returned before the ticket is taken (a wait, not an acquire fence: that would
    // invalidate the XCD's L2 for every tile)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t t = atomicAdd(ctr, 1u);
    if (t == ntiles - 1u) {
        atomicExch(ctr, 0u);
        __hip_atomic_store(epoch_word, e + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    epoch = e + 1u;
    return t;
}

// Persistent launches: of a launch's `grid` ticket-capable blocks, nblk = min(grid, ntiles)
// take part (the others leave at once: a capacity-sized launch is mostly empty for small frames).
// With ntiles <= grid every participant draws exactly one ticket (ntiles draws); otherwise each
// draws until it gets one >= ntiles (ntiles + nblk draws).  The drawer of the last ticket resets
// the counter and publishes the next epoch; every participant reads the epoch (read_epoch)
// before its first draw, so before that last one.  The grid is capped by kPersistBlocks: a
// capacity-sized grid of 10^5..10^6 mostly idle workgroups (a large rollbuffer window whose
// points mostly leave the crop box) costs more dispatch time than the work.
__device__ __forceinline__ uint32_t read_epoch(uint32_t* epoch_word) {
    const uint32_t e = __hip_atomic_load(epoch_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return e + 1u;
}

struct Tickets {
    uint32_t nblk, draws;
    bool oneshot;
};

__device__ __forceinline__ Tickets tickets(uint32_t ntiles, uint32_t grid) {
    Tickets t;
    t.oneshot = ntiles <= grid;
    t.nblk = t.oneshot ? ntiles : grid;
    t.draws = t.oneshot ? ntiles : ntiles + grid;
    return t;
}

__device__ __forceinline__ uint32_t next_ticket(uint32_t* ctr, const Tickets& tk,
                                                uint32_t* epoch_word, uint32_t epoch) {
    const uint32_t t = atomicAdd(ctr, 1u);
    if (t == tk.draws - 1u) {
        atomicExch(ctr, 0u);
        __hip_atomic_store(epoch_word, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return t;
}

// Block (256 threads) exclusive scan of one value per thread.
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t& total,
                                                         uint32_t* s_wave) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_wave[wid] = x;
    __syncthreads();
    uint32_t wbase = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        uint32_t t = s_wave[w];
        wbase += (w < wid) ? t : 0u;
        tot += t;
    }
    total = tot;
    __syncthreads();
    return wbase + x - v;
}

// Decoupled look-back over 8-byte {flag, value} granules.  flag = 2*epoch (aggregate) or
// 2*epoch+1 (inclusive prefix); epoch >= 1 grows with every launch, so granules left by earlier
// launches read as "not ready" and the status arrays never need a memset.  Each granule is
// written by ONE agent-scope atomic store and polled with agent-scope atomic loads (MI355X
// hand-off form "R2": the data is the flag, no fence needed).
// Two-level decoupled look-back, wave-cooperative, one prefix channel.  Tiles are grouped by 64:
// level 1 sums the aggregates of the tile's predecessors inside its group (one 64-wide poll);
// the group's last tile then publishes the group aggregate BEFORE resolving its own group prefix,
// so level 2 (one 64-wide poll over earlier groups, stopping at the nearest inclusive group)
// never waits on a chain of group prefixes.  ~2 round trips per tile, whatever the tile count.
// gstat granules: flag 2*epoch = group aggregate, 2*epoch+1 = group inclusive prefix.
__device__ __forceinline__ uint32_t lookback2_wave(unsigned long long* tstat,
                                                   unsigned long long* gstat, uint32_t tile,
                                                   uint32_t ntiles, uint32_t agg, uint32_t epoch,
                                                   uint32_t* err) {
    const int lane = threadIdx.x & 63;
    const unsigned long long fagg = 2ull * epoch, fincl = 2ull * epoch + 1ull;
    const uint32_t G = tile >> 6, first = G << 6, pos = tile & 63u;
    const uint32_t last = (first + 63u < ntiles - 1u) ? first + 63u : ntiles - 1u;
    if (lane == 0)
        __hip_atomic_store(&tstat[tile], (fagg << 32) | agg, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    uint32_t spins = 0;
    // level 1: aggregates of tiles [first, tile)
    uint32_t in_excl = 0;
    if (pos > 0) {
        while (true) {
            unsigned long long sv = fagg << 32;
            if ((uint32_t)lane < pos)
                sv = __hip_atomic_load(&tstat[first + lane], __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            if (__ballot((sv >> 32) < fagg)) {
                if (++spins > kSpinLimit) {
                    if (lane == 0) atomicOr(err, 1u);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
                continue;
            }
            uint32_t v = (uint32_t)lane < pos ? (uint32_t)sv : 0u;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
            in_excl = v;
            break;
        }
    }
    const uint32_t gtotal = in_excl + agg;
    if (tile == last && lane == 0)
        __hip_atomic_store(&gstat[G], (fagg << 32) | gtotal, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    // level 2: prefix of the groups before G
    uint32_t gpre = 0;
    int64_t base = (int64_t)G - 1;
    while (base >= 0) {
        const int64_t j = base - lane;
        unsigned long long sv = fincl << 32;
        if (j >= 0)
            sv = __hip_atomic_load(&gstat[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long flag = sv >> 32;
        const unsigned long long m_incl = __ballot(flag == fincl);
        const unsigned long long m_wait = __ballot(flag < fagg);
        const int firsti = m_incl ? __ffsll((long long)m_incl) - 1 : 63;
        const unsigned long long need = firsti == 63 ? ~0ull : ((2ull << firsti) - 1ull);
        if (m_wait & need) {
            if (++spins > kSpinLimit) {
                if (lane == 0) atomicOr(err, 1u);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        uint32_t v = (lane <= firsti) ? (uint32_t)sv : 0u;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        gpre += v;
        if (m_incl) break;
        base -= 64;
    }
    if (tile == last && lane == 0)
        __hip_atomic_store(&gstat[G], (fincl << 32) | (gpre + gtotal), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    return gpre + in_excl;
}

// The same two-level scheme with R channels per THREAD (the 256 R digits of a radix pass; channel
// r of thread t is t + 256 r): groups of kSortGroup (8) tiles, 8 independent polls per round trip
// (8 rather than 16: 45 fewer VGPRs in the radix pass, occupancy 4 -> 6 waves/SIMD at 4 keys per
// thread).  All R aggregates are published before the first poll.
template <int R>
__device__ __forceinline__ void lookback2_chans(unsigned long long* tstat, unsigned long long* gstat,
                                                uint32_t tile, uint32_t ntiles, const uint32_t* agg,
                                                uint32_t* excl, uint32_t epoch, uint32_t* err) {
    constexpr uint32_t kCh = 256u * R;
    const uint32_t t = threadIdx.x;
    const unsigned long long fagg = 2ull * epoch, fincl = 2ull * epoch + 1ull;
    const uint32_t G = tile / kSortGroup, first = G * kSortGroup, pos = tile - first;
    const uint32_t last = (first + kSortGroup - 1u < ntiles - 1u) ? first + kSortGroup - 1u
                                                                   : ntiles - 1u;
#pragma unroll
    for (int r = 0; r < R; ++r)
        __hip_atomic_store(&tstat[(size_t)tile * kCh + t + 256u * r], (fagg << 32) | agg[r],
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t spins = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t chan = t + 256u * r;
        uint32_t in_excl = 0;
        if (pos > 0) {
            while (true) {
                unsigned long long sv[kSortGroup];
#pragma unroll
                for (int q = 0; q < kSortGroup; ++q)
                    sv[q] = ((uint32_t)q < pos)
                                ? __hip_atomic_load(&tstat[(size_t)(first + q) * kCh + chan],
                                                    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                : (fagg << 32);
                bool wait = false;
                uint32_t v = 0;
#pragma unroll
                for (int q = 0; q < kSortGroup; ++q) {
                    wait |= (sv[q] >> 32) < fagg;
                    v += (uint32_t)q < pos ? (uint32_t)sv[q] : 0u;
                }
                if (wait) {
                    if (++spins > kSpinLimit) {
                        atomicOr(err, 2u);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                in_excl = v;
                break;
            }
        }
        excl[r] = in_excl;  // (within the group; the groups' prefix is added below)
    }
    if (tile == last)
#pragma unroll
        for (int r = 0; r < R; ++r)
            __hip_atomic_store(&gstat[(size_t)G * kCh + t + 256u * r], (fagg << 32) | (excl[r] + agg[r]),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t chan = t + 256u * r;
        uint32_t gpre = 0;
        int64_t j = (int64_t)G - 1;
        while (j >= 0) {
            unsigned long long sv[kSortGroup];
#pragma unroll
            for (int q = 0; q < kSortGroup; ++q)
                sv[q] = (j - q >= 0) ? __hip_atomic_load(&gstat[(size_t)(j - q) * kCh + chan],
                                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                     : (fincl << 32);
            int q = 0;
            bool done = false;
            for (; q < kSortGroup; ++q) {
                const unsigned long long flag = sv[q] >> 32;
                if (flag < fagg) break;
                gpre += (uint32_t)sv[q];
                if (flag == fincl) {
                    done = true;
                    break;
                }
            }
            if (done) break;
            j -= q;
            if (q < kSortGroup) {
                if (++spins > kSpinLimit) {
                    atomicOr(err, 2u);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        if (tile == last)
            __hip_atomic_store(&gstat[(size_t)G * kCh + chan], (fincl << 32) | (gpre + excl[r] + agg[r]),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        excl[r] += gpre;
    }
}

// ---- fused frame kernel ------------------------------------------------------------------------
// Camera owning global index gi; -1 when gi is outside every camera (the reference's
// out-of-bounds read, canonicalised as mask 0).  Branch-free over the (uniform) camera count so
// that the neighbour loads of one ring issue back to back.
__device__ __forceinline__ int find_cam(const CamDesc* cams, int ncams, int64_t gi) {
    int j = -1;
    for (int c = 0; c < ncams; ++c)
        j = (gi >= cams[c].off && gi < cams[c].off + (int64_t)cams[c].n) ? c : j;
    return j;
}

struct Nb {
    uint32_t d;
    float xn, yn, scale;
};

// depth + ray factors of a neighbour read by check_at (filter_flying_pixels.glsl:63-80); the
// three loads depend only on the index, so all neighbours of a ring are in flight together
__device__ __forceinline__ Nb nb_load(const CamDesc* cams, int ncams, int k, int64_t gi) {
    int j = (gi >= cams[k].off && gi < cams[k].off + (int64_t)cams[k].n) ? k
                                                                          : find_cam(cams, ncams, gi);
    // a batch of frames shares one index space: a camera's linear-index reads past its frame's
    // first camera find the previous frame's last camera, which the reference (one frame per
    // buffer) never sees - canonicalised as out of bounds like camera 0's
    if (j >= 0 && cams[j].frame != cams[k].frame) j = -1;
    Nb r;
    r.d = 0;
    r.xn = r.yn = 0.0f;
    r.scale = 0.0f;
    if (j >= 0) {
        const CamDesc& c = cams[j];
        const uint32_t local = (uint32_t)(gi - c.off);
        const uint32_t v = div_w(c, local);
        const uint32_t u = local - v * c.W;
        r.d = G(c.depth)[local];
        r.xn = G(c.xn)[u];
        r.yn = G(c.yn)[v];
        r.scale = c.scale;
    }
    return r;
}

__device__ __forceinline__ void nb_point(const Nb& n, float& x, float& y, float& z) {
    const float zz = (float)n.d * n.scale;
    x = n.xn * zz;
    y = n.yn * zz;
    z = zz;
}

// ---- depth stage bits: convert_depthmap_to_points (:83-120) -> filter_flying_pixels (:135-165)
// -> crop_points (:38-67); bit0 convert, bit1 flying, bit2 crop.
//
// Work unit of the compaction: a SEGMENT = up to 1024 consecutive pixels of one camera row (rows
// wider than 1024 are split evenly into 64-multiples), or 1024 consecutive selected rollbuffer
// points.  Segments are numbered in item order, so the ordered compaction only needs one valid
// count per segment (a plain store, no atomics) and a 16-word validity bitmask.
//
// k_mask stages the segment's depth band - rows y-h..y+h, columns x0-h..x0+len+h, h = min(F, 8) -
// in LDS with 16-byte loads, plus the column ray factors.  Every neighbour the reference reaches
// without wrapping its linear index is read from the band; the wrap cases (x < i: the previous
// row's end; y < i: the previous camera or out of bounds) and rings beyond the
// halo read global memory with the reference's linear index arithmetic.
struct SegGeo {
    int k;            // camera
    uint32_t y, x0, len;
    uint32_t item0;   // first item (global point index)
};

// The emitting camera whose segments hold segment s (the last one, 0 if none): lane c tests
// camera c, so every camera's range arrives in ONE load round - a scan over the table issued a
// dependent scalar-load round per camera (k_mask_px stamps, tools/mask_trace.py: 12.3 K of a
// block's 36.9 K cycles for 8 cameras).  Wave-uniform result.  The ballot needs lanes
// 0..ncams-1 active: a caller in divergent code (or a block not a multiple of 64 threads) takes
// the per-camera scan instead (same answer: the last match).
// uni > 0 (FrameArgs::seg_uniform, equal cameras): the camera by one scalar division - the
// descriptor fields that follow then come in one scalar-load round instead of after a vector-load
// round of every camera's range.
template <class P>
__device__ __forceinline__ int seg_camera(P cams, int ncams, uint32_t s, uint32_t uni = 0u) {
    static_assert(kMaxCams <= 64, "one camera per lane");
    if (uni) return (int)min(s / uni, (uint32_t)ncams - 1u);
    const unsigned long long need = ncams >= 64 ? ~0ull : (1ull << ncams) - 1ull;
    if ((__builtin_amdgcn_read_exec() & need) != need) {
        int k = 0;
        for (int c = 0; c < ncams; ++c)
            if (cams[c].emit && s >= cams[c].seg0 && s < cams[c].seg0 + cams[c].nseg) k = c;
        return k;
    }
    const int lane = threadIdx.x & 63;
    bool hit = false;
    if (lane < ncams) {  // (the three fields in one load round: no short-circuit between them)
        const uint32_t seg0 = cams[lane].seg0, nseg = cams[lane].nseg;
        const bool emit = cams[lane].emit != 0;
        hit = emit & (s >= seg0) & (s < seg0 + nseg);
    }
    const unsigned long long m = __ballot(hit);
    return m ? 63 - __clzll((long long)m) : 0;
}

// (P: an LDS copy of the descriptors, or the global / kernel-argument table read with scalar
// loads - the segment is block-uniform)
template <class P>
__device__ __forceinline__ SegGeo seg_geo(P cams, int ncams, uint32_t s, uint32_t uni = 0u) {
    SegGeo g{0, 0, 0, 0, 0};
    g.k = __builtin_amdgcn_readfirstlane(seg_camera(cams, ncams, s, uni));  // (scalar field loads)
    const uint32_t seg0 = cams[g.k].seg0, nchunk = cams[g.k].nchunk, segw = cams[g.k].segw;
    const uint32_t W = cams[g.k].W;
    const uint32_t i = s - seg0;
    g.y = i / nchunk;
    const uint32_t j = i - g.y * nchunk;
    g.x0 = j * segw;
    g.len = min(segw, W - g.x0);
    g.item0 = (uint32_t)cams[g.k].off + g.y * W + g.x0;
    return g;
}

struct Band {
    const uint8_t* b;   // LDS band (bytes)
    const float* xn;    // LDS xn of columns ca..cb-1 (index x - ca)
    const int* rowoff;  // LDS byte offset of column 0 of band row r (may be negative)
    uint32_t ca;        // first staged column
    int h;
};

__device__ __forceinline__ uint32_t band_d(const Band& t, int r, uint32_t x) {
    return *reinterpret_cast<const uint16_t*>(t.b + t.rowoff[r] + 2 * (int)x);
}

struct P3 {
    float x, y, z;
    bool v;  // depth != 0
};

// neighbour (x, band row r) from LDS: the reference's f32 ops x = xn·z, y = yn·z, z = d·scale
__device__ __forceinline__ P3 band_pt(const Band& t, int r, uint32_t x, float yn, float scale) {
    const uint32_t d = band_d(t, r, x);
    const float zz = (float)d * scale;
    P3 p;
    p.x = t.xn[x - t.ca] * zz;
    p.y = yn * zz;
    p.z = zz;
    p.v = d != 0u;
    return p;
}

__device__ __forceinline__ P3 glb_pt(const CamDesc* cams, int ncams, int k, int64_t gi) {
    const Nb n = nb_load(cams, ncams, k, gi);
    P3 p;
    nb_point(n, p.x, p.y, p.z);
    p.v = n.d != 0u;
    return p;
}

// sqrtf(pp) > 10.0f (max_distance, filter_flying_pixels.glsl:41,143) <=> pp > 100.00001f: the
// correctly rounded sqrt is monotonic and 0x42C80001 is the largest float whose root rounds to
// at most 10 (tests/test_oracle_kat.py::test_max_distance_square_threshold checks both sides).
__device__ __forceinline__ bool beyond_max_distance(float pp) {
    return pp > __uint_as_float(0x42C80001u);
}

// check_at / check_at_rot45 (filter_flying_pixels.glsl:74-96) on four neighbour points: invalid
// if any neighbour has depth 0 or dot(normalize(cross(down - up, right - left)), n) < thr with
// n = -normalize(p).  The exact value cv is decided first by the filter
// cva = dot3(c, na) · rsq(c·c) with na = -p · rsq(p·p): both stay within ~20 ulp(1) of the real
// value for |n| ≈ 1, so outside thr ± 1e-5 the comparison cannot differ; only lanes inside it (or
// with c·c outside the normal range, incl. the NaN of a zero cross product) run the reference
// sequence, behind a wave-uniform branch.  `live` lanes are those whose result still matters.
// the reference sequence: n = -normalize(p), c / sqrt(c·c), dot, compare.  Out of line so the
// compiler cannot hoist the exact normal of p (3 divisions + sqrt) into every pixel's prologue.
__device__ __noinline__ bool surface_exact(float cx, float cy, float cz, float dd, float thr,
                                           float px, float py, float pz) {
    float nx = px, ny = py, nz_ = pz;
    normalize3(nx, ny, nz_);
    const float len = sqrtf(dd);
    const float cv = dot3(cx / len, cy / len, cz / len, -nx, -ny, -nz_);
    return !(cv < thr);  // NaN passes
}

__device__ __forceinline__ bool ring_pass(const P3& u, const P3& d, const P3& l, const P3& r,
                                          float thr, float nax, float nay, float naz, float px,
                                          float py, float pz, bool live) {
    const bool nz = u.v & d.v & l.v & r.v;
    const float ax = d.x - u.x, ay = d.y - u.y, az = d.z - u.z;  // dy = down - up
    const float bx = r.x - l.x, by = r.y - l.y, bz = r.z - l.z;  // dx = right - left
    const float cx = ay * bz - az * by;
    const float cy = az * bx - ax * bz;
    const float cz = ax * by - ay * bx;
    const float dd = dot3(cx, cy, cz, cx, cy, cz);
    const float cva = dot3(cx, cy, cz, nax, nay, naz) * __builtin_amdgcn_rsqf(dd);
    const bool normal = (dd > 1e-30f) & (dd < 1e30f);
    const bool hi = cva > thr + 1e-5f, lo = cva < thr - 1e-5f;
    bool pass = normal & hi;
    const bool undecided = live & nz & !(normal & (hi | lo));
    if (__ballot(undecided)) {  // rare, wave-uniform
        if (undecided) pass = surface_exact(cx, cy, cz, dd, thr, px, py, pz);
    }
    return nz & pass;
}

// signed column x (>= -h on a row-start segment's own band row: the previous row's end)
__device__ __forceinline__ P3 band_pt_s(const Band& t, int r, int x, float yn, float scale) {
    const uint32_t d = *reinterpret_cast<const uint16_t*>(t.b + t.rowoff[r] + 2 * x);
    const float zz = (float)d * scale;
    P3 p;
    p.x = t.xn[x - (int)t.ca] * zz;
    p.y = yn * zz;
    p.z = zz;
    p.v = d != 0u;
    return p;
}

// waves of k_mask: every neighbour in the band (kInterior); a row-start wave of a segment with
// x0 = 0, y >= F: left neighbours of lanes x < i wrap to the previous row's end, staged in front
// of the pixel's band row (kRowStart); anything else reads the wrapping neighbours globally
constexpr int kGeneral = 0, kInterior = 1, kRowStart = 2;

// Stage bits of pixel (x, y) of camera k (band row h = the pixel's row).  Rings are evaluated
// without per-lane early exit (the reference's first-failure return only decides the same AND);
// the wave leaves the ring loop once none of its lanes is still valid.
// FT > 0: the ring count F as a compile-time constant (the launch default F = 4): unrolled rings,
// no per-ring loop bookkeeping; FT = 0: a.F at run time.
template <bool ROT45, int MODE, uint32_t FT>
__device__ __forceinline__ uint32_t depth_bits(const FrameArgs& a, const CamDesc* cams, int k,
                                               const Band& t, const float* s_yn, uint32_t x,
                                               uint32_t y, bool in) {
    const CamDesc& c = cams[k];
    const int h = t.h;
    const float scale = c.scale;
    const P3 p = in ? band_pt(t, h, x, s_yn[h], scale) : P3{0.f, 0.f, 0.f, false};
    const bool conv = in & p.v;
    bool fly = conv;
    if (a.do_flying) {
        const float pp = dot3(p.x, p.y, p.z, p.x, p.y, p.z);
        fly = fly & !beyond_max_distance(pp);
        const float rr = __builtin_amdgcn_rsqf(pp);
        const float nax = -(p.x * rr), nay = -(p.y * rr), naz = -(p.z * rr);
        const int64_t g = c.off + (int64_t)y * c.W + x;
        const uint32_t FF = FT ? FT : a.F;
#pragma unroll
        for (uint32_t i = 1; i <= FF; ++i) {
            if (!__ballot(fly)) break;  // wave-uniform exit
            fly = fly & (x + i <= c.W - 1) & (y + i <= c.H - 1);  // bounds (:60)
            const int ii = (int)i;
            const int64_t gw = (int64_t)i * c.W;
            // kInterior (wave-uniform: every lane has x >= F, y >= F, F <= h): all in the band
            constexpr bool INTERIOR = MODE != kGeneral;
            const bool L = INTERIOR || ii <= h;  // ring inside the band (uniform)
            const bool yw = !INTERIOR && y < i;  // up neighbours leave the camera (uniform)
            const bool xw = !INTERIOR && x < i;  // left neighbours wrap to the previous row
            const uint32_t xs = x, xl = xw ? x : x - i, xr = x + i;
            P3 n0, n1, n2, n3;
            // up (x, y-i), down (x, y+i), left (x-i, y), right (x+i, y)
            n0 = (L && !yw) ? band_pt(t, h - ii, xs, s_yn[h - ii], scale)
                            : glb_pt(cams, a.ncams, k, g - gw);
            n1 = L ? band_pt(t, h + ii, xs, s_yn[h + ii], scale) : glb_pt(cams, a.ncams, k, g + gw);
            if (MODE == kRowStart)  // x < i: pixel (W - i + x, y - 1), its depth before column 0
                n2 = band_pt_s(t, h, (int)x - ii, x < i ? s_yn[h - 1] : s_yn[h], scale);
            else
                n2 = (L && !xw) ? band_pt(t, h, xl, s_yn[h], scale) : glb_pt(cams, a.ncams, k, g - ii);
            n3 = L ? band_pt(t, h, xr, s_yn[h], scale) : glb_pt(cams, a.ncams, k, g + ii);
            fly = fly & ring_pass(n0, n1, n2, n3, a.thr, nax, nay, naz, p.x, p.y, p.z, fly);
            if (ROT45) {  // up (x-i, y-i), down (x+i, y+i), left (x-i, y+i), right (x+i, y-i)
                n0 = (L && !xw && !yw) ? band_pt(t, h - ii, xl, s_yn[h - ii], scale)
                                       : glb_pt(cams, a.ncams, k, g - gw - ii);
                n1 = L ? band_pt(t, h + ii, xr, s_yn[h + ii], scale)
                       : glb_pt(cams, a.ncams, k, g + gw + ii);
                n2 = (L && !xw) ? band_pt(t, h + ii, xl, s_yn[h + ii], scale)
                                : glb_pt(cams, a.ncams, k, g + gw - ii);
                n3 = (L && !yw) ? band_pt(t, h - ii, xr, s_yn[h - ii], scale)
                                : glb_pt(cams, a.ncams, k, g - gw + ii);
                fly = fly & ring_pass(n0, n1, n2, n3, a.thr, nax, nay, naz, p.x, p.y, p.z, fly);
            }
        }
    }
    bool crop = true;
    if (a.do_crop) {
        const float qx = mrow(c.Tc + 0, p.x, p.y, p.z, 1.0f);
        const float qy = mrow(c.Tc + 4, p.x, p.y, p.z, 1.0f);
        const float qz = mrow(c.Tc + 8, p.x, p.y, p.z, 1.0f);
        crop = !((qx < a.lo[0]) | (qx > a.hi[0]) | (qy < a.lo[1]) | (qy > a.hi[1]) |
                 (qz < a.lo[2]) | (qz > a.hi[2]));
    }
    return (uint32_t)conv | ((uint32_t)fly << 1) | ((uint32_t)(fly & crop) << 2);
}

// transform index of selected point i: last covered sequence starting at or before i
__device__ __forceinline__ uint32_t sel_tf(const FrameArgs& a, uint32_t i) {
    uint32_t lo = 0, hi = a.nseg;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (G(a.seg_start)[mid] <= i) lo = mid; else hi = mid;
    }
    return G(a.seg_tf)[lo];
}

// The selected points of one segment (consecutive, block-uniform): the transform of its first
// point and where the next sequence starts (sequences hold ~10^5..10^6 points, so a segment
// almost never crosses one), and the ring position of its first point - one binary search and
// one 64-bit modulo per segment instead of per point.
struct SelSeg {
    uint32_t si0;    // first selected-point index of the segment
    uint32_t tf0;    // its transform index
    uint32_t next;   // first index of the following sequence (UINT_MAX: none)
    uint64_t r0;     // ring slot of si0
};

__device__ __forceinline__ SelSeg sel_seg(const FrameArgs& a, uint32_t si0) {
    // last sequence starting at or before si0: 64-ary search by the wave (seg_start ascending,
    // seg_start[0] == 0), one round trip per factor 64 of sequences
    const int lane = threadIdx.x & 63;
    uint32_t lo = 0, hi = a.nseg;
    if (a.sel_uniform)  // equal sequences (FrameArgs::sel_uniform): no search
        lo = hi = min((si0 + a.sel_off) / a.sel_uniform, (uint32_t)a.nseg - 1u);
    while (hi - lo > 1) {
        const uint32_t step = (hi - lo + 63u) / 64u;
        const uint32_t j = lo + (uint32_t)lane * step;
        // (loaded unconditionally at a clamped index: the short-circuit form waited in a branch)
        const uint32_t sj = G(a.seg_start)[min(j, hi - 1u)];
        const unsigned long long le = __ballot(j < hi && sj <= si0);
        const uint32_t L = 63u - (uint32_t)__clzll((long long)le);  // bit 0 is always set
        lo = lo + L * step;
        hi = min(hi, lo + step);
    }
    // block-uniform values: keep them (and what is loaded through them) in scalar registers
    lo = __builtin_amdgcn_readfirstlane(lo);
    SelSeg g;
    g.si0 = si0;
    const uint32_t tf0 = G(a.seg_tf)[lo];
    const uint32_t nx = G(a.seg_start)[min(lo + 1u, a.nseg - 1u)];  // (one round with tf0)
    g.tf0 = __builtin_amdgcn_readfirstlane(tf0);
    g.next = __builtin_amdgcn_readfirstlane(lo + 1 < a.nseg ? nx : 0xFFFFFFFFu);
    g.r0 = (a.ring_first + si0) % a.ring_cap;
    return g;
}

__device__ __forceinline__ float4 sel_point(const FrameArgs& a, const SelSeg& g, uint32_t i) {
    uint64_t r = g.r0 + (i - g.si0);
    if (r >= a.ring_cap) r -= a.ring_cap;
    return gld4(a.ring, r);
}

__device__ __forceinline__ uint32_t sel_tf_in(const FrameArgs& a, const SelSeg& g, uint32_t i) {
    return i < g.next ? g.tf0 : sel_tf(a, i);
}

// selected rollbuffer point i: mask (transfer_data of the selected mask), transform_points
// _indirect (:50-69) into the crop frame, crop_points
__device__ __forceinline__ uint32_t sel_bits_m(const FrameArgs& a, const float4& p,
                                               gptr<const float> Tc) {
    if (p.w == 0.0f) return 0;  // rollbuffer mask 0
    if (a.do_crop) {
        const float qx = mrow(Tc + 0, p.x, p.y, p.z, 1.0f);
        const float qy = mrow(Tc + 4, p.x, p.y, p.z, 1.0f);
        const float qz = mrow(Tc + 8, p.x, p.y, p.z, 1.0f);
        if (qx < a.lo[0] || qx > a.hi[0] || qy < a.lo[1] || qy > a.hi[1] || qz < a.lo[2] ||
            qz > a.hi[2])
            return 3;
    }
    return 7;
}

__device__ __forceinline__ uint32_t sel_bits(const FrameArgs& a, const SelSeg& g, uint32_t i,
                                             const float4& p) {
    if (p.w == 0.0f) return 0;  // rollbuffer mask 0
    if (a.do_crop) {
        const gptr<const float> Tc = G(a.tfc + 16 * (size_t)sel_tf_in(a, g, i));
        const float qx = mrow(Tc + 0, p.x, p.y, p.z, 1.0f);
        const float qy = mrow(Tc + 4, p.x, p.y, p.z, 1.0f);
        const float qz = mrow(Tc + 8, p.x, p.y, p.z, 1.0f);
        if (qx < a.lo[0] || qx > a.hi[0] || qy < a.lo[1] || qy > a.hi[1] || qz < a.lo[2] ||
            qz > a.hi[2])
            return 3;
    }
    return 7;
}

// Camera descriptors: kernel arguments for up to kArgCams cameras, else the device copy.
// The callers read the kernel-argument table with GLOBAL loads (G()): valid because the by-value
// FrameArgs stays in the kernarg segment (a global address).  Were the compiler to keep a private
// (scratch) copy of it - an asm memory clobber did in round 4, and so did the address of the
// table escaping into a non-inlined function in the 4-pixel k_mask_px - G() would turn a
// private-aperture address into a "global" one: HSA_STATUS_ERROR_MEMORY_APERTURE_VIOLATION (round
// 4's k_mask_px_o8 fault).  tests/test_abi.py checks every kernel's scratch size
// (no copy).  (Addressing the table through __builtin_amdgcn_kernarg_segment_ptr() instead is
// immune but cost 15 % of the C2 line: 30+ more SGPRs in every frame kernel, A/B on one box.)
__device__ __forceinline__ const CamDesc* cam_table(const FrameArgs& a) {
    return a.ncams <= kArgCams ? a.cams : a.cams_dev;
}

// block-wide copy of the camera descriptors into LDS
__device__ __forceinline__ void load_cams(const FrameArgs& a, CamDesc* s_cams) {
    const uint32_t words = (uint32_t)a.ncams * (uint32_t)(sizeof(CamDesc) / 4);
    const uint32_t* src = reinterpret_cast<const uint32_t*>(cam_table(a));
    uint32_t* dst = reinterpret_cast<uint32_t*>(s_cams);
    for (uint32_t w = threadIdx.x; w < words; w += blockDim.x) dst[w] = G(src)[w];
}

// In-kernel group scan of the segment counts (replaces k_scan_reduce + k_scan_counts above
// kFusedPrefixSegs segments): after a block has written its counts, it counts itself in at its
// group of kScanGroup consecutive segments; the group's last block (agent-scope release /
// acquire: the blocks of a group may run on other XCDs) scans the group's point counts - and run
// counts - into group-local exclusive offsets and writes the group totals, then re-arms the
// counter for the next launch (graph replays included).  k_emit adds the totals of the groups
// before its own (group_partials).
// Generic form (counts stored by publish_count, from thread 0): entry `idx` of `nent` counts (cnt[q * stride + i] for series q < nser) was just
// written by thread 0 of this block; the last arriver of idx's group scans the group.
__device__ __forceinline__ void publish_count(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // global_store sc1
}

__device__ __forceinline__ void arrive_and_scan(uint32_t* done, const uint32_t* cnt, uint32_t* off,
                                                uint32_t* gtot, uint32_t idx, uint32_t nent,
                                                int nser, uint32_t stride, uint32_t* s_last) {
    const uint32_t g = idx / kScanGroup;
    const uint32_t s0 = g * kScanGroup;
    const uint32_t n = min(kScanGroup, nent - s0);
    if (threadIdx.x == 0) {
        // write-through hand-off, no fences (an agent release here is an L2 write-back per block:
        // 7x the whole kernel, measured): the counts were stored sc1 by this lane (publish_count),
        // drained before the counter add; the last arriver reads them with sc1 loads
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t old = __hip_atomic_fetch_add(done + g, 1u, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
        *s_last = old + 1u == n ? 1u : 0u;
    }
    __syncthreads();
    if (!*s_last || threadIdx.x >= 64) return;  // block-uniform, then wave 0
    const uint32_t lane = threadIdx.x;
    const uint32_t ng = (nent + kScanGroup - 1) / kScanGroup;
    // both series' counts read in one round (at a clamped index), scanned after
    const uint32_t lc = min(lane, n - 1u);
    uint32_t vs[2];
    for (int q = 0; q < 2; ++q)
        vs[q] = __hip_atomic_load(cnt + (q < nser ? q : 0) * stride + s0 + lc, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
    for (int q = 0; q < nser; ++q) {  // (k_mask: point counts, then run counts)
        const uint32_t base = q * stride;
        const uint32_t v = lane < n ? vs[q] : 0u;
        uint32_t x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (lane >= (uint32_t)o) x += y;
        }
        if (lane < n) G(off)[base + s0 + lane] = x - v;
        if (lane == 63) G(gtot)[q * ng + g] = x;
    }
    if (lane == 0) __hip_atomic_store(done + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void group_scan_tail(const FrameArgs& a, uint32_t s) {
    __shared__ uint32_t s_last;
    if (!a.grp_done) return;
    arrive_and_scan(a.grp_done, a.seg_counts, a.seg_offsets, a.grp_tot, s, a.total_segs,
                    a.run_mode ? 2 : 1, a.total_segs, &s_last);
}

// the sum of the group totals gtot[0 .. idx / kScanGroup) by one wave (every lane gets it)
__device__ __forceinline__ uint32_t wave_group_prefix(const uint32_t* gtot, uint32_t idx) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t ng = idx / kScanGroup;
    // (the first 64 totals unconditionally at a clamped index: a loop's first load waited for
    // every load issued before it)
    const uint32_t v0 = G(gtot)[min(lane, ng ? ng - 1u : 0u)];
    uint32_t sum = lane < ng ? v0 : 0u;
    for (uint32_t t = lane + 64u; t < ng; t += 64) sum += G(gtot)[t];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
    return sum;
}

// sum of the totals of the groups before segment s's group (group-scan form), into s_red per
// wave (run mode: the run totals too, into s_red + 16)
__device__ __forceinline__ void group_partials(const FrameArgs& a, uint32_t s, uint32_t* s_red) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t g = s / kScanGroup;
    const uint32_t ng = (a.total_segs + kScanGroup - 1) / kScanGroup;
    uint32_t sum = 0, rsum = 0;
    // four strides per round, loaded unconditionally at clamped indices (g >= 1 here): one load
    // round per 4 block strides, where the loop form waited on each load
    for (uint32_t t0 = threadIdx.x; t0 < g; t0 += 4u * blockDim.x) {  // (g: block-uniform)
        uint32_t v[4], w[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t t = min(t0 + (uint32_t)q * blockDim.x, g - 1u);
            v[q] = G(a.grp_tot)[t];
            w[q] = a.run_mode ? G(a.grp_tot)[ng + t] : 0u;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const bool in = t0 + (uint32_t)q * blockDim.x < g;
            sum += in ? v[q] : 0u;
            rsum += in ? w[q] : 0u;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        sum += __shfl_xor(sum, o, 64);
        rsum += __shfl_xor(rsum, o, 64);
    }
    if (lane == 0) {
        s_red[wid] = sum;
        s_red[16 + wid] = rsum;
    }
}

// group_partials in two halves (k_emit_px2): the first round's loads issued before the segment's
// own geometry and depth loads, summed after them - one load round for both instead of two
struct GroupPart {
    uint32_t v[4], w[4];
};
__device__ __forceinline__ GroupPart group_partials_issue(const FrameArgs& a, uint32_t s) {
    GroupPart p;
    const uint32_t g = s / kScanGroup;
    const uint32_t ng = (a.total_segs + kScanGroup - 1) / kScanGroup;
    const uint32_t last = g ? g - 1u : 0u;  // (clamped: entries past g are loaded, not summed)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t t = min(threadIdx.x + (uint32_t)q * blockDim.x, last);
        p.v[q] = G(a.grp_tot)[t];
        p.w[q] = a.run_mode ? G(a.grp_tot)[ng + t] : 0u;
    }
    return p;
}
__device__ __forceinline__ void group_partials_finish(const FrameArgs& a, uint32_t s,
                                                      const GroupPart& p, uint32_t* s_red) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t g = s / kScanGroup;
    const uint32_t ng = (a.total_segs + kScanGroup - 1) / kScanGroup;
    uint32_t sum = 0, rsum = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const bool in = threadIdx.x + (uint32_t)q * blockDim.x < g;
        sum += in ? p.v[q] : 0u;
        rsum += in ? p.w[q] : 0u;
    }
    for (uint32_t t = threadIdx.x + 4u * blockDim.x; t < g; t += blockDim.x) {  // (rare: > 4 strides)
        sum += G(a.grp_tot)[t];
        if (a.run_mode) rsum += G(a.grp_tot)[ng + t];
    }
    for (int o = 32; o > 0; o >>= 1) {
        sum += __shfl_xor(sum, o, 64);
        rsum += __shfl_xor(rsum, o, 64);
    }
    if (lane == 0) {
        s_red[wid] = sum;
        s_red[16 + wid] = rsum;
    }
}

// Pass 1 of the ordered compaction (apply_point_mask.glsl:42-55 made stable): one block per
// segment, one item per thread (blockDim = a.seg_threads >= every segment's length).  The ballot
// of wave w's valid bits is word w of the segment's 16-word bitmask.
template <bool ROT45, uint32_t FT>
__global__ __launch_bounds__(1024) void k_mask(FrameArgs a) {
    __shared__ CamDesc s_cams[kMaxCams];
    __shared__ float s_yn[2 * kHalo + 1];
    __shared__ int s_rowoff[2 * kHalo + 1];
    __shared__ uint32_t s_cnt[16];
    __shared__ uint32_t s_rcnt[16];
    __shared__ uint32_t s_hist[4 * 256];  // run-key digit histogram (run mode)
    extern __shared__ uint4 s_dyn[];  // band rows (a.band_rowb bytes each), then xn
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int nwaves = blockDim.x >> 6;
    // XCD-aware: blocks are dealt round-robin over the 8 XCDs (speed only, never correctness),
    // so give each XCD a contiguous run of segments - neighbouring rows' bands then share its L2
    const uint32_t n = gridDim.x, q8 = n / 8, r8 = n % 8, xcd = blockIdx.x % 8;
    const uint32_t s = xcd * q8 + min(xcd, r8) + blockIdx.x / 8;
    if (a.grid_seq_out && blockIdx.x == 0 && threadIdx.x == 0) *a.grid_seq_out = a.grid_seq;
    uint32_t bits = 0;
    uint32_t rkey = 0xFFFFFFFFu;  // run mode: sort key of a kept pixel
    const uint32_t i = threadIdx.x;
    if (a.run_mode && a.key_hist)
        for (uint32_t j = threadIdx.x; j < radix_hist_span(a.npasses); j += blockDim.x) s_hist[j] = 0;
    {
        // the block's camera from the descriptor table with scalar loads, so the band loads
        // issue at once; the LDS copy of all descriptors (neighbour lookups) overlaps them
        const gptr<const CamDesc> gcam = G(cam_table(a));
        const SegGeo sg = seg_geo(gcam, a.ncams, s, a.seg_uniform);
        struct {
            const uint16_t* depth;
            const float *xn, *yn;
            uint32_t W, H;
        } c = {gcam[sg.k].depth, gcam[sg.k].xn, gcam[sg.k].yn, gcam[sg.k].W, gcam[sg.k].H};
        const int h = a.do_flying ? (int)min(a.F, (uint32_t)kHalo) : 0;
        const uint32_t ca = sg.x0 >= (uint32_t)h ? sg.x0 - h : 0u;
        const uint32_t cb = min(c.W, sg.x0 + sg.len + h);
        const uint32_t nrows = 2 * h + 1;
        uint8_t* band = reinterpret_cast<uint8_t*>(s_dyn);
        // (kHalo floats before s_xn: the ray factors of the last h columns, s_xn[-j] = xn[W - j],
        // read by the left neighbours that wrap to the previous row's end)
        float* s_xn = reinterpret_cast<float*>(band + (size_t)nrows * a.band_rowb) + kHalo;
        // A row-start segment (x0 = 0, rows y >= h, W >= h): the pixel's own band row also stages
        // the h pixels before column 0 in linear order - the previous row's end, which the
        // reference's linear index x - i reaches for x < i (filter_flying_pixels.glsl:63-73)
        const bool wrap = a.do_flying && sg.x0 == 0 && sg.y >= (uint32_t)h && c.W >= (uint32_t)h && h > 0;
        // stage the band: 16-byte chunks, the row's first chunk aligned down (same 16-B line as
        // a needed byte, so never outside the allocation's pages); all loads before any store
        typedef uint32_t u4v __attribute__((ext_vector_type(4)));
        const uintptr_t dbase = reinterpret_cast<uintptr_t>(c.depth);
        const uint32_t nch = a.band_rowb / 16;
        const uint32_t r = (uint32_t)wid;  // one band row per wave (nrows <= 17 <= waves or looped)
        u4v v[3];
        float xv0 = 0.0f, xv1 = 0.0f;
        uint32_t n16 = 0;
        uintptr_t a16 = 0, first = 0;
        const int gy = (int)sg.y - h + (int)r;
        const bool rok = r < nrows && gy >= 0 && gy < (int)c.H;
        uintptr_t col0 = 0;  // address of column ca
        if (rok) {
            col0 = dbase + 2 * ((uintptr_t)gy * c.W + ca);
            first = col0 - (wrap && r == (uint32_t)h ? 2 * (uintptr_t)h : 0);
            const uintptr_t last = dbase + 2 * ((uintptr_t)gy * c.W + cb);  // exclusive
            a16 = first & ~(uintptr_t)15;
            n16 = min((uint32_t)((last - a16 + 15) / 16), nch);
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                const uint32_t ch = (uint32_t)lane + 64u * q;
                if (ch < n16) v[q] = *(gptr<const u4v>)(a16 + 16 * (uintptr_t)ch);
            }
        }
        if (ca + i < cb) xv0 = G(c.xn)[ca + i];
        if (ca + i + blockDim.x < cb) xv1 = G(c.xn)[ca + i + blockDim.x];
        if (i < nrows) {
            const int gyi = (int)sg.y - h + (int)i;
            s_yn[i] = (gyi >= 0 && gyi < (int)c.H) ? G(c.yn)[gyi] : 0.0f;
        }
        float xwv = 0.0f;
        if (wrap && i < (uint32_t)h) xwv = G(c.xn)[c.W - 1 - i];
        load_cams(a, s_cams);
        if (rok) {
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                const uint32_t ch = (uint32_t)lane + 64u * q;
                if (ch < n16) *reinterpret_cast<u4v*>(band + r * a.band_rowb + 16 * ch) = v[q];
            }
        }
        if (lane == 0 && r < nrows)  // rows outside the camera: any in-bounds offset (never live)
            s_rowoff[r] = (int)(r * a.band_rowb) - 2 * (int)ca + (rok ? (int)(col0 - a16) : 0);
        // bands taller than the block's waves (few waves, big F): remaining rows, plain loop
        for (uint32_t rr = (uint32_t)nwaves + r; rr < nrows; rr += (uint32_t)nwaves) {
            const int gy2 = (int)sg.y - h + (int)rr;
            const bool ok2 = gy2 >= 0 && gy2 < (int)c.H;
            uintptr_t f2 = 0, b2 = 0;
            if (ok2) {
                f2 = dbase + 2 * ((uintptr_t)gy2 * c.W + ca);
                b2 = (f2 - (wrap && rr == (uint32_t)h ? 2 * (uintptr_t)h : 0)) & ~(uintptr_t)15;
                const uint32_t m16 = min((uint32_t)((dbase + 2 * ((uintptr_t)gy2 * c.W + cb) - b2 + 15) / 16), nch);
                for (uint32_t ch = (uint32_t)lane; ch < m16; ch += 64)
                    *reinterpret_cast<u4v*>(band + rr * a.band_rowb + 16 * ch) =
                        *(gptr<const u4v>)(b2 + 16 * (uintptr_t)ch);
            }
            if (lane == 0) s_rowoff[rr] = (int)(rr * a.band_rowb) - 2 * (int)ca + (ok2 ? (int)(f2 - b2) : 0);
        }
        if (ca + i < cb) s_xn[i] = xv0;
        if (ca + i + blockDim.x < cb) s_xn[i + blockDim.x] = xv1;
        if (wrap && i < (uint32_t)h) s_xn[-1 - (int)i] = xwv;
        __syncthreads();
        const Band t{band, s_xn, s_rowoff, ca, h};
        if (64u * (uint32_t)wid < sg.len) {  // wave-uniform
            const uint32_t xw0 = sg.x0 + 64u * wid;  // x of the wave's lane 0
            if (!a.do_flying || (xw0 >= a.F && sg.y >= a.F && a.F <= (uint32_t)h))
                bits = depth_bits<ROT45, kInterior, FT>(a, s_cams, sg.k, t, s_yn, sg.x0 + i, sg.y, i < sg.len);
            else if (!ROT45 && wrap && a.F <= (uint32_t)h)  // (wrap: y >= h = F)
                bits = depth_bits<ROT45, kRowStart, FT>(a, s_cams, sg.k, t, s_yn, sg.x0 + i, sg.y, i < sg.len);
            else
                bits = depth_bits<ROT45, kGeneral, FT>(a, s_cams, sg.k, t, s_yn, sg.x0 + i, sg.y, i < sg.len);
            if (a.dbg && i < sg.len) G(a.dbg)[sg.item0 + i] = (uint8_t)bits;
            if (a.run_mode && (bits & 4u)) {  // the voxel key k_emit will compute (same f32 ops)
                const CamDesc& cd = s_cams[sg.k];
                const P3 p = band_pt(t, h, sg.x0 + i, s_yn[h], cd.scale);
                const float wx = mrow(cd.Tw + 0, p.x, p.y, p.z, 1.0f);
                const float wy = mrow(cd.Tw + 4, p.x, p.y, p.z, 1.0f);
                const float wz = mrow(cd.Tw + 8, p.x, p.y, p.z, 1.0f);
                rkey = voxel_key(wx, wy, wz, a.vlo, a.vcs, a.vrcs, a.gmax, a.gs) | (cd.frame << a.frame_shift);
            }
        }
    }
    const unsigned long long m = __ballot((bits & 4u) != 0u);
    if (lane == 0) {
        G(a.vbits)[(size_t)s * 16 + wid] = m;
        s_cnt[wid] = (uint32_t)__popcll(m);
    }
    if (a.run_mode) {  // runs of equal keys among the wave's kept lanes (k_emit's leaders)
        const unsigned long long below = m & lanemask_lt();
        const int prev = below ? 63 - __clzll((long long)below) : -1;
        const uint32_t pkey = __shfl(rkey, prev < 0 ? 0 : prev, 64);
        const bool leader = ((bits & 4u) != 0u) && (prev < 0 || pkey != rkey);
        const unsigned long long lm = __ballot(leader);
        if (lane == 0) {
            G(a.wave_runs)[(size_t)s * 16 + wid] = (uint32_t)__popcll(lm);
            s_rcnt[wid] = (uint32_t)__popcll(lm);
        }
        if (leader && a.key_hist)
            for (uint32_t p = 0; p < a.npasses; ++p)
                atomicAdd(&s_hist[p * 256 + radix_digit(rkey, p, a.npasses)], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0, r = 0;
        for (int w = 0; w < nwaves; ++w) t += s_cnt[w];
        publish_count(a.seg_counts + s, t);
        if (a.run_mode) {
            for (int w = 0; w < nwaves; ++w) r += s_rcnt[w];
            publish_count(a.seg_counts + a.total_segs + s, r);  // run counts follow the point counts
        }
    }
    if (a.run_mode && a.key_hist) {
        const gptr<uint32_t> rep = G(a.key_hist + (blockIdx.x % kHistReps) * 1024u);
        for (uint32_t j = threadIdx.x; j < radix_hist_span(a.npasses); j += blockDim.x)
            if (s_hist[j])
                __hip_atomic_fetch_add(rep + j, s_hist[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    group_scan_tail(a, s);
}

// PX pixels per thread, ring by ring in lockstep (F = 4, no rot45): pixel j of thread i is
// x0 + i + j * blockDim (blockDim = 256 / PX).  Pixel 0 is k_mask's kInterior / kRowStart wave
// of the segment's first columns, the others are interior whenever pixel 0's row is.  One
// wave-uniform ring exit and the exact-fallback ballots of a ring serve all PX pixels; the
// arithmetic of each pixel is depth_bits' (same operations, same order).
template <int AMODE, int PX>
__device__ __forceinline__ void depth_bits_px(const FrameArgs& a, const CamDesc* cams, int k,
                                              const Band& t, const float* s_yn, const uint32_t* x,
                                              uint32_t y, const bool* in, uint32_t* bits) {
    const CamDesc& c = cams[k];
    const int h = t.h;
    const float scale = c.scale;
    P3 p[PX];
    bool conv[PX], fly[PX];
    float nx[PX], ny[PX], nz[PX];
#pragma unroll
    for (int j = 0; j < PX; ++j) {
        p[j] = in[j] ? band_pt(t, h, x[j], s_yn[h], scale) : P3{0.f, 0.f, 0.f, false};
        conv[j] = in[j] & p[j].v;
        const float pp = dot3(p[j].x, p[j].y, p[j].z, p[j].x, p[j].y, p[j].z);
        fly[j] = conv[j] & !beyond_max_distance(pp);
        const float rr = __builtin_amdgcn_rsqf(pp);
        nx[j] = -(p[j].x * rr);
        ny[j] = -(p[j].y * rr);
        nz[j] = -(p[j].z * rr);
    }
#pragma unroll
    for (uint32_t i = 1; i <= 4; ++i) {
        bool any = false;
#pragma unroll
        for (int j = 0; j < PX; ++j) any |= fly[j];
        if (!__ballot(any)) break;  // wave-uniform exit
        const int ii = (int)i;
#pragma unroll
        for (int j = 0; j < PX; ++j) {
            fly[j] = fly[j] & (x[j] + i <= c.W - 1) & (y + i <= c.H - 1);
            const P3 n0 = band_pt(t, h - ii, x[j], s_yn[h - ii], scale);
            const P3 n1 = band_pt(t, h + ii, x[j], s_yn[h + ii], scale);
            const P3 n2 = (AMODE == kRowStart && j == 0)
                              ? band_pt_s(t, h, (int)x[j] - ii, x[j] < i ? s_yn[h - 1] : s_yn[h], scale)
                              : band_pt(t, h, x[j] - i, s_yn[h], scale);
            const P3 n3 = band_pt(t, h, x[j] + i, s_yn[h], scale);
            fly[j] = fly[j] & ring_pass(n0, n1, n2, n3, a.thr, nx[j], ny[j], nz[j], p[j].x, p[j].y,
                                        p[j].z, fly[j]);
        }
    }
#pragma unroll
    for (int j = 0; j < PX; ++j) {
        bool crop = true;
        if (a.do_crop) {
            const float qx = mrow(c.Tc + 0, p[j].x, p[j].y, p[j].z, 1.0f);
            const float qy = mrow(c.Tc + 4, p[j].x, p[j].y, p[j].z, 1.0f);
            const float qz = mrow(c.Tc + 8, p[j].x, p[j].y, p[j].z, 1.0f);
            crop = !((qx < a.lo[0]) | (qx > a.hi[0]) | (qy < a.lo[1]) | (qy > a.hi[1]) |
                     (qz < a.lo[2]) | (qz > a.hi[2]));
        }
        bits[j] = (uint32_t)conv[j] | ((uint32_t)fly[j] << 1) | ((uint32_t)(fly[j] & crop) << 2);
    }
}

// ---- the two pixels of a thread in packed f32 (v_pk_mul_f32 / v_pk_add_f32) --------------------
// depth_bits_px<AMODE, 2> with the arithmetic of BOTH pixels in one packed instruction per
// operation: element 0 = pixel x, element 1 = pixel x + 128.  The packed ops round exactly like
// the scalar ones (IEEE binary32, same denormal mode, no contraction: -ffp-contract=off), and
// every operation keeps depth_bits' order, so the stage bits are bit-identical.
typedef float f2v __attribute__((ext_vector_type(2)));

struct P3x2 {
    f2v x, y, z;
    bool v0, v1;
};

__device__ __forceinline__ f2v f2(float a, float b) {
    f2v r;
    r.x = a;
    r.y = b;
    return r;
}

// neighbours (col0, row r0) and (col1, row r1) from the band (rows may differ: kRowStart's wrap)
__device__ __forceinline__ P3x2 band_pt2(const Band& t, int r0, int c0, int r1, int c1, f2v yn,
                                         float scale) {
    const uint32_t d0 = *reinterpret_cast<const uint16_t*>(t.b + t.rowoff[r0] + 2 * c0);
    const uint32_t d1 = *reinterpret_cast<const uint16_t*>(t.b + t.rowoff[r1] + 2 * c1);
    P3x2 p;
    p.z = f2((float)d0, (float)d1) * f2(scale, scale);
    p.x = f2(t.xn[c0 - (int)t.ca], t.xn[c1 - (int)t.ca]) * p.z;
    p.y = yn * p.z;
    p.v0 = d0 != 0u;
    p.v1 = d1 != 0u;
    return p;
}

__device__ __forceinline__ void ring_pass2(const P3x2& u, const P3x2& d, const P3x2& l,
                                           const P3x2& r, float thr, f2v nax, f2v nay, f2v naz,
                                           f2v px, f2v py, f2v pz, bool live0, bool live1,
                                           bool& out0, bool& out1) {
    const bool nz0 = u.v0 & d.v0 & l.v0 & r.v0;
    const bool nz1 = u.v1 & d.v1 & l.v1 & r.v1;
    const f2v ax = d.x - u.x, ay = d.y - u.y, az = d.z - u.z;  // dy = down - up
    const f2v bx = r.x - l.x, by = r.y - l.y, bz = r.z - l.z;  // dx = right - left
    const f2v cx = ay * bz - az * by;
    const f2v cy = az * bx - ax * bz;
    const f2v cz = ax * by - ay * bx;
    const f2v dd = (cx * cx + cy * cy) + cz * cz;
    const f2v dt = (cx * nax + cy * nay) + cz * naz;
    const f2v cva = dt * f2(__builtin_amdgcn_rsqf(dd.x), __builtin_amdgcn_rsqf(dd.y));
    const float hi_t = thr + 1e-5f, lo_t = thr - 1e-5f;
    const bool n0 = (dd.x > 1e-30f) & (dd.x < 1e30f), n1 = (dd.y > 1e-30f) & (dd.y < 1e30f);
    const bool hi0 = cva.x > hi_t, lo0 = cva.x < lo_t, hi1 = cva.y > hi_t, lo1 = cva.y < lo_t;
    bool pass0 = n0 & hi0, pass1 = n1 & hi1;
    const bool und0 = live0 & nz0 & !(n0 & (hi0 | lo0));
    const bool und1 = live1 & nz1 & !(n1 & (hi1 | lo1));
    if (__ballot(und0 | und1)) {  // rare, wave-uniform
        if (und0) pass0 = surface_exact(cx.x, cy.x, cz.x, dd.x, thr, px.x, py.x, pz.x);
        if (und1) pass1 = surface_exact(cx.y, cy.y, cz.y, dd.y, thr, px.y, py.y, pz.y);
    }
    out0 = nz0 & pass0;
    out1 = nz1 & pass1;
}

// the world rows of transform_points (mrow's order) for two pixels at once
template <class P>
__device__ __forceinline__ f2v mrow2(P m, f2v x, f2v y, f2v z) {
    return ((f2(m[0], m[0]) * x + f2(m[1], m[1]) * y) + f2(m[2], m[2]) * z) +
           f2(m[3], m[3]) * f2(1.0f, 1.0f);
}

// voxel_key of two points: the packed quotients, then per element voxel_axis' exact-division
// guard, clamp and floor (the same operations as voxel_key)
__device__ __forceinline__ float voxel_axis_fix(float q, float d, float cs) {
    const float r = rintf(q);
    if (__builtin_expect(fabsf(q - r) <= fabsf(q) * 9.5367431640625e-07f, 0)) return d / cs;  // 2^-20
    return q;
}
__device__ __forceinline__ void voxel_key2(f2v px, f2v py, f2v pz, const float* vlo,
                                           const float* vcs, const float* vrcs,
                                           const float* gmax, const uint32_t* gs, uint32_t& k0,
                                           uint32_t& k1) {
    const f2v dx = px - f2(vlo[0], vlo[0]), dy = py - f2(vlo[1], vlo[1]), dz = pz - f2(vlo[2], vlo[2]);
    const f2v qx = dx * f2(vrcs[0], vrcs[0]), qy = dy * f2(vrcs[1], vrcs[1]), qz = dz * f2(vrcs[2], vrcs[2]);
    float f[2][3];
    f[0][0] = voxel_axis_fix(qx.x, dx.x, vcs[0]);
    f[1][0] = voxel_axis_fix(qx.y, dx.y, vcs[0]);
    f[0][1] = voxel_axis_fix(qy.x, dy.x, vcs[1]);
    f[1][1] = voxel_axis_fix(qy.y, dy.y, vcs[1]);
    f[0][2] = voxel_axis_fix(qz.x, dz.x, vcs[2]);
    f[1][2] = voxel_axis_fix(qz.y, dz.y, vcs[2]);
    uint32_t k[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const uint32_t ux = (uint32_t)floorf(fminf(fmaxf(f[j][0], 0.0f), gmax[0]));
        const uint32_t uy = (uint32_t)floorf(fminf(fmaxf(f[j][1], 0.0f), gmax[1]));
        const uint32_t uz = (uint32_t)floorf(fminf(fmaxf(f[j][2], 0.0f), gmax[2]));
        k[j] = ux + uy * gs[0] + uz * gs[0] * gs[1];
    }
    k0 = k[0];
    k1 = k[1];
}

template <int AMODE>
__device__ __forceinline__ void depth_bits_px2(const FrameArgs& a, const CamDesc* cams, int k,
                                               const Band& t, const float* s_yn, const uint32_t* x,
                                               uint32_t y, const bool* in, uint32_t* bits) {
    const CamDesc& c = cams[k];
    const int h = t.h;
    const float scale = c.scale;
    const f2v ynh = f2(s_yn[h], s_yn[h]);
    // the centre points (a pixel outside the segment reads column x0: defined, never used)
    // (a pixel past the segment's end reads inside the band row's buffer; its point is zeroed)
    P3x2 p = band_pt2(t, h, (int)x[0], h, (int)x[1], ynh, scale);
    if (!in[0]) { p.x.x = 0.f; p.y.x = 0.f; p.z.x = 0.f; p.v0 = false; }
    if (!in[1]) { p.x.y = 0.f; p.y.y = 0.f; p.z.y = 0.f; p.v1 = false; }
    const bool conv0 = in[0] & p.v0, conv1 = in[1] & p.v1;
    const f2v pp = (p.x * p.x + p.y * p.y) + p.z * p.z;
    bool fly0 = conv0 & !beyond_max_distance(pp.x);
    bool fly1 = conv1 & !beyond_max_distance(pp.y);
    const f2v rr = f2(__builtin_amdgcn_rsqf(pp.x), __builtin_amdgcn_rsqf(pp.y));
    const f2v nx = -(p.x * rr), ny = -(p.y * rr), nz = -(p.z * rr);
    const int x0 = (int)x[0], x1 = (int)x[1];
#pragma unroll
    for (uint32_t i = 1; i <= 4; ++i) {
        if (!__ballot(fly0 | fly1)) break;  // wave-uniform exit
        const int ii = (int)i;
        fly0 = fly0 & (x[0] + i <= c.W - 1) & (y + i <= c.H - 1);
        fly1 = fly1 & (x[1] + i <= c.W - 1) & (y + i <= c.H - 1);
        const P3x2 n0 = band_pt2(t, h - ii, x0, h - ii, x1, f2(s_yn[h - ii], s_yn[h - ii]), scale);
        const P3x2 n1 = band_pt2(t, h + ii, x0, h + ii, x1, f2(s_yn[h + ii], s_yn[h + ii]), scale);
        // left: kRowStart's pixel 0 may wrap to the previous row's end (staged before column 0)
        const float ynl0 = (AMODE == kRowStart && x[0] < i) ? s_yn[h - 1] : s_yn[h];
        const P3x2 n2 = band_pt2(t, h, x0 - ii, h, x1 - ii, f2(ynl0, s_yn[h]), scale);
        const P3x2 n3 = band_pt2(t, h, x0 + ii, h, x1 + ii, ynh, scale);
        bool r0, r1;
        ring_pass2(n0, n1, n2, n3, a.thr, nx, ny, nz, p.x, p.y, p.z, fly0, fly1, r0, r1);
        fly0 = fly0 & r0;
        fly1 = fly1 & r1;
    }
    const bool fl[2] = {fly0, fly1}, cv[2] = {conv0, conv1};
    const float qxv[2] = {p.x.x, p.x.y}, qyv[2] = {p.y.x, p.y.y}, qzv[2] = {p.z.x, p.z.y};
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        bool crop = true;
        if (a.do_crop) {
            const float qx = mrow(c.Tc + 0, qxv[j], qyv[j], qzv[j], 1.0f);
            const float qy = mrow(c.Tc + 4, qxv[j], qyv[j], qzv[j], 1.0f);
            const float qz = mrow(c.Tc + 8, qxv[j], qyv[j], qzv[j], 1.0f);
            crop = !((qx < a.lo[0]) | (qx > a.hi[0]) | (qy < a.lo[1]) | (qy > a.hi[1]) |
                     (qz < a.lo[2]) | (qz > a.hi[2]));
        }
        bits[j] = (uint32_t)cv[j] | ((uint32_t)fl[j] << 1) | ((uint32_t)(fl[j] & crop) << 2);
    }
}

// emit partition: the part (key range) of voxel key k (part_of below: whole occupancy-mark words)
__device__ __forceinline__ uint32_t emit_part_of(uint32_t key, uint32_t nparts, uint64_t ncells) {
    const uint32_t p = (key >> 5) / part_slice_words(nparts, ncells);
    return p < nparts ? p : nparts - 1u;
}

// the lanes of `m` whose part equals this lane's, per distinct part of the wave (wave-uniform
// loop, one iteration per part present - usually one or two); cb(part, lanes) once per part
template <class CB>
__device__ __forceinline__ unsigned long long part_lanes(unsigned long long m, bool in, uint32_t part,
                                                         const CB& cb) {
    unsigned long long mine = 0;
    unsigned long long rem = m;
    while (rem) {
        const int l = __ffsll((long long)rem) - 1;
        const uint32_t p = __shfl(part, l, 64);
        const unsigned long long pm = __ballot(in && part == p) & m;
        if (in && part == p) mine = pm;
        cb(p, pm);
        rem &= ~pm;
    }
    return mine;
}

// k_mask with PX pixels per thread (x + j * 256 / PX) for 256-pixel segments at F = 4 without
// rot45: 256 / PX threads per segment, the same band in LDS, the same outputs (validity word
// w + j * waves from pixel j of wave w; counts, runs, run-key histogram).  No debug stage bits
// (the engine launches k_mask for those).
#ifdef GDF_TRACE_GROUPS
// (diagnostic build, tools/mask_trace.py) per k_mask_px block: wall clock at entry and
// exit, then wave 0's cycles in each phase - segment geometry and camera, band loads landed, LDS
// stores + barrier, the filter, the ballots + publish barrier, the scan tail - each phase closed by
// a wait for this wave's outstanding memory operations (which the product kernel does not do)
constexpr uint32_t kMaskTraceSlots = 1u << 14;
__device__ unsigned long long g_mtrace[kMaskTraceSlots][8];
#define GDF_MSTAMP(i)               \
    __builtin_amdgcn_s_waitcnt(0);  \
    mt[i] = clock64()
#endif

template <int PX, int SEGW>
__device__ __forceinline__ void mask_px_body(const FrameArgs& a) {
#ifdef GDF_TRACE_GROUPS
    const unsigned long long mw0 = wall_clock64();
    unsigned long long mt[7] = {};
    GDF_MSTAMP(0);
#endif
    constexpr int NT = SEGW / PX, NW = NT / 64;          // threads, waves
    constexpr int NWORDS = SEGW / 64;                    // validity words of a segment
    constexpr int NBR = 2 * 4 + 1;                       // band rows (h = 4)
    constexpr int QR = (NBR + NW - 1) / NW;              // band rows per wave
    constexpr int QX = (SEGW + 2 * 4 + NT - 1) / NT;     // ray factors per thread
    constexpr int QC = (((SEGW + 8) * 2 + 15) / 16 + 1 + 63) / 64;  // 16-B chunks per lane and row
    // the segment's camera only (occupancy: 16 descriptors were 3.3 KB of LDS per block; the first
    // rows' general path reads the others from the argument table)
    __shared__ CamDesc s_cams[1];
    __shared__ float s_yn[2 * kHalo + 1];
    __shared__ int s_rowoff[2 * kHalo + 1];
    __shared__ uint32_t s_cnt[NWORDS];
    __shared__ uint32_t s_rcnt[NWORDS];
    __shared__ uint32_t s_pc[2][NWORDS][kMaxParts];  // emit partition: points, runs per (word, part)
    extern __shared__ uint4 s_dyn[];
    // run-key digit histogram: dynamic LDS behind the band, only when the launch counts digits
    uint32_t* s_hist = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(s_dyn) + a.hist_lds);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (a.nparts)
        for (uint32_t j = threadIdx.x; j < 2u * NWORDS * kMaxParts; j += NT) (&s_pc[0][0][0])[j] = 0u;
    const uint32_t n = gridDim.x, q8 = n / 8, r8 = n % 8, xcd = blockIdx.x % 8;
    const uint32_t s = xcd * q8 + min(xcd, r8) + blockIdx.x / 8;  // the block's segment
    uint32_t bits[PX], rkey[PX];
#pragma unroll
    for (int j = 0; j < PX; ++j) {
        bits[j] = 0u;
        rkey[j] = 0xFFFFFFFFu;
    }
    const uint32_t i = threadIdx.x;
    if (a.run_mode && a.key_hist)
        for (uint32_t j = threadIdx.x; j < radix_hist_span(a.npasses); j += NT) s_hist[j] = 0;
    {
        const gptr<const CamDesc> gcam = G(cam_table(a));
        SegGeo sg = seg_geo(gcam, a.ncams, s, a.seg_uniform);
        struct {
            const uint16_t* depth;
            const float *xn, *yn;
            uint32_t W, H;
        } c = {gcam[sg.k].depth, gcam[sg.k].xn, gcam[sg.k].yn, gcam[sg.k].W, gcam[sg.k].H};
#ifdef GDF_TRACE_GROUPS
        asm volatile("" ::"s"(c.depth), "s"(c.W));  // (the camera's fields before the stamp)
        GDF_MSTAMP(1);
#endif
        const int h = 4;  // (F = 4: the launch checks it)
        const uint32_t ca = sg.x0 >= (uint32_t)h ? sg.x0 - h : 0u;
        const uint32_t cb = min(c.W, sg.x0 + sg.len + h);
        const uint32_t nrows = 2 * h + 1;
        uint8_t* band = reinterpret_cast<uint8_t*>(s_dyn);
        float* s_xn = reinterpret_cast<float*>(band + (size_t)nrows * a.band_rowb) + kHalo;
        const bool wrap = sg.x0 == 0 && sg.y >= (uint32_t)h && c.W >= (uint32_t)h;
        typedef uint32_t u4v __attribute__((ext_vector_type(4)));
        const uintptr_t dbase = reinterpret_cast<uintptr_t>(c.depth);
        const uint32_t nch = a.band_rowb / 16;  // <= 64 QC (the launch checks it)
        // rows wid, wid + NW, ...: every load before any store
        u4v v[QR][QC];
        uintptr_t a16[QR], col0[QR];
        uint32_t n16[QR];
        bool rok[QR];
#pragma unroll
        for (int q = 0; q < QR; ++q) {
            const uint32_t r = (uint32_t)wid + (uint32_t)NW * q;
            const int gy = (int)sg.y - h + (int)r;
            rok[q] = r < nrows && gy >= 0 && gy < (int)c.H;
            n16[q] = 0;
            a16[q] = col0[q] = 0;
            if (rok[q]) {
                col0[q] = dbase + 2 * ((uintptr_t)gy * c.W + ca);
                // (the pixel row of a row-start segment: the previous row's end before column 0)
                const bool pix_row = r == (uint32_t)h;
                const uintptr_t first = col0[q] - (wrap && pix_row ? 2 * (uintptr_t)h : 0);
                const uintptr_t last = dbase + 2 * ((uintptr_t)gy * c.W + cb);
                a16[q] = first & ~(uintptr_t)15;
                n16[q] = min((uint32_t)((last - a16[q] + 15) / 16), nch);
#pragma unroll
                for (int cq = 0; cq < QC; ++cq) {
                    const uint32_t ch = (uint32_t)lane + 64u * cq;
                    if (ch < n16[q]) v[q][cq] = *(gptr<const u4v>)(a16[q] + 16 * (uintptr_t)ch);
                }
            }
        }
#ifdef GDF_TRACE_GROUPS
        GDF_MSTAMP(2);
#endif
        const uint32_t tb = threadIdx.x;
        float xv[QX];
#pragma unroll
        for (int q = 0; q < QX; ++q)
            xv[q] = ca + tb + (uint32_t)NT * q < cb ? G(c.xn)[ca + tb + (uint32_t)NT * q] : 0.0f;
        // the row factors, the wrap columns' ray factors and the camera descriptor: loaded
        // unconditionally at clamped indices with the band, stored after (a load in its own
        // branch waited for every load before it: a second round)
        const int gyi = (int)sg.y - h + (int)tb;
        const bool yin = tb < nrows && gyi >= 0 && gyi < (int)c.H;
        const float ynl = G(c.yn)[min((uint32_t)max(gyi, 0), c.H - 1u)];
        const float xwl = G(c.xn)[tb < c.W ? c.W - 1u - tb : 0u];
        static_assert(sizeof(CamDesc) / 4 <= (size_t)NT, "one descriptor word per thread");
        const uint32_t* csrc = reinterpret_cast<const uint32_t*>(cam_table(a) + sg.k);
        const uint32_t cdw = G(csrc)[min(threadIdx.x, (uint32_t)(sizeof(CamDesc) / 4) - 1u)];
        if (tb < nrows) s_yn[tb] = yin ? ynl : 0.0f;
        const float xwv = wrap && tb < (uint32_t)h ? xwl : 0.0f;
        if (threadIdx.x < (uint32_t)(sizeof(CamDesc) / 4))  // camera sg.k's descriptor into LDS
            reinterpret_cast<uint32_t*>(s_cams)[threadIdx.x] = cdw;
#pragma unroll
        for (int q = 0; q < QR; ++q) {
            const uint32_t r = (uint32_t)wid + (uint32_t)NW * q;
            if (r < nrows) {
#pragma unroll
                for (int cq = 0; cq < QC; ++cq) {
                    const uint32_t ch = (uint32_t)lane + 64u * cq;
                    if (rok[q] && ch < n16[q])
                        *reinterpret_cast<u4v*>(band + r * a.band_rowb + 16 * ch) = v[q][cq];
                }
                if (lane == 0)
                    s_rowoff[r] = (int)(r * a.band_rowb) - 2 * (int)ca + (rok[q] ? (int)(col0[q] - a16[q]) : 0);
            }
        }
#pragma unroll
        for (int q = 0; q < QX; ++q)
            if (ca + tb + (uint32_t)NT * q < cb) s_xn[tb + (uint32_t)NT * q] = xv[q];
        if (wrap && tb < (uint32_t)h) s_xn[-1 - (int)tb] = xwv;
        __syncthreads();
#ifdef GDF_TRACE_GROUPS
        GDF_MSTAMP(3);
#endif
        const Band t{band, s_xn, s_rowoff, ca, h};
        const float* s_ynr = s_yn;
        if (64u * (uint32_t)wid < sg.len) {  // wave-uniform
            const uint32_t xw0 = sg.x0 + 64u * wid;
            uint32_t x[PX];
            bool in[PX];
#pragma unroll
            for (int j = 0; j < PX; ++j) {
                x[j] = sg.x0 + i + (uint32_t)NT * j;
                in[j] = i + (uint32_t)NT * j < sg.len;
            }
            if (PX == 2 && a.mask_packed && sg.y >= 4u && xw0 >= 4u)
                depth_bits_px2<kInterior>(a, s_cams, 0, t, s_ynr, x, sg.y, in, bits);
            else if (PX == 2 && a.mask_packed && wrap)
                depth_bits_px2<kRowStart>(a, s_cams, 0, t, s_ynr, x, sg.y, in, bits);
            else if (sg.y >= 4u && xw0 >= 4u)
                depth_bits_px<kInterior, PX>(a, s_cams, 0, t, s_ynr, x, sg.y, in, bits);
            else if (wrap)
                depth_bits_px<kRowStart, PX>(a, s_cams, 0, t, s_ynr, x, sg.y, in, bits);
            else
#pragma unroll
                for (int j = 0; j < PX; ++j)
                    bits[j] = depth_bits<false, kGeneral, 4>(a, reinterpret_cast<const CamDesc*>(cam_table(a)), sg.k, t, s_ynr, x[j], sg.y, in[j]);
            if (a.run_mode && PX == 2 && a.mask_packed) {  // both pixels' keys in packed f32
                const CamDesc& cd = s_cams[0];
                if ((bits[0] | bits[PX - 1]) & 4u) {
                    const P3x2 p = band_pt2(t, h, (int)x[0], h, (int)x[PX - 1],
                                            f2(s_ynr[h], s_ynr[h]), cd.scale);
                    uint32_t k0, k1;
                    voxel_key2(mrow2(cd.Tw + 0, p.x, p.y, p.z), mrow2(cd.Tw + 4, p.x, p.y, p.z),
                               mrow2(cd.Tw + 8, p.x, p.y, p.z), a.vlo, a.vcs, a.vrcs, a.gmax, a.gs,
                               k0, k1);
                    if (bits[0] & 4u) rkey[0] = k0 | (cd.frame << a.frame_shift);
                    if (bits[PX - 1] & 4u) rkey[PX - 1] = k1 | (cd.frame << a.frame_shift);
                }
            } else if (a.run_mode) {
                const CamDesc& cd = s_cams[0];
#pragma unroll
                for (int j = 0; j < PX; ++j)
                    if (bits[j] & 4u) {  // the voxel key k_emit will compute (same f32 ops)
                        const P3 p = band_pt(t, h, x[j], s_ynr[h], cd.scale);
                        const float wx = mrow(cd.Tw + 0, p.x, p.y, p.z, 1.0f);
                        const float wy = mrow(cd.Tw + 4, p.x, p.y, p.z, 1.0f);
                        const float wz = mrow(cd.Tw + 8, p.x, p.y, p.z, 1.0f);
                        rkey[j] = voxel_key(wx, wy, wz, a.vlo, a.vcs, a.vrcs, a.gmax, a.gs) |
                                  (cd.frame << a.frame_shift);
                    }
            }
        }
    }
#ifdef GDF_TRACE_GROUPS
    GDF_MSTAMP(4);
#endif
#pragma unroll
    for (int j = 0; j < PX; ++j) {
        const uint32_t word = (uint32_t)wid + (uint32_t)NW * j;
        const unsigned long long m = __ballot((bits[j] & 4u) != 0u);
        if (lane == 0) {
            G(a.vbits)[(size_t)s * 16 + word] = m;
            s_cnt[word] = (uint32_t)__popcll(m);
        }
        if (a.run_mode) {
            const unsigned long long below = m & lanemask_lt();
            const int prev = below ? 63 - __clzll((long long)below) : -1;
            const uint32_t pkey = __shfl(rkey[j], prev < 0 ? 0 : prev, 64);
            const bool leader = ((bits[j] & 4u) != 0u) && (prev < 0 || pkey != rkey[j]);
            const unsigned long long lm = __ballot(leader);
            if (lane == 0) {
                G(a.wave_runs)[(size_t)s * 16 + word] = (uint32_t)__popcll(lm);
                s_rcnt[word] = (uint32_t)__popcll(lm);
            }
            if (leader && a.key_hist)
                for (uint32_t p = 0; p < a.npasses; ++p)
                    atomicAdd(&s_hist[p * 256 + radix_digit(rkey[j], p, a.npasses)], 1u);
            if (a.nparts) {  // this word's kept points and runs per part
                const bool kept = (bits[j] & 4u) != 0u;
                const uint32_t vk = a.frame_shift ? rkey[j] & ((1u << a.frame_shift) - 1u) : rkey[j];
                const uint32_t part = kept ? emit_part_of(vk, a.nparts, a.part_ncells) : 0u;
                part_lanes(m, kept, part, [&](uint32_t p, unsigned long long pm) {
                    if (lane == 0) {
                        s_pc[0][word][p] = (uint32_t)__popcll(pm);
                        s_pc[1][word][p] = (uint32_t)__popcll(pm & lm);
                    }
                });
            }
        }
    }
    __syncthreads();
#ifdef GDF_TRACE_GROUPS
    GDF_MSTAMP(5);
#endif
    // (the first wave publishes the segment)
    if (wid == 0) {
        if (a.nparts) {  // counts [points of part 0..P-1 | runs of part 0..P-1][segment]
            if ((uint32_t)lane < 2u * a.nparts) {
                const uint32_t kind = lane / a.nparts, p = lane % a.nparts;
                uint32_t c = 0;
                for (int w = 0; w < NWORDS; ++w) c += s_pc[kind][w][p];
                G(a.seg_counts)[(size_t)lane * a.total_segs + s] = c;
            }
        } else if (lane == 0) {
            uint32_t tt = 0, r = 0;
            for (int w = 0; w < NWORDS; ++w) tt += s_cnt[w];
            publish_count(a.seg_counts + s, tt);
            if (a.run_mode) {
                for (int w = 0; w < NWORDS; ++w) r += s_rcnt[w];
                publish_count(a.seg_counts + a.total_segs + s, r);
            }
        }
    }
    if (a.run_mode && a.key_hist) {
        const gptr<uint32_t> rep = G(a.key_hist + (blockIdx.x % kHistReps) * 1024u);
        for (uint32_t j = threadIdx.x; j < radix_hist_span(a.npasses); j += NT)
            if (s_hist[j])
                __hip_atomic_fetch_add(rep + j, s_hist[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // (stored after the descriptor reads: a global store before them keeps the compiler from
    // reading the camera fields with scalar loads)
    if (a.grid_seq_out && blockIdx.x == 0 && threadIdx.x == 0) *a.grid_seq_out = a.grid_seq;
    group_scan_tail(a, s);
#ifdef GDF_TRACE_GROUPS
    GDF_MSTAMP(6);
    if (threadIdx.x == 0 && blockIdx.x < kMaskTraceSlots) {
        unsigned long long* g = g_mtrace[blockIdx.x];
        g[0] = mw0;
        g[1] = wall_clock64();
        for (int k = 1; k < 7; ++k) g[k + 1] = mt[k] - mt[k - 1];
    }
#endif
}

template <int PX, int SEGW>
__global__ __launch_bounds__(SEGW / PX) void k_mask_px(FrameArgs a) {
    mask_px_body<PX, SEGW>(a);
}
// the same at 8 waves per SIMD (<= 64 VGPRs, a few spilled): tuning knob GDF_MASK_OCC8
template <int PX, int SEGW>
__global__ __launch_bounds__(SEGW / PX) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_mask_px_o8(FrameArgs a) {
    mask_px_body<PX, SEGW>(a);
}

// Exclusive scan of the segment counts by one workgroup (chunks of 4096 with a running carry);
// writes the total (m_numItemsAfterMask).  Used when there are more than kFusedPrefixSegs.
// Reduce-then-scan over chunks of 4096 counts: k_scan_reduce sums chunk b into partial[b];
// k_scan_counts block b starts from the sum of the partials before it and scans its chunk.
__device__ __forceinline__ uint32_t block_sum_1024(uint32_t v, uint32_t* s_w) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) s_w[wid] = v;
    __syncthreads();
    uint32_t t = 0;
#pragma unroll
    for (int w = 0; w < 16; ++w) t += s_w[w];
    return t;
}

// (mdev: the number of counts is ceil(*mdev / per) <= m, read on the device)
__device__ __forceinline__ uint32_t scan_len(uint32_t m, const uint32_t* mdev, uint32_t per) {
    return mdev ? min(m, (*mdev + per - 1u) / per) : m;
}

__global__ __launch_bounds__(1024) void k_scan_reduce(const uint32_t* __restrict__ counts,
                                                      uint32_t m, uint32_t* __restrict__ partial,
                                                      const uint32_t* mdev, uint32_t per) {
    __shared__ uint32_t s_w[16];
    m = scan_len(m, mdev, per);
    if (blockIdx.x * 4096u >= m && blockIdx.x) return;
    uint32_t v = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t i = blockIdx.x * 4096u + threadIdx.x * 4 + q;
        v += i < m ? counts[i] : 0u;
    }
    const uint32_t t = block_sum_1024(v, s_w);
    if (threadIdx.x == 0) partial[blockIdx.x] = t;
}

__global__ __launch_bounds__(1024) void k_scan_counts(const uint32_t* __restrict__ counts,
                                                      uint32_t m, uint32_t* __restrict__ offsets,
                                                      uint32_t* __restrict__ total,
                                                      const uint32_t* __restrict__ partial,
                                                      const uint32_t* mdev, uint32_t per) {
    __shared__ uint32_t s_w[16];
    __shared__ uint32_t s_carry;
    m = scan_len(m, mdev, per);
    const uint32_t chunks = (m + 4095u) / 4096u;
    if (blockIdx.x >= chunks && blockIdx.x) return;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    {
        uint32_t v = 0;
        for (uint32_t b = threadIdx.x; b < blockIdx.x; b += 1024) v += partial[b];
        const uint32_t c = block_sum_1024(v, s_w);
        if (threadIdx.x == 0) s_carry = c;
        __syncthreads();
    }
    // (one block: every chunk in turn with the running carry - no k_scan_reduce launch)
    const uint32_t end = gridDim.x == 1 ? m : min(m, blockIdx.x * 4096u + 4096u);
    for (uint32_t base = blockIdx.x * 4096u; base < end; base += 4096) {
        uint32_t v[4], sum = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t i = base + threadIdx.x * 4 + q;
            v[q] = i < m ? counts[i] : 0u;
            sum += v[q];
        }
        uint32_t x = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) s_w[wid] = x;
        __syncthreads();
        uint32_t wb = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < 16; ++w) {
            const uint32_t t = s_w[w];
            wb += (w < wid) ? t : 0u;
            tot += t;
        }
        uint32_t run = s_carry + wb + x - sum;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t i = base + threadIdx.x * 4 + q;
            if (i < m) offsets[i] = run;
            run += v[q];
        }
        __syncthreads();
        if (threadIdx.x == 0) s_carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0 && blockIdx.x == min(chunks ? chunks - 1u : 0u, gridDim.x - 1u) && total)
        *total = s_carry;
}

// Exclusive scan of m counts (mdev: the device-side length, see scan_len).  Up to
// kScanOneBlockChunks chunks of 4096: ONE k_scan_counts block walks them with a running carry
// (one dependent launch); above: k_scan_reduce over the chunks, then a block per chunk.
// (measured on MI355X, 8-frame VGA batches, 19.2 K counts = 5 chunks: one block walking them
// 17.4 us vs 10.8 us for reduce + 5 blocks - the walk serialises a load round trip per chunk)
constexpr uint32_t kScanOneBlockChunks = 1;
static hipError_t launch_scan(const uint32_t* counts, uint32_t m, uint32_t* offsets, uint32_t* total,
                              const uint32_t* mdev, uint32_t per, hipStream_t s) {
    const uint32_t chunks = (m + 4095u) / 4096u;
    uint32_t* partial = offsets + scan_partials_offset(m);
    if (chunks <= kScanOneBlockChunks) {
        hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(1024), 0, s, counts, m, offsets, total,
                           (const uint32_t*)partial, mdev, per);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(k_scan_reduce, dim3(chunks), dim3(1024), 0, s, counts, m, partial, mdev, per);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_scan_counts, dim3(chunks), dim3(1024), 0, s, counts, m, offsets, total,
                       (const uint32_t*)partial, mdev, per);
    return hipGetLastError();
}

// Pass 2: item-ordered emission, one block per segment.  Each valid item recomputes its world
// point with the same f32 ops as pass 1 and writes it at segment offset + rank: stable pixel
// order, cameras in add order, selected rollbuffer points after the depth points
// (fusion.cpp:1525,1559).  Optionally the voxel key (compute_voxel_coords), the occupancy mark
// (no-return atomic OR of bit 7, issued once per run of equal keys in a wave) and the key digit
// histogram.  The segment offset is the sum of the preceding counts (<= kFusedPrefixSegs
// segments) or k_scan_counts' result.
// occupancy mark + digit histogram of the wave's kept items (voxel_grid_occupancy_of_points):
// runs of equal keys among the valid lanes - the first lane of a run marks / counts
constexpr int kMarkCacheBits = 9;

__device__ __forceinline__ void mark_and_count(const FrameArgs& a, uint32_t* marks, bool valid,
                                               uint32_t key, uint32_t hkey, uint32_t* s_hist,
                                               uint32_t* s_mark) {
    const int lane = threadIdx.x & 63;
    const unsigned long long ltm = lanemask_lt();
    const unsigned long long vm = __ballot(valid);
    const unsigned long long below = vm & ltm;
    const int prev = below ? 63 - __clzll((long long)below) : -1;
    const uint32_t pkey = __shfl(key, prev < 0 ? 0 : prev, 64);
    const bool leader = valid && (prev < 0 || pkey != key);
    const unsigned long long lm = __ballot(leader);
    if (leader) {
        // a key this block already marked needs no second device-scope atomic: s_mark is a
        // direct-mapped cache of marked keys (a lane only skips a key some lane wrote AFTER
        // issuing its atomic; collisions just mark again)
        uint32_t& slot = s_mark[(key * 0x9E3779B1u) >> (32 - kMarkCacheBits)];
        if (marks && slot != key) {
            slot = key;
            __hip_atomic_fetch_or(G(marks + (key >> 5)), 1u << (key & 31u), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
        }
        if (a.key_hist && s_hist) {
            const unsigned long long after = lm & ~(ltm | (1ull << lane));
            const unsigned long long upto =
                after ? ((1ull << (__ffsll((long long)after) - 1)) - 1ull) : ~0ull;
            const uint32_t rl = (uint32_t)__popcll(vm & ~ltm & upto);
            for (uint32_t p = 0; p < a.npasses; ++p)
                atomicAdd(&s_hist[p * 256 + radix_digit(hkey, p, a.npasses)], rl);
        }
    }
}

__device__ __forceinline__ void flush_hist(const FrameArgs& a, uint32_t* s_hist) {
    if (!a.key_hist) return;
    __syncthreads();
    const gptr<uint32_t> rep = G(a.key_hist + (blockIdx.x % kHistReps) * 1024u);
    for (uint32_t j = threadIdx.x; j < radix_hist_span(a.npasses); j += blockDim.x)
        if (s_hist[j])
            __hip_atomic_fetch_add(rep + j, s_hist[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// sum of the counts of segments [0, s) by the block (fused-prefix form), into s_red per wave
// (run mode: the run counts of those segments too, into s_red + 16)
__device__ __forceinline__ void prefix_partials(const FrameArgs& a, uint32_t s, uint32_t* s_red) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t sum = 0, rsum = 0;
    for (uint32_t t = threadIdx.x; t < s; t += blockDim.x) {
        sum += G(a.seg_counts)[t];
        if (a.run_mode) rsum += G(a.seg_counts)[a.total_segs + t];
    }
    for (int o = 32; o > 0; o >>= 1) {
        sum += __shfl_xor(sum, o, 64);
        rsum += __shfl_xor(rsum, o, 64);
    }
    if (lane == 0) {
        s_red[wid] = sum;
        s_red[16 + wid] = rsum;
    }
}

// prefix of the valid counts of the waves before this one in segment s (uniform word loads)
__device__ __forceinline__ uint32_t wave_prefix(const FrameArgs& a, uint32_t s, uint32_t& tot) {
    const int wid = threadIdx.x >> 6, nwaves = blockDim.x >> 6;
    uint32_t wpre = 0;
    tot = 0;
    for (int w = 0; w < nwaves; ++w) {
        const uint32_t pc = (uint32_t)__popcll(G(a.vbits)[(size_t)s * 16 + w]);
        wpre += (w < wid) ? pc : 0u;
        tot += pc;
    }
    return wpre;
}

// Pass 2: item-ordered emission, one block per depth segment.  Each valid item recomputes its
// world point with the same f32 ops as pass 1 and writes it at segment offset + rank: stable pixel
// order, cameras in add order, selected rollbuffer points after the depth points
// (fusion.cpp:1525,1559).  Optionally the voxel key (compute_voxel_coords), the occupancy mark
// (no-return atomic OR, issued once per run of equal keys in a wave) and the key digit
// histogram.  The segment offset is the sum of the preceding counts (<= kFusedPrefixSegs
// segments) or k_scan_counts' result.
__global__ __launch_bounds__(1024) void k_emit(FrameArgs a) {
    __shared__ uint32_t s_hist[4 * 256];
    __shared__ uint32_t s_red[32];
    __shared__ uint32_t s_mark[1u << kMarkCacheBits];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int nwaves = blockDim.x >> 6;
    const uint32_t s = blockIdx.x;
    for (uint32_t j = threadIdx.x; j < (1u << kMarkCacheBits); j += blockDim.x) s_mark[j] = 0xFFFFFFFFu;
    const gptr<const CamDesc> cams = G(cam_table(a));
    const bool hist = a.key_hist && !a.run_mode;  // (run mode: k_mask counted the run keys)
    if (hist)
        for (uint32_t i = threadIdx.x; i < radix_hist_span(a.npasses); i += blockDim.x) s_hist[i] = 0;
    if (a.fused_prefix) prefix_partials(a, s, s_red);
    else if (a.grp_tot) group_partials(a, s, s_red);
    // the segment's geometry and the thread's item source, loaded before the barrier
    const uint32_t i = threadIdx.x;
    int k = seg_camera(cams, a.ncams, s, a.seg_uniform);
    // block-uniform camera: its descriptor (device copy beyond kArgCams cameras) is read with
    // scalar loads, not once per lane
    k = __builtin_amdgcn_readfirstlane(k);
    const uint32_t j = s - cams[k].seg0;
    const uint32_t y = j / cams[k].nchunk;
    const uint32_t x0 = (j - y * cams[k].nchunk) * cams[k].segw;
    const uint32_t len = min(cams[k].segw, cams[k].W - x0);
    // the validity word, the depth and the column's ray factor are independent loads: all in
    // flight together (the depth of a pixel the crop dropped is read for nothing - it is in L2
    // from k_mask - instead of waiting for the validity word first)
    const unsigned long long m = G(a.vbits)[(size_t)s * 16 + wid];
    uint32_t dval = 0;
    float xnv = 0.0f;
    if (i < len) {
        dval = G(cams[k].depth)[y * cams[k].W + x0 + i];
        xnv = G(cams[k].xn)[x0 + i];
    }
    const float ynv = G(cams[k].yn)[y];
    const bool valid = i < len && ((m >> lane) & 1ull);
    uint32_t tot;
    const uint32_t wpre = wave_prefix(a, s, tot);
    const uint32_t sbase = a.fused_prefix ? 0u : G(a.seg_offsets)[s];
    // run mode: this segment's first run (the scan over points then runs: minus all points)
    uint32_t rbase = 0, rwpre = 0, rtot = 0;
    if (a.run_mode) {
        if (!a.fused_prefix)  // (group scan: offsets local to the group's runs)
            rbase = G(a.seg_offsets)[a.total_segs + s] -
                    (a.grp_tot ? 0u : G(a.seg_offsets)[a.total_segs]);
        for (int w = 0; w < nwaves; ++w) {
            const uint32_t rc = G(a.wave_runs)[(size_t)s * 16 + w];
            rwpre += (w < wid) ? rc : 0u;
            rtot += rc;
        }
    }
    __syncthreads();
    uint32_t base = sbase;
    if (a.fused_prefix || a.grp_tot)
        for (int w = 0; w < nwaves; ++w) {
            base += s_red[w];
            rbase += s_red[16 + w];
        }
    if (s == gridDim.x - 1 && threadIdx.x == 0) {
        *G(a.out_count) = base + tot;
        if (a.run_mode) {  // the runs' end sentinel and count
            G(a.run_start)[rbase + rtot] = base + tot;
            *G(a.run_count) = rbase + rtot;
        }
    }
    const uint32_t fr = cams[k].frame;
    if (a.frame_pt_start && threadIdx.x == 0) {  // point range of each frame of a batch
        const bool first_of_frame =
            s == cams[k].seg0 && (k == 0 || !cams[k - 1].emit || cams[k - 1].frame != fr);
        if (first_of_frame) G(a.frame_pt_start)[fr] = base;
        if (s == gridDim.x - 1) G(a.frame_pt_start)[a.nframes] = base + tot;
    }
    const unsigned long long ltm = lanemask_lt();
    uint32_t key = 0xFFFFFFFFu;
    if (valid) {
        const uint32_t pos = base + wpre + (uint32_t)__popcll(m & ltm);
        const uint32_t x = x0 + i;
        const float zz = (float)dval * cams[k].scale;
        const float px = xnv * zz, py = ynv * zz, pz = zz;
        (void)x;
        const float4 w = make_float4(mrow(cams[k].Tw + 0, px, py, pz, 1.0f),
                                     mrow(cams[k].Tw + 4, px, py, pz, 1.0f),
                                     mrow(cams[k].Tw + 8, px, py, pz, 1.0f),
                                     mrow(cams[k].Tw + 12, px, py, pz, 1.0f));
        gst4(a.out_pts, pos, w);
        if (a.do_voxel) {
            key = voxel_key(w.x, w.y, w.z, a.vlo, a.vcs, a.vrcs, a.gmax, a.gs);
            G(a.out_coords)[pos] = key;
        }
    }
    if (a.run_mode) {  // run leaders: the sort key and first point of each run (k_mask's runs)
        const unsigned long long below = m & ltm;
        const int prev = below ? 63 - __clzll((long long)below) : -1;
        const uint32_t pkey = __shfl(key, prev < 0 ? 0 : prev, 64);
        const bool leader = valid && (prev < 0 || pkey != key);
        const unsigned long long lm = __ballot(leader);
        if (leader) {
            const uint32_t ri = rbase + rwpre + (uint32_t)__popcll(lm & ltm);
            G(a.run_keys)[ri] = key | (fr << a.frame_shift);
            G(a.run_start)[ri] = base + wpre + (uint32_t)__popcll(m & ltm);
        }
    }
    if (a.do_voxel)
        mark_and_count(a, a.marks ? a.marks + (size_t)fr * a.mark_words : nullptr, valid, key,
                       key | (fr << a.frame_shift), hist ? s_hist : nullptr, s_mark);
    if (hist) flush_hist(a, s_hist);
}

// k_emit for 256-pixel segments with two pixels per thread (x, x + 128; 128 threads per
// segment, k_mask_px's layout: pixel j of wave w is validity word w + 2j): the block's scalar
// work (camera lookup, counts and run prefixes of the segment's words) is shared by twice the
// pixels per wave.  Same outputs in the same order as k_emit.
// k_emit_px2 under the emit partition (FrameArgs::nparts): the same points, keys and marks; each
// kept point goes to its part (the segment's offset of the part from the one scan over [points
// per part | runs per part][segment], then the part's earlier words, then its rank among the
// word's lanes of that part), and each run (a kept pixel whose key differs from the kept pixel
// before it in the word) to its part's run list.
template <int SEGW>
__device__ __forceinline__ void emit_px2_parts(const FrameArgs& a, uint32_t* s_mark) {
    constexpr int NT = SEGW / 2, NW = NT / 64, NWORDS = SEGW / 64;
    __shared__ uint32_t s_pc[2][NWORDS][kMaxParts];
    __shared__ uint32_t s_off[2][kMaxParts], s_first[kMaxParts], s_tot;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t s = blockIdx.x, P = a.nparts, TS = a.total_segs;
    for (uint32_t j = threadIdx.x; j < 2u * NWORDS * kMaxParts; j += NT) (&s_pc[0][0][0])[j] = 0u;
    if (threadIdx.x < 2u * P) {
        const uint32_t kind = threadIdx.x / P, p = threadIdx.x % P;
        s_off[kind][p] = G(a.seg_offsets)[(size_t)threadIdx.x * TS + s];
        if (kind == 0) s_first[p] = G(a.seg_offsets)[(size_t)p * TS];
    }
    if (threadIdx.x == 0) s_tot = G(a.seg_offsets)[(size_t)P * TS];  // (the kept points)
    __syncthreads();  // (the zeroed counters and the mark cache before any wave writes them)
    const gptr<const CamDesc> cams = G(cam_table(a));
    const uint32_t i = threadIdx.x;
    int k = seg_camera(cams, a.ncams, s, a.seg_uniform);
    k = __builtin_amdgcn_readfirstlane(k);
    const uint32_t j = s - cams[k].seg0;
    const uint32_t y = j / cams[k].nchunk;
    const uint32_t x0 = (j - y * cams[k].nchunk) * cams[k].segw;
    const uint32_t len = min(cams[k].segw, cams[k].W - x0);
    uint64_t m[2];
    uint32_t dval[2] = {0u, 0u};
    float xnv[2] = {0.0f, 0.0f};
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        m[q] = G(a.vbits)[(size_t)s * 16 + wid + NW * q];
        const uint32_t ii = i + (uint32_t)NT * q;
        if (ii < len) {
            dval[q] = G(cams[k].depth)[y * cams[k].W + x0 + ii];
            xnv[q] = G(cams[k].xn)[x0 + ii];
        }
    }
    const float ynv = G(cams[k].yn)[y];
    const uint32_t fr = cams[k].frame;
    const unsigned long long ltm = lanemask_lt();
    const f2v zz2 = f2((float)dval[0], (float)dval[1]) * f2(cams[k].scale, cams[k].scale);
    const f2v px2 = f2(xnv[0], xnv[1]) * zz2, py2 = f2(ynv, ynv) * zz2, pz2 = zz2;
    const f2v wx2 = mrow2(cams[k].Tw + 0, px2, py2, pz2), wy2 = mrow2(cams[k].Tw + 4, px2, py2, pz2);
    const f2v wz2 = mrow2(cams[k].Tw + 8, px2, py2, pz2), ww2 = mrow2(cams[k].Tw + 12, px2, py2, pz2);
    uint32_t key2[2] = {0xFFFFFFFFu, 0xFFFFFFFFu};
    if (m[0] | m[1]) voxel_key2(wx2, wy2, wz2, a.vlo, a.vcs, a.vrcs, a.gmax, a.gs, key2[0], key2[1]);
    bool valid[2], lead[2];
    uint32_t part[2];
    unsigned long long mine[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const uint32_t word = (uint32_t)wid + NW * q;
        valid[q] = i + (uint32_t)NT * q < len && ((m[q] >> lane) & 1ull);
        const uint32_t key = valid[q] ? key2[q] : 0xFFFFFFFFu;
        const unsigned long long below = m[q] & ltm;
        const int prev = below ? 63 - __clzll((long long)below) : -1;
        const uint32_t pkey = __shfl(key, prev < 0 ? 0 : prev, 64);
        lead[q] = valid[q] && (prev < 0 || pkey != key);
        const unsigned long long lm = __ballot(lead[q]);
        part[q] = valid[q] ? emit_part_of(key2[q], P, a.part_ncells) : 0u;
        mine[q] = part_lanes(m[q], valid[q], part[q], [&](uint32_t p, unsigned long long pm) {
            if (lane == 0) {
                s_pc[0][word][p] = (uint32_t)__popcll(pm);
                s_pc[1][word][p] = (uint32_t)__popcll(pm & lm);
            }
        });
        mine[q] &= valid[q] ? ~0ull : 0ull;
        // (the leaders among this lane's part: runs ranked within the word)
        if (!valid[q]) lead[q] = false;
        mark_and_count(a, a.marks ? a.marks + (size_t)fr * a.mark_words : nullptr, valid[q], key,
                       key | (fr << a.frame_shift), nullptr, s_mark);
        (void)lm;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const uint32_t word = (uint32_t)wid + NW * q;
        const unsigned long long lm = __ballot(lead[q]);
        if (!valid[q]) continue;
        const uint32_t p = part[q];
        uint32_t wpre = 0, rwpre = 0;
        for (uint32_t w = 0; w < word; ++w) {
            wpre += s_pc[0][w][p];
            rwpre += s_pc[1][w][p];
        }
        const uint32_t pos = s_off[0][p] + wpre + (uint32_t)__popcll(mine[q] & ltm);
        const float4 w4 = q == 0 ? make_float4(wx2.x, wy2.x, wz2.x, ww2.x)
                                 : make_float4(wx2.y, wy2.y, wz2.y, ww2.y);
        gst4(a.part_pts, pos, w4);
        if (lead[q]) {
            const uint32_t rpos = s_off[1][p] - s_tot + rwpre + (uint32_t)__popcll(mine[q] & lm & ltm);
            G(a.part_run_keys)[rpos] = key2[q] | (fr << a.frame_shift);
            G(a.part_run_starts)[rpos] = pos - s_first[p];
        }
    }
    if (s == gridDim.x - 1 && threadIdx.x < 2u * P) {  // the parts' sizes from the scan
        const uint32_t kind = threadIdx.x / P, p = threadIdx.x % P;
        const uint32_t a0 = G(a.seg_offsets)[(size_t)threadIdx.x * TS];
        const uint32_t a1 = threadIdx.x + 1 < 2u * P ? G(a.seg_offsets)[(size_t)(threadIdx.x + 1) * TS]
                                                     : *G(a.scan_total);
        if (a.part_nseg > 1u) {  // (the nseg-segment record: this frame has no segment 1..)
            const uint32_t ns = a.part_nseg;
            G(a.part_counts)[(kind * P + p) * ns] = a1 - a0;
            for (uint32_t sg = 1; sg < ns; ++sg) G(a.part_counts)[(kind * P + p) * ns + sg] = 0u;
        } else {
            G(a.part_counts)[kind * P + p] = a1 - a0;
        }
        if (threadIdx.x == 0) *G(a.out_count) = s_tot;
    }
}

template <int SEGW>
__global__ __launch_bounds__(SEGW / 2) void k_emit_px2(FrameArgs a) {
    __shared__ uint32_t s_hist[4 * 256];
    __shared__ uint32_t s_red[32];
    __shared__ uint32_t s_mark[1u << kMarkCacheBits];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    constexpr int NT = SEGW / 2, NW = NT / 64, NWORDS = SEGW / 64;
    const uint32_t s = blockIdx.x;
    for (uint32_t j = threadIdx.x; j < (1u << kMarkCacheBits); j += NT) s_mark[j] = 0xFFFFFFFFu;
    const gptr<const CamDesc> cams = G(cam_table(a));
    const bool hist = a.key_hist && !a.run_mode;
    if (hist)
        for (uint32_t i = threadIdx.x; i < radix_hist_span(a.npasses); i += NT) s_hist[i] = 0;
    GroupPart gp{};
    if (!a.fused_prefix && a.grp_tot) gp = group_partials_issue(a, s);
    const uint32_t i = threadIdx.x;
    int k = seg_camera(cams, a.ncams, s, a.seg_uniform);
    k = __builtin_amdgcn_readfirstlane(k);
    const uint32_t j = s - cams[k].seg0;
    const uint32_t y = j / cams[k].nchunk;
    const uint32_t x0 = (j - y * cams[k].nchunk) * cams[k].segw;
    const uint32_t len = min(cams[k].segw, cams[k].W - x0);
    uint64_t m[2];
    uint32_t dval[2] = {0u, 0u};
    float xnv[2] = {0.0f, 0.0f};
    // (both pixels' loads unconditional at clamped columns, selected after: the conditional form
    // waited for each depth load inside its branch)
    uint16_t dl[2];
    float xl[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        m[q] = G(a.vbits)[(size_t)s * 16 + wid + NW * q];
        const uint32_t ic = min(i + (uint32_t)NT * q, len - 1u);
        dl[q] = G(cams[k].depth)[y * cams[k].W + x0 + ic];
        xl[q] = G(cams[k].xn)[x0 + ic];
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const bool in = i + (uint32_t)NT * q < len;
        dval[q] = in ? dl[q] : 0u;
        xnv[q] = in ? xl[q] : 0.0f;
    }
    const float ynv = G(cams[k].yn)[y];
    // counts (and runs) of the segment's 4 words: the prefix of each of this thread's words
    uint32_t pc[NWORDS], rc[NWORDS];
#pragma unroll
    for (int w = 0; w < NWORDS; ++w) {
        pc[w] = (uint32_t)__popcll(G(a.vbits)[(size_t)s * 16 + w]);
        rc[w] = 0u;
    }
    const uint32_t sbase = a.fused_prefix ? 0u : G(a.seg_offsets)[s];
    uint32_t rbase = 0;
    if (a.run_mode) {
        if (!a.fused_prefix)  // (group scan: offsets local to the group's runs)
            rbase = G(a.seg_offsets)[a.total_segs + s] -
                    (a.grp_tot ? 0u : G(a.seg_offsets)[a.total_segs]);
#pragma unroll
        for (int w = 0; w < NWORDS; ++w) rc[w] = G(a.wave_runs)[(size_t)s * 16 + w];
    }
    // (the preceding groups' totals, loaded with the segment's own loads)
    if (a.fused_prefix) prefix_partials(a, s, s_red);
    else if (a.grp_tot) group_partials_finish(a, s, gp, s_red);
    __syncthreads();
    uint32_t base = sbase;
    if (a.fused_prefix || a.grp_tot)
        for (int w = 0; w < NW; ++w) {
            base += s_red[w];
            rbase += s_red[16 + w];
        }
    uint32_t tot = 0, rtot = 0;
#pragma unroll
    for (int w = 0; w < NWORDS; ++w) {
        tot += pc[w];
        rtot += rc[w];
    }
    if (s == gridDim.x - 1 && threadIdx.x == 0) {
        *G(a.out_count) = base + tot;
        if (a.run_mode) {
            G(a.run_start)[rbase + rtot] = base + tot;
            *G(a.run_count) = rbase + rtot;
        }
    }
    const uint32_t fr = cams[k].frame;
    if (a.frame_pt_start && threadIdx.x == 0) {
        const bool first_of_frame =
            s == cams[k].seg0 && (k == 0 || !cams[k - 1].emit || cams[k - 1].frame != fr);
        if (first_of_frame) G(a.frame_pt_start)[fr] = base;
        if (s == gridDim.x - 1) G(a.frame_pt_start)[a.nframes] = base + tot;
    }
    const unsigned long long ltm = lanemask_lt();
    // the world points (and keys) of the thread's two pixels in packed f32 (the same operations
    // as k_emit: convert, transform_points' rows, compute_voxel_coords)
    const f2v zz2 = f2((float)dval[0], (float)dval[1]) * f2(cams[k].scale, cams[k].scale);
    const f2v px2 = f2(xnv[0], xnv[1]) * zz2, py2 = f2(ynv, ynv) * zz2, pz2 = zz2;
    const f2v wx2 = mrow2(cams[k].Tw + 0, px2, py2, pz2), wy2 = mrow2(cams[k].Tw + 4, px2, py2, pz2);
    const f2v wz2 = mrow2(cams[k].Tw + 8, px2, py2, pz2), ww2 = mrow2(cams[k].Tw + 12, px2, py2, pz2);
    uint32_t key2[2] = {0xFFFFFFFFu, 0xFFFFFFFFu};
    if (a.do_voxel && (m[0] | m[1]))
        voxel_key2(wx2, wy2, wz2, a.vlo, a.vcs, a.vrcs, a.gmax, a.gs, key2[0], key2[1]);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const uint32_t word = (uint32_t)wid + NW * q;
        uint32_t wpre = 0, rwpre = 0;
#pragma unroll
        for (int w = 0; w < NWORDS; ++w) {
            wpre += (uint32_t)w < word ? pc[w] : 0u;
            rwpre += (uint32_t)w < word ? rc[w] : 0u;
        }
        const bool valid = i + (uint32_t)NT * q < len && ((m[q] >> lane) & 1ull);
        uint32_t key = 0xFFFFFFFFu;
        if (valid) {
            const uint32_t pos = base + wpre + (uint32_t)__popcll(m[q] & ltm);
            const float4 w4 = q == 0 ? make_float4(wx2.x, wy2.x, wz2.x, ww2.x)
                                     : make_float4(wx2.y, wy2.y, wz2.y, ww2.y);
            gst4(a.out_pts, pos, w4);
            if (a.do_voxel) {
                key = key2[q];
                G(a.out_coords)[pos] = key;
            }
        }
        if (a.run_mode) {
            const unsigned long long below = m[q] & ltm;
            const int prev = below ? 63 - __clzll((long long)below) : -1;
            const uint32_t pkey = __shfl(key, prev < 0 ? 0 : prev, 64);
            const bool leader = valid && (prev < 0 || pkey != key);
            const unsigned long long lm = __ballot(leader);
            if (leader) {
                const uint32_t ri = rbase + rwpre + (uint32_t)__popcll(lm & ltm);
                G(a.run_keys)[ri] = key | (fr << a.frame_shift);
                G(a.run_start)[ri] = base + wpre + (uint32_t)__popcll(m[q] & ltm);
            }
        }
        if (a.do_voxel)
            mark_and_count(a, a.marks ? a.marks + (size_t)fr * a.mark_words : nullptr, valid, key,
                           key | (fr << a.frame_shift), hist ? s_hist : nullptr, s_mark);
    }
    if (hist) flush_hist(a, s_hist);
}

// the emit partition's k_emit_px2 (its own kernel: the part bookkeeping's registers would otherwise
// raise the plain kernel's VGPR count, 32 -> 54, and cost it 10 us per 8-frame batch)
template <int SEGW>
__global__ __launch_bounds__(SEGW / 2) void k_emit_px2_parts(FrameArgs a) {
    __shared__ uint32_t s_mark[1u << kMarkCacheBits];
    for (uint32_t j = threadIdx.x; j < (1u << kMarkCacheBits); j += SEGW / 2) s_mark[j] = 0xFFFFFFFFu;
    emit_px2_parts<SEGW>(a, s_mark);
}

// Selected rollbuffer points (insertSelectedPointSequence + transformPointSequence + crop +
// applyPointMask + computeVoxelCoords + occupancy marks for the rollbuffer part).  The window is
// large (10^8 points) and mostly cropped away: each block owns a tile of kSelSegs x blockDim
// consecutive selected points (tiles in ticket order), reads them once, counts its survivors
// (and, run mode, their runs of equal keys), resolves the survivors / runs before it by two
// decoupled look-backs (wave 0: points, wave 1: runs) and writes its survivors (world point +
// voxel key) and run records straight to their place behind the depth compaction's - one pass
// over the window, in selection order.  The last tile writes the frame's totals.  Stage bits go
// to the debug buffer as before.
#ifdef GDF_TRACE_GROUPS
// (diagnostic build, tools/sel_trace.py) per k_sel tile: the wall clock (100 MHz) at block entry,
// ticket, end of the counting pass (every wave past the barrier), end of the look-back, and block
// end; the hardware id of wave 0
constexpr uint32_t kSelTraceSlots = 1u << 16;
__device__ unsigned long long g_strace[kSelTraceSlots][8];
#endif
template <uint32_t kSegs>
__global__ __launch_bounds__(1024) void k_sel(FrameArgs a) {
    constexpr uint32_t kSelSegs = kSegs;
    __shared__ uint32_t s_wc[kSelSegs * 16];  // kept items per (segment j, wave w), j-major
    __shared__ uint32_t s_rc[kSelSegs * 16];  // run mode: runs per (segment j, wave w)
    static_assert(kSelSegs * 16 <= 256, "k_sel scan covers 256 entries");
    __shared__ uint32_t s_mark[1u << kMarkCacheBits];
    __shared__ uint32_t s_tile, s_epoch, s_tot[2], s_ex[2];
    extern __shared__ uint32_t s_key[];  // [kSegs * blockDim] with sel_key_lds: item keys
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int nwaves = blockDim.x >> 6;
    const uint32_t B = blockDim.x, i = threadIdx.x;
    const bool stash = a.sel_key_lds != 0;  // (run mode, keys)
    const Tickets tk = tickets(a.sel_tiles, gridDim.x);  // (one tile per block: oneshot)
#ifdef GDF_TRACE_GROUPS
    const unsigned long long sw0 = wall_clock64();
#endif
    // the depth compaction's totals (k_emit, earlier on the stream; the rollbuffer points and runs
    // go behind them): read now, in flight with the ticket, not after the look-back
    const uint32_t d = __builtin_amdgcn_readfirstlane(*G(a.out_count));
    const uint32_t rd = __builtin_amdgcn_readfirstlane(a.run_mode ? *G(a.run_count) : 0u);
    if (i == 0) {
        const uint32_t ep = read_epoch(a.epoch_word);
        s_epoch = ep;
        s_tile = next_ticket(a.sel_ctr, tk, a.epoch_word, ep);
    }
    __syncthreads();
    const uint32_t tile = s_tile, epoch = s_epoch;
    if (a.grid_seq_out && tile == 0 && i == 0) *a.grid_seq_out = a.grid_seq;  // (as k_mask)
#ifdef GDF_TRACE_GROUPS
    const unsigned long long sw1 = wall_clock64();
#endif
    const uint32_t si0 = tile * kSelSegs * B;
    float tc[12], tw[16];
    // the ring loads (their slots need no search; 32-bit slot arithmetic: ring_cap < 2^32),
    // branch-free (a point past the selection re-reads the tile's first slot and is dropped);
    // otherwise the sequence search runs while they fly
    float4 p[kSelSegs];
    {
        const uint32_t cap = (uint32_t)a.ring_cap;
        const uint32_t r0 = (uint32_t)((a.ring_first + si0) % a.ring_cap);
#pragma unroll
        for (uint32_t j = 0; j < kSelSegs; ++j) {
            const uint32_t si = si0 + j * B + i;
            uint32_t q = r0 + j * B + i;
            q = q >= cap ? q - cap : q;
            p[j] = gld4(a.ring, si < a.sel_count ? q : r0);
        }
    }
    const SelSeg g = sel_seg(a, si0);
    // the whole tile inside one sequence (all but ~1 in 10^2..10^3 tiles): its crop transform is
    // block-uniform, read once into scalar registers, and the stage bits are computed without
    // branches; a tile reaching into the next sequence takes the per-point lookup
    const bool one_seq = si0 + kSelSegs * B <= g.next;
    if (a.marks)  // (rollbuffer frames of processFrame take their marks from the voxel groups)
        for (uint32_t j = i; j < (1u << kMarkCacheBits); j += B) s_mark[j] = 0xFFFFFFFFu;
    uint32_t bits[kSelSegs];
    if (one_seq) {
        // both matrices in one load round (the world one's was a second round, after the bits)
        const gptr<const float> Tc = G(a.tfc + 16 * (size_t)g.tf0);
        const gptr<const float> Tw = G(a.tfw + 16 * (size_t)g.tf0);
        // (block-uniform: into scalar registers as they arrive, not held in VGPRs beside the points)
        float tcl[12], twl[16];
#pragma unroll
        for (int q = 0; q < 12; ++q) tcl[q] = Tc[q];
#pragma unroll
        for (int q = 0; q < 16; ++q) twl[q] = Tw[q];
#pragma unroll
        for (int q = 0; q < 12; ++q)
            tc[q] = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, tcl[q])));
#pragma unroll
        for (int q = 0; q < 16; ++q)
            tw[q] = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, twl[q])));
#pragma unroll
        for (uint32_t j = 0; j < kSelSegs; ++j) {
            const float x = p[j].x, y = p[j].y, z = p[j].z;
            const float qx = mrow(tc + 0, x, y, z, 1.0f);
            const float qy = mrow(tc + 4, x, y, z, 1.0f);
            const float qz = mrow(tc + 8, x, y, z, 1.0f);
            const bool out = a.do_crop && ((qx < a.lo[0]) | (qx > a.hi[0]) | (qy < a.lo[1]) |
                                           (qy > a.hi[1]) | (qz < a.lo[2]) | (qz > a.hi[2]));
            const bool live = (si0 + j * B + i < a.sel_count) & (p[j].w != 0.0f);
            bits[j] = live ? (out ? 3u : 7u) : 0u;
        }
    } else {
#pragma unroll
        for (uint32_t j = 0; j < kSelSegs; ++j) {
            const uint32_t si = si0 + j * B + i;
            bits[j] = si < a.sel_count ? sel_bits(a, g, si, p[j]) : 0u;
        }
    }
    uint32_t keep = 0;  // bit j: item j of this thread survives the crop
    const unsigned long long ltm = lanemask_lt();
    const gptr<const float> T0 = G(a.tfw + 16 * (size_t)g.tf0);
    // a tile inside one sequence: its world matrix in registers, read once (through the pointer
    // the compiler re-read the 64-B matrix for every item - 16 dependent cache round trips per
    // wave per pass - as it cannot move those loads above the debug-byte stores)

    // the world point of selected item j (transform_points_indirect, world matrix)
    auto world = [&](uint32_t j) {
        const float x = p[j].x, y = p[j].y, z = p[j].z;
        if (one_seq)  // (block-uniform)
            return make_float4(mrow(tw + 0, x, y, z, 1.0f), mrow(tw + 4, x, y, z, 1.0f),
                               mrow(tw + 8, x, y, z, 1.0f), mrow(tw + 12, x, y, z, 1.0f));
        const uint32_t si = si0 + j * B + i;
        const gptr<const float> Tw = si < g.next ? T0 : G(a.tfw + 16 * (size_t)sel_tf(a, si));
        return make_float4(mrow(Tw + 0, x, y, z, 1.0f), mrow(Tw + 4, x, y, z, 1.0f),
                           mrow(Tw + 8, x, y, z, 1.0f), mrow(Tw + 12, x, y, z, 1.0f));
    };
    uint32_t rlead = 0;  // run mode: bit j - item j starts a run of equal keys in its wave
#pragma unroll
    for (uint32_t j = 0; j < kSelSegs; ++j) {
        const uint32_t si = si0 + j * B + i;
        if (a.dbg && si < a.sel_count) G(a.dbg)[a.depth_total + si] = (uint8_t)bits[j];
        keep |= ((bits[j] >> 2) & 1u) << j;
        const unsigned long long m = __ballot((bits[j] & 4u) != 0u);
        if (lane == 0) s_wc[j * nwaves + wid] = (uint32_t)__popcll(m);
        if (a.run_mode) {
            uint32_t key = 0xFFFFFFFFu;
            if (bits[j] & 4u) {
                const float4 w = world(j);
                key = voxel_key(w.x, w.y, w.z, a.vlo, a.vcs, a.vrcs, a.gmax, a.gs);
                p[j] = w;  // (the store pass writes this world point: the raw one is not read again)
            }
            if (stash) s_key[j * B + i] = key;  // (read back by the same thread: no barrier)
            const unsigned long long below = m & ltm;
            const int prev = below ? 63 - __clzll((long long)below) : -1;
            const uint32_t pkey = __shfl(key, prev < 0 ? 0 : prev, 64);
            const bool leader = ((bits[j] & 4u) != 0u) && (prev < 0 || pkey != key);
            rlead |= (uint32_t)leader << j;
            const unsigned long long lm = __ballot(leader);
            if (lane == 0) s_rc[j * nwaves + wid] = (uint32_t)__popcll(lm);
        }
    }
    __syncthreads();
#ifdef GDF_TRACE_GROUPS
    const unsigned long long sw2 = wall_clock64();
#endif
    // exclusive scans of the (segment, wave) counts in item order: points by wave 0, runs by
    // wave 1 (<= 256 entries each)
    const uint32_t ne = kSelSegs * (uint32_t)nwaves;
    if (wid == 0 || (wid == 1 && a.run_mode)) {
        uint32_t* sc = wid == 0 ? s_wc : s_rc;
        uint32_t carry = 0;
        for (uint32_t e0 = 0; e0 < ne; e0 += 64) {  // uniform
            const uint32_t e = e0 + (uint32_t)lane;
            const uint32_t v = e < ne ? sc[e] : 0u;
            uint32_t x = v;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(x, o, 64);
                if (lane >= o) x += y;
            }
            if (e < ne) sc[e] = carry + x - v;
            carry += __shfl(x, 63, 64);
        }
        // the survivors (runs) of the tiles before this one
        const uint32_t words = a.sel_tiles + a.sel_tiles / 64u + 2u;
        unsigned long long* st = a.sel_status + (wid == 0 ? 0u : 2u * (size_t)words);
        const uint32_t ex =
            lookback2_wave(st, st + words, tile, a.sel_tiles, carry, epoch, a.err);
        if (lane == 0) {
            s_tot[wid] = carry;
            s_ex[wid] = ex;
        }
    }
    __syncthreads();
#ifdef GDF_TRACE_GROUPS
    const unsigned long long sw3 = wall_clock64();
#endif
    const uint32_t pbase = d + s_ex[0], rbase = rd + (a.run_mode ? s_ex[1] : 0u);
    if (tile == a.sel_tiles - 1u && i == 0) {  // the frame's totals
        *G(a.final_count) = pbase + s_tot[0];
        if (a.run_mode) {
            const uint32_t rtot = rbase + s_tot[1];
            *G(a.run_total) = rtot;
            G(a.run_start)[rtot] = pbase + s_tot[0];
        }
        if (a.sel_splits)  // (the partition's unused cuts: empty segments at the end)
            for (uint32_t c = a.sel_ncuts; c < kMaxSegs - 2u; ++c) G(a.sel_splits)[1u + c] = pbase + s_tot[0];
    }
    if (a.sel_splits && tile == 0u && i == 0) G(a.sel_splits)[0] = d;  // (depth | rollbuffer)
#pragma unroll
    for (uint32_t j = 0; j < kSelSegs; ++j) {
        const bool valid = (keep >> j) & 1u;
        const unsigned long long m = __ballot(valid);
        const uint32_t pos = pbase + s_wc[j * nwaves + wid] + (uint32_t)__popcll(m & ltm);
        // a cut of the selection (sharded window: where the next piece this rank holds starts):
        // the survivors before that item, kept or not
        for (uint32_t c = 0; c < a.sel_ncuts; ++c)  // (uniform; sel_ncuts <= kMaxSegs - 2)
            if (si0 + j * B + i == a.sel_cut_at[c]) G(a.sel_splits)[1u + c] = pos;
        if (!m) continue;  // wave-uniform
        uint32_t key = 0xFFFFFFFFu;
        if (valid) {
            // (run mode: the world point was computed for the run keys above, 24 VALU per item)
            const float4 w = a.run_mode ? p[j] : world(j);
            gst4(a.out_pts, pos, w);
            if (a.do_voxel) {
                key = stash ? s_key[j * B + i] : voxel_key(w.x, w.y, w.z, a.vlo, a.vcs, a.vrcs, a.gmax, a.gs);
                G(a.out_coords)[pos] = key;
            }
        }
        if (a.run_mode) {  // the run records: key, first point
            const bool lead = (rlead >> j) & 1u;
            const unsigned long long lm = __ballot(lead);
            if (lead) {
                const uint32_t rpos = rbase + s_rc[j * nwaves + wid] + (uint32_t)__popcll(lm & ltm);
                G(a.run_keys)[rpos] = key;
                G(a.run_start)[rpos] = pos;
            }
        }
        if (a.do_voxel && a.marks) mark_and_count(a, a.marks, valid, key, key, nullptr, s_mark);
    }
#ifdef GDF_TRACE_GROUPS
    __syncthreads();
    if (i == 0 && tile < kSelTraceSlots) {
        unsigned long long* t = g_strace[tile];
        t[0] = sw0;
        t[1] = sw1;
        t[2] = sw2;
        t[3] = sw3;
        t[4] = wall_clock64();
        t[5] = ((unsigned)__builtin_amdgcn_s_getreg(4 | (15 << 11)) & 0xFFFFu) |  // HW_ID
               (((unsigned long long)__builtin_amdgcn_s_getreg(20 | (15 << 11)) & 0xFu) << 16);  // XCC
        t[6] = blockIdx.x;
    }
#endif
}

struct HookScope {  // begin/end of one profiled launch
    LaunchHook* h;
    int slot;
    HookScope(LaunchHook* h_, int s_) : h(h_), slot(s_) {
        if (h) h->begin(slot);
    }
    ~HookScope() {
        if (h) h->end(slot);
    }
};

// k_sel's key stash (FrameArgs::sel_key_lds) can exceed the default 64 KB of dynamic LDS per
// workgroup (16 x 1024 items: 64 KB + the static arrays): allowed once per process
bool sel_key_lds_allowed(uint32_t bytes) {
    static const bool ok = [] {
        const int cap = 96 * 1024;
        return hipFuncSetAttribute(reinterpret_cast<const void*>(&k_sel<4>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, cap) == hipSuccess &&
               hipFuncSetAttribute(reinterpret_cast<const void*>(&k_sel<8>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, cap) == hipSuccess &&
               hipFuncSetAttribute(reinterpret_cast<const void*>(&k_sel<16>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, cap) == hipSuccess;
    }();
    return ok && bytes <= 96u * 1024u;
}

hipError_t launch_frame(const FrameArgs& a, hipStream_t s, LaunchHook* hook) {
    hipError_t e;
    if (a.total_segs == 0) {  // no depth survivors to count
        if ((e = hipMemsetAsync(a.out_count, 0, 4, s)) != hipSuccess) return e;
        if (a.run_mode && (e = hipMemsetAsync(a.run_count, 0, 4, s)) != hipSuccess) return e;
        if (a.grid_seq_out && !a.sel_tiles &&  // no kernel of this frame stores the ticket
            (e = hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(a.grid_seq_out),
                                   (int)a.grid_seq, 1, s)) != hipSuccess)
            return e;
    } else {
        {
            HookScope hs(hook, GDF_KERNEL_MASK);
            const size_t lds = (size_t)a.band_lds;
            const void* km = mask_kernel(a);
            if (km == reinterpret_cast<const void*>(&k_mask_px<2, 256>))
                hipLaunchKernelGGL((k_mask_px<2, 256>), dim3(a.total_segs), dim3(128), lds, s, a);
            else if (km == reinterpret_cast<const void*>(&k_mask_px_o8<2, 256>))
                hipLaunchKernelGGL((k_mask_px_o8<2, 256>), dim3(a.total_segs), dim3(128), lds, s, a);
            else if (km == reinterpret_cast<const void*>(&k_mask_px<2, 640>))
                hipLaunchKernelGGL((k_mask_px<2, 640>), dim3(a.total_segs), dim3(320), lds, s, a);
            else if (km == reinterpret_cast<const void*>(&k_mask<true, 4>))
                hipLaunchKernelGGL((k_mask<true, 4>), dim3(a.total_segs), dim3(a.seg_threads), lds, s, a);
            else if (km == reinterpret_cast<const void*>(&k_mask<false, 4>))
                hipLaunchKernelGGL((k_mask<false, 4>), dim3(a.total_segs), dim3(a.seg_threads), lds, s, a);
            else if (a.rot45)
                hipLaunchKernelGGL((k_mask<true, 0>), dim3(a.total_segs), dim3(a.seg_threads), lds, s, a);
            else
                hipLaunchKernelGGL((k_mask<false, 0>), dim3(a.total_segs), dim3(a.seg_threads), lds, s, a);
            if ((e = hipGetLastError()) != hipSuccess) return e;
        }
        if (!a.fused_prefix && !a.grp_done) {  // (run mode: the point counts, then the run counts)
            HookScope hs(hook, GDF_KERNEL_SCAN);
            const uint32_t m = a.nparts ? 2u * a.nparts * a.total_segs
                                        : a.run_mode ? 2u * a.total_segs : a.total_segs;
            if ((e = launch_scan(a.seg_counts, m, a.seg_offsets, a.scan_total, nullptr, 1u, s)) != hipSuccess)
                return e;
        }
        HookScope hs(hook, GDF_KERNEL_EMIT);
        const void* ke = emit_kernel(a);
        if (ke == reinterpret_cast<const void*>(&k_emit_px2_parts<256>))
            hipLaunchKernelGGL(k_emit_px2_parts<256>, dim3(a.total_segs), dim3(128), 0, s, a);
        else if (ke == reinterpret_cast<const void*>(&k_emit_px2<256>))
            hipLaunchKernelGGL(k_emit_px2<256>, dim3(a.total_segs), dim3(128), 0, s, a);
        else if (ke == reinterpret_cast<const void*>(&k_emit_px2<640>))
            hipLaunchKernelGGL(k_emit_px2<640>, dim3(a.total_segs), dim3(320), 0, s, a);
        else
            hipLaunchKernelGGL(k_emit, dim3(a.total_segs), dim3(a.seg_threads), 0, s, a);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if (a.sel_tiles) {  // rollbuffer points: one pass, behind the depth survivors
        HookScope hs(hook, GDF_KERNEL_SEL);
        const uint32_t thr = a.sel_tile / a.sel_segs;
        const size_t lds = a.sel_key_lds;
        if (a.sel_segs == 4)
            hipLaunchKernelGGL(k_sel<4>, dim3(a.sel_tiles), dim3(thr), lds, s, a);
        else if (a.sel_segs == 16)
            hipLaunchKernelGGL(k_sel<16>, dim3(a.sel_tiles), dim3(thr), lds, s, a);
        else
            hipLaunchKernelGGL(k_sel<8>, dim3(a.sel_tiles), dim3(thr), lds, s, a);
    }
    return hipGetLastError();
}

// 640-pixel segments (single frames under 1 Mi pixels): two pixels per thread only from this many
// segments (measured on MI355X, A/B on one box: 720p single frames, 1440 segments, 13.7 -> 14.4-14.9
// Gpoints/s; VGA single frames, 480 segments = 2400 waves of 320 threads, 8.3 -> 7.6-8.1)
constexpr uint32_t kPx640MinSegs = 1024;

// k_mask_px (2 pixels per thread) serves 256-pixel segments at F = 4 without rot45 (tuning knob
// GDF_MASK_PX; 0 or 1: k_mask); k_mask everything else.  (The 4-pixel form is gone: slower, and its
// compiler-made private copy of FrameArgs broke the G() camera-table reads, cam_table above.)  Measured on MI355X
// (A/B on one box, dense frames, 2 pixels per thread vs k_mask): VGA 8-frame batches
// 22.1 -> 23.7, 720p 4-frame batches 29.8 -> 32.6, 4K 30.9 -> 32.4 Gpoints/s
const void* mask_kernel(const FrameArgs& a) {
    const Tuning& T = *a.tune;
    if (T.mask_px2 >= 2 && a.do_flying && a.F == 4 && !a.rot45 && a.seg_threads == 256 && !a.dbg &&
        a.band_rowb <= 64 * 16)
        return T.mask_occ8 ? reinterpret_cast<const void*>(&k_mask_px_o8<2, 256>)
                           : reinterpret_cast<const void*>(&k_mask_px<2, 256>);
    // (half 720p rows: single frames under 1 Mi pixels with enough segments to fill the chip)
    if (T.mask_px2 >= 2 && a.do_flying && a.F == 4 && !a.rot45 && a.seg_threads == 640 && !a.dbg &&
        a.band_rowb <= 2 * 64 * 16 && a.total_segs >= kPx640MinSegs)
        return reinterpret_cast<const void*>(&k_mask_px<2, 640>);
    return frame_kernel(0, a.rot45, a.do_flying ? a.F : 0u);
}


// k_emit_px2 (two pixels per thread) for 256-pixel segments unless Tuning::emit_px2 is cleared
// the compaction kernels that write the emit partition (FrameArgs::nparts)
bool emit_partition_kernels(const FrameArgs& a) {
    const void* km = mask_kernel(a);
    FrameArgs plain = a;
    plain.nparts = 0;
    return (km == reinterpret_cast<const void*>(&k_mask_px<2, 256>) ||
            km == reinterpret_cast<const void*>(&k_mask_px_o8<2, 256>)) &&
           emit_kernel(plain) == reinterpret_cast<const void*>(&k_emit_px2<256>);
}

const void* emit_kernel(const FrameArgs& a) {
    if (a.nparts) return reinterpret_cast<const void*>(&k_emit_px2_parts<256>);
    if (a.tune->emit_px2 && a.seg_threads == 256) return reinterpret_cast<const void*>(&k_emit_px2<256>);
    if (a.tune->emit_px2 && a.seg_threads == 640 && a.total_segs >= kPx640MinSegs)
        return reinterpret_cast<const void*>(&k_emit_px2<640>);
    return reinterpret_cast<const void*>(&k_emit);
}

const void* frame_kernel(int which, int rot45, uint32_t F) {
    if (which == 1) return reinterpret_cast<const void*>(&k_emit);
    if (which == 2) return reinterpret_cast<const void*>(&k_sel<8>);
    if (which == 4) return reinterpret_cast<const void*>(&k_sel<4>);
    if (which == 5) return reinterpret_cast<const void*>(&k_sel<16>);
    if (F == 4)  // the launch default: rings unrolled
        return rot45 ? reinterpret_cast<const void*>(&k_mask<true, 4>)
                     : reinterpret_cast<const void*>(&k_mask<false, 4>);
    return rot45 ? reinterpret_cast<const void*>(&k_mask<true, 0>)
                 : reinterpret_cast<const void*>(&k_mask<false, 0>);
}

// per-camera ray factors (sh/convert_depthmap_to_points.glsl:68-69), one f32 division each
__global__ __launch_bounds__(256) void k_tables(uint32_t W, uint32_t H, float fx, float fy,
                                                float cx, float cy, float* __restrict__ xn,
                                                float* __restrict__ yn) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < W) xn[i] = ((float)i - cx) / fx;
    if (i < H) yn[i] = ((float)i - cy) / fy;
}

hipError_t launch_tables(uint32_t W, uint32_t H, float fx, float fy, float cx, float cy, float* xn,
                         float* yn, hipStream_t s) {
    const uint32_t n = W > H ? W : H;
    hipLaunchKernelGGL(k_tables, dim3((n + 255) / 256), dim3(256), 0, s, W, H, fx, fy, cx, cy, xn,
                       yn);
    return hipGetLastError();
}

// ---- point-sequence filter + rollbuffer insert --------------------------------------------------
// filter_point_sequence.glsl:49-76 neighbour test
__device__ __forceinline__ bool ps_ok(const float4* pts, float px, float py, float pz, float nx,
                                      float ny, float nz, uint32_t other, float thr) {
    const float4 q = pts[other];
    float dx = q.x - px, dy = q.y - py, dz = q.z - pz;
    normalize3(dx, dy, dz);
    float c = fabsf(dot3(dx, dy, dz, nx, ny, nz));
    return !(1.0f - c < thr);
}

// new points [src0, src0 + cnt) of the n uploaded (a sharded engine's own sequences; the
// filter's neighbours range over all n) into ring slots first, first + 1, ...
__global__ __launch_bounds__(256) void k_ps_filter_insert(const float4* __restrict__ pts,
                                                          uint32_t n, int do_filter, float thr,
                                                          uint32_t F, float4* __restrict__ ring,
                                                          uint64_t cap, uint64_t first,
                                                          uint32_t src0, uint32_t cnt) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= cnt) return;
    const uint32_t g = src0 + t;
    const float4 p = pts[g];
    bool valid = true;
    if (do_filter) {
        if (sqrtf(dot3(p.x, p.y, p.z, p.x, p.y, p.z)) < 1e-3f) {
            valid = false;
        } else {
            float nx = p.x, ny = p.y, nz = p.z;
            normalize3(nx, ny, nz);
            nx = -nx; ny = -ny; nz = -nz;
            for (uint32_t i = 0; i < F && valid; ++i) {
                const uint32_t j0 = g + i - 1u;
                if (j0 < n && !ps_ok(pts, p.x, p.y, p.z, nx, ny, nz, j0, thr)) valid = false;
                const uint32_t j1 = g + i + 1u;
                if (valid && j1 < n && !ps_ok(pts, p.x, p.y, p.z, nx, ny, nz, j1, thr))
                    valid = false;
            }
        }
    }
    ring[(first + t) % cap] = make_float4(p.x, p.y, p.z, valid ? 1.0f : 0.0f);
}

hipError_t launch_ps_filter_insert(const float4* new_pts, uint32_t n, int do_filter, float thr,
                                   uint32_t F, float4* ring, uint64_t cap, uint64_t first,
                                   hipStream_t s, uint32_t src0, uint32_t cnt) {
    if (cnt == 0xFFFFFFFFu) cnt = n - src0;
    if (cnt == 0) return hipSuccess;
    hipLaunchKernelGGL(k_ps_filter_insert, dim3((cnt + 255) / 256), dim3(256), 0, s, new_pts, n,
                       do_filter, thr, F, ring, cap, first, src0, cnt);
    return hipGetLastError();
}

// addPointSequence for device-resident PointCloud2 records (fusion.cpp:777-780: x, y, z floats at
// byte offsets 0/4/8 of each point_step record, w = 1).  step is a multiple of 4; the common
// step 16 (16-byte aligned records) reads one 16-byte vector per point.
__global__ __launch_bounds__(256) void k_gather_records(const uint8_t* __restrict__ rec,
                                                        uint32_t n, uint32_t step, int vec16,
                                                        float4* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float4 p;
    if (vec16) {
        p = reinterpret_cast<const float4*>(rec)[i];
    } else {
        const float* r = reinterpret_cast<const float*>(rec + (size_t)i * step);
        p = make_float4(r[0], r[1], r[2], 0.0f);
    }
    p.w = 1.0f;
    out[i] = p;
}

hipError_t launch_gather_records(const void* rec, uint32_t n, uint32_t step, float4* out,
                                 hipStream_t s) {
    if (n == 0) return hipSuccess;
    const int vec16 = step == 16 && (reinterpret_cast<uintptr_t>(rec) & 15u) == 0;
    hipLaunchKernelGGL(k_gather_records, dim3((n + 255) / 256), dim3(256), 0, s,
                       static_cast<const uint8_t*>(rec), n, step, vec16, out);
    return hipGetLastError();
}

// ---- historic occupancy grid ---------------------------------------------------------------------
// Occupancy marks of a frame are a bitmask (cell c -> bit c % 32 of word c / 32), set by k_emit /
// k_scatter and consumed - read and cleared - by the grid update.  hist' = max(sat_dec(hist),
// mark·L) (decrement_uints.glsl:31-51 + max_with_uints_times_scalar.glsl:36-46); the output byte is
// hist & 0xFF (uints_to_chars.glsl:31-50).  With L <= 255 the u8 grid IS the history.
// Grid updates are applied in engine order even when consecutive frames run on different
// streams (frame pipelining): update f waits until ctl[0] == f (updates completed), and the last
// of its blocks to finish publishes ctl[0] = f + 1.  f comes from the host (the kernel argument,
// or a per-slot word the frame's k_mask stored).  ctl == nullptr: no ordering (one stream).
// COHERENT: the block reads the grid with agent-coherent loads (grid_load), so no per-block L2
// invalidate (an agent acquire fence, buffer_inv) is needed after the wait
template <bool COHERENT = false>
__device__ __forceinline__ uint32_t grid_seq_enter(const GridSeq& q) {
    __shared__ uint32_t s_f;
    if (!q.ctl) return 0;
    if (threadIdx.x == 0) {
        const uint32_t f = q.fptr ? __hip_atomic_load(q.fptr, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT) : q.f;
        uint32_t spins = 0;
        while ((int32_t)(__hip_atomic_load(&q.ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) -
                         f) < 0) {
            if (++spins > kSpinLimit) {
                atomicOr(q.err, 4u);
                break;
            }
            __builtin_amdgcn_s_sleep(8);
        }
        if (!COHERENT) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // the previous update's grid
        s_f = f;
    }
    __syncthreads();
    return s_f;
}

// COHERENT: the block wrote the grid with agent-coherent stores (grid_store): once they have
// completed they are visible to every XCD, and no per-block L2 write-back (an agent release fence,
// buffer_wbl2, issued by each of hundreds of blocks) is needed before the block counts itself in.
// This covers ONLY the sc1 grid stores: the plain stores of the same blocks (a single frame's grid
// delta, a batch's sparse snapshots) are read by later kernels of the SAME stream (k_download,
// k_snap_expand), ordered by the kernel boundary's release, never by the next slot's update.
template <bool COHERENT = false>
__device__ __forceinline__ void grid_seq_leave(const GridSeq& q, uint32_t f, uint32_t nblocks) {
    if (!q.ctl) return;
    __builtin_amdgcn_s_waitcnt(0);  // this wave's grid stores have completed
    __syncthreads();
    if (threadIdx.x == 0) {
        if (!COHERENT) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // L2 write-back: visible to all XCDs
        const uint32_t c = atomicAdd(&q.ctl[1], 1u);
        if (c == nblocks - 1u) {
            atomicExch(&q.ctl[1], 0u);
            __hip_atomic_store(&q.ctl[0], f + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

__device__ __forceinline__ uint32_t grid_byte(uint32_t h, uint32_t m, uint32_t L) {
    const uint32_t dec = h ? h - 1u : 0u;
    return m ? (dec > L ? dec : L) : dec;
}

// 4 cells of a u32 word of the u8 grid, marks in bits 0..3 of mb
__device__ __forceinline__ uint32_t grid_word(uint32_t w, uint32_t mb, uint32_t L) {
    return grid_byte(w & 0xFFu, mb & 1u, L) | (grid_byte((w >> 8) & 0xFFu, (mb >> 1) & 1u, L) << 8) |
           (grid_byte((w >> 16) & 0xFFu, (mb >> 2) & 1u, L) << 16) |
           (grid_byte(w >> 24, (mb >> 3) & 1u, L) << 24);
}

// blocks [0, nblocks) of a launch update the u8 grid: 32 cells (two 16-byte vectors and one mark
// word) per thread and step; the grid allocation is padded to 32 bytes
// two grid words of 16 cells each as agent-scope (sc1) 64-bit stores: coherent across the XCDs
// without an L2 write-back (grid_seq_leave<true>)
__device__ __forceinline__ void grid_store(uint4* grid, uint64_t j, const uint4& v) {
    unsigned long long* p = reinterpret_cast<unsigned long long*>(grid + j);
    __hip_atomic_store(p, ((unsigned long long)v.y << 32) | v.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(p + 1, ((unsigned long long)v.w << 32) | v.z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The wave's 64 grid words (2 KB from uint4 2 i0) through 2 KB of LDS per wave: two coalesced 1-KB
// agent-coherent (sc1) buffer accesses per direction.  Per lane at a 32-B stride, the coherent
// accesses reach memory sector by sector - four 8-B stores per 32-B sector measured the grid's
// writes at ~4x its bytes (PMC WRITE_SIZE of the carrying radix pass).  Past the grid (the last
// wave's idle lanes) the buffer range check returns 0 / drops the store.  Grids of 2 GB and more
// take the per-lane form.
__device__ __forceinline__ uint4* grid_xbuf() {
    __shared__ uint4 s_gx[4][128];
    return &s_gx[threadIdx.x >> 6][0];
}
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
typedef uint32_t gx4 __attribute__((ext_vector_type(4)));
constexpr int kCpolSc1 = 16;  // buffer cache policy: sc1 (agent scope)

__device__ __forceinline__ uint4 grid_load(const uint4* grid, uint64_t j);
__device__ __forceinline__ void grid_store(uint4* grid, uint64_t j, const uint4& v);

__device__ __forceinline__ void grid_wave_load(const uint4* grid, uint64_t nwords, uint64_t i0,
                                               uint4& v0, uint4& v1) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t bytes = nwords * 32u;
    if (bytes < (1ull << 31)) {
        uint4* sx = grid_xbuf();
        const __amdgpu_buffer_rsrc_t r =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(grid), 0, (int)bytes, 0x00020000);
        const uint32_t base = (uint32_t)(i0 * 32u) + lane * 16u;
        const gx4 a = __builtin_amdgcn_raw_buffer_load_b128(r, base, 0, kCpolSc1);
        const gx4 b = __builtin_amdgcn_raw_buffer_load_b128(r, base + 1024u, 0, kCpolSc1);
        sx[lane] = make_uint4(a.x, a.y, a.z, a.w);
        sx[64 + lane] = make_uint4(b.x, b.y, b.z, b.w);
        wave_lds_sync();
        v0 = sx[2 * lane];
        v1 = sx[2 * lane + 1];
        wave_lds_sync();  // (the buffer is free again)
    } else if (i0 + lane < nwords) {
        v0 = grid_load(grid, 2 * (i0 + lane));
        v1 = grid_load(grid, 2 * (i0 + lane) + 1);
    } else {
        v0 = v1 = make_uint4(0u, 0u, 0u, 0u);
    }
}

__device__ __forceinline__ void grid_wave_store(uint4* grid, uint64_t nwords, uint64_t i0,
                                                const uint4& v0, const uint4& v1) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t bytes = nwords * 32u;
    if (bytes < (1ull << 31)) {
        uint4* sx = grid_xbuf();
        sx[2 * lane] = v0;
        sx[2 * lane + 1] = v1;
        wave_lds_sync();
        const uint4 a = sx[lane], b = sx[64 + lane];
        wave_lds_sync();
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(grid, 0, (int)bytes, 0x00020000);
        const uint32_t base = (uint32_t)(i0 * 32u) + lane * 16u;
        gx4 va, vb;
        va.x = a.x; va.y = a.y; va.z = a.z; va.w = a.w;
        vb.x = b.x; vb.y = b.y; vb.z = b.z; vb.w = b.w;
        __builtin_amdgcn_raw_buffer_store_b128(va, r, base, 0, kCpolSc1);
        __builtin_amdgcn_raw_buffer_store_b128(vb, r, base + 1024u, 0, kCpolSc1);
    } else if (i0 + lane < nwords) {
        grid_store(grid, 2 * (i0 + lane), v0);
        grid_store(grid, 2 * (i0 + lane) + 1, v1);
    }
}

__device__ __forceinline__ uint4 grid_load(const uint4* grid, uint64_t j) {
    const unsigned long long* p = reinterpret_cast<const unsigned long long*>(grid + j);
    const unsigned long long a = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long b = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
}

__device__ __forceinline__ void grid_u8_part(uint4* __restrict__ grid, uint32_t* __restrict__ marks,
                                             uint64_t nwords, uint32_t L, uint32_t block,
                                             uint32_t nblocks, const GridSeq& q) {
    const uint64_t stride = (uint64_t)nblocks * blockDim.x;
    // wave-uniform loop (the delta's ballots need every lane)
    for (uint64_t i0 = block * (uint64_t)blockDim.x + (threadIdx.x & ~63u); i0 < nwords; i0 += stride) {
        const uint64_t i = i0 + (threadIdx.x & 63u);
        const bool act = i < nwords;
        uint4 o0 = make_uint4(0u, 0u, 0u, 0u), o1 = o0;
        uint32_t m = 0;
        grid_wave_load(grid, nwords, i0, o0, o1);
        if (act) m = marks[i];
        uint4 v0, v1;
        v0.x = grid_word(o0.x, m, L);
        v0.y = grid_word(o0.y, m >> 4, L);
        v0.z = grid_word(o0.z, m >> 8, L);
        v0.w = grid_word(o0.w, m >> 12, L);
        v1.x = grid_word(o1.x, m >> 16, L);
        v1.y = grid_word(o1.y, m >> 20, L);
        v1.z = grid_word(o1.z, m >> 24, L);
        v1.w = grid_word(o1.w, m >> 28, L);
        grid_wave_store(grid, nwords, i0, v0, v1);
        if (act && m) marks[i] = 0u;
        if (q.dcnt) {  // the changed groups (a frame: the grid's ~1-2 % non-zero cells)
            const bool ch = act && ((o0.x ^ v0.x) | (o0.y ^ v0.y) | (o0.z ^ v0.z) | (o0.w ^ v0.w) |
                                    (o1.x ^ v1.x) | (o1.y ^ v1.y) | (o1.z ^ v1.z) | (o1.w ^ v1.w)) != 0u;
            const unsigned long long b = __ballot(ch);
            if (b) {  // wave-uniform: one append per wave step
                uint32_t base = 0;
                if ((threadIdx.x & 63u) == 0)
                    base = __hip_atomic_fetch_add(q.dcnt, (uint32_t)__popcll(b), __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
                base = __shfl(base, 0, 64);
                if (ch) {
                    const uint32_t e = base + (uint32_t)__popcll(b & lanemask_lt());
                    q.didx[e] = (uint32_t)i;
                    q.ddata[2 * (uint64_t)e] = v0;
                    q.ddata[2 * (uint64_t)e + 1] = v1;
                }
            }
        }
    }
}

// Sparse per-frame grid snapshots of a batch (the u8 grid the reference downloads after every
// frame, fusion.cpp:1824-1839): the grid after frame f < nframes - 1 is kept as the list of its
// NON-ZERO 32-cell groups (word index + 32 bytes), written by the grid update itself.  A dense
// copy per frame would write (B - 1) C bytes per batch (23.5 MB at B = 8 and the launch-default
// grid) to serve a download that may never come; the groups a launch-default frame keeps
// non-zero (its last `lifetime` frames' voxels) are ~1 % of them.  Every wave of the update owns a
// segment of snap.seg entries per frame, compacted by ballot (no atomics); snap.cnt[f * W + w]
// is wave w's count.  gdf_download_batch_occupancy_grid expands a frame with k_snap_expand.
__device__ __forceinline__ void snap_layout(uint64_t nwords, uint32_t nblocks, uint32_t& waves,
                                            uint32_t& seg) {
    const uint64_t stride = (uint64_t)nblocks * 256u;
    waves = nblocks * 4u;
    seg = (uint32_t)((nwords + stride - 1) / stride) * 64u;
}

// the grid updates of a batch of `nframes` frames, frame f's marks at marks + f * mark_words,
// applied in frame order in registers (blocks [0, nblocks) of a launch, 256 threads); the grid
// after frame f < nframes - 1 goes to the sparse snapshots, the last one is the grid itself.
// Marks are cleared.
// (mk(f, i): the marks word i of frame f - read and cleared, or OR-ed over ranks)
// (fill(i, mf): every frame's marks word i at once into mf[0 .. nframes), nframes <= kMaxCams)
template <class Marks, class Fill>
__device__ __forceinline__ void grid_u8_frames(uint4* __restrict__ grid, uint64_t nwords,
                                               uint32_t L, uint32_t block, uint32_t nblocks,
                                               uint32_t nframes, const Marks& mk,
                                               const SnapArgs& sn, const Fill& fill) {
    __shared__ uint32_t s_sc[4][kMaxCams];  // per wave: snapshot entries so far, per frame
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    // (the host passes snapshots only for <= kMaxCams frames; anything else keeps none)
    const bool keep_snaps = sn.idx != nullptr && nframes <= (uint32_t)kMaxCams;
    uint32_t W, seg;
    snap_layout(nwords, nblocks, W, seg);
    const uint32_t wave = block * 4u + wid;
    if (lane < (uint32_t)kMaxCams) s_sc[wid][lane] = 0u;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint64_t stride = (uint64_t)nblocks * blockDim.x;
    for (uint64_t i0 = (uint64_t)block * blockDim.x + (threadIdx.x & ~63u); i0 < nwords;
         i0 += stride) {  // wave-uniform
        const uint64_t i = i0 + lane;
        const bool act = i < nwords;
        uint4 v0 = make_uint4(0u, 0u, 0u, 0u), v1 = v0;
        grid_wave_load(grid, nwords, i0, v0, v1);
        auto step = [&](uint32_t f, uint32_t m) {
            v0.x = grid_word(v0.x, m, L);
            v0.y = grid_word(v0.y, m >> 4, L);
            v0.z = grid_word(v0.z, m >> 8, L);
            v0.w = grid_word(v0.w, m >> 12, L);
            v1.x = grid_word(v1.x, m >> 16, L);
            v1.y = grid_word(v1.y, m >> 20, L);
            v1.z = grid_word(v1.z, m >> 24, L);
            v1.w = grid_word(v1.w, m >> 28, L);
            if (f + 1 < nframes && keep_snaps) {
                const bool nz = act && ((v0.x | v0.y | v0.z | v0.w | v1.x | v1.y | v1.z | v1.w) != 0u);
                const unsigned long long b = __ballot(nz);
                if (b) {  // wave-uniform
                    const uint32_t base = s_sc[wid][f];
                    if (nz) {
                        const uint64_t e = ((uint64_t)f * W + wave) * seg + base +
                                           (uint32_t)__popcll(b & lanemask_lt());
                        sn.idx[e] = (uint32_t)i;
                        sn.data[2 * e] = v0;
                        sn.data[2 * e + 1] = v1;
                    }
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    if (lane == 0) s_sc[wid][f] = base + (uint32_t)__popcll(b);
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                }
            }
        };
        if (nframes <= (uint32_t)kMaxCams) {
            // every frame's marks word first: the loads are in flight together, not one memory
            // latency per frame (the batched update was ~B dependent round trips per word)
            uint32_t mf[kMaxCams];
#pragma unroll
            for (uint32_t f = 0; f < (uint32_t)kMaxCams; ++f) mf[f] = 0u;
            if (act) fill(i, mf);
#pragma unroll
            for (uint32_t f = 0; f < (uint32_t)kMaxCams; ++f) {
                if (f >= nframes) break;
                step(f, mf[f]);
            }
        } else {
            for (uint32_t f = 0; f < nframes; ++f) step(f, act ? mk(f, i) : 0u);
        }
        grid_wave_store(grid, nwords, i0, v0, v1);
    }
    if (keep_snaps && lane + 1 < nframes) sn.cnt[(uint64_t)lane * W + wave] = s_sc[wid][lane];
}

__device__ __forceinline__ void grid_u8_part_frames(uint4* __restrict__ grid,
                                                    uint32_t* __restrict__ marks, uint64_t nwords,
                                                    uint32_t L, uint32_t block, uint32_t nblocks,
                                                    uint32_t nframes, uint64_t mark_words,
                                                    const SnapArgs& sn) {
    grid_u8_frames(grid, nwords, L, block, nblocks, nframes,
                   [&](uint32_t f, uint64_t i) {
                       const uint32_t m = marks[f * mark_words + i];
                       if (m) marks[f * mark_words + i] = 0u;
                       return m;
                   },
                   sn,
                   [&](uint64_t i, uint32_t (&mf)[kMaxCams]) {
#pragma unroll
                       for (uint32_t f = 0; f < (uint32_t)kMaxCams; ++f)
                           if (f < nframes) mf[f] = marks[f * mark_words + i];
#pragma unroll
                       for (uint32_t f = 0; f < (uint32_t)kMaxCams; ++f)
                           if (f < nframes && mf[f]) marks[f * mark_words + i] = 0u;
                   });
}

// frame f's sparse snapshot into a zeroed dense u8 grid: one block per update wave
__global__ __launch_bounds__(256) void k_snap_expand(const uint32_t* __restrict__ idx,
                                                     const uint4* __restrict__ data,
                                                     const uint32_t* __restrict__ cnt, uint32_t f,
                                                     uint32_t W, uint32_t seg,
                                                     uint4* __restrict__ out) {
    const uint32_t w = blockIdx.x;
    const uint32_t n = cnt[(uint64_t)f * W + w];
    const uint64_t e0 = ((uint64_t)f * W + w) * seg;
    for (uint32_t j = threadIdx.x; j < n; j += blockDim.x) {
        const uint32_t i = idx[e0 + j];
        out[2 * (uint64_t)i] = data[2 * (e0 + j)];
        out[2 * (uint64_t)i + 1] = data[2 * (e0 + j) + 1];
    }
}

void snap_dims(uint64_t ncells, uint32_t nblocks, uint32_t* waves, uint32_t* seg) {
    const uint64_t nwords = (ncells + 31) / 32;
    const uint64_t stride = (uint64_t)nblocks * 256u;
    *waves = nblocks * 4u;
    *seg = (uint32_t)((nwords + stride - 1) / stride) * 64u;
}

hipError_t launch_snap_expand(const SnapArgs& sn, uint32_t frame, uint32_t nblocks,
                              uint64_t ncells, uint8_t* out, hipStream_t s) {
    uint32_t W, seg;
    snap_dims(ncells, nblocks, &W, &seg);
    hipError_t e = hipMemsetAsync(out, 0, (ncells + 31) / 32 * 32, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_snap_expand, dim3(W), dim3(256), 0, s, sn.idx, sn.data, sn.cnt, frame, W,
                       seg, reinterpret_cast<uint4*>(out));
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_grid_u8(uint4* __restrict__ grid,
                                                 uint32_t* __restrict__ marks, uint64_t nwords,
                                                 uint32_t L, GridSeq q) {
    const uint32_t f = grid_seq_enter<true>(q);
    grid_u8_part(grid, marks, nwords, L, blockIdx.x, gridDim.x, q);
    grid_seq_leave<true>(q, f, gridDim.x);
}

static unsigned grid_blocks(uint64_t work, unsigned per_block) {
    uint64_t b = (work + per_block - 1) / per_block;
    if (b > 2048) b = 2048;
    if (b == 0) b = 1;
    return (unsigned)b;
}

hipError_t launch_grid_u8(uint8_t* grid, uint32_t* marks, uint64_t ncells, uint32_t lifetime,
                          const GridSeq& q, hipStream_t s) {
    const uint64_t nwords = (ncells + 31) / 32;
    hipLaunchKernelGGL(k_grid_u8, dim3(grid_blocks(nwords, 256)), dim3(256), 0, s,
                       reinterpret_cast<uint4*>(grid), marks, nwords, lifetime, q);
    return hipGetLastError();
}

// nframes consecutive grid updates in one pass (batched multi-GPU exchange): frame f's marks are
// the OR over ranks of bits[r * rank_stride + f * frame_stride + word]; the updates are applied
// in frame order in registers, so the grid equals nframes sequential k_grid_u8 updates; sparse
// snapshots of the frames but the last as the fused pass writes them
__global__ __launch_bounds__(256) void k_grid_u8_batch(uint4* __restrict__ grid,
                                                       const uint32_t* __restrict__ bits,
                                                       uint64_t nwords, uint32_t nranks,
                                                       uint32_t nframes, uint64_t frame_stride,
                                                       uint64_t rank_stride, uint32_t L,
                                                       GridSeq q, SnapArgs sn) {
    const uint32_t f0 = grid_seq_enter<true>(q);
    grid_u8_frames(grid, nwords, L, blockIdx.x, gridDim.x, nframes,
                   [&](uint32_t f, uint64_t i) {
                       uint32_t m = 0;
                       for (uint32_t r = 0; r < nranks; ++r) m |= bits[r * rank_stride + f * frame_stride + i];
                       return m;
                   },
                   sn,
                   [&](uint64_t i, uint32_t (&mf)[kMaxCams]) {
                       for (uint32_t r = 0; r < nranks; ++r) {  // (a rank's frames in flight together)
                           const uint32_t* b = bits + r * rank_stride + i;
#pragma unroll
                           for (uint32_t f = 0; f < (uint32_t)kMaxCams; ++f)
                               if (f < nframes) mf[f] |= b[f * frame_stride];
                       }
                   });
    grid_seq_leave<true>(q, f0, gridDim.x);
}

uint32_t fused_grid_blocks(uint64_t ncells, uint32_t wpt) { return grid_blocks((ncells + 31) / 32, 256 * wpt); }
uint32_t batch_grid_blocks(uint64_t ncells) { return grid_blocks((ncells + 31) / 32, 256); }

hipError_t launch_grid_u8_batch(uint8_t* grid, const uint32_t* bits, uint64_t ncells,
                                uint32_t nranks, uint32_t nframes, uint64_t frame_stride,
                                uint64_t rank_stride, uint32_t lifetime, const GridSeq& q,
                                const SnapArgs& snap, hipStream_t s) {
    const uint64_t nwords = (ncells + 31) / 32;
    hipLaunchKernelGGL(k_grid_u8_batch, dim3(batch_grid_blocks(ncells)), dim3(256), 0, s,
                       reinterpret_cast<uint4*>(grid), bits, nwords, nranks, nframes,
                       frame_stride, rank_stride, lifetime, q, snap);
    return hipGetLastError();
}

// general u32 history (lifetime > 255) with a separate u8 output grid; 32 cells per thread
__global__ __launch_bounds__(256) void k_grid_u32(uint32_t* __restrict__ hist,
                                                  uint32_t* __restrict__ marks,
                                                  uint8_t* __restrict__ out8, uint64_t ncells,
                                                  uint32_t L, GridSeq q) {
    const uint32_t f = grid_seq_enter(q);
    const uint64_t nwords = (ncells + 31) / 32;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nwords;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t m = marks[i];
        for (uint32_t b = 0; b < 32; ++b) {
            const uint64_t c = 32 * i + b;
            if (c >= ncells) break;
            const uint32_t h = hist[c];
            const uint32_t dec = h >= 1u ? h - 1u : 0u;
            const uint32_t mv = ((m >> b) & 1u) ? L : 0u;
            const uint32_t nv = dec > mv ? dec : mv;
            hist[c] = nv;
            out8[c] = (uint8_t)(nv & 0xFFu);
        }
        if (m) marks[i] = 0u;
    }
    grid_seq_leave(q, f, gridDim.x);
}

hipError_t launch_grid_u32(uint32_t* hist, uint32_t* marks, uint8_t* out8, uint64_t ncells,
                           uint32_t lifetime, const GridSeq& q, hipStream_t s) {
    hipLaunchKernelGGL(k_grid_u32, dim3(grid_blocks((ncells + 31) / 32, 256)), dim3(256), 0, s,
                       hist, marks, out8, ncells, lifetime, q);
    return hipGetLastError();
}

// u8 history -> u32 history (switch to lifetime > 255)
__global__ __launch_bounds__(256) void k_widen(const uint8_t* __restrict__ g8,
                                               uint32_t* __restrict__ hist, uint64_t ncells,
                                               GridSeq q) {
    const uint32_t f = grid_seq_enter(q);
    for (uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; c < ncells;
         c += (uint64_t)gridDim.x * blockDim.x)
        hist[c] = g8[c];
    grid_seq_leave(q, f, gridDim.x);
}

hipError_t launch_widen_grid(const uint8_t* grid8, uint32_t* hist, uint64_t ncells,
                             const GridSeq& q, hipStream_t s) {
    hipLaunchKernelGGL(k_widen, dim3(grid_blocks(ncells, 256)), dim3(256), 0, s, grid8, hist,
                       ncells, q);
    return hipGetLastError();
}

// ---- standalone voxel keys / occupancy marks (stage-by-stage API) --------------------------------
__global__ __launch_bounds__(256) void k_coords(const float4* __restrict__ pts,
                                                const uint32_t* __restrict__ count,
                                                uint32_t* __restrict__ coords, VoxelParams v) {
    const uint32_t n = *count;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const float4 p = pts[i];
        coords[i] = voxel_key(p.x, p.y, p.z, v.vlo, v.vcs, v.vrcs, v.gmax, v.gs);
    }
}

hipError_t launch_coords(const float4* pts, const uint32_t* count, uint32_t nmax,
                         uint32_t* coords, const VoxelParams& v, hipStream_t s) {
    hipLaunchKernelGGL(k_coords, dim3(grid_blocks(nmax, 256)), dim3(256), 0, s, pts, count,
                       coords, v);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_scatter(const uint32_t* __restrict__ coords,
                                                 const uint32_t* __restrict__ count,
                                                 uint32_t* __restrict__ marks) {
    const uint32_t n = *count;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t k = coords[i];
        atomicOr(&marks[k >> 5], 1u << (k & 31u));
    }
}

hipError_t launch_scatter(const uint32_t* coords, const uint32_t* count, uint32_t nmax,
                          uint32_t* marks, hipStream_t s) {
    hipLaunchKernelGGL(k_scatter, dim3(grid_blocks(nmax, 256)), dim3(256), 0, s, coords, count,
                       marks);
    return hipGetLastError();
}

// ---- GPU voxelize: onesweep LSD radix sort + ordered group mean ---------------------------------
// Digit histograms of all passes in one read of the keys (when the compaction did not build
// them: large frames).  Keys of neighbouring points repeat, so each wave adds run lengths: the
// first lane of a run of equal digits adds the run (few LDS atomics on hot bins); each thread
// keeps 4 chunk loads in flight.
// Packed run keys (VoxelizeArgs::pack_runs): the engine's own runs are at most 64 points long (a
// run never leaves a 64-lane wave word of the compaction), so the first radix pass stores the
// run's length - 1 in key bits 26..31 - above every digit the passes extract (sort keys of <= 25
// bits) - and sorts the run's first point as the value instead of its index: the group phase then
// reads each sorted run's points range from its own key / value, not by a gather of
// run_start[index] (8 useful bytes per 64-128-B line: most of k_group_runs' traffic on C3).
constexpr uint32_t kRunLenShift = 26, kRunKeyMask = (1u << kRunLenShift) - 1u;

// frame of compacted point `idx` in a batch: the number of frame starts (after frame 0) <= idx
__device__ __forceinline__ uint32_t frame_of(const uint32_t* s_fstart, uint32_t nframes,
                                             uint32_t idx) {
    uint32_t f = 0;
    for (uint32_t j = 1; j < nframes; ++j) f += idx >= s_fstart[j] ? 1u : 0u;
    return f;
}

__device__ __forceinline__ void load_fstart(uint32_t* s_fstart, const uint32_t* fstart,
                                            uint32_t nframes) {
    if (nframes > 1)
        for (uint32_t j = threadIdx.x; j <= nframes; j += blockDim.x) s_fstart[j] = fstart[j];
}

__global__ __launch_bounds__(256) void k_sort_hist(const uint32_t* __restrict__ keys,
                                                   const uint32_t* __restrict__ count,
                                                   uint32_t npasses, uint32_t* __restrict__ hist,
                                                   uint32_t nframes, uint32_t fshift,
                                                   const uint32_t* __restrict__ fstart) {
    __shared__ uint32_t s_h[4 * 256];
    __shared__ uint32_t s_fstart[kMaxCams + 1];
    // (the item count and the frame starts read in one round, before the barrier)
    const uint32_t n = *count;
    const bool fr = fstart && nframes > 1;
    const uint32_t fsv = (fr ? fstart : count)[fr ? min(threadIdx.x, nframes) : 0u];
    for (uint32_t i = threadIdx.x; i < 4 * 256; i += 256) s_h[i] = 0;
    if (fr && threadIdx.x <= nframes) s_fstart[threadIdx.x] = fsv;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const uint32_t stride = gridDim.x * 256u;
    for (uint32_t base = blockIdx.x * 256u; base < n; base += 4u * stride) {  // block-uniform
        uint32_t k[4];
        // (the four keys loaded unconditionally at clamped indices first: loaded one by one
        // between the frame lookups, each waited for the one before)
#pragma unroll
        for (int q = 0; q < 4; ++q) k[q] = keys[min(base + q * stride + threadIdx.x, n - 1u)];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t i = base + q * stride + threadIdx.x;
            if (i >= n) k[q] = 0u;
            else if (fr) k[q] |= frame_of(s_fstart, nframes, i) << fshift;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t i = base + q * stride + threadIdx.x;
            const unsigned long long vm = __ballot(i < n);  // valid lanes: a prefix of the wave
            if (!vm) break;
            const uint32_t nv = (uint32_t)__popcll(vm);
            for (uint32_t p = 0; p < npasses; ++p) {
                const uint32_t d = radix_digit(k[q], p, npasses);
                const uint32_t pd = __shfl_up(d, 1, 64);
                const bool leader = (uint32_t)lane < nv && (lane == 0 || pd != d);
                const unsigned long long lm = __ballot(leader);
                if (leader) {
                    const unsigned long long after = lane == 63 ? 0ull : lm & (~0ull << (lane + 1));
                    const uint32_t end = after ? (uint32_t)(__ffsll((long long)after) - 1) : nv;
                    atomicAdd(&s_h[p * 256 + d], end - (uint32_t)lane);
                }
            }
        }
    }
    __syncthreads();
    uint32_t* rep = hist + (blockIdx.x % kHistReps) * 1024u;
    for (uint32_t i = threadIdx.x; i < radix_hist_span(npasses); i += 256)
        if (s_h[i]) atomicAdd(&rep[i], s_h[i]);
}

// Stable scatter of one 8-bit (NB = 256) or 9-bit (NB = 512, the last pass of a 25-bit batch key)
// digit.  Tile = 256 threads x PT keys: wave w owns keys
// [w*64*PT, (w+1)*64*PT) of the tile in slot-major order (slot j, lane l -> w*64*PT + j*64 + l),
// so ranking the slots in order with wave ballots keeps the sort stable.  Per-digit tile offsets
// come from a decoupled look-back over epoch-tagged {flag, count} granules.
template <int PT, int NB>
__global__ __launch_bounds__(kSortThreads) void k_sort_pass(
    const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin,
    uint32_t* __restrict__ kout, uint32_t* __restrict__ vout, const uint32_t* __restrict__ count,
    const uint32_t* __restrict__ ghist, unsigned long long* status, unsigned long long* gstatus,
    uint32_t* tile_ctr, uint32_t* epoch_word, uint32_t* err, uint32_t shift, uint32_t dbits,
    uint32_t grid_block0, uint4* grid, uint32_t* marks, uint64_t grid_nwords, uint32_t lifetime,
    GridSeq q, uint32_t nframes, uint32_t fshift, const uint32_t* __restrict__ fstart,
    uint64_t mark_words, SnapArgs snap, uint32_t* qreset, const uint32_t* __restrict__ pack_rs) {
    constexpr int kTile = kSortThreads * PT;
    // (first pass: the run-group queue counters start from zero for this voxelize's k_group_runs)
    if (qreset && blockIdx.x == 0 && threadIdx.x == 0) {
        qreset[0] = 0u;
        qreset[1] = 0u;
        qreset[2] = 0u;
    }
    if (blockIdx.x >= grid_block0) {  // fused historic-grid update (first pass only)
        const uint32_t f = grid_seq_enter<true>(q);
        if (nframes > 1)
            grid_u8_part_frames(grid, marks, grid_nwords, lifetime, blockIdx.x - grid_block0,
                                gridDim.x - grid_block0, nframes, mark_words, snap);
        else
            grid_u8_part(grid, marks, grid_nwords, lifetime, blockIdx.x - grid_block0,
                         gridDim.x - grid_block0, q);
        grid_seq_leave<true>(q, f, gridDim.x - grid_block0);
        return;
    }
    __shared__ uint32_t s_fstart[kMaxCams + 1];
    constexpr int R = NB / 256;  // digits per thread in the offset phase
    __shared__ uint32_t s_cnt[4][NB];
    __shared__ uint32_t s_base[NB];
    __shared__ uint32_t s_excl[NB];
    __shared__ uint32_t s_wave[4];
    __shared__ uint32_t s_tile, s_epoch;
    const uint32_t n = *count;
    const uint32_t ntiles = (n + kTile - 1) / kTile;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned long long ltm = lanemask_lt();
    const Tickets tk = tickets(ntiles, grid_block0);
    if (blockIdx.x >= tk.nblk) return;
    // first pass of a batch: the frame index joins the key above its voxel bits
    const bool add_frame = nframes > 1 && vin == nullptr && fstart != nullptr;
    // the block's prologue reads in one round: the digit counts (the kHistReps replicas of this
    // thread's digits), the frame starts (unconditionally, at a clamped index), then the epoch,
    // whose wait covers them (issued one after the other they were three dependent rounds)
    uint32_t hv0 = 0, hv1 = 0;
    {
        const uint32_t d = NB == 256 ? threadIdx.x : 2u * threadIdx.x;
#pragma unroll
        for (int r = 0; r < kHistReps; ++r) {
            hv0 += ghist[r * 1024 + d];
            if constexpr (NB == 512) hv1 += ghist[r * 1024 + d + 1];
        }
    }
    static_assert(kMaxCams + 1 <= kSortThreads, "one frame start per thread");
    const uint32_t fsv = (add_frame ? fstart : ghist)[min(threadIdx.x, nframes)];
    if (threadIdx.x == 0) s_epoch = read_epoch(epoch_word);
    if (add_frame && threadIdx.x <= nframes) s_fstart[threadIdx.x] = fsv;
    // the digit bases do not depend on the tile
    {
        uint32_t total;
        const uint32_t e = block_exclusive_scan(hv0 + hv1, total, s_wave);
        if constexpr (NB == 256) {
            s_base[threadIdx.x] = e;
        } else {
            s_base[2u * threadIdx.x] = e;
            s_base[2u * threadIdx.x + 1u] = e + hv0;
        }
    }
    for (bool first = true;; first = false) {  // persistent: tiles in ticket order
        if (!first && tk.oneshot) return;
        if (threadIdx.x == 0) s_tile = next_ticket(tile_ctr, tk, epoch_word, s_epoch);
        for (uint32_t i = threadIdx.x; i < 4 * NB; i += kSortThreads) (&s_cnt[0][0])[i] = 0;
        __syncthreads();
        const uint32_t tile = s_tile, epoch = s_epoch;
        if (tile >= ntiles) return;  // block-uniform

        uint32_t key[PT], val[PT], rank[PT];
        const uint32_t wbase = tile * kTile + w * 64 * PT;
#pragma unroll
        for (int j = 0; j < PT; ++j) {
            const uint32_t idx = wbase + j * 64 + lane;
            const bool ok = idx < n;
            key[j] = ok ? kin[idx] : 0xFFFFFFFFu;
            val[j] = ok ? (vin ? vin[idx] : idx) : 0u;
            if (add_frame && ok) key[j] |= frame_of(s_fstart, nframes, idx) << fshift;
            if (pack_rs && ok) {  // (first pass: the run's first point and its length in the key)
                const uint32_t ps = pack_rs[idx], len = pack_rs[idx + 1] - ps;
                if (len - 1u > 63u) atomicOr(err, 16u);  // (invariant: runs inside a wave word)
                val[j] = ps;
                key[j] |= (min(max(len, 1u), 64u) - 1u) << kRunLenShift;
            }
        }
#pragma unroll
        for (int j = 0; j < PT; ++j) {
            const uint32_t idx = wbase + j * 64 + lane;
            const bool ok = idx < n;
            const uint32_t d = (key[j] >> shift) & (NB - 1u);
            unsigned long long m = __ballot(ok);
            for (uint32_t b = 0; b < dbits; ++b) {
                const bool bit = (d >> b) & 1u;
                const unsigned long long bb = __ballot(bit);
                m &= bit ? bb : ~bb;
            }
            const uint32_t before = (uint32_t)__popcll(m & ltm);
            uint32_t base = 0;
            if (ok) base = s_cnt[w][d];
            rank[j] = base + before;
            __builtin_amdgcn_wave_barrier();
            if (ok && before == 0) s_cnt[w][d] = base + (uint32_t)__popcll(m);
            __builtin_amdgcn_wave_barrier();
        }
        __syncthreads();
        uint32_t tot[R], ex[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t d = threadIdx.x + 256u * r;
            tot[r] = 0;
#pragma unroll
            for (int ww = 0; ww < 4; ++ww) {
                const uint32_t c = s_cnt[ww][d];
                s_cnt[ww][d] = tot[r];
                tot[r] += c;
            }
        }
        lookback2_chans<R>(status, gstatus, tile, ntiles, tot, ex, epoch, err);
#pragma unroll
        for (int r = 0; r < R; ++r) s_excl[threadIdx.x + 256u * r] = ex[r];
        __syncthreads();
#pragma unroll
        for (int j = 0; j < PT; ++j) {
            const uint32_t idx = wbase + j * 64 + lane;
            if (idx < n) {
                const uint32_t dd = (key[j] >> shift) & (NB - 1u);
                const uint32_t pos = s_base[dd] + s_excl[dd] + s_cnt[w][dd] + rank[j];
                kout[pos] = key[j];
                vout[pos] = val[j];
            }
        }
        __syncthreads();  // LDS reused by the next tile
    }
}


// Voxel groups of the sorted keys and their outputs in ONE kernel (RadixGrouper::makeGroups,
// inc/radix_grouper.h:35-64, + averageGridCells / occupiedGridCells, inc/voxelize.h:9-71).
// Tile = 256 sorted keys: group starts (key != previous key), their ids by a block scan plus a
// decoupled look-back over tiles, then the outputs of the groups that START in this tile.
// average: the sequential f32 sum in stable (index) order, x/y/z divided by the count, w the
// un-divided sum.  The points of the tile's groups (up to kStagePts) are gathered into LDS by the
// whole block, then each group is summed by its owning thread; groups reaching past the staged
// range are summed by a wave (chunks staged through LDS, lanes 0..3 each run one component's
// dependent add chain).  !average: the voxel's lower corner (GridMeta::worldCoord).
// Block 0 also clears the digit histogram for the next voxelize (its last reader was the final
// sort pass).
constexpr int kStagePts = 512;   // points of a tile's groups staged in LDS (8 KiB)
constexpr uint32_t kPersistBlocks = 2048;  // blocks of a persistent sort / group launch
// above (capacity in 256-key tiles): group-id offsets by count + scan instead of the ticketed
// look-back in k_group (measured on MI355X: a batch of four VGA frames, ~1.8 K tiles, runs its
// group phase 1.7x faster through count + scan than through the look-back chain; one VGA frame,
// 1.2 K tiles of capacity, 4 % faster per frame): Tuning::group_scan_tiles.
// Staged groups of up to Tuning::small_group points are summed by their own thread
// (thread_group_sum: the four component chains side by side, one group per lane, the groups of a
// tile in parallel); longer ones by a wave (gdf_voxsum.hpp's stretch sums: a wave per group,
// serial over a block's groups).  Tuning::points_lane: k_group's staged long groups by 4-lane
// chains (measured slower on single VGA / 720p frames: 5.7 / 9.9 vs 6.1 / 11.6 Gpoints/s).

// p[0] + ... + p[n-1] per component, in order, by one thread: blocks of 4 points alternate between
// two register sets, the next block read while the current one is added (LDS latency off the
// add chains).  Reads stay inside [0, n) (no padding needed).
__device__ __forceinline__ float4 thread_group_sum(const float4* p, uint32_t n) {
    float ax = 0.f, ay = 0.f, az = 0.f, aw = 0.f;
    auto add = [&](const float4& q) {
        ax = ax + q.x;
        ay = ay + q.y;
        az = az + q.z;
        aw = aw + q.w;
    };
    uint32_t k = 0;
    if (n >= 8) {
        float4 a[4], b[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) a[q] = p[q];
#pragma unroll 1
        for (; k + 8 <= n; k += 8) {
#pragma unroll
            for (int q = 0; q < 4; ++q) b[q] = p[k + 4 + q];
            asm volatile("" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int q = 0; q < 4; ++q) add(a[q]);
            const uint32_t kn = k + 8 + 4 <= n ? k + 8 : k;  // (in range; unused past the loop)
#pragma unroll
            for (int q = 0; q < 4; ++q) a[q] = p[kn + q];
            asm volatile("" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int q = 0; q < 4; ++q) add(b[q]);
        }
        if (k + 4 <= n) {  // a[] holds points k .. k+3 exactly when k + 4 <= n here
#pragma unroll
            for (int q = 0; q < 4; ++q) add(a[q]);
            k += 4;
        }
    }
    for (; k < n; ++k) add(p[k]);
    return make_float4(ax, ay, az, aw);
}

constexpr uint32_t kChainPad = 16;  // LDS padding of staged point buffers
constexpr uint32_t kGatherChunk = 256;  // points per gathered chunk of a k_group wave
constexpr uint32_t kExtraRuns = 64;  // runs past a k_group_runs tile read for its last group
constexpr uint32_t kRunPasses = 4;   // staging windows per k_group_runs tile (mode 2)
constexpr uint32_t kHugeGroup = 32768;  // queued groups drawn first by k_group_runs_big (points)
constexpr uint32_t kHugeRuns = 2048;    // ... or runs (a crossing group's point estimate can be low)

// k_group_runs staging: positions [base, base + staged) of a tile's run stream (staged <=
// kRunStage) into s_pts.  Position q lies in the last run r with s_off[r] <= q (a branch-free
// search of the nruns <= 320 run offsets) at point s_ps[r] + q - s_off[r].  A thread resolves 4 of
// its positions, issues their 4 loads together and stores them after: the loop form waited on each
// load before its LDS store - up to 8 dependent gathers per 2048-position window, the staged-sums
// phase 82 % of a C2 tile (tools/gruns_trace.py).  (8 loads at once: 108 VGPRs and a spill.)
template <int kRunStage>
__device__ __forceinline__ void stage_run_points(float4* s_pts, const float4* __restrict__ pts,
                                                 const uint32_t* s_ps, const uint32_t* s_off,
                                                 uint32_t nruns, uint32_t base, uint32_t staged) {
    constexpr int kPer = kRunStage / kGroupThreads;
    constexpr int kB = kPer < 4 ? kPer : 4;
#pragma unroll
    for (int b0 = 0; b0 < kPer; b0 += kB) {
        if ((uint32_t)b0 * kGroupThreads >= staged) break;  // (block-uniform)
        uint32_t src[kB];
#pragma unroll
        for (int j = 0; j < kB; ++j) {
            const uint32_t k = threadIdx.x + (uint32_t)(b0 + j) * kGroupThreads;
            const uint32_t q = base + k;
            uint32_t lo = 0;
#pragma unroll
            for (uint32_t step = 256; step; step >>= 1)
                if (lo + step < nruns && s_off[lo + step] <= q) lo += step;
            src[j] = k < staged ? s_ps[lo] + (q - s_off[lo]) : 0u;  // (past the window: point 0, dropped)
        }
        // unconditional loads and stores (a conditional pair became a branch, a load and a wait
        // each); positions past `staged` hold point 0, never summed (s_pts has kRunStage slots)
        float4 v[kB];
#pragma unroll
        for (int j = 0; j < kB; ++j) v[j] = pts[src[j]];
#pragma unroll
        for (int j = 0; j < kB; ++j) s_pts[threadIdx.x + (uint32_t)(b0 + j) * kGroupThreads] = v[j];
    }
}

// comp[0] + comp[4] + ... + comp[4 (n - 1)] in order: one component of a staged group by one lane
// (its 4 lanes hold the group's 4 components); blocks of 8 values alternate between two register
// sets so the LDS reads of the next block overlap the additions of the current one.
__device__ __forceinline__ float lane_comp_chain_from(const float* comp, uint32_t n, float acc) {
    uint32_t k = 0;
    if (n >= 16) {
        float a[8], b[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) a[q] = comp[4 * q];
#pragma unroll 1
        for (; k + 16 <= n; k += 16) {
#pragma unroll
            for (int q = 0; q < 8; ++q) b[q] = comp[4 * (k + 8 + q)];
            asm volatile("" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int q = 0; q < 8; ++q) acc = acc + a[q];
            const uint32_t kn = k + 16 + 8 <= n ? k + 16 : k;  // (in range; unused past the loop)
#pragma unroll
            for (int q = 0; q < 8; ++q) a[q] = comp[4 * (kn + q)];
            asm volatile("" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int q = 0; q < 8; ++q) acc = acc + b[q];
        }
        if (k + 8 <= n) {  // a[] holds values k .. k+7 exactly when k + 8 <= n here
#pragma unroll
            for (int q = 0; q < 8; ++q) acc = acc + a[q];
            k += 8;
        }
    }
    for (; k < n; ++k) acc = acc + comp[4 * k];
    return acc;
}
__device__ __forceinline__ float lane_comp_chain(const float* comp, uint32_t n) {
    return lane_comp_chain_from(comp, n, 0.0f);
}

// (the wave's LDS writes visible to its own lanes)
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Voxel sums, one component per wave (gdf_voxsum.hpp): wave c of a 4-wave group sums component c.
// A staged group of cnt points (float4 AoS in LDS)
__device__ __forceinline__ float lds_group_comp(const float4* pts, uint32_t c, uint32_t cnt) {
    const float* f = reinterpret_cast<const float*>(pts) + c;
    return comp_stretch_sum<4>([&](uint32_t i) { return f[4 * i]; }, 0, cnt, 0.0f);
}
// a group's points pts[vals[k]], k in [s, e) (points mode), gathered from global memory
__device__ __forceinline__ float gather_group_comp(const uint32_t* __restrict__ vals,
                                                   const float4* __restrict__ pts, uint32_t c,
                                                   uint32_t s, uint32_t e) {
    const float* f = reinterpret_cast<const float*>(pts) + c;
    return comp_stretch_sum<4>([&](uint32_t i) { return f[4 * (size_t)vals[s + i]]; }, 0, e - s,
                               0.0f);
}

// Group starts per tile of kGroupThreads sorted keys (large frames: the tiles' group-id offsets
// then come from a scan of these counts instead of tickets and look-back in k_group).
// group starts per tile of the sorted keys; with gdone, also their group scan (arrive_and_scan:
// local offsets into offsets[], group totals into gtot[]) - no scan launches
__global__ __launch_bounds__(256) void k_group_count(const uint32_t* __restrict__ keys,
                                                     const uint32_t* __restrict__ count,
                                                     uint32_t* __restrict__ counts,
                                                     uint32_t* gdone, uint32_t* offsets,
                                                     uint32_t* gtot, uint32_t km,
                                                     uint32_t* __restrict__ first) {
    __shared__ uint32_t s_w[4], s_f[4];
    __shared__ uint32_t s_last;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t n = *count;
    const uint32_t ntiles = (n + kGroupThreads - 1) / kGroupThreads;
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {  // block-uniform
        const uint32_t i = t * kGroupThreads + threadIdx.x;
        // (both keys loaded unconditionally at clamped indices: one load round, where the
        // conditional second load waited for the first)
        const uint32_t kc = keys[min(i, n - 1u)] & km, kp = keys[i ? min(i - 1u, n - 1u) : 0u] & km;
        const uint32_t key = i < n ? kc : 0u;
        const uint32_t prev = (i < n && i > 0) ? kp : ~key;
        const unsigned long long b = __ballot(i < n && (i == 0 || key != prev));
        if (lane == 0) {
            s_w[wid] = (uint32_t)__popcll(b);
            s_f[wid] = b ? t * kGroupThreads + 64u * wid + (uint32_t)(__ffsll((long long)b) - 1) : 0xFFFFFFFFu;
        }
        __syncthreads();
        if (threadIdx.x == 0) publish_count(counts + t, s_w[0] + s_w[1] + s_w[2] + s_w[3]);
        if (first && threadIdx.x == 0) first[t] = min(min(s_f[0], s_f[1]), min(s_f[2], s_f[3]));
        if (gdone) arrive_and_scan(gdone, counts, offsets, gtot, t, ntiles, 1, 0u, &s_last);
        __syncthreads();
    }
}

__device__ __forceinline__ void group_corner(uint32_t key, const VoxelParams& vp, float* o) {
    const uint32_t gx = key % vp.gs[0];
    const uint32_t gy = (key / vp.gs[0]) % vp.gs[1];
    const uint32_t gz = key / (vp.gs[0] * vp.gs[1]);
    o[0] = (float)gx * vp.vcs[0] + vp.vlo[0];
    o[1] = (float)gy * vp.vcs[1] + vp.vlo[1];
    o[2] = (float)gz * vp.vcs[2] + vp.vlo[2];
    o[3] = 0.0f;
}

__global__ __launch_bounds__(kGroupThreads) __attribute__((amdgpu_waves_per_eu(7, 8))) void k_group(
    const uint32_t* __restrict__ keys, const uint32_t* __restrict__ vals,
    const uint32_t* __restrict__ count, const float4* __restrict__ pts, float* __restrict__ out,
    uint32_t* __restrict__ out_count, unsigned long long* status, unsigned long long* gstatus,
    uint32_t* tile_ctr, uint32_t* epoch_word, uint32_t* err, uint32_t* hist, int average,
    VoxelParams vp, uint32_t* marks, const uint32_t* tile_base, uint4* __restrict__ bigq,
    uint32_t* __restrict__ bigcnt, uint32_t bigcap, uint32_t nframes, uint32_t fshift,
    uint32_t* __restrict__ fvox, uint32_t small_max, uint32_t lane_chains,
    const uint32_t* tile_gtot) {
    __shared__ uint32_t s_wave[4];
    __shared__ uint32_t s_tile, s_epoch, s_excl, s_nbig, s_nq;
    __shared__ uint32_t s_start[kGroupThreads + 1];
    __shared__ uint32_t s_big[kGroupThreads];
    __shared__ float4 s_pts[kStagePts + kChainPad];
    __shared__ float4 s_gbuf[4][kGatherChunk];  // per-wave chunks of gathered groups
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t n = *count;
    const uint32_t ntiles = (n + kGroupThreads - 1) / kGroupThreads;
    // a batch's keys carry the frame above bit fshift: kmask strips it
    const uint32_t kmask = nframes > 1 ? (1u << fshift) - 1u : 0xFFFFFFFFu;
    if (blockIdx.x == 0) {
        for (uint32_t i = threadIdx.x; i < kHistWords; i += kGroupThreads) hist[i] = 0;
        if (ntiles == 0 && threadIdx.x == 0) *out_count = 0;  // n == 0
        if (ntiles == 0 && fvox)
            for (uint32_t f = threadIdx.x; f <= nframes; f += kGroupThreads) fvox[f] = 0;
    }
    // tile_base (large frames): the group-id offset of every tile is known (k_group_count + scan),
    // so blocks walk the tiles by index with no ticket and no look-back; otherwise tickets +
    // decoupled look-back in one launch
    const Tickets tk = tickets(ntiles, gridDim.x);
    if (!tile_base && blockIdx.x >= tk.nblk) return;
    if (!tile_base && threadIdx.x == 0) s_epoch = read_epoch(epoch_word);
    if (threadIdx.x == 0) s_nq = 0;
    uint32_t walk = blockIdx.x;
    for (bool first = true;; first = false) {  // persistent
    if (!first && !tile_base && tk.oneshot) return;
    // (group-scanned offsets: the group-local offset + the totals of the groups before)
    const uint32_t gpre = tile_base && tile_gtot && wid == 0 && walk < ntiles
                              ? wave_group_prefix(tile_gtot, walk) : 0u;
    if (threadIdx.x == 0) {
        if (tile_base) {
            s_tile = walk;
            s_excl = walk < ntiles ? tile_base[walk] + gpre : 0u;
        } else {
            s_tile = next_ticket(tile_ctr, tk, epoch_word, s_epoch);
        }
        s_nbig = 0;
    }
    walk += gridDim.x;
    __syncthreads();
    const uint32_t tile = s_tile, epoch = s_epoch;
    if (tile >= ntiles) {  // block-uniform
        if (bigq && threadIdx.x == 0) bigcnt[blockIdx.x] = s_nq;
        return;
    }
    const uint32_t i = tile * kGroupThreads + threadIdx.x;
    const uint32_t tend = min(n, (tile + 1) * kGroupThreads);
    const uint32_t key = i < n ? keys[i] : 0u;
    const uint32_t prev = (i < n && i > 0) ? keys[i - 1] : ~key;
    const bool start = i < n && (i == 0 || key != prev);
    uint32_t total;
    const uint32_t local = block_exclusive_scan(start ? 1u : 0u, total, s_wave);
    if (start) s_start[local] = i;
    __syncthreads();
    // Overlapped: every lane issues the staging gather of the points from the tile's first group
    // start on (kStagePts positions; extra positions are harmless), wave 0 resolves the group-id
    // prefix (look-back) and wave 1 finds where the tile's last group ends.
    // (a tile without a group start - inside a group that began earlier - still publishes its
    // zero count for the look-back)
    const uint32_t S0 = total ? s_start[0] : n;
    const uint32_t staged = min(n - S0, (uint32_t)kStagePts);
    float4 sp[kStagePts / kGroupThreads];
    if (average) {
#pragma unroll
        for (int q = 0; q < kStagePts / kGroupThreads; ++q) {
            const uint32_t j = threadIdx.x + kGroupThreads * q;
            if (j < staged) sp[q] = pts[vals[S0 + j]];
        }
    }
    if (wid == 0) {
        const uint32_t ex = tile_base ? s_excl
                                      : lookback2_wave(status, gstatus, tile, ntiles, total, epoch, err);
        if (lane == 0) {
            s_excl = ex;
            if (tile == ntiles - 1) {
                *out_count = ex + total;
                if (fvox)  // frames after the last point's frame start at the end
                    for (uint32_t f = (keys[n - 1] >> fshift) + 1; f <= nframes; ++f)
                        fvox[f] = ex + total;
            }
        }
    } else if (wid == 1 && total) {
        // end of the tile's last group = first index >= tend whose (sorted) key exceeds the
        // tile's last key: the next 64 keys, then a 64-ary search of the rest (groups of
        // thousands of points: a few round trips instead of one per 64 keys)
        const uint32_t lastkey = keys[tend - 1];
        uint32_t lo = tend, hi = n;  // keys[tend, lo) <= lastkey; hi = n or keys[hi] > lastkey
        while (lo < hi) {
            const uint32_t len = hi - lo;
            const uint32_t step = len <= 64u || lo == tend ? 1u : (len + 63u) / 64u;
            const uint32_t j = lo + (uint32_t)lane * step;
            const unsigned long long ch = __ballot(j < hi && keys[j] > lastkey);
            if (ch) {
                const uint32_t f = (uint32_t)(__ffsll((long long)ch) - 1);
                hi = lo + f * step;
                if (step == 1u) break;
                lo = f ? lo + (f - 1u) * step + 1u : lo;
            } else {
                const uint32_t lastp = lo + min(63u, (len - 1u) / step) * step;  // last probe
                lo = lastp + 1u;
            }
        }
        if (lane == 0) s_start[total] = hi;
    }
    if (average) {
#pragma unroll
        for (int q = 0; q < kStagePts / kGroupThreads; ++q) {
            const uint32_t j = threadIdx.x + kGroupThreads * q;
            if (j < staged) s_pts[j] = sp[q];
        }
    }
    __syncthreads();
    if (total == 0) continue;  // block-uniform (nothing of this tile is read after the barrier)
    // one group per thread: staged groups summed here in index order, the rest queued for waves
    if (threadIdx.x < total) {
        const uint32_t g = s_excl + threadIdx.x;
        const uint32_t s = s_start[threadIdx.x], e = s_start[threadIdx.x + 1];
        float* o = out + 4 * (size_t)g;
        if (marks) {  // voxel_grid_occupancy_of_points: one mark per occupied voxel
            const uint32_t key = keys[s] & kmask;
            atomicOr(marks + (key >> 5), 1u << (key & 31u));
        }
        if (fvox) {  // a batch: the first voxel of each frame (frames without points share it)
            const uint32_t fc = keys[s] >> fshift;
            const uint32_t f0 = s == 0 ? 0u : (keys[s - 1] >> fshift) + 1u;
            for (uint32_t f = f0; f <= fc; ++f) fvox[f] = g;
        }
        if (!average) {
            float c[4];
            group_corner(keys[s] & kmask, vp, c);
            *reinterpret_cast<float4*>(o) = make_float4(c[0], c[1], c[2], c[3]);
        } else if (e - S0 <= staged && e - s <= small_max) {
            const float4 a = thread_group_sum(s_pts + (s - S0), e - s);
            const float fc = (float)(e - s);
            *reinterpret_cast<float4*>(o) = make_float4(a.x / fc, a.y / fc, a.z / fc, a.w);
        } else if (bigq && e - S0 > staged) {
            // a voxel reaching past the staged points (at most the tile's last group): summed
            // by k_group_big, so this block's other waves do not wait at the tile barrier for
            // its chain (a block walks ~20 tiles; a voxel can hold 10^4 points)
            bigq[(size_t)blockIdx.x * bigcap + s_nq] = make_uint4(g, s, e, 0u);
            s_nq = s_nq + 1u;
        } else {
            s_big[atomicAdd(&s_nbig, 1u)] = threadIdx.x;
        }
    }
    __syncthreads();
    const uint32_t nbig = s_nbig;
    // staged long groups: 4 lanes each, one component chain per lane (16 groups per wave), or
    // (lane_chains = 0) the 4 waves' stretch sums, wave = component
    for (uint32_t b = ((uint32_t)lane >> 2) * 4u + (uint32_t)wid; lane_chains && b < nbig; b += 64u) {
        const uint32_t li = s_big[b];
        const uint32_t s = s_start[li], e = s_start[li + 1];
        if (e - S0 > staged) continue;
        const uint32_t c = (uint32_t)lane & 3u;
        const float acc = lane_comp_chain(reinterpret_cast<const float*>(s_pts + (s - S0)) + c, e - s);
        out[4 * (size_t)(s_excl + li) + c] = c < 3 ? acc / (float)(e - s) : acc;
    }
    for (uint32_t b = 0; !lane_chains && b < nbig; ++b) {  // staged: the 4 waves, wave = component
        const uint32_t li = s_big[b];
        const uint32_t s = s_start[li], e = s_start[li + 1];
        if (e - S0 > staged) continue;  // (block-uniform)
        store_comp_mean(out + 4 * (size_t)(s_excl + li), wid,
                        lds_group_comp(s_pts + (s - S0), wid, e - s), e - s);
    }
    // groups past the staged points (small frames: no queue): a wave per group, chunks of
    // kGatherChunk points gathered through vals into the wave's LDS buffer - the next chunk's
    // loads in flight while lanes 0..3 chain the current one, one component each
    for (uint32_t b = wid; b < nbig; b += 4u) {
        const uint32_t li = s_big[b];
        const uint32_t s = s_start[li], e = s_start[li + 1];
        if (e - S0 <= staged) continue;  // (wave-uniform)
        float4 r[kGatherChunk / 64];
#pragma unroll
        for (int q = 0; q < (int)kGatherChunk / 64; ++q) {
            const uint32_t k = s + q * 64u + (uint32_t)lane;
            r[q] = k < e ? pts[vals[k]] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        float acc = 0.0f;
#pragma unroll 1
        for (uint32_t c = s; c < e; c += kGatherChunk) {
#pragma unroll
            for (int q = 0; q < (int)kGatherChunk / 64; ++q) s_gbuf[wid][q * 64 + lane] = r[q];
            const uint32_t cn = c + kGatherChunk;
#pragma unroll
            for (int q = 0; q < (int)kGatherChunk / 64; ++q) {
                const uint32_t k = cn + q * 64u + (uint32_t)lane;
                r[q] = k < e ? pts[vals[k]] : make_float4(0.f, 0.f, 0.f, 0.f);
            }
            wave_sync();
            if (lane < 4)
                acc = lane_comp_chain_from(reinterpret_cast<const float*>(&s_gbuf[wid][0]) + lane,
                                           min(e - c, kGatherChunk), acc);
            wave_sync();
        }
        if (lane < 4) out[4 * (size_t)(s_excl + li) + lane] = lane < 3 ? acc / (float)(e - s) : acc;
    }
    __syncthreads();  // LDS reused by the next tile
    }
}

// The long voxels queued by k_group (large frames): one block (4 waves, one per component) per
// voxel, independent of tiles and block barriers; the same sums as k_group's wave path.
__global__ __launch_bounds__(256) void k_group_big(const uint32_t* __restrict__ vals,
                                                   const float4* __restrict__ pts,
                                                   float* __restrict__ out,
                                                   const uint4* __restrict__ bigq,
                                                   const uint32_t* __restrict__ bigcnt,
                                                   uint32_t nblocks, uint32_t bigcap) {
    const uint32_t wid = threadIdx.x >> 6;  // (the component)
    const uint64_t nslots = (uint64_t)nblocks * bigcap;
    for (uint64_t slot = blockIdx.x; slot < nslots; slot += gridDim.x) {  // block-uniform
        const uint32_t b = (uint32_t)(slot / bigcap), k = (uint32_t)(slot % bigcap);
        if (k >= bigcnt[b]) continue;
        const uint4 q = bigq[slot];
        const float sum = gather_group_comp(vals, pts, wid, q.y, q.z);
        store_comp_mean(out + 4 * (size_t)q.x, wid, sum, q.z - q.y);
    }
}

// ---- voxel groups over sorted RUNS (run mode) ---------------------------------------------------
// The sort ordered runs of equal keys (run r = points run_start[r] .. run_start[r+1]-1, contiguous
// in the compaction); a voxel group is a maximal sequence of sorted runs with one key and its
// points are the concatenation of its runs' points - the same stable index order the reference
// sums in (inc/voxelize.h:29-35), read as contiguous ranges with no per-point (key, index) list.
// k_group_runs: points of a tile's groups staged in LDS (Tuning::run_stage: 512 or 2048), and the
// size up to which a staged group is summed in-block (Tuning::run_inblock; larger ones are queued;
// measured: C2 / 720p x4 / 4K best or within noise of best at 1024).  Staged groups above
// small_group (Tuning::run_wave): 0 queued for k_group_runs_big, 1 a wave's stretch sums
// (wave_group_sum), 2 four lanes' chains (lane_comp_chain, default).
// Persistent grids of the radix passes and of the group phase, at most (Tuning::sort_blocks /
// group_blocks): the launches are sized by the capacity (the item count is on the device), and a
// run sort's ~10x fewer items leave most blocks with no tile.
// Chunks of k_group_runs_big (one 4-wave block per queued group; grid Tuning::run_big_blocks): 1 K
// points (Q = 16) or 512 (Q = 8); Tuning::run_q16 0 never 1 K, 1 always, 2 (default) for single
// frames - 4K depth frames (voxels of ~20 K points) and rollbuffer windows (C3: 4.72 -> 4.49 ms per
// frame with 1 K chunks) - and 512 for multi-frame batches.  k_group_runs_big sums the groups below
// the huge region one per wave (wave_stream_sum) when the queue is long (Tuning::run_wave_mode 1;
// 0: every group in block mode, 2: wave mode whatever the queue's length).


// Wave64 inclusive sum scan on DPP (gdf_voxsum.hpp dpp_iscan).
__device__ __forceinline__ uint32_t dpp_sum_scan(uint32_t x) { return (uint32_t)dpp_iscan((int)x); }

struct RunRec {
    uint32_t ps, len;
};

// A group's points stream through a 4-wave block in order: batches of 256 sorted runs (4 per lane,
// runs 4 l .. 4 l + 3 in lane l; the records rps / rlen - first point, length - are indexed by
// sorted run, contiguous, and read two batches ahead), their points in chunks of 64 x Q positions
// - position -> run by a max-scan of the runs' first positions - loaded coalesced one chunk ahead
// (across batch boundaries too); wave w loads rows w, w + 4, ... of a chunk, the block transposes
// the chunk into LDS rows per component and wave c sums component c (gdf_voxsum.hpp
// rows_chunk_sum) - the reference's sequential f32 sum, in stable order.  256-run batches keep
// chunks nearly full where runs are short (4K frames: ~100 points per run of a long voxel, C3
// windows ~11): a chunk never spans two batches.
constexpr int kRunsPerLane = 4;
struct RunRecs {
    uint32_t ps[kRunsPerLane], len[kRunsPerLane];
};
struct RunBatch {
    uint32_t off[kRunsPerLane], len[kRunsPerLane];  // runs 4 lane + j: first batch position, length
    uint32_t base[kRunsPerLane];                    // first point - first batch position
    uint32_t T;                                     // the batch's points (wave-uniform)
};

__device__ __forceinline__ RunBatch run_batch(const RunRecs& r) {
    RunBatch b;
    uint32_t acc = 0;
#pragma unroll
    for (int j = 0; j < kRunsPerLane; ++j) {
        b.off[j] = acc;
        acc += r.len[j];
    }
    const uint32_t x = dpp_sum_scan(acc);
#pragma unroll
    for (int j = 0; j < kRunsPerLane; ++j) {
        b.off[j] += x - acc;
        b.len[j] = r.len[j];
        b.base[j] = r.ps[j] - b.off[j];
    }
    b.T = (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
    return b;
}

__device__ __forceinline__ RunRecs run_recs(const uint32_t* __restrict__ rps,
                                            const uint32_t* __restrict__ rlen, uint32_t r0,
                                            uint32_t re) {
    RunRecs q;
    const uint32_t r = r0 + kRunsPerLane * (threadIdx.x & 63);
#pragma unroll
    for (int j = 0; j < kRunsPerLane; ++j) {
        const bool ok = r + j < re;
        q.ps[j] = ok ? rps[r + j] : 0u;
        q.len[j] = ok ? rlen[r + j] : 0u;
    }
    return q;
}

// This wave's copy of a batch's run bases (s_base[wave][run]) for fetch_rows4.
__device__ __forceinline__ void put_bases(const RunBatch& bt, uint32_t* s_base) {
    const uint32_t lane = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < kRunsPerLane; ++j) s_base[kRunsPerLane * lane + j] = bt.base[j];
}

// N independent inclusive wave64 max-scans on DPP, step by step (values >= -1: row shifts inside
// the 16-lane rows, then the row broadcasts of lanes 15 and 31)
template <int N>
__device__ __forceinline__ void dpp_max_scan_n(int (&v)[N]) {
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = max(v[i], __builtin_amdgcn_update_dpp(-1, v[i], 0x111, 0xf, 0xf, false));
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = max(v[i], __builtin_amdgcn_update_dpp(-1, v[i], 0x112, 0xf, 0xf, false));
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = max(v[i], __builtin_amdgcn_update_dpp(-1, v[i], 0x114, 0xf, 0xf, false));
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = max(v[i], __builtin_amdgcn_update_dpp(-1, v[i], 0x118, 0xf, 0xf, false));
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = max(v[i], __builtin_amdgcn_update_dpp(-1, v[i], 0x142, 0xa, 0xf, false));
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = max(v[i], __builtin_amdgcn_update_dpp(-1, v[i], 0x143, 0xc, 0xf, false));
}

// This wave's Q / 4 consecutive rows of the chunk at batch position c: the first positions of the
// runs starting in them marked in s_mark (disjoint between the waves; a run outside them marks a
// scratch slot past the chunk - no branches), the rows max-scanned side by side, the first one
// carried in by the last run starting before it (a ballot count: every run holds >= 1 point, so
// the runs' first positions increase with the run index) and each next one by the row before; a
// position's point is base[run] + position (s_base: this wave's copy of the batch's bases).
// Positions past the batch load point 0 (never summed), and no select touches the loaded values:
// the loads stay in flight until the chunk is stored.
// WAVE: the wave fetches a chunk of its own, Q / 4 rows from batch position c (wave mode of
// k_group_runs_big; s_mark then holds 64 (Q / 4 + 1) marks of this wave).
template <int Q, bool WAVE = false>
__device__ __forceinline__ void fetch_rows4(const RunBatch& bt, uint32_t c, int* s_mark,
                                            const uint32_t* s_base, const float4* __restrict__ pts,
                                            float4 (&p)[Q / 4]) {
    constexpr int RPW = Q / 4;  // rows per wave
    constexpr uint32_t CH = WAVE ? 64u * RPW : 64u * Q;
    const uint32_t lane = threadIdx.x & 63, wid = WAVE ? 0u : threadIdx.x >> 6;
    const uint32_t row0 = wid * RPW, pos_w = c + 64u * row0;
#pragma unroll
    for (int i = 0; i < RPW; ++i) s_mark[64u * (row0 + i) + lane] = -1;
    wave_sync();
#pragma unroll
    for (int j = 0; j < kRunsPerLane; ++j) {
        const uint32_t o = bt.off[j];
        const bool mine = bt.len[j] != 0u && o - pos_w < 64u * RPW;
        s_mark[mine ? o - c : CH + lane] = (int)(kRunsPerLane * lane + j);
    }
    wave_sync();
    int before = 0;
#pragma unroll
    for (int j = 0; j < kRunsPerLane; ++j)
        before += (int)__popcll(__ballot(bt.len[j] != 0u && bt.off[j] < pos_w));
    int mk[RPW];
#pragma unroll
    for (int i = 0; i < RPW; ++i) mk[i] = s_mark[64u * (row0 + i) + lane];
    dpp_max_scan_n<RPW>(mk);
    int carry = before - 1;  // (wave-uniform)
    uint32_t b[RPW];
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
        const int m = max(mk[i], carry);
        carry = max(carry, __builtin_amdgcn_readlane(mk[i], 63));
        b[i] = s_base[max(m, 0)];
    }
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
        const uint32_t pos = pos_w + 64u * i + lane;
        p[i] = pts[pos < bt.T ? b[i] + pos : 0u];
    }
}

#ifdef GDF_TRACE_GROUPS
// (diagnostic build, tools/group_trace.py) per queued group: wall clock start / end, points,
// chunks, cycles in the sums / at the barriers / in the fetches, and the CU it ran on
constexpr uint32_t kTraceSlots = 1u << 16;
__device__ unsigned long long g_gtrace[kTraceSlots][8];
#define GDF_TCLK(var) const unsigned long long var = clock64()
#else
#define GDF_TCLK(var)
#endif

// The sum of component wid of sorted runs [rs, re) (one 4-wave block); npts = the group's points.
template <int Q>
__device__ __forceinline__ float block_stream_sum(const uint32_t* __restrict__ rps,
                                                  const uint32_t* __restrict__ rlen, uint32_t rs,
                                                  uint32_t re, const float4* __restrict__ pts,
                                                  int* s_mark, uint32_t* s_base,
                                                  float (*s_soa)[kRowStride * Q], uint32_t& npts,
                                                  unsigned long long* tr) {
    static_assert(Q % 4 == 0 && Q <= 16, "rows_chunk_sum takes up to 16 rows");
    constexpr uint32_t CH = 64u * Q, NB = 64u * kRunsPerLane;  // chunk points, batch runs
    const uint32_t wid = threadIdx.x >> 6;
    npts = 0;
    float s = 0.0f;
    ChainMode cm;
    RunBatch cur = run_batch(run_recs(rps, rlen, rs, re));
    RunRecs rec1 = run_recs(rps, rlen, rs + NB, re);      // batch 1
    RunRecs rec2 = run_recs(rps, rlen, rs + 2u * NB, re);  // batch 2
    float4 p[Q / 4];
    put_bases(cur, s_base);
    wave_sync();
    fetch_rows4<Q>(cur, 0, s_mark, s_base, pts, p);
    uint32_t rb = rs, c = 0;
    while (true) {  // block-uniform: one chunk per iteration
        const uint32_t n = min(CH, cur.T - c);
        GDF_TCLK(b0);
        __syncthreads();  // every wave has summed the previous chunk
        GDF_TCLK(b1);
#pragma unroll
        for (int i = 0; i < Q / 4; ++i) {
            const uint32_t k = kRowStride * (wid * (Q / 4) + i) + (threadIdx.x & 63);
            s_soa[0][k] = p[i].x;
            s_soa[1][k] = p[i].y;
            s_soa[2][k] = p[i].z;
            s_soa[3][k] = p[i].w;
        }
        // the next chunk, loaded while this one is summed: the rest of this batch, or the next
        // batch's first chunk (whose records were read two batches ago); none: T = 0
        const bool more = c + CH < cur.T;
        const bool next_batch = !more && rb + NB < re;
        RunBatch fb = cur;
        uint32_t cn = c + CH;
        if (next_batch) {
            fb = run_batch(rec1);
            rec1 = rec2;
            rec2 = run_recs(rps, rlen, rb + 3u * NB, re);
            cn = 0;
        } else if (!more) {
            fb.T = 0;
        }
        GDF_TCLK(b2);
        __syncthreads();  // the chunk is in LDS
        GDF_TCLK(b3);
        if (next_batch) {
            put_bases(fb, s_base);
            wave_sync();
        }
        if (more || next_batch) fetch_rows4<Q>(fb, cn, s_mark, s_base, pts, p);
        GDF_TCLK(b4);
        s = rows_chunk_sum(s_soa[wid], n, s, cm);
        GDF_TCLK(b5);
#ifdef GDF_TRACE_GROUPS
        if (tr) {
            tr[0] += (b1 - b0) + (b3 - b2);  // barriers
            tr[1] += b2 - b1;                // LDS stores (waits for the loads)
            tr[2] += b4 - b3;                // fetch issue
            tr[3] += b5 - b4;                // sum
            tr[4] += 1;
        }
#else
        (void)tr;
#endif
        npts += n;
        if (more) {
            cur = fb;
            c += CH;
        } else if (next_batch) {
            rb += NB;
            cur = fb;
            c = 0;
        } else {
            break;
        }
    }
    return s;
}

// Wave mode of k_group_runs_big: a queued group streamed by ONE wave, its 4 components side by
// side (rows4c_chunk: lanes 16 c .. 16 c + 15 sum component c, stretch rows or the chain per
// component), chunks of 256 points (4 rows) fetched by the wave itself TWO chunks ahead (a
// chunk's adds take ~1 K cycles, a fetch's memory latency more), the run batches as
// block_stream_sum's.  A block's 4 waves sum 4 different groups, so a SIMD runs as many chains
// (the z sums of a window's floor: chain rows) as it holds waves, where the block form ran one per
// group and its other 3 waves waited at the chunk barriers.  Returns this lane's component sum;
// npts = the group's points.
struct WaveCursor {  // the fetch position: batch (records of the next two read ahead), chunk
    RunBatch b;
    RunRecs rec1, rec2;
    uint32_t rb, c;
    bool live;
};

__device__ __forceinline__ uint32_t wave_fetch(WaveCursor& f, const uint32_t* __restrict__ rps,
                                               const uint32_t* __restrict__ rlen, uint32_t re,
                                               const float4* __restrict__ pts, int* s_mark,
                                               uint32_t* s_base, float4 (&p)[4]) {
    constexpr uint32_t CH = 256u, NB = 64u * kRunsPerLane;
    if (!f.live) return 0u;  // (wave-uniform)
    fetch_rows4<16, true>(f.b, f.c, s_mark, s_base, pts, p);
    const uint32_t n = min(CH, f.b.T - f.c);
    if (f.c + CH < f.b.T) {
        f.c += CH;
    } else if (f.rb + NB < re) {
        f.b = run_batch(f.rec1);
        f.rec1 = f.rec2;
        f.rec2 = run_recs(rps, rlen, f.rb + 3u * NB, re);
        f.rb += NB;
        f.c = 0;
        wave_sync();  // (this fetch's base reads are done)
        put_bases(f.b, s_base);
        wave_sync();
    } else {
        f.live = false;
    }
    return n;
}

__device__ __forceinline__ void wave_store_chunk(float* wsoa, const float4 (&p)[4], uint32_t n) {
    const uint32_t lane = threadIdx.x & 63;
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // values past n: -0.0, which leaves any sum as it is
        const bool in = 64u * i + lane < n;
        const uint32_t k = i * kRowStride + lane;
        wsoa[0 * kWaveCompStride + k] = in ? p[i].x : -0.0f;
        wsoa[1 * kWaveCompStride + k] = in ? p[i].y : -0.0f;
        wsoa[2 * kWaveCompStride + k] = in ? p[i].z : -0.0f;
        wsoa[3 * kWaveCompStride + k] = in ? p[i].w : -0.0f;
    }
}

__device__ __forceinline__ float wave_stream_sum(const uint32_t* __restrict__ rps,
                                                 const uint32_t* __restrict__ rlen, uint32_t rs,
                                                 uint32_t re, const float4* __restrict__ pts,
                                                 int* s_mark, uint32_t* s_base, float* wsoa,
                                                 uint32_t& npts) {
    constexpr uint32_t NB = 64u * kRunsPerLane;
    WaveCursor f;
    f.b = run_batch(run_recs(rps, rlen, rs, re));
    f.rec1 = run_recs(rps, rlen, rs + NB, re);
    f.rec2 = run_recs(rps, rlen, rs + 2u * NB, re);
    f.rb = rs;
    f.c = 0;
    f.live = true;
    put_bases(f.b, s_base);
    wave_sync();
    float4 p0[4], p1[4];
    uint32_t n0 = wave_fetch(f, rps, rlen, re, pts, s_mark, s_base, p0);
    uint32_t n1 = wave_fetch(f, rps, rlen, re, pts, s_mark, s_base, p1);
    float s = 0.0f;
    npts = 0;
    while (n0) {  // wave-uniform: two chunks per iteration, the buffers alternating
        wave_sync();  // (the previous chunk's rows are read)
        wave_store_chunk(wsoa, p0, n0);
        wave_sync();
        const uint32_t m0 = n0;
        n0 = wave_fetch(f, rps, rlen, re, pts, s_mark, s_base, p0);
        s = rows4c_chunk(wsoa, m0, s);
        npts += m0;
        if (!n1) break;
        wave_sync();
        wave_store_chunk(wsoa, p1, n1);
        wave_sync();
        const uint32_t m1 = n1;
        n1 = wave_fetch(f, rps, rlen, re, pts, s_mark, s_base, p1);
        s = rows4c_chunk(wsoa, m1, s);
        npts += m1;
    }
    return s;
}

// Groups of one tile of 256 sorted runs: group starts (key != previous run's key), group ids by a
// block scan plus the tile's offset (count + scan, or tickets + look-back as k_group), the end of
// the tile's last group (a search of the run keys past the tile).  The points of the tile's groups
// are staged (up to kRunStage from the first group start); groups of <= small_max staged points
// are summed by their thread, longer staged ones by a wave from LDS, and the others (past the
// staged points, or continuing past the tile) are queued for k_group_runs_big - one append per
// group, so a block never waits on a long chain.  Marks, frame voxel starts and corners as k_group.
// WAVE (Tuning::run_wave): staged groups above small_max are 0 queued like the unstaged ones, 1 summed
// by a wave from LDS (wave_group_sum: per-wave transpose buffers, 59.4 instead of 37.6 KB of LDS -
// 2 blocks per CU, not 4), 2 summed by 4 lanes each, one component chain per lane (16 groups per
// wave, the tile's long groups dealt round-robin over the 4 waves).
#ifdef GDF_TRACE_GROUPS
// (diagnostic build, tools/gruns_trace.py) per k_group_runs tile: the wall clock (100 MHz) at block
// entry, tile start, after the run records and block scans, after the tile's offset / last-group
// end, after the staged sums, at the tile's end; the hardware id of wave 0, the block
constexpr uint32_t kRunTraceSlots = 1u << 14;
__device__ unsigned long long g_rtrace[kRunTraceSlots][8];
#define GDF_RSTAMP(var) const unsigned long long var = wall_clock64()
#else
#define GDF_RSTAMP(var)
#endif
template <int kRunStage, int WAVE>
__global__ __launch_bounds__(kGroupThreads) void k_group_runs(
    const uint32_t* __restrict__ keys, const uint32_t* __restrict__ rvals,
    const uint32_t* __restrict__ count, const uint32_t* __restrict__ run_start,
    const float4* __restrict__ pts, float* __restrict__ out, uint32_t* __restrict__ out_count,
    unsigned long long* status, unsigned long long* gstatus, uint32_t* tile_ctr,
    uint32_t* epoch_word, uint32_t* err, uint32_t* hist, int average, VoxelParams vp,
    uint32_t* marks, const uint32_t* tile_base, uint4* __restrict__ bigq, uint32_t bigq_cap,
    uint32_t* __restrict__ qctr, uint32_t nframes, uint32_t fshift, uint32_t* __restrict__ fvox,
    uint32_t inblock_max, uint32_t* __restrict__ rps, uint32_t* __restrict__ rlen,
    uint32_t small_max, const uint32_t* tile_gtot, uint64_t mark_stride, uint32_t packed,
    const uint32_t* __restrict__ tile_first) {
    __shared__ uint32_t s_wave[4];
    __shared__ uint32_t s_tile, s_epoch, s_excl, s_nbig, s_nq, s_qbase, s_wend, s_nx, s_nbase;
    __shared__ uint32_t s_nh, s_hbase;
    __shared__ uint32_t s_start[kGroupThreads + 1];  // group starts (run index); [total] = end
    // the tile's runs, then up to kExtraRuns runs of the next tiles (the rest of the tile's last
    // group): first points and the exclusive scan of their lengths
    __shared__ uint32_t s_ps[kGroupThreads + kExtraRuns];
    __shared__ uint32_t s_off[kGroupThreads + kExtraRuns + 1];
    __shared__ uint32_t s_big[kGroupThreads];
    __shared__ float4 s_pts[kRunStage + kChainPad];
    __shared__ __attribute__((aligned(16))) float s_wsoa[WAVE == 1 ? 4 : 1][WAVE == 1 ? kWaveSoa : 4];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (WAVE == 1) wave_soa_init(s_wsoa[wid]);
    if (WAVE == 0) inblock_max = min(inblock_max, small_max);  // longer groups: k_group_runs_big
    const uint32_t n = *count;  // runs
    // packed run keys: the length bits above the key (kRunLenShift), the first point as the value
    const uint32_t km = packed ? kRunKeyMask : 0xFFFFFFFFu;
    auto K = [&](uint32_t j) { return keys[j] & km; };
    const uint32_t ntiles = (n + kGroupThreads - 1) / kGroupThreads;
    const uint32_t kmask = nframes > 1 ? (1u << fshift) - 1u : 0xFFFFFFFFu;
    if (blockIdx.x == 0) {
        for (uint32_t i = threadIdx.x; i < kHistWords; i += kGroupThreads) hist[i] = 0;
        if (ntiles == 0 && threadIdx.x == 0) *out_count = 0;
        if (ntiles == 0 && fvox)
            for (uint32_t f = threadIdx.x; f <= nframes; f += kGroupThreads) fvox[f] = 0;
    }
    const Tickets tk = tickets(ntiles, gridDim.x);
    if (!tile_base && blockIdx.x >= tk.nblk) return;
    if (!tile_base && threadIdx.x == 0) s_epoch = read_epoch(epoch_word);
    uint32_t walk = blockIdx.x;
    GDF_RSTAMP(rw0);
    for (bool first = true;; first = false) {  // persistent
        if (!first && !tile_base && tk.oneshot) return;
        // the tile's run records (key, predecessor's key, value), loaded unconditionally at clamped
        // indices in one round - with tile offsets (tile_base) the tile is the walk index and they
        // are issued before the barrier, with the offset and group-prefix loads
        uint32_t kraw = 0, kpraw = 0, vraw = 0;
        auto load_recs = [&](uint32_t tl) {
            const uint32_t ii = tl * kGroupThreads + threadIdx.x;
            const uint32_t ic = min(ii, n - 1u);
            kraw = keys[ic];
            kpraw = keys[ii ? min(ii - 1u, n - 1u) : 0u];
            vraw = rvals[ic];
        };
        if (tile_base && walk < ntiles) load_recs(walk);
        const uint32_t tb0 = tile_base && threadIdx.x == 0 && walk < ntiles ? tile_base[walk] : 0u;
        // (group-scanned offsets: the group-local offset + the totals of the groups before)
        const uint32_t gpre = tile_base && tile_gtot && wid == 0 && walk < ntiles
                                  ? wave_group_prefix(tile_gtot, walk) : 0u;
        if (threadIdx.x == 0) {
            if (tile_base) {
                s_tile = walk;
                s_excl = walk < ntiles ? tb0 + gpre : 0u;
            } else {
                s_tile = next_ticket(tile_ctr, tk, epoch_word, s_epoch);
            }
            s_nbig = 0;
            s_nq = 0;
            s_wend = 0;
            s_nx = 0;
            s_nbase = 0xFFFFFFFFu;
            s_nh = 0;
        }
        walk += gridDim.x;
        __syncthreads();
        const uint32_t tile = s_tile, epoch = s_epoch;
        if (tile >= ntiles) return;  // block-uniform
        GDF_RSTAMP(rw1);
        const uint32_t t0 = tile * kGroupThreads;
        const uint32_t i = t0 + threadIdx.x;
        const uint32_t tend = min(n, t0 + kGroupThreads);
        if (!tile_base) load_recs(tile);
        // the reads for the end of the tile's last group (wave 1, below), issued before the scans
        // by every wave (no branch: a load in one waited for the ones before it): the last key, the
        // next tiles' first starts
        const uint32_t lkraw = keys[tend - 1];
        const uint32_t tt1 = tile + 1u + (uint32_t)lane;
        const bool has_tf = tile_first != nullptr;
        const uint32_t pfr = (has_tf ? tile_first : keys)[min(tt1, ntiles - 1u)];
        const uint32_t pf = (has_tf & (tt1 < ntiles)) ? pfr : 0xFFFFFFFFu;
        // ... and the records of the (up to kExtraRuns) runs past the tile
        const uint32_t xi = min(tend + (uint32_t)lane, n - 1u);
        const uint32_t xvr = rvals[xi], xkr = keys[xi];
        const uint32_t kp = kpraw & km;
        const uint32_t key = i < n ? kraw & km : 0u;
        const uint32_t prev = (i < n && i > 0) ? kp : ~key;
        const bool start = i < n && (i == 0 || key != prev);
        RunRec rr{0u, 0u};
        if (average && i < n) {  // (and the sorted run records for k_group_runs_big)
            const uint32_t v = vraw;
            rr.ps = packed ? v : run_start[v];
            rr.len = packed ? (kraw >> kRunLenShift) + 1u : run_start[v + 1] - rr.ps;
            rps[i] = rr.ps;
            rlen[i] = rr.len;
        }
        uint32_t total, ptotal;
        const uint32_t local = block_exclusive_scan(start ? 1u : 0u, total, s_wave);
        if (start) s_start[local] = i;
        const uint32_t poff = block_exclusive_scan(rr.len, ptotal, s_wave);
        s_ps[threadIdx.x] = rr.ps;
        s_off[threadIdx.x] = poff;
        if (threadIdx.x == 0) s_off[kGroupThreads] = ptotal;
        __syncthreads();
        GDF_RSTAMP(rw2);
        if (wid == 0) {
            const uint32_t ex = tile_base ? s_excl
                                          : lookback2_wave(status, gstatus, tile, ntiles, total, epoch, err);
            if (lane == 0) {
                s_excl = ex;
                if (tile == ntiles - 1) {
                    *out_count = ex + total;
                    if (fvox)
                        for (uint32_t f = (K(n - 1) >> fshift) + 1; f <= nframes; ++f)
                            fvox[f] = ex + total;
                }
            }
        } else if (wid == 1 && total) {  // end of the tile's last group (as k_group, over runs)
            const uint32_t lastkey = lkraw & km;
            uint32_t lo = tend, hi = n;
            if (tile_first) {
                // the first group start of the next tiles that hold one (k_group_count): 64 tiles
                // (16 K runs) per probe of a small cached array, not ~4 rounds of 64 scattered key
                // reads - a window's long groups sent those over the whole run array per tile
                // (most of this kernel's 1.67 GB per C3 frame)
                hi = n;
                for (uint32_t t0x = tile + 1; t0x < ntiles; t0x += 64u) {  // (wave-uniform)
                    const uint32_t tt = t0x + (uint32_t)lane;
                    const uint32_t f = t0x == tile + 1u ? pf : tt < ntiles ? tile_first[tt] : 0xFFFFFFFFu;
                    const unsigned long long has = __ballot(f != 0xFFFFFFFFu);
                    if (has) {
                        hi = (uint32_t)__shfl((int)f, __ffsll((long long)has) - 1, 64);
                        break;
                    }
                }
                lo = hi;  // (done)
            }
            while (lo < hi) {
                const uint32_t len = hi - lo;
                const uint32_t step = len <= 64u || lo == tend ? 1u : (len + 63u) / 64u;
                const uint32_t j = lo + (uint32_t)lane * step;
                const unsigned long long ch = __ballot(j < hi && K(j) > lastkey);
                if (ch) {
                    const uint32_t f = (uint32_t)(__ffsll((long long)ch) - 1);
                    hi = lo + f * step;
                    if (step == 1u) break;
                    lo = f ? lo + (f - 1u) * step + 1u : lo;
                } else {
                    const uint32_t lastp = lo + min(63u, (len - 1u) / step) * step;
                    lo = lastp + 1u;
                }
            }
            // the rest of a last group continuing past the tile, when short: its runs' records
            // (the tile is full here) - so a group is queued only when long
            if (average && hi > tend && hi - tend <= kExtraRuns) {
                const uint32_t nx = hi - tend;
                uint32_t ps = 0, len = 0;
                if ((uint32_t)lane < nx) {  // (lane's record preloaded: xvr, xkr)
                    ps = packed ? xvr : run_start[xvr];
                    len = packed ? (xkr >> kRunLenShift) + 1u : run_start[xvr + 1] - ps;
                }
                const uint32_t inc = dpp_sum_scan(len);
                if ((uint32_t)lane < nx) {
                    s_ps[kGroupThreads + lane] = ps;
                    s_off[kGroupThreads + 1 + lane] = ptotal + inc;
                }
                if (lane == 0) s_nx = nx;
            }
            if (lane == 0) s_start[total] = hi;
        }
        // the groups summed in-block: inside the tile, <= kRunInBlock points, ending within
        // kRunStage positions of the first group start; their points are staged (positions of the
        // tile's run stream up to the last such group's end; position -> run by a binary search
        // of the run offsets), the other groups are queued
        const uint32_t W0 = total ? s_off[s_start[0] - t0] : 0u;
        __syncthreads();  // (the last group's end, s_start[total]; the extra runs)
        GDF_RSTAMP(rw3);
        const uint32_t rend = tend + s_nx;  // runs with records here
        if constexpr (WAVE == 2) {
            // Windows of kRunStage staged positions, up to kRunPasses per tile: each window starts
            // at the first group not summed yet and takes every group that ends inside it; its
            // groups are summed by their thread (<= small_max points) or by 4 lanes, one component
            // chain each.  Groups longer than inblock_max, continuing past the tile's records, or
            // left after the last window are queued for k_group_runs_big.
            uint32_t gs = 0, ge = 0;
            bool elig = false, done = false;
            if (threadIdx.x < total && average) {
                const uint32_t s = s_start[threadIdx.x], e = s_start[threadIdx.x + 1];
                if (e <= rend) {
                    gs = s_off[s - t0];
                    ge = s_off[e - t0];
                    elig = ge - gs <= inblock_max;
                }
            }
            uint32_t base = W0;
#pragma unroll 1
            for (uint32_t pass = 0; pass < kRunPasses; ++pass) {
                const bool in = elig && !done && gs >= base && ge - base <= (uint32_t)kRunStage;
                // (shared counters: each is reset by thread 0 between the barrier after its last
                // read and the barrier before its next update)
                if (in) atomicMax(&s_wend, ge - base);
                __syncthreads();  // A
                const uint32_t staged = s_wend;
                if (threadIdx.x == 0) s_nbase = 0xFFFFFFFFu;  // (read before A by everyone)
                if (staged == 0) break;  // block-uniform
                stage_run_points<kRunStage>(s_pts, pts, s_ps, s_off, kGroupThreads + s_nx, base, staged);
                __syncthreads();  // B
                if (threadIdx.x == 0) s_wend = 0;
                if (in && ge - gs <= small_max) {
                    const float4 acc = thread_group_sum(s_pts + (gs - base), ge - gs);
                    const float fc = (float)(ge - gs);
                    *reinterpret_cast<float4*>(out + 4 * (size_t)(s_excl + threadIdx.x)) =
                        make_float4(acc.x / fc, acc.y / fc, acc.z / fc, acc.w);
                } else if (in) {
                    s_big[atomicAdd(&s_nbig, 1u)] = threadIdx.x;
                }
                __syncthreads();  // C
                const uint32_t nbig = s_nbig;
                for (uint32_t bi = ((uint32_t)lane >> 2) * 4u + (uint32_t)wid; bi < nbig; bi += 64u) {
                    const uint32_t li = s_big[bi];  // staged long groups: 4 lanes, lane = component
                    const uint32_t g0 = s_off[s_start[li] - t0] - base;
                    const uint32_t g1 = s_off[s_start[li + 1] - t0] - base;
                    const uint32_t c = (uint32_t)lane & 3u;
                    const float acc = lane_comp_chain(reinterpret_cast<const float*>(s_pts + g0) + c, g1 - g0);
                    out[4 * (size_t)(s_excl + li) + c] = c < 3 ? acc / (float)(g1 - g0) : acc;
                }
                done = done || in;
                if (elig && !done) atomicMin(&s_nbase, gs);
                __syncthreads();  // D (s_pts read; s_nbase complete)
                base = s_nbase;
                if (threadIdx.x == 0) s_nbig = 0;
                if (base == 0xFFFFFFFFu) break;  // block-uniform: nothing eligible left
            }
            __syncthreads();
            GDF_RSTAMP(rw4);
#ifdef GDF_TRACE_GROUPS
            auto rtrace = [&]() {
                if (threadIdx.x == 0 && tile < kRunTraceSlots) {
                    unsigned long long* g = g_rtrace[tile];
                    g[0] = rw0;
                    g[1] = rw1;
                    g[2] = rw2;
                    g[3] = rw3;
                    g[4] = rw4;
                    g[5] = wall_clock64();
                    g[6] = ((unsigned)__builtin_amdgcn_s_getreg(4 | (15 << 11)) & 0xFFFFu) |
                           (((unsigned long long)__builtin_amdgcn_s_getreg(20 | (15 << 11)) & 0xFu) << 16);
                    g[7] = blockIdx.x;
                }
            };
            if (total == 0) rtrace();
#endif
            if (total == 0) continue;  // block-uniform
            // queued groups: huge ones (>= kHugeGroup points) into the region at the top of the
            // queue that k_group_runs_big draws first (longest first bounds the tail: the C3
            // window's 10^5-point groups otherwise start late).  A group continuing past the
            // tile's records is sized by its runs times the mean length of its own runs inside the
            // tile (an estimate: it only orders the queue; the tile's other groups can have much
            // shorter runs).
            uint32_t qlocal = 0xFFFFFFFFu, hlocal = 0xFFFFFFFFu;
            if (threadIdx.x < total && average && !done) {
                const uint32_t s = s_start[threadIdx.x], e = s_start[threadIdx.x + 1];
                const uint32_t nin = tend - s, pin = s_off[tend - t0] - s_off[s - t0];
                const uint64_t est = e > rend ? (uint64_t)(e - s) * pin / max(nin, 1u)
                                              : (uint64_t)(ge - gs);
                const bool huge = est >= kHugeGroup || e - s >= kHugeRuns;
                if (huge) hlocal = atomicAdd(&s_nh, 1u);
                else qlocal = atomicAdd(&s_nq, 1u);
            }
            __syncthreads();
            if (threadIdx.x == 0 && s_nq) s_qbase = atomicAdd(qctr, s_nq);  // one append per tile
            if (threadIdx.x == 64 && s_nh) s_hbase = atomicAdd(qctr + 2, s_nh);
            __syncthreads();
            if (threadIdx.x < total) {
                const uint32_t g = s_excl + threadIdx.x;
                const uint32_t s = s_start[threadIdx.x], e = s_start[threadIdx.x + 1];
                if (marks) {  // (mark_stride: a batch's frame f at f * mark_stride words)
                    const uint32_t k = K(s) & kmask;
                    const uint64_t fo = mark_stride && nframes > 1 ? (uint64_t)(K(s) >> fshift) * mark_stride : 0u;
                    atomicOr(marks + fo + (k >> 5), 1u << (k & 31u));
                }
                if (fvox) {
                    const uint32_t fc = K(s) >> fshift;
                    const uint32_t f0 = s == 0 ? 0u : (K(s - 1) >> fshift) + 1u;
                    for (uint32_t f = f0; f <= fc; ++f) fvox[f] = g;
                }
                if (!average) {
                    float c[4];
                    group_corner(K(s) & kmask, vp, c);
                    *reinterpret_cast<float4*>(out + 4 * (size_t)g) = make_float4(c[0], c[1], c[2], c[3]);
                } else if (qlocal != 0xFFFFFFFFu) {  // k_group_runs_big
                    const uint32_t slot = s_qbase + qlocal;
                    if (slot < bigq_cap) bigq[slot] = make_uint4(g, s, e, 0u);
                    else atomicOr(err, 8u);
                } else if (hlocal != 0xFFFFFFFFu) {  // from the top (the regions never meet: the
                    const uint32_t h = s_hbase + hlocal;  // queue holds every group, bigq_cap >= groups)
                    if (h < bigq_cap) bigq[bigq_cap - 1u - h] = make_uint4(g, s, e, 0u);
                    else atomicOr(err, 8u);
                }
            }
#ifdef GDF_TRACE_GROUPS
            rtrace();
#endif
        } else {
            bool inblock = false;
            if (threadIdx.x < total && average) {
                const uint32_t s = s_start[threadIdx.x], e = s_start[threadIdx.x + 1];
                if (e <= rend) {
                    const uint32_t ge = s_off[e - t0] - W0;
                    inblock = ge <= (uint32_t)kRunStage && ge - (s_off[s - t0] - W0) <= inblock_max;
                    if (inblock) atomicMax(&s_wend, ge);
                }
            }
            __syncthreads();
            const uint32_t staged = s_wend;
            stage_run_points<kRunStage>(s_pts, pts, s_ps, s_off, kGroupThreads + s_nx, W0, staged);
            __syncthreads();
            if (total == 0) continue;  // block-uniform
            uint32_t qlocal = 0xFFFFFFFFu;  // this thread's group in the tile's queue appends
            if (threadIdx.x < total && average && !inblock) qlocal = atomicAdd(&s_nq, 1u);
            __syncthreads();
            if (threadIdx.x == 0 && s_nq) s_qbase = atomicAdd(qctr, s_nq);  // one append per tile
            __syncthreads();
            if (threadIdx.x < total) {
                const uint32_t g = s_excl + threadIdx.x;
                const uint32_t s = s_start[threadIdx.x], e = s_start[threadIdx.x + 1];
                float* o = out + 4 * (size_t)g;
                if (marks) {  // (mark_stride: a batch's frame f at f * mark_stride words)
                    const uint32_t k = K(s) & kmask;
                    const uint64_t fo = mark_stride && nframes > 1 ? (uint64_t)(K(s) >> fshift) * mark_stride : 0u;
                    atomicOr(marks + fo + (k >> 5), 1u << (k & 31u));
                }
                if (fvox) {
                    const uint32_t fc = K(s) >> fshift;
                    const uint32_t f0 = s == 0 ? 0u : (K(s - 1) >> fshift) + 1u;
                    for (uint32_t f = f0; f <= fc; ++f) fvox[f] = g;
                }
                const uint32_t g0 = s_off[s - t0] - W0;  // staged positions of the group
                const uint32_t g1 = e <= rend ? s_off[e - t0] - W0 : 0xFFFFFFFFu;
                if (!average) {
                    float c[4];
                    group_corner(K(s) & kmask, vp, c);
                    *reinterpret_cast<float4*>(o) = make_float4(c[0], c[1], c[2], c[3]);
                } else if (qlocal != 0xFFFFFFFFu) {  // past the staged points: k_group_runs_big
                    const uint32_t slot = s_qbase + qlocal;
                    if (slot < bigq_cap) bigq[slot] = make_uint4(g, s, e, 0u);
                    else atomicOr(err, 8u);
                } else if (g1 - g0 <= small_max) {
                    const float4 a = thread_group_sum(s_pts + g0, g1 - g0);
                    const float fc = (float)(g1 - g0);
                    *reinterpret_cast<float4*>(o) = make_float4(a.x / fc, a.y / fc, a.z / fc, a.w);
                } else {
                    s_big[atomicAdd(&s_nbig, 1u)] = threadIdx.x;
                }
            }
            __syncthreads();
            const uint32_t nbig = WAVE ? s_nbig : 0u;
            if (WAVE == 2) {  // staged long groups: 4 lanes each, lane = component
                for (uint32_t bi = ((uint32_t)lane >> 2) * 4u + (uint32_t)wid; bi < nbig; bi += 64u) {
                    const uint32_t li = s_big[bi];
                    const uint32_t s = s_start[li], e = s_start[li + 1];
                    const uint32_t g0 = s_off[s - t0] - W0, g1 = s_off[e - t0] - W0;
                    const uint32_t c = (uint32_t)lane & 3u;
                    const float acc = lane_comp_chain(reinterpret_cast<const float*>(s_pts + g0) + c, g1 - g0);
                    out[4 * (size_t)(s_excl + li) + c] = c < 3 ? acc / (float)(g1 - g0) : acc;
                }
            }
            for (uint32_t bi = wid; WAVE == 1 && bi < nbig; bi += 4) {  // staged: a wave per group
                const uint32_t li = s_big[bi];
                const uint32_t g = s_excl + li;
                const uint32_t s = s_start[li], e = s_start[li + 1];
                const uint32_t g0 = s_off[s - t0] - W0, g1 = s_off[e - t0] - W0;
                const float sum = wave_group_sum(s_pts + g0, g1 - g0, s_wsoa[WAVE == 1 ? wid : 0]);
                if ((lane & 15) == 0) {
                    const uint32_t c = (uint32_t)lane >> 4;
                    out[4 * (size_t)g + c] = c < 3 ? sum / (float)(g1 - g0) : sum;
                }
            }
        }
        __syncthreads();  // LDS reused by the next tile
    }
}

// The groups queued by k_group_runs: block b of a resident-sized grid takes queue slot b, then
// draws further slots (qctr[1]) while any remain and streams the runs of each (records rps / rlen by sorted run, written by k_group_runs) from global memory
// (block_stream_sum).  The queue was complete when this launch began; the first sort pass of the
// next voxelize zeroes the counters.
// OCC4: compiled for 4 waves per SIMD (128 VGPRs, ~40 of them spilled; tuning knob
// GDF_RUN_BIG_OCC4), else 3 (167 VGPRs)
template <int Q, bool OCC4 = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC4 ? 4 : 1, 8))) void k_group_runs_big(const uint32_t* __restrict__ rps,
                                                       const uint32_t* __restrict__ rlen,
                                                       const float4* __restrict__ pts,
                                                       float* __restrict__ out,
                                                       const uint4* __restrict__ bigq,
                                                       uint32_t bigq_cap, uint32_t* qctr,
                                                       uint32_t wave_mode) {
    // block mode: s_mark[64 Q + 64], s_soa[4][kRowStride Q]; wave mode: s_mark[4][320] and a
    // kWaveSoa SoA chunk per wave (the same bytes)
    constexpr uint32_t kMarkN = 64 * Q + 64 > 4 * 320 ? 64 * Q + 64 : 4 * 320;
    constexpr uint32_t kSoaN = 4 * kRowStride * Q > 4 * kWaveSoa ? 4 * kRowStride * Q : 4 * kWaveSoa;
    __shared__ int s_mark[kMarkN];  // (+ a scratch row: marks of runs outside a wave's rows)
    __shared__ uint32_t s_base[4][64 * kRunsPerLane];  // (a copy per wave)
    __shared__ __attribute__((aligned(16))) float s_soa_raw[kSoaN];
    float (*s_soa)[kRowStride * Q] = reinterpret_cast<float (*)[kRowStride * Q]>(s_soa_raw);
    __shared__ uint32_t s_t;
    const uint32_t wid = threadIdx.x >> 6;  // (the component, in block mode)
    // logical slot j: the huge region (appended from the top, drawn first), then the others
    const uint32_t na = __hip_atomic_load(qctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t nh = __hip_atomic_load(qctr + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t nq = min(na + nh, bigq_cap);
    auto slot_of = [&](uint32_t j) { return j < nh ? bigq_cap - 1u - j : j - nh; };
#ifdef GDF_TRACE_GROUPS
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // (the queue's two regions, in the last slot)
        g_gtrace[kTraceSlots - 1][0] = 0;
        g_gtrace[kTraceSlots - 1][1] = na;
        g_gtrace[kTraceSlots - 1][2] = nh;
        g_gtrace[kTraceSlots - 1][3] = bigq_cap;
    }
#endif
    // Every resident block / wave takes a first slot, further ones are drawn from the counter.
    // The grid is sized to the blocks the chip holds at once (launch_voxelize): a block that is
    // not resident yet must not hold a slot - with 1024 blocks, the C3 window's 100 K-point
    // groups in slots ~800-1000 started only when the rest of the queue was drained (1.0 ms into
    // a 1.7 ms kernel, tools/group_trace.py --c3); drawing the first slot from the counter too
    // serialised 10^3 atomics at the start (4K: groups starting up to 13 us late, an empty queue
    // 14 us).  One slot per draw: queued groups range over 10^3x in length (C3: up to 139 K
    // points), and draws of 8 consecutive slots measured 1.7 -> 2.8 ms of tail imbalance on the
    // C3 window.  The huge region is summed in block mode (wave c: component c, 1 K-point chunks:
    // the shortest critical path for the longest groups); with wave_mode the other groups are
    // summed one per wave (wave_stream_sum): blocks past the huge region start in wave mode, a
    // block mode block switches to it at its first draw past the region (C3 group phase 1.58 ->
    // 1.33 ms, profiles/r05/wavemode/).
    // Wave mode only for a long queue (>= 4 normal groups per block: the C3 window's 22 K groups,
    // not a 4K frame's ~650 - one wave's chain per group lengthens each group's sum, and with
    // about one group per block that is the launch's critical path: 4K 125 -> 184 us)
    const uint32_t G = gridDim.x;
    if (wave_mode == 1 && na < 4u * G) wave_mode = 0;  // (2: always, the tests' knob)
    const uint32_t nb0 = wave_mode ? min(nh, G) : G;  // blocks starting in block mode
    const uint32_t start0 = nb0 + (G - nb0) * 4u;     // the first drawn slot
    uint32_t t = blockIdx.x;
    if (blockIdx.x < nb0) {
        while (true) {  // block-uniform
            if (t >= nq) return;
            if (wave_mode && t >= nh) break;  // (a normal slot: wave mode from here)
            const uint4 q = bigq[slot_of(t)];
            uint32_t np = 0;
#ifdef GDF_TRACE_GROUPS
            unsigned long long tr[5] = {0, 0, 0, 0, 0};
            const unsigned long long w0 = wall_clock64(), c0 = clock64();
            const float sum = block_stream_sum<Q>(rps, rlen, q.y, q.z, pts, s_mark, s_base[wid], s_soa, np, tr);
            if (threadIdx.x == 128 && t < kTraceSlots) {  // (wave 2: z)
                unsigned long long* g = g_gtrace[t];
                g[0] = w0;
                g[1] = wall_clock64();
                g[2] = ((unsigned long long)np << 32) | (unsigned)tr[4];
                g[3] = clock64() - c0;
                g[4] = tr[0];
                g[5] = tr[1];
                g[6] = tr[2];
                // HW_ID (hwreg 4: wave, simd, pipe, cu, sh, se) and XCC_ID (hwreg 20) bits 0..15
                const unsigned long long hw = (unsigned)__builtin_amdgcn_s_getreg(4 | (15 << 11)) & 0xFFFFu;
                const unsigned long long xcc = (unsigned)__builtin_amdgcn_s_getreg(20 | (15 << 11)) & 0xFu;
                g[7] = tr[3] | (hw << 40) | (xcc << 56);
            }
#else
            const float sum = block_stream_sum<Q>(rps, rlen, q.y, q.z, pts, s_mark, s_base[wid], s_soa, np,
                                                       nullptr);
#endif
            store_comp_mean(out + 4 * (size_t)q.x, wid, sum, np);
            if (threadIdx.x == 0) s_t = atomicAdd(qctr + 1, 1u);
            __syncthreads();
            const uint32_t d = s_t;
            __syncthreads();  // (also: every wave is done with the block mode's LDS)
            t = start0 + d;
        }
        // wave mode from slot t: wave 0 keeps it, the others draw
        if (wid != 0) t = 0xFFFFFFFFu;
    } else {
        t = nb0 + (blockIdx.x - nb0) * 4u + wid;
    }
    // ---- wave mode ----
    const uint32_t lane = threadIdx.x & 63;
    int* wmark = s_mark + wid * 320u;
    float* wsoa = s_soa_raw + wid * kWaveSoa;
    wave_soa_init(wsoa);
    while (true) {  // wave-uniform
        if (t == 0xFFFFFFFFu) {
            uint32_t d = 0;
            if (lane == 0) d = atomicAdd(qctr + 1, 1u);
            t = start0 + (uint32_t)__builtin_amdgcn_readfirstlane((int)d);
        }
        if (t >= nq) return;
        const uint4 q = bigq[slot_of(t)];
        uint32_t np = 0;
#ifdef GDF_TRACE_GROUPS
        const unsigned long long w0 = wall_clock64(), c0 = clock64();
#endif
        const float sum = wave_stream_sum(rps, rlen, q.y, q.z, pts, wmark, s_base[wid], wsoa, np);
        const uint32_t c = lane >> 4;
        if ((lane & 15u) == 0) out[4 * (size_t)q.x + c] = c < 3 ? sum / (float)np : sum;
#ifdef GDF_TRACE_GROUPS
        if (lane == 0 && t < kTraceSlots) {
            unsigned long long* g = g_gtrace[t];
            g[0] = w0;
            g[1] = wall_clock64();
            g[2] = ((unsigned long long)np << 32) | ((np + 255u) / 256u);
            g[3] = clock64() - c0;
            g[4] = g[5] = g[6] = 0;
            const unsigned long long hw = (unsigned)__builtin_amdgcn_s_getreg(4 | (15 << 11)) & 0xFFFFu;
            const unsigned long long xcc = (unsigned)__builtin_amdgcn_s_getreg(20 | (15 << 11)) & 0xFu;
            g[7] = (hw << 40) | (xcc << 56);
        }
#endif
        t = 0xFFFFFFFFu;
    }
}

#ifdef GDF_TRACE_GROUPS
extern "C" int gdf_debug_group_trace(void* dst, size_t bytes) {  // (diagnostic build only)
    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_gtrace), std::min(bytes, sizeof(g_gtrace)), 0,
                                    hipMemcpyDeviceToHost);
}
extern "C" int gdf_debug_group_trace_clear() {
    static unsigned long long zero[kTraceSlots][8];
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_gtrace), zero, sizeof(zero), 0, hipMemcpyHostToDevice);
}
extern "C" int gdf_debug_sel_trace(void* dst, size_t bytes) {  // (diagnostic build only)
    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_strace), std::min(bytes, sizeof(g_strace)), 0,
                                    hipMemcpyDeviceToHost);
}
extern "C" int gdf_debug_sel_trace_clear() {
    static unsigned long long zero[kSelTraceSlots][8];
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_strace), zero, sizeof(zero), 0, hipMemcpyHostToDevice);
}
extern "C" int gdf_debug_runs_trace(void* dst, size_t bytes) {  // (diagnostic build only)
    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_rtrace), std::min(bytes, sizeof(g_rtrace)), 0,
                                    hipMemcpyDeviceToHost);
}
extern "C" int gdf_debug_runs_trace_clear() {
    static unsigned long long zero[kRunTraceSlots][8];
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_rtrace), zero, sizeof(zero), 0, hipMemcpyHostToDevice);
}
extern "C" int gdf_debug_mask_trace(void* dst, size_t bytes) {  // (diagnostic build only)
    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_mtrace), std::min(bytes, sizeof(g_mtrace)), 0,
                                    hipMemcpyDeviceToHost);
}
#endif

uint32_t seg_sort_tiles(uint32_t nmax, uint32_t nframes) {
    return (nmax + kSortThreads * 8 - 1) / (kSortThreads * 8) + std::max<uint32_t>(nframes, 1u);
}
uint32_t seg_sort_groups(uint32_t nmax, uint32_t nframes) {
    return (seg_sort_tiles(nmax, nframes) + kSortGroup - 1) / kSortGroup + std::max<uint32_t>(nframes, 1u);
}

size_t voxelize_status_words(uint32_t nmax, uint32_t key_bits) {  // (tiles of >= 4 keys per thread)
    return (size_t)((nmax + kSortThreads * 4 - 1) / (kSortThreads * 4) + 1) *
           (radix_wide_last(key_bits) ? 512 : 256);
}
size_t voxelize_group_tiles(uint32_t nmax) {
    return (size_t)((nmax + kGroupThreads - 1) / kGroupThreads + 1);
}

template <int PT, int NB>
static void launch_sort_pass(uint32_t tiles, hipStream_t s, const uint32_t* kin, const uint32_t* vin,
                             uint32_t* kout, uint32_t* vout, const VoxelizeArgs& a, uint32_t p,
                             uint32_t dbits) {
    // the first pass also carries the historic-grid update in extra blocks
    const bool g = p == 0 && a.grid8 != nullptr;
    const uint64_t nwords = g ? (a.ncells + 31) / 32 : 0;
    const uint32_t gb = g ? fused_grid_blocks(a.ncells, a.tune->grid_wpt) : 0;
    hipLaunchKernelGGL((k_sort_pass<PT, NB>), dim3(tiles + gb), dim3(kSortThreads), 0, s, kin, vin, kout,
                       vout, a.count, a.hist + 256 * p, a.status, a.sgstatus,
                       reinterpret_cast<uint32_t*>(a.ctrs + kCtrSort0 + p),
                       reinterpret_cast<uint32_t*>(a.ctrs + kCtrEpoch), a.err, 8 * p, dbits, tiles,
                       reinterpret_cast<uint4*>(a.grid8), a.marks, nwords, a.lifetime, a.gseq,
                       a.nframes, a.frame_shift, a.frame_pt_start, a.mark_words,
                       a.snap,
                       p == 0 ? reinterpret_cast<uint32_t*>(a.ctrs + kCtrRunQueue) : nullptr,
                       p == 0 && a.pack_runs ? a.run_start : nullptr);
}

// Blocks of k_group_runs_big<8> / <16> the current device holds at once, cached per device (an
// engine is bound to one device, but a process may drive several; the value is computed once per
// device and kernel variant, races only recompute the same number)
static uint32_t resident_big_blocks(bool q16, bool occ4) {
    constexpr int kDev = 64;
    static std::atomic<uint32_t> cache[kDev][4];
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::atomic<uint32_t>* slot = dev >= 0 && dev < kDev ? &cache[dev][(q16 ? 1 : 0) + (occ4 ? 2 : 0)] : nullptr;
    uint32_t rb = slot ? slot->load(std::memory_order_relaxed) : 0u;
    if (rb) return rb;
    int per_cu = 0, cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &per_cu, occ4 ? (q16 ? reinterpret_cast<const void*>(&k_group_runs_big<16, true>)
                             : reinterpret_cast<const void*>(&k_group_runs_big<8, true>))
                      : (q16 ? reinterpret_cast<const void*>(&k_group_runs_big<16>)
                             : reinterpret_cast<const void*>(&k_group_runs_big<8>)), 256, 0);
    // (the API can report one block per CU too many, MI355X_MICROARCH.md)
    rb = per_cu > 1 && cus > 0 ? (uint32_t)((per_cu - 1) * cus) : 256u;
    if (slot) slot->store(rb, std::memory_order_relaxed);
    return rb;
}

hipError_t launch_voxelize(const VoxelizeArgs& a, hipStream_t s, LaunchHook* hook) {
    const Tuning& T = *a.tune;
    const uint32_t npasses = radix_passes(a.key_bits);
    const int pt = a.sort_pt == 4 || a.sort_pt == 8 ? a.sort_pt : 16;
    const uint32_t tile = kSortThreads * pt;
    // persistent blocks (ticket loop): at most kPersistBlocks, fewer when the capacity is small
    // a run sort's items are ~10x fewer than the capacity's points: a grid of an eighth (at least
    // 256 blocks) holds them, and the empty blocks of a full grid only delay the grid-update
    // blocks behind them (C2 +1 %, profiles/r05/knobs/)
    const uint32_t cap_tiles = (a.nmax + tile - 1) / tile;
    const uint32_t run_cap = a.run_start ? std::max<uint32_t>(256u, cap_tiles / 8) : cap_tiles;
    const uint32_t sort_tiles = std::min<uint32_t>(std::min(cap_tiles, run_cap),
                                                   std::min<uint32_t>(kPersistBlocks, T.sort_blocks));
    hipError_t e;
    const uint32_t* kin = a.keys;
    const uint32_t* vin = nullptr;
    uint32_t* kbuf[2] = {a.keys_a, a.keys_b};
    uint32_t* vbuf[2] = {a.vals_a, a.vals_b};
    const bool runs = a.run_start != nullptr;  // keys are run keys: sort runs, then expand
    const uint32_t sorted_passes = npasses;  // (the free pair: kbuf[passes & 1])
    if (!a.hist_ready) {
        unsigned hb = grid_blocks(a.nmax, 256 * 4);
        if (hb > 512) hb = 512;
        hipLaunchKernelGGL(k_sort_hist, dim3(hb), dim3(256), 0, s, a.keys, a.count, npasses, a.hist,
                           a.nframes, a.frame_shift, a.frame_pt_start);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    for (uint32_t p = 0; p < npasses; ++p) {
        const uint32_t remaining = a.key_bits > 8 * p ? a.key_bits - 8 * p : 0u;
        // (a 9-bit last digit: radix_wide_last)
        const bool wide = p + 1 == npasses && remaining == 9;
        const uint32_t dbits = wide ? 9u : remaining >= 8 ? 8u : (remaining ? remaining : 1u);
        const bool gate = p == 0 && a.grid8 != nullptr;
        if (gate && a.grid_wait && (e = hipStreamWaitEvent(s, a.grid_wait, 0)) != hipSuccess) return e;
        if (gate && a.grid_rec && a.grid_rec_early && (e = hipEventRecord(a.grid_rec, s)) != hipSuccess) return e;
        if (sort_tiles) {
            HookScope hs(hook, GDF_KERNEL_SORT);
            if (wide) {
                if (pt == 4)
                    launch_sort_pass<4, 512>(sort_tiles, s, kin, vin, kbuf[p & 1], vbuf[p & 1], a, p, dbits);
                else if (pt == 8)
                    launch_sort_pass<8, 512>(sort_tiles, s, kin, vin, kbuf[p & 1], vbuf[p & 1], a, p, dbits);
                else
                    launch_sort_pass<16, 512>(sort_tiles, s, kin, vin, kbuf[p & 1], vbuf[p & 1], a, p, dbits);
            } else if (pt == 4)
                launch_sort_pass<4, 256>(sort_tiles, s, kin, vin, kbuf[p & 1], vbuf[p & 1], a, p, dbits);
            else if (pt == 8)
                launch_sort_pass<8, 256>(sort_tiles, s, kin, vin, kbuf[p & 1], vbuf[p & 1], a, p, dbits);
            else
                launch_sort_pass<16, 256>(sort_tiles, s, kin, vin, kbuf[p & 1], vbuf[p & 1], a, p, dbits);
            if ((e = hipGetLastError()) != hipSuccess) return e;
        }
        if (gate && a.grid_rec && !a.grid_rec_early && (e = hipEventRecord(a.grid_rec, s)) != hipSuccess) return e;
        kin = kbuf[p & 1];
        vin = vbuf[p & 1];
    }
    const uint32_t* gcount = a.count;  // items of the group phase (points, or runs)
    const uint32_t max_tiles = (a.nmax + kGroupThreads - 1) / kGroupThreads;
    const uint32_t group_tiles = std::min<uint32_t>(max_tiles, std::min<uint32_t>(kPersistBlocks, T.group_blocks));
    HookScope hs(hook, GDF_KERNEL_GROUP);
    const uint32_t* tile_base = nullptr;
    const uint32_t* tile_gtot = nullptr;
    const uint32_t* tile_first = nullptr;
    const uint32_t bigcap = (max_tiles + std::max<uint32_t>(group_tiles, 1u) - 1) /
                            std::max<uint32_t>(group_tiles, 1u);  // tiles per block (walk)
    if (a.group_counts && max_tiles > T.group_scan_tiles) {
        // many tiles: their group-id offsets from a count + scan instead of one ticket each
        // (a single ticket counter serves ~10^2 draws per microsecond)
        // (up to kMaxGroupScanTiles tiles the count kernel scans its groups of kScanGroup tiles
        // itself and the group kernels add the group totals: no scan launches)
        const bool gscan = a.group_done && max_tiles <= kMaxGroupScanTiles;
        hipLaunchKernelGGL(k_group_count, dim3(group_tiles), dim3(256), 0, s, kin, gcount,
                           a.group_counts, gscan ? a.group_done : nullptr, a.group_offsets,
                           a.group_gtot, runs && a.pack_runs ? kRunKeyMask : 0xFFFFFFFFu,
                           runs ? a.group_first : nullptr);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        if (!gscan && (e = launch_scan(a.group_counts, max_tiles, a.group_offsets, nullptr, gcount,
                                       (uint32_t)kGroupThreads, s)) != hipSuccess)
            return e;
        tile_base = a.group_offsets;
        tile_gtot = gscan ? a.group_gtot : nullptr;
        tile_first = runs ? a.group_first : nullptr;
    }
    if (runs) {  // groups of sorted runs; the long ones by k_group_runs_big
        const uint32_t gb = std::max<uint32_t>(group_tiles, 1u);
        uint32_t* qctr = reinterpret_cast<uint32_t*>(a.ctrs + kCtrRunQueue);
        auto kg = T.run_wave == 1 ? (T.run_stage >= 2048 ? k_group_runs<2048, 1> : k_group_runs<512, 1>)
                : T.run_wave == 2 ? (T.run_stage >= 2048 ? k_group_runs<2048, 2> : k_group_runs<512, 2>)
                                  : (T.run_stage >= 2048 ? k_group_runs<2048, 0> : k_group_runs<512, 0>);
        hipLaunchKernelGGL(kg, dim3(gb), dim3(kGroupThreads), 0, s, kin, vin, gcount,
                           a.run_start, a.pts, reinterpret_cast<float*>(a.out), a.out_count,
                           a.gstatus, a.ggstatus, reinterpret_cast<uint32_t*>(a.ctrs + kCtrGroup),
                           reinterpret_cast<uint32_t*>(a.ctrs + kCtrEpoch), a.err, a.hist,
                           a.average, a.vp, a.group_marks, tile_base, a.bigq, a.bigq_cap, qctr,
                           a.nframes, a.frame_shift, a.frame_vox_start,
                           std::min<uint32_t>(T.run_inblock, T.run_stage >= 2048 ? 2048u : 512u),
                           kbuf[sorted_passes & 1], vbuf[sorted_passes & 1], T.small_group,  // (free after the sort)
                           tile_gtot, a.group_mark_stride, a.pack_runs ? 1u : 0u, tile_first);
        if (a.average) {
            if ((e = hipGetLastError()) != hipSuccess) return e;
            const bool q16 = T.run_q16 == 1 || (T.run_q16 == 2 && a.nframes <= 1);
            const bool occ4 = T.run_big_occ4 != 0;
            const uint32_t rb = resident_big_blocks(q16, occ4);
            const uint32_t big_blocks = std::min(std::min(T.run_big_blocks, rb), a.big_cap ? a.big_cap : rb);
            auto kb = occ4 ? (q16 ? k_group_runs_big<16, true> : k_group_runs_big<8, true>)
                           : (q16 ? k_group_runs_big<16, false> : k_group_runs_big<8, false>);
            hipLaunchKernelGGL(kb, dim3(big_blocks), dim3(256), 0, s, kbuf[sorted_passes & 1],
                               vbuf[sorted_passes & 1], a.pts, reinterpret_cast<float*>(a.out), a.bigq,
                               a.bigq_cap, qctr, T.run_wave_mode);
        }
        return hipGetLastError();
    }
    hipLaunchKernelGGL(k_group, dim3(group_tiles ? group_tiles : 1), dim3(kGroupThreads), 0, s, kin,
                       vin, gcount, a.pts, reinterpret_cast<float*>(a.out), a.out_count,
                       a.gstatus, a.ggstatus, reinterpret_cast<uint32_t*>(a.ctrs + kCtrGroup),
                       reinterpret_cast<uint32_t*>(a.ctrs + kCtrEpoch), a.err, a.hist, a.average,
                       a.vp, a.group_marks, tile_base, tile_base ? a.bigq : nullptr,
                       a.bigcnt, bigcap, a.nframes, a.frame_shift, a.frame_vox_start,
                       T.small_group, T.points_lane, tile_gtot);
    if (tile_base && a.bigq && a.average) {
        if ((e = hipGetLastError()) != hipSuccess) return e;
        hipLaunchKernelGGL(k_group_big, dim3(2048), dim3(256), 0, s, vin, a.pts,
                           reinterpret_cast<float*>(a.out), a.bigq, a.bigcnt, group_tiles, bigcap);
    }
    return hipGetLastError();
}

// ---- orphan shaders of the reference --------------------------------------
// mask_dilate (sh/mask_dilate.glsl:40-67): per pixel, a zero anywhere in the (2F+1)^2 window
// (clipped to the image) writes 0; as written the shader writes 0 for the other pixels too
// (:67), the intended erosion keeps the pixel's value.  The window AND is separable: a block
// stages a (16 + 2F) x (64 + 2F) tile of "non-zero" bytes in LDS (outside the image = 1: those
// neighbours are skipped), ANDs along rows, then along columns - O(F) per pixel, not O(F^2).
constexpr uint32_t kDilTW = 64, kDilTH = 16;

__global__ __launch_bounds__(256) void k_mask_dilate(const uint32_t* __restrict__ in,
                                                     uint32_t* __restrict__ out, uint32_t W,
                                                     uint32_t H, uint32_t F, int as_written) {
    __shared__ uint8_t s_in[(kDilTH + 2 * kDilateMaxF) * (kDilTW + 2 * kDilateMaxF)];
    __shared__ uint8_t s_h[(kDilTH + 2 * kDilateMaxF) * kDilTW];
    const uint32_t x0 = blockIdx.x * kDilTW, y0 = blockIdx.y * kDilTH;
    const uint32_t cols = kDilTW + 2 * F, rows = kDilTH + 2 * F;
    for (uint32_t e = threadIdx.x; e < rows * cols; e += blockDim.x) {
        const uint32_t r = e / cols, c = e - r * cols;
        const int64_t gx = (int64_t)x0 - F + c, gy = (int64_t)y0 - F + r;
        uint8_t v = 1;
        if (gx >= 0 && gx < W && gy >= 0 && gy < H) v = in[(size_t)gy * W + gx] != 0u;
        s_in[e] = v;
    }
    __syncthreads();
    for (uint32_t e = threadIdx.x; e < rows * kDilTW; e += blockDim.x) {
        const uint32_t r = e / kDilTW, c = e - r * kDilTW;
        const uint8_t* row = s_in + r * cols + c;
        uint8_t a = 1;
        for (uint32_t k = 0; k <= 2 * F; ++k) a &= row[k];
        s_h[e] = a;
    }
    __syncthreads();
    for (uint32_t e = threadIdx.x; e < kDilTH * kDilTW; e += blockDim.x) {
        const uint32_t ty = e / kDilTW, tx = e - ty * kDilTW;
        const uint32_t x = x0 + tx, y = y0 + ty;
        if (x >= W || y >= H) continue;
        uint8_t a = 1;
        for (uint32_t k = 0; k <= 2 * F; ++k) a &= s_h[(ty + k) * kDilTW + tx];
        const size_t idx = (size_t)y * W + x;
        out[idx] = (as_written || !a) ? 0u : in[idx];
    }
}

hipError_t launch_mask_dilate(const uint32_t* in, uint32_t* out, uint32_t W, uint32_t H,
                              uint32_t F, int as_written, hipStream_t s) {
    if (W == 0 || H == 0) return hipSuccess;
    hipLaunchKernelGGL(k_mask_dilate, dim3((W + kDilTW - 1) / kDilTW, (H + kDilTH - 1) / kDilTH),
                       dim3(256), 0, s, in, out, W, H, F, as_written);
    return hipGetLastError();
}

// transform_points (sh/transform_points.glsl:37-54): out[i] = T * in[i] where mask[i] != 0
__global__ __launch_bounds__(256) void k_transform_points(const float4* __restrict__ in,
                                                          const uint32_t* __restrict__ mask,
                                                          float4* __restrict__ out, uint32_t n,
                                                          Mat4 T) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        if (mask[i] == 0u) continue;
        const float4 p = in[i];
        out[i] = make_float4(mrow(T.m + 0, p.x, p.y, p.z, p.w), mrow(T.m + 4, p.x, p.y, p.z, p.w),
                             mrow(T.m + 8, p.x, p.y, p.z, p.w), mrow(T.m + 12, p.x, p.y, p.z, p.w));
    }
}

hipError_t launch_transform_points(const float4* in, const uint32_t* mask, float4* out, uint32_t n,
                                   const float* T, hipStream_t s) {
    if (n == 0) return hipSuccess;
    Mat4 m;
    for (int i = 0; i < 16; ++i) m.m[i] = T[i];
    hipLaunchKernelGGL(k_transform_points, dim3(grid_blocks(n, 256)), dim3(256), 0, s, in, mask,
                       out, n, m);
    return hipGetLastError();
}

// ---- multi-GPU fused cloud: stable partition of the compacted (point, key) list by key range -----
// part(key) = min(floor((key / 32) / S), nparts - 1) with S = ceil(ceil(C / 32) / nparts) (part_slice_words):
// rank j owns the keys of the occupancy-mark words [j S, (j + 1) S) - whole words, so the marks
// of rank j's voxels fill exactly slice j of every frame's bitmask and one in-place all-gather of
// equal slices is the union (gdf_fused.cpp) - and after an all-to-all every rank holds, in rank
// (= camera) order and pixel order within a
// camera, exactly the points of its key range - the stable order the reference's single voxelize
// sees for them (fusion.cpp:1743-1756 over the concatenated cameras).  Tiles of 1024 items: counts
// per (part, tile) dest-major, scanned by k_scan_*, then a stable scatter (wave ballots on the
// 4-bit part, per-wave counters in LDS).
constexpr uint32_t kPartTile = 1024;

__device__ __forceinline__ uint32_t part_of(uint32_t key, uint32_t nparts, uint64_t ncells) {
    return emit_part_of(key, nparts, ncells);
}

// RUNS: the partition also cuts each part's points into runs of equal (frame | voxel) keys - a
// run starts at a tile's first item or where the key differs from the item before it (equal keys
// share a part, so a run never straddles parts) - and writes them part-major behind the points'
// counts: run keys (with the frame bits) and run starts relative to the part's first point.  The
// receiver then sorts runs, not points (gdf_voxelize_runs), and no per-point key travels.
__device__ __forceinline__ uint32_t sent_key(const uint32_t* __restrict__ keys, uint32_t i,
                                             const uint32_t* s_fstart, uint32_t nframes,
                                             uint32_t fshift, bool batch) {
    const uint32_t k = keys[i];
    return batch ? k | (frame_of(s_fstart, nframes, i) << fshift) : k;
}

// the segment cuts of a partition (launch_partition's splits): item i lies in segment
// #{cuts <= i}; a cut starts a run
struct SegCuts {
    uint32_t c[kMaxSegs - 1];
    __device__ SegCuts(const uint32_t* splits, uint32_t nsplit, uint32_t stride) {
#pragma unroll
        for (uint32_t k = 0; k < kMaxSegs - 1; ++k) c[k] = k < nsplit ? splits[k * stride] : 0xFFFFFFFFu;
    }
    __device__ uint32_t seg(uint32_t i) const {
        uint32_t s = 0;
#pragma unroll
        for (uint32_t k = 0; k < kMaxSegs - 1; ++k) s += i >= c[k] ? 1u : 0u;
        return s;
    }
    __device__ bool at(uint32_t i) const {
        bool b = false;
#pragma unroll
        for (uint32_t k = 0; k < kMaxSegs - 1; ++k) b |= i == c[k];
        return b;
    }
};

template <bool RUNS>
__global__ __launch_bounds__(256) void k_part_count(const uint32_t* __restrict__ keys,
                                                    const uint32_t* __restrict__ count,
                                                    uint32_t nparts, uint64_t ncells,
                                                    uint32_t ntiles, uint32_t* __restrict__ counts,
                                                    const uint32_t* __restrict__ fstart,
                                                    uint32_t nframes, uint32_t fshift,
                                                    const uint32_t* __restrict__ splits,
                                                    uint32_t nsplit, uint32_t stride) {
    __shared__ uint32_t s_c[2 * kMaxBuckets];
    __shared__ uint32_t s_fstart[kMaxCams + 1];
    const bool batch = RUNS && fstart != nullptr && nframes > 1;
    if (batch) load_fstart(s_fstart, fstart, nframes);
    const uint32_t n = *count;
    const SegCuts cut(splits, nsplit, stride);
    const uint32_t nseg = nsplit + 1u;
    const uint32_t nb = nparts * nseg;
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {  // block-uniform
        if (threadIdx.x < 2 * kMaxBuckets) s_c[threadIdx.x] = 0;
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t i = t * kPartTile + q * 256 + threadIdx.x;
            if (i < n) {
                const uint32_t key = keys[i];
                const uint32_t b = part_of(key, nparts, ncells) * nseg + cut.seg(i);
                atomicAdd(&s_c[b], 1u);
                if (RUNS && (i == t * kPartTile || cut.at(i) ||
                             sent_key(keys, i - 1, s_fstart, nframes, fshift, batch) !=
                                 (batch ? key | (frame_of(s_fstart, nframes, i) << fshift) : key)))
                    atomicAdd(&s_c[kMaxBuckets + b], 1u);
            }
        }
        __syncthreads();
        if (threadIdx.x < nb) {
            counts[threadIdx.x * ntiles + t] = s_c[threadIdx.x];
            if (RUNS) counts[(nb + threadIdx.x) * ntiles + t] = s_c[kMaxBuckets + threadIdx.x];
        }
        __syncthreads();
    }
}

// lanes of this wave in the same bucket as this lane, among the lanes of `m` (buckets < 32)
__device__ __forceinline__ unsigned long long same_part(unsigned long long m, uint32_t part) {
#pragma unroll
    for (int b = 0; b < 5; ++b) {
        const bool bit = (part >> b) & 1u;
        const unsigned long long bb = __ballot(bit);
        m &= bit ? bb : ~bb;
    }
    return m;
}

template <bool RUNS>
__global__ __launch_bounds__(256) void k_part_scatter(const float4* __restrict__ pts,
                                                      const uint32_t* __restrict__ keys,
                                                      const uint32_t* __restrict__ count,
                                                      uint32_t nparts, uint64_t ncells,
                                                      uint32_t ntiles,
                                                      const uint32_t* __restrict__ offsets,
                                                      const uint32_t* __restrict__ total,
                                                      float4* __restrict__ out_pts,
                                                      uint32_t* __restrict__ out_keys,
                                                      uint32_t* __restrict__ part_counts,
                                                      const uint32_t* __restrict__ fstart,
                                                      uint32_t nframes, uint32_t fshift,
                                                      uint32_t* __restrict__ out_run_keys,
                                                      uint32_t* __restrict__ out_run_start,
                                                      const uint32_t* __restrict__ splits,
                                                      uint32_t nsplit, uint32_t stride) {
    __shared__ uint32_t s_w[4][kMaxBuckets];  // per-wave running counts (slot-major order)
    __shared__ uint32_t s_rw[4][kMaxBuckets];  // (runs)
    __shared__ uint32_t s_base[kMaxBuckets];
    __shared__ uint32_t s_rbase[kMaxBuckets];
    __shared__ uint32_t s_pfirst[kMaxBuckets];  // the bucket's first send position
    __shared__ uint32_t s_fstart[kMaxCams + 1];
    // a batch (fstart): the sent key carries the point's frame above the voxel key, the part
    // comes from the voxel key alone
    const bool batch = fstart != nullptr && nframes > 1;
    if (batch) load_fstart(s_fstart, fstart, nframes);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t n = *count;
    const SegCuts cut(splits, nsplit, stride);
    const uint32_t nseg = nsplit + 1u;
    const uint32_t nb = nparts * nseg;
    const uint32_t mp = nb * ntiles;  // (RUNS: the run counts' offsets follow the points')
    if (blockIdx.x == 0 && threadIdx.x < nb) {
        const uint32_t a = offsets[threadIdx.x * ntiles];
        const uint32_t b = threadIdx.x + 1 < nb ? offsets[(threadIdx.x + 1) * ntiles]
                                               : (RUNS ? offsets[mp] : *total);
        part_counts[threadIdx.x] = b - a;
        if (RUNS) {
            const uint32_t ra = offsets[mp + threadIdx.x * ntiles];
            const uint32_t rb = threadIdx.x + 1 < nb ? offsets[mp + (threadIdx.x + 1) * ntiles] : *total;
            part_counts[nb + threadIdx.x] = rb - ra;
        }
    }
    const unsigned long long ltm = lanemask_lt();
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {  // block-uniform
        if (threadIdx.x < 4 * kMaxBuckets) {
            (&s_w[0][0])[threadIdx.x] = 0;
            if (RUNS) (&s_rw[0][0])[threadIdx.x] = 0;
        }
        if (threadIdx.x < nb) {
            s_base[threadIdx.x] = offsets[threadIdx.x * ntiles + t];
            if (RUNS) {
                s_rbase[threadIdx.x] = offsets[mp + threadIdx.x * ntiles + t] - offsets[mp];
                s_pfirst[threadIdx.x] = offsets[threadIdx.x * ntiles];
            }
        }
        __syncthreads();
        // wave w owns items [t*1024 + w*256, + 256) in 4 slots of 64: stable within the tile
        uint32_t part[4], rank[4], key[4], rrank[4];
        bool lead[4];
        float4 p[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t i = t * kPartTile + w * 256 + q * 64 + lane;
            const bool ok = i < n;
            key[q] = ok ? keys[i] : 0u;
            if (ok) p[q] = pts[i];
            part[q] = ok ? part_of(key[q], nparts, ncells) * nseg + cut.seg(i) : 0u;
            if (batch && ok) key[q] |= frame_of(s_fstart, nframes, i) << fshift;
            const unsigned long long m = same_part(__ballot(ok), part[q]);
            const uint32_t before = (uint32_t)__popcll(m & ltm);
            const uint32_t base = ok ? s_w[w][part[q]] : 0u;
            rank[q] = base + before;
            if (RUNS) {
                lead[q] = ok && (i == t * kPartTile || cut.at(i) ||
                                 sent_key(keys, i - 1, s_fstart, nframes, fshift, batch) != key[q]);
                const unsigned long long lm = same_part(__ballot(lead[q]), part[q]);
                const uint32_t rbefore = (uint32_t)__popcll(lm & ltm);
                const uint32_t rb0 = ok ? s_rw[w][part[q]] : 0u;
                rrank[q] = rb0 + rbefore;
                __builtin_amdgcn_wave_barrier();
                if (ok && before == 0) {
                    s_w[w][part[q]] = base + (uint32_t)__popcll(m);
                    s_rw[w][part[q]] = rb0 + (uint32_t)__popcll(lm);
                }
            } else {
                __builtin_amdgcn_wave_barrier();
                if (ok && before == 0) s_w[w][part[q]] = base + (uint32_t)__popcll(m);
            }
            __builtin_amdgcn_wave_barrier();
        }
        __syncthreads();
        // waves before this one in the tile
        if (threadIdx.x < nb) {
            uint32_t run = 0, rrun = 0;
            for (int ww = 0; ww < 4; ++ww) {
                const uint32_t c = s_w[ww][threadIdx.x];
                s_w[ww][threadIdx.x] = run;
                run += c;
                if (RUNS) {
                    const uint32_t rc = s_rw[ww][threadIdx.x];
                    s_rw[ww][threadIdx.x] = rrun;
                    rrun += rc;
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t i = t * kPartTile + w * 256 + q * 64 + lane;
            if (i < n) {
                const uint32_t pos = s_base[part[q]] + s_w[w][part[q]] + rank[q];
                out_pts[pos] = p[q];
                if (out_keys) out_keys[pos] = key[q];
                if (RUNS && lead[q]) {
                    const uint32_t rpos = s_rbase[part[q]] + s_rw[w][part[q]] + rrank[q];
                    out_run_keys[rpos] = key[q];
                    out_run_start[rpos] = pos - s_pfirst[part[q]];
                }
            }
        }
        __syncthreads();
    }
}

uint32_t part_tiles(uint32_t nmax) { return (nmax + kPartTile - 1) / kPartTile; }

hipError_t launch_partition(const float4* pts, const uint32_t* keys, const uint32_t* count,
                            uint32_t nmax, uint32_t nparts, uint64_t ncells, uint32_t* counts,
                            uint32_t* offsets, uint32_t* total, float4* out_pts,
                            uint32_t* out_keys, uint32_t* part_counts, hipStream_t s,
                            const uint32_t* fstart, uint32_t nframes, uint32_t fshift,
                            uint32_t* out_run_keys, uint32_t* out_run_start,
                            const uint32_t* splits, uint32_t nsplit, uint32_t stride) {
    if (nparts == 0 || nparts > kMaxParts) return hipErrorInvalidValue;
    if (!splits) nsplit = 0;
    if (nsplit > kMaxSegs - 1 || nparts * (nsplit + 1) > kMaxBuckets) return hipErrorInvalidValue;
    const uint32_t ntiles = std::max<uint32_t>(part_tiles(nmax), 1u);
    const uint32_t blocks = std::min<uint32_t>(ntiles, 2048u);
    const bool runs = out_run_keys != nullptr;
    if (runs)
        hipLaunchKernelGGL(k_part_count<true>, dim3(blocks), dim3(256), 0, s, keys, count, nparts,
                           ncells, ntiles, counts, fstart, nframes, fshift, splits, nsplit, stride);
    else
        hipLaunchKernelGGL(k_part_count<false>, dim3(blocks), dim3(256), 0, s, keys, count, nparts,
                           ncells, ntiles, counts, fstart, nframes, fshift, splits, nsplit, stride);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const uint32_t nb = nparts * (nsplit + 1u);
    const uint32_t m = (runs ? 2u : 1u) * nb * ntiles;
    if ((e = launch_scan(counts, m, offsets, total, nullptr, 1u, s)) != hipSuccess) return e;
    if (runs)
        hipLaunchKernelGGL(k_part_scatter<true>, dim3(blocks), dim3(256), 0, s, pts, keys, count,
                           nparts, ncells, ntiles, offsets, total, out_pts, out_keys, part_counts,
                           fstart, nframes, fshift, out_run_keys, out_run_start, splits, nsplit, stride);
    else
        hipLaunchKernelGGL(k_part_scatter<false>, dim3(blocks), dim3(256), 0, s, pts, keys, count,
                           nparts, ncells, ntiles, offsets, total, out_pts, out_keys, part_counts,
                           fstart, nframes, fshift, out_run_keys, out_run_start, splits, nsplit, stride);
    return hipGetLastError();
}

// gdf_download_frame prefetch (DlArgs): one grid-stride pass over [counters | points | coords |
// voxelized | delta indices | delta data], 16-B stores where the items are 16 B (the host link
// takes coalesced wave stores at DMA-like rates).
__global__ __launch_bounds__(256) void k_download(DlArgs d) {
    const uint32_t n = (d.parts & DL_POINTS) ? min(d.misc[d.i_count], d.pts_cap) : 0u;
    const uint32_t nv = (d.parts & DL_VOX) ? min(d.misc[d.i_vox], d.vox_cap) : 0u;
    const uint32_t nd = (d.parts & DL_DELTA) && d.delta_cap ? min(d.misc[d.i_delta], d.delta_cap) : 0u;
    const uint64_t e0 = (d.parts & DL_MISC) ? d.misc_words : 0u, e1 = e0 + n, e2 = e1 + n,
                   e3 = e2 + nv, e4 = e3 + nd,
                   e5 = e4 + 2ull * nd;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < e5; i += stride) {
        if (i < e0) d.h_misc[i] = d.misc[i];
        else if (i < e1) d.h_pts[i - e0] = d.pts[i - e0];
        else if (i < e2) d.h_coords[i - e1] = d.coords[i - e1];
        else if (i < e3) d.h_vox[i - e2] = d.vox[i - e2];
        else if (i < e4) d.h_didx[i - e3] = d.didx[i - e3];
        else d.h_ddata[i - e4] = d.ddata[i - e4];
    }
}

hipError_t launch_download(const DlArgs& d, hipStream_t s) {
    hipLaunchKernelGGL(k_download, dim3(512), dim3(256), 0, s, d);
    return hipGetLastError();
}

// The received run lists of gdf_voxelize_runs: source q's run starts are relative to its point
// segment - add its point base; close the list (run_start[R] = n) and store the counts the
// voxelize reads (misc words: points, runs).  The multi-GPU step's own buckets are read from its
// send lists here (run starts rebased on the way, points and run keys copied), and the key range's
// mark words are cleared: one grid-stride pass over [runs | own points | mark words].
__global__ __launch_bounds__(256) void k_run_rebase(uint32_t* __restrict__ run_start, RebaseArgs r,
                                                    uint32_t* __restrict__ n_points,
                                                    uint32_t* __restrict__ n_runs) {
    const uint32_t R = r.run_base[r.nsrc];
    uint64_t own_pts = 0;
    for (uint32_t k = 0; k < r.n_own; ++k)
        own_pts += r.point_base[r.own_src[k] + 1] - r.point_base[r.own_src[k]];
    const uint64_t e0 = R, e1 = e0 + own_pts, e2 = e1 + r.zero_row_words * r.zero_rows;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < e2; t += stride) {
        if (t < e0) {
            const uint32_t i = (uint32_t)t;
            uint32_t q = 0;
            while (q + 1 < r.nsrc && r.run_base[q + 1] <= i) ++q;
            int own = -1;
            for (uint32_t k = 0; k < r.n_own; ++k)
                if (r.own_src[k] == q) own = (int)k;
            if (own < 0) {
                run_start[i] += r.point_base[q];
            } else {
                const uint32_t j = i - r.run_base[q];
                run_start[i] = r.own_run_starts[own][j] + r.point_base[q];
                r.run_keys[i] = r.own_run_keys[own][j];
            }
        } else if (t < e1) {
            uint64_t j = t - e0;
            uint32_t k = 0;
            for (; k + 1 < r.n_own; ++k) {
                const uint32_t c = r.point_base[r.own_src[k] + 1] - r.point_base[r.own_src[k]];
                if (j < c) break;
                j -= c;
            }
            r.pts[r.point_base[r.own_src[k]] + j] = r.own_pts[k][j];
        } else {
            const uint64_t w = t - e1, row = w / r.zero_row_words;
            r.zero[row * r.zero_stride + (w - row * r.zero_row_words)] = 0u;
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        run_start[R] = r.point_base[r.nsrc];
        *n_points = r.point_base[r.nsrc];
        *n_runs = R;
    }
}

hipError_t launch_run_rebase(uint32_t* run_start, const RebaseArgs& r, uint32_t* n_points,
                             uint32_t* n_runs, hipStream_t s) {
    uint64_t own_pts = 0;
    for (uint32_t k = 0; k < r.n_own; ++k)
        own_pts += r.point_base[r.own_src[k] + 1] - r.point_base[r.own_src[k]];
    const uint64_t items = (uint64_t)r.run_base[r.nsrc] + own_pts + r.zero_row_words * r.zero_rows;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>(std::max<uint64_t>((items + 255) / 256, 1), 4096);
    hipLaunchKernelGGL(k_run_rebase, dim3(blocks), dim3(256), 0, s, run_start, r, n_points, n_runs);
    return hipGetLastError();
}

// ---- runs of equal keys in an external (point, key) list -----------------------------------------
// What a rank received in the fused-cloud exchange (every source's points of the rank's key range,
// stable) keeps each camera's runs of equal keys (consecutive kept pixels of one voxel, ~10 points
// each on dense frames): found here, the voxelize sorts runs instead of points (k_group_runs sums
// each voxel's runs in run order = point order, the same sequential chain).  Tiles of 4096 keys,
// 16 contiguous keys per thread; a leader is a key that differs from the one before it.  Counts
// per tile -> launch_scan -> emit (run key, first point); the last tile closes run_start[R] = n.
constexpr uint32_t kXRunTile = 4096;

__device__ __forceinline__ uint32_t xrun_leaders(const uint32_t* __restrict__ keys, uint32_t n,
                                                 uint32_t i0, bool vec, uint32_t (&k)[16]) {
    if (vec && i0 + 16u <= n) {
        const uint4* k4 = reinterpret_cast<const uint4*>(keys + i0);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint4 v = k4[q];
            k[4 * q] = v.x;
            k[4 * q + 1] = v.y;
            k[4 * q + 2] = v.z;
            k[4 * q + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int j = 0; j < 16; ++j) k[j] = i0 + j < n ? keys[i0 + j] : 0u;
    }
    if (i0 >= n) return 0u;
    uint32_t prev = i0 ? keys[i0 - 1] : ~k[0];
    uint32_t m = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        m |= (uint32_t)((i0 + j < n) & (k[j] != prev)) << j;
        prev = k[j];
    }
    return m;
}

__global__ __launch_bounds__(256) void k_xruns_count(const uint32_t* __restrict__ keys,
                                                     const uint32_t* __restrict__ count,
                                                     uint32_t nmax, int vec,
                                                     uint32_t* __restrict__ tcounts) {
    __shared__ uint32_t s_w[4];
    const uint32_t n = min(*count, nmax);
    if (blockIdx.x * kXRunTile >= n) return;  // (tiles past n are not scanned)
    uint32_t k[16];
    const uint32_t m = xrun_leaders(keys, n, blockIdx.x * kXRunTile + threadIdx.x * 16u, vec != 0, k);
    uint32_t c = (uint32_t)__popc(m);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) tcounts[blockIdx.x] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
}

__global__ __launch_bounds__(256) void k_xruns_emit(const uint32_t* __restrict__ keys,
                                                    const uint32_t* __restrict__ count,
                                                    uint32_t nmax, int vec,
                                                    const uint32_t* __restrict__ offsets,
                                                    const uint32_t* __restrict__ total,
                                                    uint32_t* __restrict__ run_keys,
                                                    uint32_t* __restrict__ run_start) {
    __shared__ uint32_t s_w[4];
    const uint32_t n = min(*count, nmax);
    const uint32_t last = n ? (n - 1u) / kXRunTile : 0u;  // the tile that closes the run list
    if (blockIdx.x > last) return;
    if (blockIdx.x == last && threadIdx.x == 0) run_start[*total] = n;
    if (n == 0) return;
    const uint32_t i0 = blockIdx.x * kXRunTile + threadIdx.x * 16u;
    uint32_t k[16];
    uint32_t m = xrun_leaders(keys, n, i0, vec != 0, k);
    const uint32_t c = (uint32_t)__popc(m);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t x = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_w[wid] = x;
    __syncthreads();
    uint32_t pos = offsets[blockIdx.x] + x - c;
    for (int w = 0; w < wid; ++w) pos += s_w[w];
    while (m) {
        const int j = __builtin_ctz(m);
        m &= m - 1u;
        run_keys[pos] = k[j];
        run_start[pos] = i0 + (uint32_t)j;
        ++pos;
    }
}

uint32_t xrun_tiles(uint32_t nmax) { return (nmax + kXRunTile - 1) / kXRunTile; }

hipError_t launch_xruns(const uint32_t* keys, const uint32_t* count, uint32_t nmax,
                        uint32_t* tcounts, uint32_t* offsets, uint32_t* run_keys,
                        uint32_t* run_start, uint32_t* run_total, hipStream_t s) {
    const uint32_t tiles = std::max<uint32_t>(xrun_tiles(nmax), 1u);
    const int vec = (reinterpret_cast<uintptr_t>(keys) & 15u) == 0;
    hipLaunchKernelGGL(k_xruns_count, dim3(tiles), dim3(256), 0, s, keys, count, nmax, vec, tcounts);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if ((e = launch_scan(tcounts, tiles, offsets, run_total, count, kXRunTile, s)) != hipSuccess)
        return e;
    hipLaunchKernelGGL(k_xruns_emit, dim3(tiles), dim3(256), 0, s, keys, count, nmax, vec, offsets,
                       (const uint32_t*)run_total, run_keys, run_start);
    return hipGetLastError();
}

// ---- multi-GPU occupancy marks -------------------------------------------------------------------
// The engine's marks already are the exchange format (1 bit per cell): export is a copy, import
// ORs the all-gathered masks of every rank into them.
__global__ __launch_bounds__(256) void k_import_marks(uint32_t* __restrict__ marks,
                                                      const uint32_t* __restrict__ bits,
                                                      uint64_t words, uint32_t nranks,
                                                      uint64_t stride) {
    for (uint64_t w = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; w < words;
         w += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t v = marks[w];
        for (uint32_t r = 0; r < nranks; ++r) v |= bits[(uint64_t)r * stride + w];
        marks[w] = v;
    }
}

// export that also clears: the frame's marks leave the engine (batched multi-GPU exchange; the
// next frame of this slot starts from an empty mask, the union comes back through the import)
__global__ __launch_bounds__(256) void k_take_marks(uint32_t* __restrict__ marks,
                                                    uint32_t* __restrict__ bits, uint64_t words) {
    for (uint64_t w = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; w < words;
         w += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t v = marks[w];
        bits[w] = v;
        if (v) marks[w] = 0u;
    }
}

// take + sparse form: besides the bitmask, the non-zero words as (index, word) pairs -
// pairs[0] = number of non-zero words (may exceed cap: then only the bitmask is complete),
// pairs[1 + 2k], pairs[2 + 2k] = k-th pair (any order; OR-merged on import).  pairs[0] must be 0
// on entry.
__global__ __launch_bounds__(256) void k_take_marks_sparse(uint32_t* __restrict__ marks,
                                                           uint32_t* __restrict__ bits,
                                                           uint64_t words,
                                                           uint32_t* __restrict__ pairs,
                                                           uint32_t cap) {
    const int lane = threadIdx.x & 63;
    for (uint64_t base = blockIdx.x * (uint64_t)blockDim.x; base < words;
         base += (uint64_t)gridDim.x * blockDim.x) {  // wave-uniform
        const uint64_t w = base + threadIdx.x;
        const uint32_t v = w < words ? marks[w] : 0u;
        if (w < words) {
            bits[w] = v;
            if (v) marks[w] = 0u;
        }
        const unsigned long long nz = __ballot(v != 0u);
        if (!nz) continue;
        uint32_t first = 0;
        if (lane == 0) first = atomicAdd(pairs, (uint32_t)__popcll(nz));
        first = __shfl(first, 0, 64);
        if (v) {
            const uint32_t k = first + (uint32_t)__popcll(nz & lanemask_lt());
            if (k < cap) {
                pairs[1 + 2 * k] = (uint32_t)w;
                pairs[2 + 2 * k] = v;
            }
        }
    }
}

// OR the pairs of `nranks` x `nframes` sparse masks into union[f * words + index]; union zeroed
// on entry.  Record (r, f) sits at pairs + (r * frames_per_rank + f) * rec_words (an all-gathered
// [rank, batch, record] buffer of which the first nframes frames are live); a record holds at
// most cap = (rec_words - 1) / 2 pairs, whatever its count word says (a count above cap means the
// caller exchanged bitmasks instead, so such records are never visited - the cap only keeps a
// stale record inside its own slot).
__global__ __launch_bounds__(256) void k_union_pairs(uint32_t* __restrict__ uni, uint64_t words,
                                                     const uint32_t* __restrict__ pairs,
                                                     uint32_t nframes, uint32_t frames_per_rank,
                                                     uint64_t rec_words) {
    const uint32_t rec = blockIdx.y;  // r * nframes + f
    const uint32_t r = rec / nframes, f = rec % nframes;
    const uint32_t* p = pairs + ((uint64_t)r * frames_per_rank + f) * rec_words;
    const uint32_t cap = (uint32_t)((rec_words - 1) / 2);
    const uint32_t n = min(p[0], cap);
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
        const uint32_t idx = p[1 + 2 * k], v = p[2 + 2 * k];
        if (idx < words) atomicOr(uni + (uint64_t)f * words + idx, v);
    }
}

hipError_t launch_take_marks_sparse(uint32_t* marks, uint64_t words, uint32_t* bits,
                                    uint32_t* pairs, uint32_t cap, hipStream_t s) {
    hipError_t e = hipMemsetAsync(pairs, 0, 4, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_take_marks_sparse, dim3(grid_blocks(words, 256)), dim3(256), 0, s, marks,
                       bits, words, pairs, cap);
    return hipGetLastError();
}

hipError_t launch_union_pairs(uint32_t* uni, uint64_t words, const uint32_t* pairs,
                              uint32_t nranks, uint32_t nframes, uint32_t frames_per_rank,
                              uint64_t rec_words, hipStream_t s) {
    hipError_t e = hipMemsetAsync(uni, 0, (size_t)nframes * words * 4, s);
    if (e != hipSuccess || nranks * nframes == 0 || rec_words < 3) return e;
    hipLaunchKernelGGL(k_union_pairs, dim3(8, nranks * nframes), dim3(256), 0, s, uni, words,
                       pairs, nframes, frames_per_rank, rec_words);
    return hipGetLastError();
}

hipError_t launch_export_marks(const uint32_t* marks, uint64_t words, uint32_t* bits,
                               hipStream_t s) {
    return hipMemcpyAsync(bits, marks, words * 4, hipMemcpyDeviceToDevice, s);
}

hipError_t launch_take_marks(uint32_t* marks, uint64_t words, uint32_t* bits, hipStream_t s) {
    hipLaunchKernelGGL(k_take_marks, dim3(grid_blocks(words, 256)), dim3(256), 0, s, marks, bits,
                       words);
    return hipGetLastError();
}

hipError_t launch_import_marks(uint32_t* marks, uint64_t words, const uint32_t* bits,
                               uint32_t nranks, uint64_t stride, hipStream_t s) {
    hipLaunchKernelGGL(k_import_marks, dim3(grid_blocks(words, 256)), dim3(256), 0, s, marks, bits,
                       words, nranks, stride);
    return hipGetLastError();
}

}  // namespace gdf
