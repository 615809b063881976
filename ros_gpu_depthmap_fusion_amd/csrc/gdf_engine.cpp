// gdf_engine.cpp — host runtime of the MI355X depth-fusion engine and the C-ABI of include/gdf.h.
//
// Replaces the reference's GL host layer (src/gpu_depthmap_fusion.cpp:29-1839 + the
// StorageBuffer/ComputeProgram runtime in include/gpu_depthmap_fusion/*.h) with:
//   - a grow-only device arena (DevBuf) instead of glBufferData-backed StorageBuffers;
//   - one HIP stream per engine; stream order replaces every glMemoryBarrier;
//   - a rollbuffer RING of points with the mask in w (O(new) insert, O(1) roll) instead of the
//     reference's A/B double buffers that copy the whole window twice per frame
//     (fusion.cpp:1005-1032, 1174-1207);
//   - host mirrors of the sequence headers so roll/select need no device->host download
//     (the reference downloads them, fusion.cpp:1102 and :1369);
//   - deferred stage calls: convert/flying/crop/transform only record their parameters and
//     run as ONE fused compaction launch (k_frame) when applyPointMask needs the result.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <atomic>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "gdf.h"
#include "gdf_kernels.hpp"

using namespace gdf;

namespace {
thread_local std::string g_last_error;
}  // namespace

namespace gdf {
void set_last_error(const std::string& msg) { g_last_error = msg; }
}  // namespace gdf

namespace {

struct GdfError {
    int code;
    std::string msg;
};

[[noreturn]] void fail(int code, const std::string& msg) { throw GdfError{code, msg}; }

#define HIPCHK(expr)                                                                       \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess)                                                              \
            fail(GDF_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));          \
    } while (0)

// Host -> pinned-staging copies of host depth maps, split over worker threads: one thread's
// memcpy (~8-15 GB/s, box-dependent) bounded the host-map line at half the device-map rate
// (VERDICT r2 weak #11).  The caller works too; workers are created on first use and block on a
// condition variable between calls.  Threads: GDF_H2D_THREADS (default 4: the caller + 3
// workers).  Round 3 measured no gain from threads (8 DMAs per batch with command gaps bounded
// the line); with one coalesced DMA per batch (upload_depthmaps) the single-thread memcpy is the
// bound - trace: 107-us DMA, next batch's DMA issued ~240 us later - and 1 / 4 / 8 threads give
// 28.6 / 34.5 / 32.6 GB/s on one box (profiles/r04/h2d/).
class StagingCopier {
  public:
    struct Job {
        uint8_t* dst;
        const uint8_t* src;
        size_t bytes;
    };
    ~StagingCopier() {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    void run(const std::vector<Job>& jobs) {
        size_t total = 0;
        for (const Job& j : jobs) total += j.bytes;
        if (total == 0) return;
        const unsigned nt = threads();
        // (one frame - the synchronous component path - is copied by the caller alone: waking
        // the workers costs more latency than they save on 0.6 MB; batches use them)
        if (nt <= 1 || total < kMinParallel) {
            for (const Job& j : jobs) std::memcpy(j.dst, j.src, j.bytes);
            return;
        }
        // one generation per call: its own chunk list, captured by the workers under the lock, so
        // a worker that wakes late (after this call returned) holds the OLD list - already fully
        // claimed - and can never read the next call's list while it is being built
        auto g = std::make_shared<Gen>();
        for (const Job& j : jobs)
            for (size_t o = 0; o < j.bytes; o += kChunk)
                g->chunks.push_back({j.dst + o, j.src + o, std::min(kChunk, j.bytes - o)});
        g->left = g->chunks.size();
        {
            std::lock_guard<std::mutex> lk(m_);
            if (th_.empty())
                for (unsigned i = 1; i < nt; ++i) th_.emplace_back([this] { worker(); });
            cur_ = g;
            ++gen_;
        }
        cv_.notify_all();
        work(*g);
        std::unique_lock<std::mutex> lk(m_);
        done_cv_.wait(lk, [&] { return g->left == 0; });  // every chunk copied
        cur_.reset();
    }

  private:
    struct Gen {
        std::vector<Job> chunks;  // fixed once published
        std::atomic<size_t> next{0};
        size_t left = 0;          // chunks not yet copied (guarded by m_)
    };
    static constexpr size_t kChunk = 256 << 10;
    static constexpr size_t kMinParallel = 2 << 20;
    unsigned threads() {
        if (!nthreads_) {
            const char* s = std::getenv("GDF_H2D_THREADS");
            const int v = s ? std::atoi(s) : 4;
            nthreads_ = (unsigned)std::max(1, std::min(v, 16));
        }
        return nthreads_;
    }
    void work(Gen& g) {  // claim chunks until none is left (caller and workers alike)
        size_t done = 0;
        for (size_t i; (i = g.next.fetch_add(1)) < g.chunks.size(); ++done)
            std::memcpy(g.chunks[i].dst, g.chunks[i].src, g.chunks[i].bytes);
        if (!done) return;
        std::lock_guard<std::mutex> lk(m_);
        g.left -= done;
        if (g.left == 0) done_cv_.notify_all();
    }
    void worker() {
        uint64_t seen = 0;
        for (;;) {
            std::shared_ptr<Gen> g;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                g = cur_;
            }
            if (g) work(*g);
        }
    }
    unsigned nthreads_ = 0;
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_cv_;
    std::shared_ptr<Gen> cur_;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    // grow-only; contents are NOT preserved (like StorageBuffer::resize, storage_buffer.h:25-44)
    bool ensure(size_t need) {
        if (need <= bytes) return false;
        size_t nb = std::max(need, bytes + bytes / 2);
        nb = (nb + 255) & ~size_t(255);
        void* q = nullptr;
        if (p) {
            HIPCHK(hipDeviceSynchronize());
            HIPCHK(hipFree(p));
            p = nullptr;
            bytes = 0;
        }
        hipError_t e = hipMalloc(&q, nb);
        if (e != hipSuccess) fail(GDF_ERR_NOMEM, "hipMalloc of " + std::to_string(nb) + " bytes failed");
        p = q;
        bytes = nb;
        return true;
    }
    // grow-only and zero-filled on growth (look-back granules / counters must start at 0)
    bool ensure_zero(size_t need, hipStream_t s) {
        if (!ensure(need)) return false;
        HIPCHK(hipMemsetAsync(p, 0, bytes, s));
        return true;
    }
    template <class T>
    T* as() const { return static_cast<T*>(p); }
};

struct CamTable {  // cached per-camera ray factors (xn per column, yn per row)
    uint32_t W = 0, H = 0;
    float fx = 0, fy = 0, cx = 0, cy = 0;
    bool valid = false;
    DevBuf xn, yn;
};

struct Hdr {  // PointSequence, gpu_depthmap_fusion.h:178-204
    uint32_t sec, nsec, start, num;
    float T[16];
    // (not in the reference) rollbuffer sharding, gdf_set_rollbuffer_shard: the sequence's arrival
    // number and its point count before sharding (num = 0 for a sequence another shard holds)
    uint64_t id = 0;
    uint32_t num_global = 0;
};

// Where the points of collected sequences come from: a run of `n` points at collect offset `dst`,
// either host xyzw at pts[4*hsrc] (copied at add time) or borrowed device records (`dev`, `step`).
struct PsRun {
    uint32_t dst = 0, n = 0, step = 0;
    const void* dev = nullptr;
    size_t hsrc = 0;
};

struct PsBuf {  // PointSequences, gpu_depthmap_fusion.h:206-217
    uint32_t total = 0;
    size_t host_total = 0;
    std::vector<Hdr> seqs;
    std::vector<float> pts;
    std::vector<PsRun> runs;
    void clear() {
        total = 0;
        host_total = 0;
        seqs.clear();
        pts.clear();
        runs.clear();
    }
    void add_run(const PsRun& r) {
        if (!r.n) return;
        if (!r.dev && !runs.empty() && !runs.back().dev && runs.back().dst + runs.back().n == r.dst &&
            runs.back().hsrc + runs.back().n == r.hsrc) {
            runs.back().n += r.n;  // contiguous host points: one copy
            return;
        }
        runs.push_back(r);
    }
};

struct Cam {
    const uint16_t* host = nullptr;
    const uint16_t* dev = nullptr;
    uint32_t frame = 0;  // frame of a multi-frame batch
    uint32_t W, H, n;
    float scale, fx, fy, cx, cy;
    float Tw[16], Tc[16];
};

int compare_time(uint32_t sa, uint32_t na, uint32_t sb, uint32_t nb) {  // fusion.cpp:1089-1096
    if (sa < sb) return -1;
    if (sa > sb) return +1;
    if (na < nb) return -1;
    if (na > nb) return +1;
    return 0;
}

// R = A·B row-major, ((a0·b0 + a1·b1) + a2·b2) + a3·b3 (rollbuffer_transfer_selected_transforms
// .glsl:60-65 computes Move^T·World^T on the transposed storage = (T_world_move·T_move)^T)
void mat_mul(const float* A, const float* B, float* R) {
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c)
            R[4 * r + c] = ((A[4 * r + 0] * B[0 * 4 + c] + A[4 * r + 1] * B[1 * 4 + c]) +
                            A[4 * r + 2] * B[2 * 4 + c]) + A[4 * r + 3] * B[3 * 4 + c];
}

// ros::Time - ros::Duration(double) as in roscpp_core (DurationBase::fromSec,
// normalizeSecNSecSigned/Unsigned); false where ROS would throw.
bool ros_time_minus(uint32_t sec, uint32_t nsec, double seconds, uint32_t* os, uint32_t* ons) {
    int64_t dsec64 = (int64_t)std::floor(seconds);
    if (dsec64 < INT32_MIN || dsec64 > INT32_MAX) return false;
    int32_t dsec = (int32_t)dsec64;
    int32_t dnsec = (int32_t)std::round((seconds - (double)dsec) * 1e9);
    int32_t rollover = (int32_t)((int64_t)dnsec / 1000000000LL);
    dsec += rollover;
    dnsec = (int32_t)((int64_t)dnsec % 1000000000LL);
    int64_t ns = -(int64_t)dnsec, ss = -(int64_t)dsec;
    int64_t np = ns % 1000000000LL, sp = ss + ns / 1000000000LL;
    if (np < 0) { np += 1000000000LL; --sp; }
    if (sp < INT32_MIN || sp > INT32_MAX) return false;
    int64_t sec_sum = (int64_t)sec + sp, nsec_sum = (int64_t)nsec + np;
    int64_t np2 = nsec_sum % 1000000000LL, sp2 = sec_sum + nsec_sum / 1000000000LL;
    if (np2 < 0) { np2 += 1000000000LL; --sp2; }
    if (sp2 < 0 || sp2 > 0xFFFFFFFFLL) return false;
    *os = (uint32_t)sp2;
    *ons = (uint32_t)np2;
    return true;
}

enum MiscSlot {
    kCount = 0, kTileCtr = 1, kErr = 2, kVoxCount = 3, kGridTicket = 4, kDepthCount = 5,
    kSelTotal = 6, kPartTotal = 7, kRecvCount = 8, kRunCount = 9, kScanTotal = 10, kRunTotal = 11,
    kRecvRuns = 12, kDeltaCount = 13,
    kSplit0 = 16,  // [kMaxSegs - 1] the partition's segment cuts of a rollbuffer frame (k_sel)
    kMiscWords = 20
};

}  // namespace


// every environment variable that selects a launch shape or an alternative form (none changes a
// result: DESIGN.md §5 "Tuning knobs"); read at gdf_create only
constexpr const char* kTuningVars[] = {
    "GDF_MASK_PX", "GDF_MASK_OCC8", "GDF_EMIT_PX2", "GDF_GRID_WPT", "GDF_SORT_BLOCKS",
    "GDF_GROUP_BLOCKS", "GDF_GROUP_SCAN_TILES", "GDF_GROUP_FIRST", "GDF_RUN_STAGE",
    "GDF_RUN_INBLOCK", "GDF_RUN_WAVE", "GDF_SMALL_GROUP", "GDF_POINTS_LANE", "GDF_RUN_WAVE_MODE",
    "GDF_RUN_BIG_OCC4", "GDF_RUN_BIG_BLOCKS", "GDF_RUN_Q16", "GDF_SORT_PT", "GDF_SEG_ITEMS",
    "GDF_SEL_SHAPE", "GDF_H2D_THREADS", "GDF_NO_GRAPHS", "GDF_NO_RUNS", "GDF_FORCE_RUNS",
    "GDF_RUN_HIST_SORT", "GDF_RUN_HIST_ALL", "GDF_NO_PACK_RUNS", "GDF_NO_XRUNS",
    "GDF_NO_GROUP_SCAN", "GDF_NO_MASK_PACKED", "GDF_NO_GRID_DELTA", "GDF_NO_EMIT_PART",
    "GDF_NO_DL_PREFETCH", "GDF_DL_FORK", "GDF_GRID_GATE", "GDF_NO_SEL_KEY_LDS",
    "GDF_NO_SEG_UNIFORM"};

constexpr int kMaxPipe = 4;
// batches of frames of at most this many depth pixels each run k_group_runs_big on this many blocks
constexpr uint64_t kSmallFramePixels = 640 * 480;
constexpr uint32_t kSmallFrameBigBlocks = 32;

// Everything one frame writes.  Frames rotate over npipe slots (gdf_clear starts a frame), so a
// new frame's compaction runs while the previous frame's sort / grouping still execute.  The
// occupancy grid is ordered on the device (GridSeq: updates apply in ticket order whatever stream
// they run on); other shared state (rollbuffer ring, selection and camera tables) is rewritten
// only after the host has drained the other slots (serialize) - a cross-stream event wait costs
// ~20 us of GPU time per frame on this device (tools/graph_probe.hip).
struct Slot {
    hipStream_t own = nullptr;
    hipStream_t ext = nullptr;      // caller-owned stream of this slot (gdf_set_slot_streams)
    hipStream_t stream() const { return ext ? ext : own; }
    DevBuf d_depth;                 // host depth maps uploaded for this frame
    void* h_stage = nullptr;        // pinned staging of pageable host depth maps
    size_t h_stage_bytes = 0;
    hipEvent_t h2d_done = nullptr;  // the slot's last staged copy has been read
    bool h2d_pending = false;
    DevBuf d_camdesc;
    DevBuf d_ctrs;                  // tile tickets of the look-back launches
    DevBuf d_khist;                 // digit histogram of the voxel keys [4*256]
    bool khist_pending = false;     // accumulated by the fused compaction, not yet consumed
    DevBuf d_pts, d_coords, d_stage, d_vbits, d_tcounts, d_toffsets;
    DevBuf d_selstat;  // k_sel's look-back granules
    DevBuf d_misc;
    uint32_t* h_misc = nullptr;     // pinned
    bool compacted = false, coords_valid = false, marks_set = false;
    bool group_marks = false;       // this frame's marks are set by the voxel groups (k_group)
    uint32_t dbg_count = 0;
    DevBuf d_ka, d_kb, d_va, d_vb, d_sstatus, d_sgstatus, d_gstatus, d_ggstatus, d_vox;
    DevBuf d_gcnt, d_goff;          // group starts per tile + their scan (large frames)
    DevBuf d_gfirst;                // the first group start of each tile (run groups)
    DevBuf d_bigq, d_bigcnt;        // long voxels queued for k_group_big (large frames)
    bool vox_valid = false;
    DevBuf d_markbits;              // this frame's occupancy marks (1 bit per cell; per batch frame)
    uint32_t marks_gen = ~0u;
    uint32_t marks_frames = 0;      // frames the zeroed mark buffer covers
    DevBuf d_fstart, d_fvox;        // batch: first point / first voxel of each frame [nframes + 1]
    // batch: sparse snapshots of the u8 grid after each frame but the last (SnapArgs), valid
    // when this batch's grid update wrote them (snap_blocks: that update's grid size)
    DevBuf d_snap_idx, d_snap_data, d_snap_cnt;
    bool snap_valid = false;
    uint32_t snap_blocks = 0, snap_frames = 0;
    DevBuf d_pcnt, d_poff;          // multi-GPU key-range partition workspace
    DevBuf d_xcnt, d_xoff, d_xrk, d_xrs;  // runs of a received (point, key) list
    DevBuf d_grpdone, d_grptot;     // in-kernel group scan of the segment counts
    struct Pinned {                 // pinned host mirror (gdf_download_frame)
        void* p = nullptr;
        size_t bytes = 0;
        void* ensure(size_t need) {
            if (need <= bytes) return p;
            if (p) (void)hipHostFree(p);
            p = nullptr;
            bytes = 0;
            const size_t nb = std::max(need, bytes + bytes / 2);
            if (hipHostMalloc(&p, nb, hipHostMallocDefault) != hipSuccess) {
                p = nullptr;
                return nullptr;
            }
            bytes = nb;
            return p;
        }
        ~Pinned() {
            if (p) (void)hipHostFree(p);
        }
    };
    // Two sets of mirrors: gdf_download_frame hands out set `mir_out`, and the next downloads
    // (k_download's prefetch, or the copies of a later gdf_download_frame) go to the other set,
    // so the views a caller holds stay intact until its next gdf_download_frame (gdf.h).
    struct Mirrors {
        Pinned pts, coords, vox, delta, misc;
    } mir[2];
    int mir_out = -1;               // the set last handed out (-1: none)
    int mir_pf = 0;                 // the set this slot's valid prefetch wrote
    int mir_next() const { return mir_out == 0 ? 1 : 0; }
    bool pf_valid = false;          // this slot's last frame wrote its downloads (k_download)
    bool sel_frame = false;         // this slot's last frame compacted rollbuffer points (k_sel)
    bool part_emitted = false;      // this slot's last compaction wrote the emit partition
    hipStream_t dl_aux = nullptr;   // k_download of the points / coords, after the compaction,
    hipEvent_t dl_ev = nullptr;     // overlapping the voxelize (an event after the compaction)
    DevBuf d_didx, d_ddata;         // the grid delta of this slot's single-frame update
    bool delta_valid = false;
    uint32_t delta_ticket = 0;      // ... and that update's sequence number
    DevBuf d_ggdone, d_ggtot;       // ... and of the group phase's tile counts
    DevBuf d_wruns, d_runkeys, d_runstart;  // runs of equal keys
    bool runs_sel = false;          // ... counted in kRunTotal (frame with rollbuffer points)
    bool runs_valid = false;        // this frame's voxelize may sort runs
    uint32_t nframes = 1;           // frames of the slot's last processed batch
    uint32_t n_total = 0;
    // steady-state frames as HIP graphs (the fused frame + voxelize launches of this slot): one
    // graph launch and two kernel-node argument updates (depth pointers, grid ticket) per frame
    // instead of six direct launches.  A graph is replayed while the frame's launch arguments -
    // minus those two fields - equal its capture's; captured once they repeat on two frames.  Up to
    // kGraphCache argument sets per slot keep their graphs (least recently used evicted), so a
    // caller alternating between parameter sets (e.g. the component's runtime config topics,
    // component.cpp:970-990) replays instead of re-capturing.
    static constexpr int kGraphCache = 4;
    struct GraphEntry {
        hipGraph_t g = nullptr;
        hipGraphExec_t x = nullptr;
        // the compaction kernel nodes (k_mask, k_emit, k_emit_sel): they take the FrameArgs
        std::vector<std::pair<hipGraphNode_t, hipKernelNodeParams>> frame_nodes;
        FrameArgs key_a;
        VoxelizeArgs key_v;
        bool valid = false;
        uint64_t used = 0;  // last use (Graphs::tick)
        void reset() {
            if (x) (void)hipGraphExecDestroy(x);
            if (g) (void)hipGraphDestroy(g);
            x = nullptr;
            g = nullptr;
            valid = false;
            used = 0;
            frame_nodes.clear();
        }
    };
    struct Graphs {
        GraphEntry e[kGraphCache];
        // argument sets seen once (direct launches): a second sighting captures
        FrameArgs cand_a[kGraphCache];
        VoxelizeArgs cand_v[kGraphCache];
        bool cand[kGraphCache] = {};
        int cand_next = 0;
        uint64_t tick = 0;
        uint64_t captures = 0, replays = 0;  // instrumentation (gdf_get_graph_stats)
        void reset() {
            for (GraphEntry& x : e) x.reset();
            for (bool& c : cand) c = false;
        }
    } graph;
};

struct gdf_engine {
    int device = 0;
    StagingCopier copier;  // host depth maps -> pinned staging
    // frame slots: per-frame buffers on their own streams (pipeline depth 1..kMaxPipe)
    Slot slots[kMaxPipe];
    int cur = 0;
    int ring = 0;  // slot of the most recent gdf_clear (gdf_select_slot moves cur, not ring)
    int npipe = 1;
    hipStream_t user_stream = nullptr;  // gdf_set_stream: single slot on the caller's stream
    bool serialized = false;            // this frame already waits for the previous one
    Slot& sl() { return slots[cur]; }
    const Slot& sl() const { return slots[cur]; }
    Slot& prev_slot() { return slots[(cur + npipe - 1) % npipe]; }
    std::mutex ps_mutex;
    int voxel_group_size = 1024;

    // point-sequence collect/upload double buffer (fusion.cpp:734-746)
    PsBuf psA, psB;
    PsBuf* collect = &psA;
    PsBuf* upload = &psB;

    // frame inputs
    std::vector<Cam> cams;
    uint32_t nframes = 1;           // frames of the batch being assembled (gdf_next_frame_in_batch)
    uint32_t depth_total = 0;
    std::vector<CamDesc> halo;      // halo cameras (multi-GPU), negative offsets (built per frame)
    std::vector<Cam> halo_cams;     // gdf_add_halo_depthmap_device inputs of this frame
    std::vector<uint32_t> halo_tail;  // pixels present at the end of each halo camera
    std::vector<CamTable> tables = std::vector<CamTable>(kMaxCams);
    std::vector<CamDesc> h_cams;
    uint32_t mask_blocks = 0;       // compaction segments over the emitting cameras
    uint64_t index_end = 0;         // end of the cameras' index space (halo gaps included)
    uint32_t last_sort_items = 0;   // items the last synchronous frame's voxelize sorted
    bool last_sort_runs = false;    // ... runs of equal keys (else points)
    uint32_t max_segw = 0;          // widest segment (sizes k_mask's LDS band)
    bool depth_uploaded = false;

    // new sequences on the device
    DevBuf d_new;
    uint32_t n_new = 0;
    std::vector<Hdr> new_hdrs;
    bool ps_filter_set = false;
    float ps_thr = 0.f;
    uint32_t ps_F = 0;

    // rollbuffer ring + host header mirrors of the A (after insert) / B (after roll) buffers
    DevBuf d_ring;
    uint64_t ring_cap = 0, ring_head = 0;
    std::vector<Hdr> hdrA, hdrB;
    // rollbuffer sharding (gdf_set_rollbuffer_shard): sequence id keeps its points on shard
    // (id / shard_block) % nshards; every shard holds every header
    uint32_t shard = 0, nshards = 1, shard_block = 1;
    uint64_t seq_counter = 0;  // sequences inserted so far (their ids)
    gdf_rollbuffer_state rb{};

    // selected rollbuffer points
    bool prepared = false, sel_inserted = false;
    DevBuf d_seg_start, d_seg_tf, d_tfw, d_tfc;
    uint32_t sel_uniform = 0, sel_off = 0;  // (FrameArgs::sel_uniform)
    uint32_t nseg = 0;
    // a sharded window: where the 2nd, 3rd .. piece of the selection this shard holds starts
    // (selected-item index), the partition cutting its rollbuffer points there
    std::vector<uint32_t> sel_cuts;

    // deferred depth plan
    bool converted = false, flying_set = false, crop_set = false;
    uint32_t F = 0;
    float thr = 0.f;
    int rot45 = 0;
    float lo[3] = {0, 0, 0}, hi[3] = {0, 0, 0};

    Tuning tune;                    // launch shapes, a snapshot at gdf_create
    std::string tuning_set;         // the GDF_* tuning variables set at creation ("K=V K=V")
    int sort_pt = 0;  // radix keys per thread (4, 8, 16); 0: chosen by frame capacity
    uint32_t sel_segs = kSelSegs, sel_threads = kSelThreads;  // k_sel tile shape
    bool sel_shape_set = false;     // GDF_SEL_SHAPE given (else the shape follows the window)
    uint32_t seg_items = 0;  // max pixels per depth compaction segment (64..1024); 0: by frame size
    bool use_graphs = !getenv("GDF_NO_GRAPHS");  // gdf_set_graphs
    bool use_runs = !getenv("GDF_NO_RUNS");      // voxelize runs of equal keys (depth frames)
    bool force_runs = getenv("GDF_FORCE_RUNS") != nullptr;    // tuning knob: runs at every size
    bool run_hist_in_sort = getenv("GDF_RUN_HIST_SORT") != nullptr;  // tuning knob
    // the runs' lengths packed into the sort keys, their first points as the sorted values (the
    // group phase reads no run_start[index] gathers); GDF_NO_PACK_RUNS: the index form
    bool pack_runs = !getenv("GDF_NO_PACK_RUNS");
    bool run_hist_all = getenv("GDF_RUN_HIST_ALL") != nullptr;  // tuning knob: k_mask counts the
                                                               // run digits at any segment count
    bool xruns = !getenv("GDF_NO_XRUNS");  // voxelize_points sorts the received list's runs
    bool group_scan = !getenv("GDF_NO_GROUP_SCAN");  // segment offsets without scan launches
    bool mask_packed = !getenv("GDF_NO_MASK_PACKED");  // k_mask_px<2>: packed f32 pixel pairs
    bool sel_key_lds = !getenv("GDF_NO_SEL_KEY_LDS");  // k_sel: the keys kept in LDS (A/B)
    bool seg_uniform = !getenv("GDF_NO_SEG_UNIFORM");  // equal cameras: segment -> camera by division
    // host mirror of the u8 grid (gdf_download_frame): after the first grid download, single-frame
    // updates also list the 32-cell groups they changed, and the next download moves only those
    bool grid_delta = false;
    bool grid_delta_allowed = !getenv("GDF_NO_GRID_DELTA");
    Slot::Pinned h_mirror;
    // after a single-frame gdf_download_frame of points / coords / voxels: single frames end with
    // k_download into the slot's pinned mirrors (the next download_frame waits once)
    bool dl_prefetch = false;
    // gdf_set_emit_partition: the next deferred frame's send lists (device), armed until used
    struct EmitPart {
        uint32_t nparts = 0, cap = 0;
        float* pts = nullptr;
        uint32_t *run_keys = nullptr, *run_starts = nullptr, *counts = nullptr;
        uint32_t nseg = 1;  // gdf_set_partition_segments: [depth | rollbuffer pieces] buckets
    } epart;
    bool emit_part = !getenv("GDF_NO_EMIT_PART");  // (else: compaction, then the partition pass)
    // a frame armed with gdf_set_emit_partition sets its occupancy marks (gdf_set_partition_marks:
    // off when the caller builds the union from the key-range voxelize, gdf_voxelize_runs_marked)
    bool part_marks = true;
    bool dl_prefetch_allowed = !getenv("GDF_NO_DL_PREFETCH");
    // tuning knob GDF_DL_FORK: the points / coords part on a second stream right after the
    // compaction (direct launches) instead of in the chain's last kernel (graph replays)
    bool dl_fork = getenv("GDF_DL_FORK") != nullptr;
    bool mirror_valid = false;
    uint32_t mirror_ticket = 0, mirror_gen = 0;

    // compaction outputs

    // voxel grid
    bool grid_set = false;
    float vlo[3] = {0, 0, 0}, vhi[3] = {0, 0, 0}, vcs[3] = {0, 0, 0};
    uint32_t gs[3] = {0, 0, 0};
    uint64_t ncells = 0;
    uint32_t key_bits = 0;
    VoxelParams vp{};
    DevBuf d_grid8, d_hist32, d_out8;
    DevBuf d_snap_dense;  // a batch frame's grid expanded from its sparse snapshot (download)
    DevBuf d_gridctl;               // GridSeq counters [0] updates done, [1] blocks finished
    uint32_t grid_ticket = 0;       // sequence number of the next grid update
    // The grid updates' order on the device is the ticket (GridSeq: a carrying launch's grid
    // blocks wait until the updates before theirs are done).  That wait cannot stall: tickets
    // follow the host's submission order, so the awaited update was submitted earlier - ahead of
    // the waiter in any hardware queue the two share (in-order dispatch) - and the waiters of at
    // most 4 slots (<= 4 x ~205 blocks of one wave each) leave the chip's other ~7 K wave slots to
    // it; kSpinLimit turns a stall into GDF_ERR_DEVICE regardless.
    // GDF_GRID_GATE=1 orders direct launches by the streams as well: a launch carrying an update
    // waits for the event recorded after the previous update when that one ran on another stream
    // (GDF_GRID_GATE=early: recorded right before it - next in its stream, dispatchable), so no
    // block ever waits for work queued on another stream.  Measured on MI355X (A/B, one box, 2000
    // steps each, profiles/r06/grid_gate/): C2 30.2 (tickets) vs 28.7 (gate) / 28.9 (early) -
    // each cross-stream wait costs the batch's chain more than the spin it removes.
    const char* grid_gate_env = getenv("GDF_GRID_GATE");
    bool grid_gate = grid_gate_env != nullptr;
    bool grid_gate_early = grid_gate_env && std::strcmp(grid_gate_env, "early") == 0;
    hipEvent_t grid_ev = nullptr;       // recorded after the last gated update
    hipStream_t grid_ev_stream = nullptr;  // ... on this stream (nullptr: none yet)
    uint32_t grid_gen = 0;          // bumped when the grid is (re)allocated: slots re-zero marks
    int grid_mode = 0;  // 0: u8 grid = history (lifetime <= 255); 1: u32 history + u8 output
    bool grid_alloc = false;
    bool invoked_once = false;

    // voxelize

    bool debug = false;

    // live timing: event pairs per launch, resolved on query
    bool profiling = false;
    struct EvPair { hipEvent_t a, b; int slot; };
    std::vector<EvPair> ev_pending;
    std::vector<hipEvent_t> ev_pool;
    double prof_ms[GDF_KERNEL_SLOTS] = {};
    uint64_t prof_n[GDF_KERNEL_SLOTS] = {};

    hipStream_t s() const { return user_stream ? user_stream : sl().stream(); }

    hipEvent_t take_event() {
        if (!ev_pool.empty()) {
            hipEvent_t ev = ev_pool.back();
            ev_pool.pop_back();
            return ev;
        }
        hipEvent_t ev;
        HIPCHK(hipEventCreate(&ev));
        return ev;
    }
    // brackets one launch (or launch group) of `slot` with an event pair when profiling
    template <class F>
    void timed(int slot, F&& launch) { timed_on(slot, s(), launch); }
    template <class F>
    void timed_on(int slot, hipStream_t st, F&& launch) {
        if (!profiling) {
            launch();
            return;
        }
        EvPair p{take_event(), take_event(), slot};
        HIPCHK(hipEventRecord(p.a, st));
        launch();
        HIPCHK(hipEventRecord(p.b, st));
        ev_pending.push_back(p);
        if (ev_pending.size() > 4096) resolve_events();
    }
    // per-kernel event pairs inside launch_frame / launch_voxelize
    struct Hook : LaunchHook {
        gdf_engine* e;
        std::vector<hipEvent_t> open;
        explicit Hook(gdf_engine* e_) : e(e_) {}
        void begin(int) override {
            hipEvent_t a = e->take_event();
            HIPCHK(hipEventRecord(a, e->s()));
            open.push_back(a);
        }
        void end(int slot) override {
            hipEvent_t b = e->take_event();
            HIPCHK(hipEventRecord(b, e->s()));
            e->ev_pending.push_back(EvPair{open.back(), b, slot});
            open.pop_back();
        }
    };
    Hook hook{this};
    LaunchHook* hook_ptr() { return profiling ? &hook : nullptr; }
    void resolve_events() {
        for (EvPair& p : ev_pending) {
            HIPCHK(hipEventSynchronize(p.b));
            float ms = 0.f;
            HIPCHK(hipEventElapsedTime(&ms, p.a, p.b));
            prof_ms[p.slot] += ms;
            prof_n[p.slot] += 1;
            ev_pool.push_back(p.a);
            ev_pool.push_back(p.b);
        }
        ev_pending.clear();
    }

    void sync() {
        Slot& c = sl();
        HIPCHK(hipStreamSynchronize(s()));
        if (c.h_misc && c.h_misc[kErr]) {
            const uint32_t code = c.h_misc[kErr];
            c.h_misc[kErr] = 0;
            HIPCHK(hipMemsetAsync(c.d_misc.as<uint32_t>() + kErr, 0, 4, s()));
            fail(GDF_ERR_DEVICE, "device error flags (code " + std::to_string(code) +
                                     ": 1/2/4 look-back / grid spin limit, 8 run-group queue full, 16 run over 64 points)");
        }
    }
    // read the small device counters into pinned memory (after the producing kernels)
    void read_misc() {
        HIPCHK(hipMemcpyAsync(sl().h_misc, sl().d_misc.p, kMiscWords * 4, hipMemcpyDeviceToHost, s()));
        sync();
    }
    // once per frame, before rewriting state the frames in flight may still read (rollbuffer
    // ring, selection / camera tables, grid allocation): drain the other slots on the host
    void serialize() {
        if (npipe <= 1 || serialized) return;
        for (int i = 0; i < npipe; ++i)
            if (i != cur && slots[i].stream()) HIPCHK(hipStreamSynchronize(slots[i].stream()));
        serialized = true;
    }
    // the ordering of one historic-grid update: ticket f (or the ticket the frame's k_mask stored)
    // (one stream: stream order suffices, no device ordering)
    GridSeq grid_seq(uint32_t f, const uint32_t* fptr = nullptr) {
        GridSeq q{};
        q.ctl = npipe > 1 ? d_gridctl.as<uint32_t>() : nullptr;
        q.fptr = fptr;
        q.f = f;
        q.err = sl().d_misc.as<uint32_t>() + kErr;
        return q;
    }
    // the stream gate of a grid update launched on st: the event to wait for before it (null:
    // none - the previous gated update ran on st, or there was none) and the one to record after
    hipEvent_t grid_gate_wait(hipStream_t st) const {
        return grid_gate && npipe > 1 && grid_ev_stream && grid_ev_stream != st ? grid_ev : nullptr;
    }
    hipEvent_t grid_gate_record(hipStream_t st) {
        if (!grid_gate || npipe <= 1) return nullptr;
        if (!grid_ev) HIPCHK(hipEventCreateWithFlags(&grid_ev, hipEventDisableTiming));
        grid_ev_stream = st;
        return grid_ev;
    }
    // a grid-update launch of its own on st, between the gate's wait and record
    template <class F>
    void grid_gated(hipStream_t st, F&& launch) {
        if (hipEvent_t w = grid_gate_wait(st)) HIPCHK(hipStreamWaitEvent(st, w, 0));
        launch();
        if (hipEvent_t r = grid_gate_record(st)) HIPCHK(hipEventRecord(r, st));
    }
};

namespace {

void create_slot(Slot& sl) {
    if (sl.own) return;
    HIPCHK(hipStreamCreateWithFlags(&sl.own, hipStreamNonBlocking));
    HIPCHK(hipHostMalloc((void**)&sl.h_misc, kMiscWords * 4, hipHostMallocDefault));
    std::memset(sl.h_misc, 0, kMiscWords * 4);
}

void sync_all(gdf_engine* e) {
    if (e->user_stream) HIPCHK(hipStreamSynchronize(e->user_stream));
    for (Slot& sl : e->slots)
        if (sl.stream()) HIPCHK(hipStreamSynchronize(sl.stream()));
}

// frame boundary (gdf_clear): the next frame goes to the next slot
void next_slot(gdf_engine* e) {
    if (e->npipe <= 1) return;
    e->ring = (e->ring + 1) % e->npipe;
    e->cur = e->ring;
    e->serialized = false;
}

// ---- frame inputs ---------------------------------------------------------------------------------
void engine_clear(gdf_engine* e) {  // fusion.cpp:725-732
    next_slot(e);
    e->sl().pf_valid = false;
    e->nframes = 1;
    e->rb.selection_point_count = 0;
    e->rb.selection_sequence_count = 0;
    e->depth_total = 0;
    e->cams.clear();
    e->halo_cams.clear();
    e->halo_tail.clear();
    e->depth_uploaded = false;
    e->converted = e->flying_set = e->crop_set = false;
    e->prepared = e->sel_inserted = false;
}

void add_depthmap(gdf_engine* e, const uint16_t* host, const uint16_t* dev, uint32_t W, uint32_t H,
                  float scale, float fx, float fy, float cx, float cy, const float* Tw,
                  const float* Tc) {
    if ((!host && !dev) || !Tw || !Tc || W == 0 || H == 0) fail(GDF_ERR_ARG, "addDepthmap: bad argument");
    if (e->cams.size() >= GDF_MAX_CAMERAS) fail(GDF_ERR_ARG, "addDepthmap: too many cameras");
    if ((uint64_t)W * H >= (1ull << 24))
        fail(GDF_ERR_ARG, "addDepthmap: W*H must stay below 2^24 (exact f32 pixel coordinates)");
    if ((uint64_t)e->depth_total + (uint64_t)W * H >= (1ull << 31))
        fail(GDF_ERR_ARG, "addDepthmap: total pixels exceed 2^31");
    Cam c;
    c.host = host;
    c.dev = dev;
    c.frame = e->nframes - 1;
    c.W = W; c.H = H; c.n = W * H;
    c.scale = scale; c.fx = fx; c.fy = fy; c.cx = cx; c.cy = cy;
    std::memcpy(c.Tw, Tw, 64);
    std::memcpy(c.Tc, Tc, 64);
    e->cams.push_back(c);
    e->depth_total += c.n;
    e->depth_uploaded = false;
}

void add_point_sequence(gdf_engine* e, const void* rec, uint32_t n, uint32_t step, uint32_t sec,
                        uint32_t nsec, const float* Tm) {  // fusion.cpp:747-796
    if ((n && (!rec || step < 12)) || !Tm) fail(GDF_ERR_ARG, "addPointSequence: bad argument");
    std::lock_guard<std::mutex> lk(e->ps_mutex);
    PsBuf* b = e->collect;
    if ((uint64_t)b->total + n > 0xFFFFFFFFull) fail(GDF_ERR_CAPACITY, "addPointSequence: too many points");
    Hdr h;
    h.sec = sec; h.nsec = nsec; h.start = b->total; h.num = n;
    std::memcpy(h.T, Tm, 64);
    PsRun run;
    run.dst = b->total;
    run.n = n;
    run.hsrc = b->host_total;
    b->pts.resize((b->host_total + n) * 4);
    const uint8_t* r = static_cast<const uint8_t*>(rec);
    float* o = b->pts.data() + b->host_total * 4;
    for (uint32_t k = 0; k < n; ++k) {
        std::memcpy(o + 4 * (size_t)k, r + (size_t)k * step, 12);
        o[4 * (size_t)k + 3] = 1.0f;
    }
    b->host_total += n;
    b->total += n;
    b->seqs.push_back(h);
    b->add_run(run);
}

// addPointSequence with the PointCloud2 records in device memory of the engine's GPU: borrowed
// (like addDepthmap's pointer) until the next uploadPointSequences, gathered on the device there.
void add_point_sequence_device(gdf_engine* e, const void* rec, uint32_t n, uint32_t step,
                               uint32_t sec, uint32_t nsec, const float* Tm) {
    if ((n && (!rec || step < 12 || step % 4 || reinterpret_cast<uintptr_t>(rec) % 4)) || !Tm)
        fail(GDF_ERR_ARG, "addPointSequenceDevice: bad argument (records need 4-byte alignment)");
    std::lock_guard<std::mutex> lk(e->ps_mutex);
    PsBuf* b = e->collect;
    if ((uint64_t)b->total + n > 0xFFFFFFFFull) fail(GDF_ERR_CAPACITY, "addPointSequence: too many points");
    Hdr h;
    h.sec = sec; h.nsec = nsec; h.start = b->total; h.num = n;
    std::memcpy(h.T, Tm, 64);
    PsRun run;
    run.dst = b->total;
    run.n = n;
    run.step = step;
    run.dev = rec;
    b->total += n;
    b->seqs.push_back(h);
    b->add_run(run);
}

// ---- point-sequence chain -----------------------------------------------------------------------
void upload_point_sequences(gdf_engine* e) {  // fusion.cpp:819-857
    std::lock_guard<std::mutex> lk(e->ps_mutex);
    if (e->collect == &e->psA) { e->upload = &e->psA; e->collect = &e->psB; }
    else { e->collect = &e->psA; e->upload = &e->psB; }
    e->collect->clear();
    e->n_new = e->upload->total;
    e->new_hdrs = e->upload->seqs;
    if (e->n_new) {
        e->serialize();  // d_new / the ring are shared with the previous frame
        e->d_new.ensure((size_t)e->n_new * 16);
        float4* dst = e->d_new.as<float4>();
        for (const PsRun& r : e->upload->runs) {
            if (r.dev)
                HIPCHK(launch_gather_records(r.dev, r.n, r.step, dst + r.dst, e->s()));
            else
                HIPCHK(hipMemcpyWithStream(dst + r.dst, e->upload->pts.data() + 4 * r.hsrc,
                                           (size_t)r.n * 16, hipMemcpyHostToDevice, e->s()));
        }
    }
    e->ps_filter_set = false;
}

void ensure_ring(gdf_engine* e, uint64_t need) {
    if (need <= e->ring_cap) return;
    uint64_t cap = std::max<uint64_t>(need + need / 2, 1u << 20);
    void* q = nullptr;
    HIPCHK(hipStreamSynchronize(e->s()));
    if (hipMalloc(&q, cap * 16) != hipSuccess) fail(GDF_ERR_NOMEM, "rollbuffer ring allocation failed");
    const uint64_t R = e->rb.num_points;
    if (R && e->d_ring.p) {  // linearise the live window into the new ring
        const uint64_t first = e->ring_head % e->ring_cap;
        const uint64_t a = std::min<uint64_t>(R, e->ring_cap - first);
        HIPCHK(hipMemcpyAsync(q, e->d_ring.as<float4>() + first, a * 16, hipMemcpyDeviceToDevice, e->s()));
        if (R > a)
            HIPCHK(hipMemcpyAsync(static_cast<float4*>(q) + a, e->d_ring.p, (R - a) * 16,
                                  hipMemcpyDeviceToDevice, e->s()));
        HIPCHK(hipStreamSynchronize(e->s()));
    }
    if (e->d_ring.p) HIPCHK(hipFree(e->d_ring.p));
    e->d_ring.p = q;
    e->d_ring.bytes = cap * 16;
    e->ring_cap = cap;
    e->ring_head = 0;
}

void insert_new_point_sequences(gdf_engine* e) {  // fusion.cpp:979-1087
    if (e->n_new) e->serialize();  // ring writes; without new points only host headers change
    const uint32_t R = e->rb.num_points, S = e->rb.num_seqs;
    if (e->hdrB.size() < S) fail(GDF_ERR_STATE, "insert: rollbuffer headers out of sync");
    if ((uint64_t)R + e->n_new >= (1ull << 31)) fail(GDF_ERR_CAPACITY, "rollbuffer exceeds 2^31 points");
    // sequence ids; a sharded engine keeps the points of its own sequences only (the filter still
    // reads every new point: its neighbours cross sequences, filter_point_sequence.glsl:78-122)
    uint32_t kept = 0;
    std::vector<std::pair<uint32_t, uint32_t>> spans;  // own (first new point, count), merged
    for (Hdr& h : e->new_hdrs) {
        h.id = e->seq_counter++;
        h.num_global = h.num;
        const bool own = e->nshards <= 1 || (h.id / e->shard_block) % e->nshards == e->shard;
        if (own && h.num) {
            if (!spans.empty() && spans.back().first + spans.back().second == h.start)
                spans.back().second += h.num;
            else
                spans.emplace_back(h.start, h.num);
            kept += h.num;
        }
        if (!own) h.num = 0;
    }
    ensure_ring(e, (uint64_t)R + kept);
    if (kept)
        e->timed(GDF_KERNEL_PS_INSERT, [&] {
            uint32_t at = 0;
            for (const auto& sp : spans) {
                HIPCHK(launch_ps_filter_insert(e->d_new.as<float4>(), e->n_new, e->ps_filter_set ? 1 : 0,
                                               e->ps_thr, e->ps_F, e->d_ring.as<float4>(), e->ring_cap,
                                               (e->ring_head + R + at) % e->ring_cap, e->s(),
                                               sp.first, sp.second));
                at += sp.second;
            }
        });
    e->hdrA.assign(e->hdrB.begin(), e->hdrB.begin() + S);
    e->hdrA.insert(e->hdrA.end(), e->new_hdrs.begin(), e->new_hdrs.end());
    e->rb.num_points = R + kept;
    e->rb.num_seqs = S + (uint32_t)e->new_hdrs.size();
    if (!e->new_hdrs.empty()) {
        e->rb.last_time_sec = e->new_hdrs.back().sec;
        e->rb.last_time_nsec = e->new_hdrs.back().nsec;
    }
}

void roll_rollbuffer(gdf_engine* e, uint32_t min_sec, uint32_t min_nsec) {  // fusion.cpp:1098-1217
    // host-side only (headers and the ring head); ring slots it frees are rewritten by a later
    // insert, which serializes on the previous frame
    uint32_t d_seqs = 0, d_pts = 0;
    const uint32_t nseq = (uint32_t)e->hdrA.size();
    for (uint32_t i = 0; i < nseq; ++i) {
        const Hdr& q = e->hdrA[i];
        if (compare_time(q.sec, q.nsec, min_sec, min_nsec) < 0) {
            d_pts += q.num;
        } else {
            d_seqs = i;
            break;
        }
    }
    if (nseq > d_seqs) {
        e->rb.earliest_time_sec = e->hdrA[d_seqs].sec;
        e->rb.earliest_time_nsec = e->hdrA[d_seqs].nsec;
    } else {
        e->rb.earliest_time_sec = e->rb.earliest_time_nsec = 0;
        e->rb.last_time_sec = e->rb.last_time_nsec = 0;
    }
    if (d_pts > e->rb.num_points || d_seqs > e->rb.num_seqs)
        fail(GDF_ERR_STATE, "roll: discarded points exceed the rollbuffer (reference uint underflow)");
    if (e->ring_cap) e->ring_head = (e->ring_head + d_pts) % e->ring_cap;
    e->hdrB.assign(e->hdrA.begin() + d_seqs, e->hdrA.end());
    e->rb.num_points -= d_pts;
    e->rb.num_seqs -= d_seqs;
}

void select_timespan(gdf_engine* e, uint32_t mins, uint32_t minn, uint32_t maxs,
                     uint32_t maxn) {  // fusion.cpp:1358-1416
    const uint32_t num_seqs = e->rb.num_seqs;
    int64_t start = num_seqs, last = 0;
    uint32_t pcount = 0, pstart = 0;
    for (uint32_t i = 0; i < e->hdrB.size(); ++i) {
        const Hdr& q = e->hdrB[i];
        if (compare_time(mins, minn, q.sec, q.nsec) <= 0 && compare_time(q.sec, q.nsec, maxs, maxn) <= 0) {
            if ((int64_t)i < start) start = i;
            if ((int64_t)i > last) last = i;
            pcount += q.num;
        }
    }
    const int64_t count = last < start ? 0 : 1 + last - start;
    // a sharded window is the unsharded one spread over the shards only when the selected
    // sequences are the contiguous run [start, last] (time-ordered headers, as a sensor's are):
    // an unselected sequence with points inside it would shift each shard's point range differently
    if (e->nshards > 1)
        for (int64_t i = start; i <= last && i < (int64_t)e->hdrB.size(); ++i) {
            const Hdr& q = e->hdrB[i];
            if (q.num_global && !(compare_time(mins, minn, q.sec, q.nsec) <= 0 &&
                                  compare_time(q.sec, q.nsec, maxs, maxn) <= 0))
                fail(GDF_ERR_STATE, "sharded rollbuffer: the selected sequences are not contiguous "
                                    "(point sequences out of time order)");
        }
    for (int64_t i = 0; i < start && i < (int64_t)e->hdrB.size(); ++i) pstart += e->hdrB[i].num;
    e->rb.selection_point_start = pstart;
    e->rb.selection_point_count = pcount;
    e->rb.selection_sequence_start = (uint32_t)start;
    e->rb.selection_sequence_count = (uint32_t)count;
}

void prepare_buffers(gdf_engine* e) {  // fusion.cpp:1497-1508
    const uint64_t n = (uint64_t)e->depth_total + e->rb.selection_point_count;
    if (n >= (1ull << 31)) fail(GDF_ERR_CAPACITY, "more than 2^31 points in one frame");
    e->sl().n_total = (uint32_t)n;
    e->sl().d_pts.ensure((size_t)(n ? n : 1) * 16);
    e->sl().d_coords.ensure((size_t)(n ? n : 1) * 4);
    e->prepared = true;
}

void insert_selected(gdf_engine* e, const float* Twm, const float* Tcm) {  // fusion.cpp:1509-1553
    if (!Twm || !Tcm) fail(GDF_ERR_ARG, "insertSelectedPointSequence: null transform");
    if (!e->prepared) fail(GDF_ERR_STATE, "insertSelectedPointSequence before preparePointAndMaskBuffers");
    const uint32_t ps = e->rb.selection_point_start, cnt = e->rb.selection_point_count;
    const uint32_t ss = e->rb.selection_sequence_start, sc = e->rb.selection_sequence_count;
    if ((uint64_t)e->depth_total + cnt > e->sl().n_total) fail(GDF_ERR_STATE, "selection exceeds prepared buffers");
    if (cnt && (uint64_t)ps + cnt > e->rb.num_points) fail(GDF_ERR_STATE, "selection exceeds rollbuffer points");
    if (sc && (uint64_t)ss + sc > e->hdrB.size()) fail(GDF_ERR_STATE, "selection exceeds rollbuffer sequences");
    e->sel_cuts.clear();
    if (e->nshards > 1 && sc) {
        // the selection's pieces: maximal stretches of selected sequences (with points) held by one
        // shard, in order; this shard's rollbuffer points are cut where its 2nd, 3rd .. piece
        // starts (the exchange places every piece at its place in the unsharded order).  Every
        // shard sees the same headers, so every shard accepts or rejects the window alike.
        std::vector<uint32_t> pieces(e->nshards, 0);
        int64_t cur = -1;
        uint64_t own = 0;
        for (uint32_t j = ss; j < ss + sc; ++j) {
            const Hdr& h = e->hdrB[j];
            if (!h.num_global) continue;
            const int64_t k = (int64_t)((h.id / e->shard_block) % e->nshards);
            if (k != cur) {
                if (k == (int64_t)e->shard && pieces[k]) e->sel_cuts.push_back((uint32_t)own);
                ++pieces[k];
                cur = k;
            }
            if (k == (int64_t)e->shard) own += h.num;
        }
        const uint32_t most = *std::max_element(pieces.begin(), pieces.end());
        const uint32_t room = std::min<uint32_t>(kMaxSegs, std::max<uint32_t>(e->epart.nseg, 2u)) - 1u;
        if (most > room)
            fail(GDF_ERR_STATE, "sharded rollbuffer: a shard holds " + std::to_string(most) +
                                " separate pieces of the selected window, the exchange carries " +
                                std::to_string(room) + " (raise the block size: the window spans " +
                                "too many blocks)");
    }
    if (cnt == 0) {  // nothing selected: the frame kernels read no selection table
        e->nseg = 0;
        e->sel_inserted = true;
        return;
    }
    e->serialize();  // the selection tables are shared with the previous frame
    // transforms of the selected sequences (kernel 19 of SURVEY §2b, computed host-side)
    std::vector<float> tfw((size_t)std::max<uint32_t>(sc, 1) * 16), tfc(tfw.size());
    for (uint32_t j = 0; j < sc; ++j) {
        mat_mul(Twm, e->hdrB[ss + j].T, tfw.data() + 16 * (size_t)j);
        mat_mul(Tcm, e->hdrB[ss + j].T, tfc.data() + 16 * (size_t)j);
    }
    // transform index per point = seq_idx[p] - seq_idx[sel_point_start] (kernel 18): the points
    // of sequence j get index j - s0, s0 = sequence containing point sel_point_start.
    std::vector<uint32_t> seg_start, seg_tf;
    if (cnt) {
        uint64_t cum = 0;
        int64_t s0 = -1;
        if (e->nshards > 1) {  // the unsharded engine's s0: the first selected sequence with points
            for (uint32_t j = ss; j < e->hdrB.size() && s0 < 0; ++j)
                if (e->hdrB[j].num_global) s0 = j;
        }
        for (uint32_t j = 0; j < e->hdrB.size(); ++j) {
            const uint64_t a = cum, b = cum + e->hdrB[j].num;
            cum = b;
            if (b <= ps || a == b) continue;
            if (a >= (uint64_t)ps + cnt) break;
            if (s0 < 0) s0 = j;
            const uint64_t rel = a > ps ? a - ps : 0;
            const uint32_t t = (uint32_t)(j - s0);
            if (t >= sc) fail(GDF_ERR_STATE, "transform index outside the selected sequences");
            seg_start.push_back((uint32_t)rel);
            seg_tf.push_back(t);
        }
        if (seg_start.empty()) fail(GDF_ERR_STATE, "selected points not covered by sequences");
    }
    e->nseg = (uint32_t)seg_start.size();
    // equal sequences (FrameArgs::sel_uniform): every start after the first k * S - off
    e->sel_uniform = e->sel_off = 0;
    if (e->nseg >= 2) {
        const uint64_t S = e->nseg >= 3 ? (uint64_t)seg_start[2] - seg_start[1] : seg_start[1];
        const uint64_t off = S >= seg_start[1] ? S - seg_start[1] : S;
        bool uni = S > 0 && S >= seg_start[1] && off < S && (uint64_t)cnt + off < (1ull << 32);
        for (uint32_t k = 1; uni && k < e->nseg; ++k) uni = (uint64_t)seg_start[k] + off == k * S;
        if (uni) {
            e->sel_uniform = (uint32_t)S;
            e->sel_off = (uint32_t)off;
        }
    }
    if (e->nseg) {
        e->d_seg_start.ensure(e->nseg * 4);
        e->d_seg_tf.ensure(e->nseg * 4);
        HIPCHK(hipMemcpyWithStream(e->d_seg_start.p, seg_start.data(), e->nseg * 4, hipMemcpyHostToDevice, e->s()));
        HIPCHK(hipMemcpyWithStream(e->d_seg_tf.p, seg_tf.data(), e->nseg * 4, hipMemcpyHostToDevice, e->s()));
    }
    e->d_tfw.ensure(tfw.size() * 4);
    e->d_tfc.ensure(tfc.size() * 4);
    HIPCHK(hipMemcpyWithStream(e->d_tfw.p, tfw.data(), tfw.size() * 4, hipMemcpyHostToDevice, e->s()));
    HIPCHK(hipMemcpyWithStream(e->d_tfc.p, tfc.data(), tfc.size() * 4, hipMemcpyHostToDevice, e->s()));
    e->sel_inserted = true;
}

// ---- depth chain ------------------------------------------------------------------------------------
void ensure_table(gdf_engine* e, size_t slot, const Cam& c) {
    CamTable& t = e->tables[slot];
    if (t.valid && t.W == c.W && t.H == c.H && t.fx == c.fx && t.fy == c.fy && t.cx == c.cx &&
        t.cy == c.cy)
        return;
    e->serialize();  // the previous frame may still read the old table
    t.xn.ensure((size_t)c.W * 4);
    t.yn.ensure((size_t)c.H * 4);
    HIPCHK(launch_tables(c.W, c.H, c.fx, c.fy, c.cx, c.cy, t.xn.as<float>(), t.yn.as<float>(), e->s()));
    t.W = c.W; t.H = c.H; t.fx = c.fx; t.fy = c.fy; t.cx = c.cx; t.cy = c.cy;
    t.valid = true;
}

// Host depth maps (the reference's blocking glBufferSubData, fusion.cpp:1583-1593) are copied
// into the slot's pinned staging buffer (after the slot's previous copy from it has finished; the
// frame's maps in one parallel copy, StagingCopier) and sent to the slot's device buffer with
// hipMemcpyAsync on the slot's own stream: the caller's buffer is free again when
// gdf_upload_depthmaps returns, as in the reference, and the DMA of frame f+1 overlaps the kernels
// of frame f (another slot, another stream) with no cross-stream event.  Every host map is
// staged, pinned or not.  (Measured on MI355X, tools/h2d_probe.py: a VGA frame costs +9 us per
// frame this way at 3 frames in flight; a DMA straight from the caller's hipHostMalloc buffer was
// slower, +160 us.)
struct HostUpload {
    uint16_t* dst;
    uint8_t* stage;
    const void* src;
    size_t bytes;
};

void stage_host_depth(gdf_engine* e, uint16_t* dst, const Cam& c, size_t& staged,
                      std::vector<HostUpload>& ups) {
    Slot& q = e->sl();
    const size_t bytes = (size_t)c.n * 2;
    if (q.h2d_pending) {  // the slot's previous frame may still read the staging
        HIPCHK(hipEventSynchronize(q.h2d_done));
        q.h2d_pending = false;
    }
    if (q.h_stage_bytes < staged + bytes) fail(GDF_ERR_STATE, "depth staging not sized");
    ups.push_back({dst, static_cast<uint8_t*>(q.h_stage) + staged, c.host, bytes});
    staged += bytes;
}

void upload_depthmaps(gdf_engine* e) {  // fusion.cpp:1583-1593
    uint64_t host_px = 0;
    for (const Cam& c : e->cams)
        if (!c.dev) host_px += c.n;
    if (host_px) e->sl().d_depth.ensure(host_px * 2);
    if (host_px && e->sl().h_stage_bytes < host_px * 2) {  // grow the staging once per frame
        Slot& q = e->sl();
        if (q.h2d_pending) HIPCHK(hipEventSynchronize(q.h2d_done));
        q.h2d_pending = false;
        if (q.h_stage) HIPCHK(hipHostFree(q.h_stage));
        q.h_stage = nullptr;
        q.h_stage_bytes = 0;
        HIPCHK(hipHostMalloc(&q.h_stage, host_px * 2, hipHostMallocDefault));
        q.h_stage_bytes = host_px * 2;
    }
    size_t staged = 0;
    std::vector<HostUpload> ups;
    if (e->cams.size() + e->halo_cams.size() > (size_t)kMaxCams) fail(GDF_ERR_ARG, "too many cameras (incl. halo)");
    // halo cameras (multi-GPU): the cameras that precede this engine's first one in the
    // reference's concatenated buffer, at negative offsets; only their last `tail` pixels exist
    // (a virtual base pointer: the flying-pixel reads reach back at most F rows + F pixels,
    // checked in frame_args)
    // Index space: a frame's halo camera sits right before the frame's first depth map (frame 0's
    // at negative offsets, later frames' in a gap after the previous frame's cameras), so every
    // frame's top-border reads resolve exactly as in the reference's concatenated buffer.
    e->halo.clear();
    auto halo_desc = [&](size_t j, int64_t off) {
        const Cam& c = e->halo_cams[j];
        CamDesc d{};
        d.off = off;
        d.depth = c.dev - (c.n - e->halo_tail[j]);
        ensure_table(e, j, c);
        d.xn = e->tables[j].xn.as<float>();
        d.yn = e->tables[j].yn.as<float>();
        d.W = c.W; d.H = c.H; d.n = c.n; d.emit = 0;
        d.scale = c.scale;
        d.wmagic = ((1ull << 40) + c.W - 1) / c.W;
        d.frame = c.frame;
        std::memcpy(d.Tw, c.Tw, 64);
        std::memcpy(d.Tc, c.Tc, 64);
        return d;
    };
    e->h_cams.clear();
    e->mask_blocks = 0;
    e->max_segw = 0;
    int64_t off = 0;
    uint64_t hoff = 0;
    size_t hj = 0;  // next halo camera (in frame order)
    std::vector<CamDesc> ordered;  // halo of frame f, then frame f's depth maps
    for (size_t k = 0; k < e->cams.size(); ++k) {
        const Cam& c = e->cams[k];
        if (hj < e->halo_cams.size() && e->halo_cams[hj].frame == c.frame &&
            (k == 0 || e->cams[k - 1].frame != c.frame)) {
            const int64_t hn = (int64_t)e->halo_cams[hj].n;
            const int64_t hstart = hj == 0 && k == 0 ? -hn : off;
            ordered.push_back(halo_desc(hj, hstart));
            e->halo.push_back(ordered.back());
            if (hstart >= 0) off += hn;  // (later frames: the halo takes a gap in the index space)
            ++hj;
        }
        CamDesc d{};
        d.off = off;
        if (c.dev) {
            d.depth = c.dev;
        } else {
            uint16_t* dst = e->sl().d_depth.as<uint16_t>() + hoff;
            stage_host_depth(e, dst, c, staged, ups);
            d.depth = dst;
            hoff += c.n;
        }
        ensure_table(e, e->halo_cams.size() + k, c);
        d.xn = e->tables[e->halo_cams.size() + k].xn.as<float>();
        d.yn = e->tables[e->halo_cams.size() + k].yn.as<float>();
        d.W = c.W; d.H = c.H; d.n = c.n; d.emit = 1;
        d.frame = c.frame;
        d.scale = c.scale;
        d.wmagic = ((1ull << 40) + c.W - 1) / c.W;
        // compaction segments: rows split into nchunk pieces of segw (a multiple of 64) pixels
        // segment width: whole rows (up to 1024 px) for small frames, 256 px for frames (or
        // batches) over 1 Mi pixels, where more, smaller blocks per CU hide the band loads
        // (measured on MI355X, dense frames, mask + emit: 4K 1024 -> 256 px 311 -> 237 us,
        // 720p x4 140 -> 107 us; 128 px and 64 px lose again in the mask)
        const uint32_t seg_items = e->seg_items ? e->seg_items : (e->depth_total > (1u << 20) ? 256u : kSegItems);
        d.nchunk = (c.W + seg_items - 1) / seg_items;
        d.segw = ((c.W + d.nchunk - 1) / d.nchunk + 63) / 64 * 64;
        d.nseg = c.H * d.nchunk;
        d.seg0 = e->mask_blocks;
        e->mask_blocks += d.nseg;
        e->max_segw = std::max(e->max_segw, d.segw);
        std::memcpy(d.Tw, c.Tw, 64);
        std::memcpy(d.Tc, c.Tc, 64);
        e->h_cams.push_back(d);
        ordered.push_back(d);
        off += c.n;
    }
    if (hj != e->halo_cams.size()) fail(GDF_ERR_STATE, "a halo camera without a depth map in its frame");
    e->index_end = (uint64_t)std::max<int64_t>(off, 0);
    if (staged) {  // the staging is free again once these copies have run
        std::vector<StagingCopier::Job> jobs;
        for (const HostUpload& u : ups) jobs.push_back({u.stage, static_cast<const uint8_t*>(u.src), u.bytes});
        e->copier.run(jobs);
        // one DMA per contiguous run of staged maps (a batch's maps are staged and placed back to
        // back): 8 VGA frames as one 4.9 MB copy instead of 8 copies with a command gap each
        // (~8 us between 17-us copies in the trace, profiles/r04/h2d/)
        for (size_t i = 0; i < ups.size();) {
            size_t j = i + 1, bytes = ups[i].bytes;
            while (j < ups.size() &&
                   reinterpret_cast<uint8_t*>(ups[j].dst) == reinterpret_cast<uint8_t*>(ups[i].dst) + bytes &&
                   ups[j].stage == ups[i].stage + bytes)
                bytes += ups[j++].bytes;
            HIPCHK(hipMemcpyAsync(ups[i].dst, ups[i].stage, bytes, hipMemcpyHostToDevice, e->s()));
            i = j;
        }
        Slot& q = e->sl();
        if (!q.h2d_done) HIPCHK(hipEventCreateWithFlags(&q.h2d_done, hipEventDisableTiming));
        HIPCHK(hipEventRecord(q.h2d_done, e->s()));
        q.h2d_pending = true;
    }
    // every frame's halo right before the frame's depth maps: sorted by offset (k_emit finds a
    // frame's first camera by its predecessor)
    e->h_cams = ordered;
    e->depth_uploaded = true;
}

// the slot's mark bitmask exists and is zero for the current grid
void ensure_marks(gdf_engine* e) {
    Slot& sl = e->sl();
    if (sl.marks_gen == e->grid_gen && sl.marks_frames >= e->nframes) return;
    const uint32_t nf = std::max(e->nframes, sl.marks_gen == e->grid_gen ? sl.marks_frames : 1u);
    const size_t bytes = (size_t)((e->ncells + 31) / 32) * 4 * nf;
    sl.d_markbits.ensure(bytes);
    HIPCHK(hipMemsetAsync(sl.d_markbits.p, 0, bytes, e->s()));
    sl.marks_gen = e->grid_gen;
    sl.marks_frames = nf;
}

// bits of the sort key: the voxel key, plus the frame index of a batch above it
uint32_t frame_bits(const gdf_engine* e) {
    return e->nframes > 1 ? 32u - (uint32_t)__builtin_clz(e->nframes - 1) : 0u;
}
uint32_t sort_bits(const gdf_engine* e) { return e->key_bits + frame_bits(e); }

void set_grid(gdf_engine* e, const float* lo, const float* hi, const float* cs) {
    // shader grid size (fusion.cpp:1693-1698) and VoxelGridMeta (grid_meta.h:140-158) must agree
    uint32_t g[3];
    uint64_t cells = 1;
    for (int a = 0; a < 3; ++a) {
        const float f = (hi[a] - lo[a]) / cs[a];
        if (!(f > 0.0f) || !(f < 4294967040.0f)) fail(GDF_ERR_ARG, "voxel grid: need lower < upper and cell_size > 0");
        g[a] = (uint32_t)std::ceil(f);
        cells *= g[a];
    }
    if (cells >= 0xFFFFFFFFull) fail(GDF_ERR_ARG, "voxel grid: more than 2^32-1 cells");
    std::memcpy(e->vlo, lo, 12);
    std::memcpy(e->vhi, hi, 12);
    std::memcpy(e->vcs, cs, 12);
    std::memcpy(e->gs, g, 12);
    for (int a = 0; a < 3; ++a) {
        e->vp.vlo[a] = lo[a];
        e->vp.vcs[a] = cs[a];
        e->vp.vrcs[a] = 1.0f / cs[a];  // IEEE, correctly rounded
        e->vp.gmax[a] = (float)(g[a] - 1u);
        e->vp.gs[a] = g[a];
    }
    e->key_bits = cells <= 1 ? 0u : 64u - (uint32_t)__builtin_clzll(cells - 1);
    const bool changed = !e->grid_alloc || cells != e->ncells;
    e->ncells = cells;
    e->grid_set = true;
    if (changed) {  // historic grid cleared on first use / resize (fusion.cpp:1759-1773)
        sync_all(e);  // no grid update in flight on any stream
        const size_t padded = (size_t)((cells + 31) / 32) * 32;
        e->d_grid8.ensure(padded);
        HIPCHK(hipMemsetAsync(e->d_grid8.p, 0, padded, e->s()));
        e->d_gridctl.ensure(64);
        HIPCHK(hipMemsetAsync(e->d_gridctl.p, 0, 64, e->s()));
        e->grid_ticket = 0;
        HIPCHK(hipStreamSynchronize(e->s()));  // the other streams see the cleared counters
        e->grid_mode = 0;
        e->grid_alloc = true;
        e->grid_gen++;
        e->sl().marks_set = false;
    }
    ensure_marks(e);
}

// the frame's occupancy marks: 1 bit per cell, consumed (and cleared) by the grid update
uint32_t* marks_ptr(const gdf_engine* e) { return e->sl().d_markbits.as<uint32_t>(); }
uint64_t mark_words(const gdf_engine* e) { return (e->ncells + 31) / 32; }

void ensure_misc(gdf_engine* e);

// The delta outputs (changed 32-cell groups) of the single-frame u8 grid update about to be
// issued with sequence number t on the current slot - once a grid download asked for them.
void delta_args(gdf_engine* e, GridSeq& q, uint32_t t, bool single) {
    Slot& sl = e->sl();
    sl.delta_valid = false;
    if (!e->grid_delta || !single || e->grid_mode != 0) return;
    const uint64_t nw = mark_words(e);
    sl.d_didx.ensure(nw * 4);
    sl.d_ddata.ensure(nw * 32);
    ensure_misc(e);
    HIPCHK(hipMemsetAsync(sl.d_misc.as<uint32_t>() + kDeltaCount, 0, 4, e->s()));
    q.dcnt = sl.d_misc.as<uint32_t>() + kDeltaCount;
    q.didx = sl.d_didx.as<uint32_t>();
    q.ddata = sl.d_ddata.as<uint4>();
    sl.delta_valid = true;
    sl.delta_ticket = t;
}

// switch to the general u32 history once a lifetime no longer fits the u8 grid
void widen_if_needed(gdf_engine* e, uint32_t lifetime, hipStream_t st) {
    if (e->grid_mode != 0 || lifetime <= 255) return;
    ensure_misc(e);
    e->d_hist32.ensure((size_t)e->ncells * 4);
    e->d_out8.ensure((size_t)((e->ncells + 31) / 32) * 32);
    e->grid_gated(st, [&] {
        HIPCHK(launch_widen_grid(e->d_grid8.as<uint8_t>(), e->d_hist32.as<uint32_t>(), e->ncells,
                                 e->grid_seq(e->grid_ticket++), st));
    });
    e->grid_mode = 1;
}

void ensure_misc(gdf_engine* e) {
    if (!e->sl().d_misc.p) {
        e->sl().d_misc.ensure(kMiscWords * 4);
        HIPCHK(hipMemsetAsync(e->sl().d_misc.p, 0, kMiscWords * 4, e->s()));
    }
    if (!e->sl().d_ctrs.p) e->sl().d_ctrs.ensure_zero(kCtrSlots * 8, e->s());
    if (!e->sl().d_khist.p) e->sl().d_khist.ensure_zero(kHistWords * 4, e->s());
}

// Arguments of the fused compaction launch: convert + flying + crop + selected-point transform +
// ordered compaction (+ voxel keys and occupancy marks when fused_voxel).
FrameArgs frame_args(gdf_engine* e, bool fused_voxel, bool compaction_marks = false) {
    if (!e->prepared) prepare_buffers(e);
    if (!e->depth_uploaded) upload_depthmaps(e);
    ensure_misc(e);
    FrameArgs a;
    std::memset(&a, 0, sizeof(a));  // padding too: graph keys compare the bytes
    a.tune = &e->tune;
    a.ncams = (int32_t)e->h_cams.size();
    if (a.ncams <= kArgCams) {
        for (size_t k = 0; k < e->h_cams.size(); ++k) a.cams[k] = e->h_cams[k];
    } else {  // pageable source: the copy is staged before hipMemcpyAsync returns
        e->sl().d_camdesc.ensure(e->h_cams.size() * sizeof(CamDesc));
        HIPCHK(hipMemcpyAsync(e->sl().d_camdesc.p, e->h_cams.data(), e->h_cams.size() * sizeof(CamDesc),
                              hipMemcpyHostToDevice, e->s()));
        a.cams_dev = e->sl().d_camdesc.as<const CamDesc>();
    }
    if (e->seg_uniform && !e->h_cams.empty()) {  // (FrameArgs::seg_uniform)
        uint32_t u = e->h_cams[0].nseg;
        for (size_t k = 0; k < e->h_cams.size(); ++k) {
            const CamDesc& d = e->h_cams[k];
            if (!d.emit || d.nseg != u || d.seg0 != (uint32_t)k * u) u = 0;
        }
        a.seg_uniform = u;
    }
    a.depth_total = e->depth_total;
    const uint32_t sel = e->sel_inserted ? e->rb.selection_point_count : 0u;
    a.depth_segs = e->mask_blocks;
    // one item per thread: blocks as wide as the widest segment
    a.seg_threads = e->max_segw ? std::max<uint32_t>(64, e->max_segw) : kSegItems;
    a.total_segs = a.depth_segs;
    // k_sel tiles: 4 K points; 16 K for windows over 16 Mi points, whose ~10^4..10^5 tiles would
    // otherwise queue on the one ticket counter (measured on MI355X, C3's 236 M-point window:
    // 57.6 K tiles 2.92 ms, 14.4 K tiles 2.11 ms per frame)
    const bool big_window = !e->sel_shape_set && sel > (1u << 24);
    a.sel_segs = big_window ? 16u : e->sel_segs;
    a.sel_tile = big_window ? 16u * 1024u : e->sel_segs * e->sel_threads;
    a.sel_tiles = (uint32_t)(((uint64_t)sel + a.sel_tile - 1) / a.sel_tile);
    if (a.sel_tiles) {  // rollbuffer compaction (k_sel) + placement behind the depth points
        Slot& q = e->sl();
        // (epoch-tagged granules: zeroed once when allocated, never between frames)
        q.d_selstat.ensure_zero((size_t)4 * (a.sel_tiles + a.sel_tiles / 64 + 2) * 8, e->s());
        a.sel_status = q.d_selstat.as<unsigned long long>();
        a.sel_ctr = reinterpret_cast<uint32_t*>(q.d_ctrs.as<unsigned long long>() + kCtrSel);
        a.epoch_word = reinterpret_cast<uint32_t*>(q.d_ctrs.as<unsigned long long>() + kCtrEpoch);
    }
    a.do_flying = e->flying_set ? 1 : 0;
    a.F = e->F;
    a.thr = e->thr;
    a.rot45 = e->rot45;
    a.do_crop = e->crop_set ? 1 : 0;
    std::memcpy(a.lo, e->lo, 12);
    std::memcpy(a.hi, e->hi, 12);
    a.sel_count = sel;
    a.ring = e->d_ring.as<const float4>();
    a.ring_cap = e->ring_cap ? e->ring_cap : 1;
    a.ring_first = e->ring_cap ? (e->ring_head + e->rb.selection_point_start) % e->ring_cap : 0;
    a.nseg = e->nseg;
    a.seg_start = e->d_seg_start.as<uint32_t>();
    a.sel_uniform = e->sel_uniform;
    a.sel_off = e->sel_off;
    a.seg_tf = e->d_seg_tf.as<uint32_t>();
    a.tfw = e->d_tfw.as<float>();
    a.tfc = e->d_tfc.as<float>();
    if (a.sel_tiles) {  // (the partition's segment cuts: depth | the pieces of the selection)
        a.sel_splits = e->sl().d_misc.as<uint32_t>() + kSplit0;
        a.sel_ncuts = (uint32_t)std::min<size_t>(e->sel_cuts.size(), kMaxSegs - 2);
        for (uint32_t c = 0; c < a.sel_ncuts; ++c) a.sel_cut_at[c] = e->sel_cuts[c];
    }
    a.do_voxel = fused_voxel ? 1 : 0;
    e->sl().group_marks = fused_voxel && a.sel_tiles && !compaction_marks;
    if (fused_voxel) {
        // With rollbuffer points (10^7 survivors of a window that re-observes the same voxels) the
        // occupancy marks come from the voxel groups after the sort - one per voxel - instead of
        // device-scope atomics per run of survivors; the grid update is then its own launch.
        // A frame whose voxelize is deferred (multi-GPU: the rank with the rollbuffer sends its
        // points away to the key-range owners) has no local groups: k_sel marks them itself.
        // Otherwise: marks from the compaction, and the sequence number the grid update fused
        // into the first radix pass will take.
        if (!e->sl().group_marks) {
            a.grid_seq_out = e->sl().d_misc.as<uint32_t>() + kGridTicket;
            a.grid_seq = e->grid_ticket;
            if (!(compaction_marks && e->epart.nparts && !e->part_marks)) a.marks = marks_ptr(e);
        }
        std::memcpy(a.vlo, e->vp.vlo, 12);
        std::memcpy(a.vcs, e->vp.vcs, 12);
        std::memcpy(a.vrcs, e->vp.vrcs, 12);
        std::memcpy(a.gmax, e->vp.gmax, 12);
        std::memcpy(a.gs, e->vp.gs, 12);
        if (e->sl().khist_pending) HIPCHK(hipMemsetAsync(e->sl().d_khist.p, 0, kHistWords * 4, e->s()));
        // digit histogram of the keys from the compaction blocks (frees the sort of a separate
        // pass) - but not over a large rollbuffer window, where tens of thousands of blocks would
        // each flush their histogram with device-scope atomics; k_sort_hist counts those keys
        a.key_hist = a.total_segs <= kFusedPrefixSegs && !a.sel_tiles ? e->sl().d_khist.as<uint32_t>()
                                                                      : nullptr;
        a.npasses = radix_passes(sort_bits(e));
        // depth-only frames sort runs of equal keys (8-20x fewer items on dense frames); k_mask
        // counts the runs and their key digits (one flush per segment: few runs, few bins)
        // (measured on MI355X, dense frames: 4K 18.2 -> 24.0 Gpoints/s, a batch of four VGA frames
        // 14.6 -> 16.8; a single VGA frame (0.3 Mi pixels) gains nothing: the extra key in k_mask
        // costs what the shorter sort saves, so frames under 1 Mi pixels sort points)
        // Rollbuffer windows (10^7 points re-observing the same voxels) always sort runs: k_sel
        // counts them per tile.
        // (a deferred voxelize - the multi-GPU exchange - sorts what the rank RECEIVES, whose runs
        // gdf_voxelize_points finds itself: the compaction counts none)
        a.run_mode = e->use_runs && !compaction_marks &&
                             (a.sel_tiles || (a.total_segs && (e->force_runs ||
                                                               a.depth_total >= (1u << 20))))
                         ? 1 : 0;
        // the run-key digits: k_mask's per-segment flush while there are few segments; above,
        // k_sort_hist over the runs (tens of thousands of flushes contend at the atomic units)
        if (a.run_mode)
            a.key_hist = (a.total_segs <= kFusedPrefixSegs || e->run_hist_all) && !e->run_hist_in_sort &&
                         !a.sel_tiles
                             ? e->sl().d_khist.as<uint32_t>() : nullptr;
    }
    // k_sel keeps the voxel keys of its run detection in LDS for its store pass (run mode; not for
    // the debug stage bits' launches).  GDF_NO_SEL_KEY_LDS: the store pass recomputes them.
    if (a.sel_tiles && a.run_mode && a.do_voxel && e->sel_key_lds && sel_key_lds_allowed(a.sel_tile * 4u))
        a.sel_key_lds = a.sel_tile * 4u;
    a.out_pts = e->sl().d_pts.as<float4>();
    a.out_coords = e->sl().d_coords.as<uint32_t>();
    // with rollbuffer points the depth compaction counts into kDepthCount and k_sel writes
    // the frame's total
    a.out_count = e->sl().d_misc.as<uint32_t>() + (a.sel_tiles ? kDepthCount : kCount);
    a.final_count = e->sl().d_misc.as<uint32_t>() + kCount;
    const uint32_t segs = std::max<uint32_t>(a.total_segs, 1);
    e->sl().d_vbits.ensure((size_t)segs * 16 * 8);
    e->sl().d_tcounts.ensure((size_t)segs * 2 * 4);  // point counts, then run counts
    e->sl().d_toffsets.ensure(seg_offsets_words(2 * segs) * 4);
    a.scan_total = e->sl().d_misc.as<uint32_t>() + kScanTotal;
    if (a.run_mode) {
        Slot& q = e->sl();
        q.d_wruns.ensure((size_t)segs * 16 * 4);
        q.d_runkeys.ensure((size_t)std::max<uint32_t>(q.n_total, 1) * 4);
        q.d_runstart.ensure(((size_t)q.n_total + 1) * 4);
        a.wave_runs = q.d_wruns.as<uint32_t>();
        a.run_keys = q.d_runkeys.as<uint32_t>();
        a.run_start = q.d_runstart.as<uint32_t>();
        a.run_count = q.d_misc.as<uint32_t>() + kRunCount;
        if (a.sel_tiles) a.run_total = q.d_misc.as<uint32_t>() + kRunTotal;
    }
    e->sl().runs_sel = a.run_mode && a.sel_tiles;
    a.vbits = e->sl().d_vbits.as<unsigned long long>();
    a.seg_counts = e->sl().d_tcounts.as<uint32_t>();
    a.seg_offsets = e->sl().d_toffsets.as<uint32_t>();
    a.fused_prefix = a.total_segs <= kFusedPrefixSegs ? 1 : 0;
    a.mask_packed = e->mask_packed ? 1 : 0;
    // above: the last k_mask block of each group of kScanGroup segments scans the group (no scan
    // launches); k_emit sums the group totals before its own
    const uint32_t ngroups = (a.total_segs + kScanGroup - 1) / kScanGroup;
    if (!a.fused_prefix && e->group_scan && ngroups <= kMaxScanGroups) {
        Slot& q = e->sl();
        q.d_grpdone.ensure_zero((size_t)ngroups * 4, e->s());  // (self-resetting afterwards)
        q.d_grptot.ensure((size_t)ngroups * 2 * 4);
        a.grp_done = q.d_grpdone.as<uint32_t>();
        a.grp_tot = q.d_grptot.as<uint32_t>();
    }
    // k_mask's LDS band: 2h+1 rows of 16-B chunks covering segw + 2h columns (+1 chunk of
    // alignment), then the columns' ray factors
    {
        const uint32_t h = a.do_flying ? std::min<uint32_t>(a.F, kHalo) : 0u;
        const uint32_t cols = e->max_segw + 2 * h;
        a.band_rowb = ((cols * 2 + 15) / 16 + 1) * 16;
        a.band_lds = (2 * h + 1) * a.band_rowb + (kHalo + a.seg_threads * 2) * 4;
        a.hist_lds = (a.band_lds + 15) & ~15u;  // (k_mask_px: the digit histogram, when counted)
        if (a.run_mode && a.key_hist) a.band_lds = a.hist_lds + 4 * 256 * 4;
    }
    if (e->debug) {  // (stage bits by global index: halo gaps included)
        e->sl().d_stage.ensure(std::max<size_t>({(size_t)e->sl().n_total, (size_t)e->index_end + sel, 1}));
        a.dbg = e->sl().d_stage.as<uint8_t>();
    }
    e->sl().dbg_count = e->sl().n_total;
    a.err = e->sl().d_misc.as<uint32_t>() + kErr;
    if (!e->halo_cams.empty() && a.do_flying && !e->cams.empty()) {
        for (size_t j = 0; j < e->halo_cams.size(); ++j) {  // each halo against its frame's camera
            const Cam* first = nullptr;
            for (const Cam& c : e->cams)
                if (c.frame == e->halo_cams[j].frame) { first = &c; break; }
            if (!first) continue;
            const uint64_t reach = (uint64_t)a.F * first->W + a.F;  // deepest read into the halo
            if (reach > e->halo_cams[j].n)
                fail(GDF_ERR_ARG, "halo camera shorter than F rows of the frame's first camera "
                                  "(reads would reach the camera before it)");
            if (e->halo_tail[j] < reach)
                fail(GDF_ERR_ARG, "halo depth map tail shorter than F rows + F pixels of the frame's first camera");
        }
    }
    a.nframes = e->nframes;
    a.frame_shift = e->nframes > 1 ? e->key_bits : 0u;
    a.mark_words = mark_words(e);
    e->sl().sel_frame = a.sel_tiles != 0;  // (the partition pass's [depth | rollbuffer] split)
    // (2 segments: a frame without a selection has no rollbuffer segment - the counts take the
    // 2-segment layout, segment 1 empty)
    if (fused_voxel && compaction_marks && e->epart.nparts && e->emit_part && !a.sel_tiles &&
        a.total_segs && !e->debug) {
        // the compaction writes the key-range partition itself (k_mask_px + k_emit_px2 only;
        // anything else compacts, then partitions: gdf_process_frame)
        FrameArgs t = a;
        t.run_mode = 1;
        t.key_hist = nullptr;
        t.fused_prefix = 0;
        t.grp_done = t.grp_tot = nullptr;
        if (emit_partition_kernels(t)) {
            Slot& q = e->sl();
            const uint32_t segs = std::max<uint32_t>(a.total_segs, 1);
            const uint32_t P = e->epart.nparts;
            q.d_tcounts.ensure((size_t)segs * 2 * P * 4);
            q.d_toffsets.ensure(seg_offsets_words(2 * P * segs) * 4);
            q.d_wruns.ensure((size_t)segs * 16 * 4);
            t.seg_counts = q.d_tcounts.as<uint32_t>();
            t.seg_offsets = q.d_toffsets.as<uint32_t>();
            t.wave_runs = q.d_wruns.as<uint32_t>();
            t.nparts = P;
            t.part_ncells = e->ncells;
            t.part_pts = reinterpret_cast<float4*>(e->epart.pts);
            t.part_run_keys = e->epart.run_keys;
            t.part_run_starts = e->epart.run_starts;
            t.part_counts = e->epart.counts;
            t.part_nseg = e->epart.nseg;
            a = t;
        }
    }
    e->sl().nframes = e->nframes;
    e->sl().snap_valid = false;  // (set by this batch's grid update when it keeps the frames' grids)
    if (e->nframes > 1) {
        e->sl().d_fstart.ensure((size_t)(e->nframes + 1) * 4);
        a.frame_pt_start = e->sl().d_fstart.as<uint32_t>();
    }
    return a;
}

void frame_launched(gdf_engine* e, bool fused_voxel, bool key_hist, bool runs = false) {
    e->sl().khist_pending = fused_voxel && key_hist;
    e->sl().runs_valid = fused_voxel && runs;
    e->sl().compacted = true;
    e->sl().coords_valid = fused_voxel;
    e->sl().marks_set = fused_voxel;
    e->sl().vox_valid = false;
}

void run_frame(gdf_engine* e, bool fused_voxel, bool compaction_marks = false) {
    e->sl().pf_valid = false;
    const FrameArgs a = frame_args(e, fused_voxel, compaction_marks);
    e->sl().part_emitted = a.nparts != 0;
    if (e->profiling) e->timed(GDF_KERNEL_EVENT_FLOOR, [] {});  // calibrates the event overhead
    e->timed(GDF_KERNEL_FRAME, [&] { HIPCHK(launch_frame(a, e->s(), e->hook_ptr())); });
    frame_launched(e, fused_voxel, a.key_hist != nullptr, a.run_mode != 0);
    if (fused_voxel && !a.marks && !e->sl().group_marks) e->sl().marks_set = false;  // (no marks)
    if (a.nparts) {  // (the points went to the send lists only: no compaction-order outputs)
        e->sl().coords_valid = false;
        e->sl().runs_valid = false;
    }
}

void compute_voxel_coords(gdf_engine* e, const float* lo, const float* hi, const float* cs) {
    if (!e->sl().compacted) fail(GDF_ERR_STATE, "computeVoxelCoords before applyPointMask");
    set_grid(e, lo, hi, cs);
    HIPCHK(launch_coords(e->sl().d_pts.as<float4>(), e->sl().d_misc.as<uint32_t>() + kCount,
                         std::max<uint32_t>(e->sl().n_total, 1), e->sl().d_coords.as<uint32_t>(), e->vp, e->s()));
    e->sl().coords_valid = true;
    e->sl().marks_set = false;
    e->sl().runs_valid = false;  // the keys were recomputed: no runs for them
}

// an external (point, key) list to voxelize instead of the frame's compaction (multi-GPU fused
// cloud: the lists all-to-all'ed by key range)
struct VoxSource {
    const float4* pts = nullptr;
    const uint32_t* keys = nullptr;
    uint32_t n = 0;
    const uint32_t* run_keys = nullptr;  // its runs of equal keys (launch_xruns), or none
    const uint32_t* run_start = nullptr;
};

// the slot's sparse snapshot buffers for a grid update of `nblocks` blocks over `nframes` frames
// (the batch's frames but the last are kept); marks the slot's snapshots valid
SnapArgs snap_args(gdf_engine* e, uint32_t nblocks, uint32_t nframes) {
    Slot& q = e->sl();
    uint32_t W = 0, seg = 0;
    snap_dims(e->ncells, nblocks, &W, &seg);
    const size_t entries = (size_t)W * seg * (nframes - 1);
    q.d_snap_idx.ensure(entries * 4);
    q.d_snap_data.ensure(entries * 32);
    q.d_snap_cnt.ensure((size_t)W * (nframes - 1) * 4);
    q.snap_valid = true;
    q.snap_blocks = nblocks;
    q.snap_frames = nframes;
    return SnapArgs{q.d_snap_idx.as<uint32_t>(), q.d_snap_data.as<uint4>(), q.d_snap_cnt.as<uint32_t>()};
}

VoxelizeArgs voxelize_args(gdf_engine* e, int average, int fused_grid_lifetime,
                           const VoxSource* src = nullptr) {  // fusion.cpp:1743-1756
    if (!e->grid_set || (!src && !e->sl().coords_valid))
        fail(GDF_ERR_STATE, "voxelize before computeVoxelCoords");
    const uint32_t nmax = std::max<uint32_t>(src ? src->n : e->sl().n_total, 1);
    if (nmax >= (1u << 31)) fail(GDF_ERR_CAPACITY, "voxelize supports < 2^31 points");
    ensure_misc(e);
    e->sl().d_ka.ensure((size_t)nmax * 4);
    e->sl().d_kb.ensure((size_t)nmax * 4);
    e->sl().d_va.ensure((size_t)nmax * 4);
    e->sl().d_vb.ensure((size_t)nmax * 4);
    const size_t swords = voxelize_status_words(nmax, sort_bits(e));
    e->sl().d_sstatus.ensure_zero(swords * 8, e->s());
    e->sl().d_sgstatus.ensure_zero((swords / kSortGroup + 512) * 8, e->s());
    e->sl().d_gstatus.ensure_zero(voxelize_group_tiles(nmax) * 8, e->s());
    e->sl().d_ggstatus.ensure_zero((voxelize_group_tiles(nmax) / 64 + 2) * 8, e->s());
    e->sl().d_vox.ensure((size_t)nmax * 16);
    const uint32_t gtiles = (uint32_t)voxelize_group_tiles(nmax);
    e->sl().d_gcnt.ensure((size_t)gtiles * 4);
    e->sl().d_gfirst.ensure((size_t)gtiles * 4);
    e->sl().d_goff.ensure(seg_offsets_words(gtiles) * 4);
    if (e->group_scan) {  // k_group_count's own group scan (kernels skip it above their bound)
        const size_t ng = ((size_t)gtiles + kScanGroup - 1) / kScanGroup;
        e->sl().d_ggdone.ensure_zero(ng * 4, e->s());  // (self-resetting afterwards)
        e->sl().d_ggtot.ensure(ng * 4);
    }
    // point mode: <= 1 long voxel per tile; run mode: one queue entry per long group, at most
    // one per voxel of the batch
    const uint64_t qcap = std::min<uint64_t>(nmax, (uint64_t)std::max<uint32_t>(e->nframes, 1) * e->ncells);
    const uint64_t bigq_n = std::max<uint64_t>((uint64_t)gtiles + 2048, qcap);
    e->sl().d_bigq.ensure((size_t)bigq_n * 16);
    e->sl().d_bigcnt.ensure(2048 * 4);
    VoxelizeArgs v;
    std::memset(&v, 0, sizeof(v));
    v.tune = &e->tune;
    v.keys = e->sl().d_coords.as<uint32_t>();
    v.pts = e->sl().d_pts.as<float4>();
    v.count = e->sl().d_misc.as<uint32_t>() + kCount;
    if (src && src->run_keys) {  // the received list's runs (gdf_voxelize_points)
        v.keys = src->run_keys;
        v.pts = src->pts;
        v.count = e->sl().d_misc.as<uint32_t>() + kRecvRuns;
        v.run_start = src->run_start;
        v.point_count = e->sl().d_misc.as<uint32_t>() + kRecvCount;
    } else if (src) {
        v.keys = src->keys;
        v.pts = src->pts;
        v.count = e->sl().d_misc.as<uint32_t>() + kRecvCount;
    } else if (e->sl().runs_valid) {  // sort the frame's runs of equal keys, then expand
        v.keys = e->sl().d_runkeys.as<uint32_t>();
        v.count = e->sl().d_misc.as<uint32_t>() + (e->sl().runs_sel ? kRunTotal : kRunCount);
        v.run_start = e->sl().d_runstart.as<uint32_t>();
        v.point_count = e->sl().d_misc.as<uint32_t>() + kCount;
        v.pack_runs = e->pack_runs && sort_bits(e) <= 25 ? 1 : 0;
        // a batch of depth frames of at most VGA size each: a voxel rarely gathers the > 1 K
        // points of one frame that queue it for k_group_runs_big (profiles/r06/knob_big/: a VGA
        // batch queues none) - 32 blocks instead of the resident grid (queued groups still run)
        if (!e->sl().runs_sel && e->nframes > 1 &&
            e->depth_total <= (uint64_t)e->nframes * kSmallFramePixels)
            v.big_cap = kSmallFrameBigBlocks;
    }
    v.nmax = nmax;
    v.key_bits = sort_bits(e);
    v.average = average;
    v.hist_ready = e->sl().khist_pending && !src ? 1 : 0;
    v.vp = e->vp;
    v.keys_a = e->sl().d_ka.as<uint32_t>();
    v.keys_b = e->sl().d_kb.as<uint32_t>();
    v.vals_a = e->sl().d_va.as<uint32_t>();
    v.vals_b = e->sl().d_vb.as<uint32_t>();
    v.hist = e->sl().d_khist.as<uint32_t>();
    v.status = e->sl().d_sstatus.as<unsigned long long>();
    v.sgstatus = e->sl().d_sgstatus.as<unsigned long long>();
    v.gstatus = e->sl().d_gstatus.as<unsigned long long>();
    v.ggstatus = e->sl().d_ggstatus.as<unsigned long long>();
    v.ctrs = e->sl().d_ctrs.as<unsigned long long>();
    // keys per thread of a radix tile: small frames want many tiles (latency), big ones few
    // (each tile publishes 256 look-back words: 2 KiB per 1 Ki keys at PT=4)
    v.group_counts = e->sl().d_gcnt.as<uint32_t>();
    v.group_first = e->tune.group_first ? e->sl().d_gfirst.as<uint32_t>() : nullptr;
    v.group_offsets = e->sl().d_goff.as<uint32_t>();
    v.group_done = e->group_scan ? e->sl().d_ggdone.as<uint32_t>() : nullptr;
    v.group_gtot = e->group_scan ? e->sl().d_ggtot.as<uint32_t>() : nullptr;
    v.bigq = e->sl().d_bigq.as<uint4>();
    v.bigq_cap = (uint32_t)std::min<uint64_t>(bigq_n, 0xFFFFFFFFu);
    v.bigcnt = e->sl().d_bigcnt.as<uint32_t>();
    v.sort_pt = e->sort_pt ? e->sort_pt : nmax <= (1u << 20) ? 4 : nmax <= (1u << 24) ? 8 : 16;
    v.err = e->sl().d_misc.as<uint32_t>() + kErr;
    v.out = e->sl().d_vox.as<float4>();
    v.out_count = e->sl().d_misc.as<uint32_t>() + kVoxCount;
    if (e->sl().group_marks) v.group_marks = marks_ptr(e);
    v.nframes = e->nframes;
    v.frame_shift = e->nframes > 1 ? e->key_bits : 0u;
    v.mark_words = mark_words(e);
    if (e->nframes > 1) {
        // (frame bits from the point ranges - not for runs, whose keys carry them, nor for an
        // external list, whose keys carry them too: gdf_partition_points of a batch)
        v.frame_pt_start = v.run_start || src ? nullptr : e->sl().d_fstart.as<uint32_t>();
        e->sl().d_fvox.ensure((size_t)(e->nframes + 1) * 4);
        v.frame_vox_start = e->sl().d_fvox.as<uint32_t>();
    }
    if (fused_grid_lifetime >= 0 && !e->sl().group_marks) {  // processFrame: the grid update rides on the first sort pass
        v.grid8 = e->d_grid8.as<uint8_t>();
        v.marks = marks_ptr(e);
        v.ncells = e->ncells;
        v.lifetime = (uint32_t)fused_grid_lifetime;
        // the ticket was stored by this frame's k_mask (run_frame: grid_seq = grid_ticket)
        v.gseq = e->grid_seq(0, e->sl().d_misc.as<uint32_t>() + kGridTicket);
        delta_args(e, v.gseq, e->grid_ticket, e->nframes == 1);
        e->grid_ticket++;
        if (e->nframes > 1) v.snap = snap_args(e, fused_grid_blocks(e->ncells, e->tune.grid_wpt), e->nframes);
    }
    return v;
}

void voxelize_launched(gdf_engine* e, int fused_grid_lifetime) {
    if (e->sl().group_marks) {
        e->sl().marks_set = true;  // set by k_group; the grid update follows separately
    } else if (fused_grid_lifetime >= 0) {
        e->sl().marks_set = false;
        e->invoked_once = true;
    }
    e->sl().khist_pending = false;
    e->sl().vox_valid = true;
}

// the stream gate of the grid update a direct voxelize launch carries (its first radix pass)
VoxelizeArgs gated(gdf_engine* e, VoxelizeArgs v, hipStream_t st) {
    if (v.grid8) {
        v.grid_wait = e->grid_gate_wait(st);
        v.grid_rec = e->grid_gate_record(st);
        v.grid_rec_early = e->grid_gate_early ? 1 : 0;
    }
    return v;
}

void voxelize(gdf_engine* e, int average, int fused_grid_lifetime = -1) {
    e->sl().pf_valid = false;
    const VoxelizeArgs v = gated(e, voxelize_args(e, average, fused_grid_lifetime), e->s());
    e->timed(GDF_KERNEL_VOXELIZE, [&] { HIPCHK(launch_voxelize(v, e->s(), e->hook_ptr())); });
    voxelize_launched(e, fused_grid_lifetime);
}

void occupancy_grid(gdf_engine* e, uint32_t lifetime, hipStream_t st);

// graph key: the launch arguments without the per-frame fields (depth pointers, grid ticket)
void graph_key(const FrameArgs& a, FrameArgs& k) {
    k = a;
    for (int c = 0; c < kArgCams; ++c) k.cams[c].depth = nullptr;
    k.grid_seq = 0;
}

bool same_key(const FrameArgs& a, const VoxelizeArgs& v, const FrameArgs& ka, const VoxelizeArgs& kv) {
    FrameArgs k;
    graph_key(a, k);
    return std::memcmp(&k, &ka, sizeof(k)) == 0 && std::memcmp(&v, &kv, sizeof(v)) == 0;
}

// processFrame's fused frame (compaction + voxelize + grid update) on the slot's stream:
// direct launches, or the slot's captured graph when the launch arguments repeat
// gdf_download_frame prefetch: a single frame's downloads written by k_download at the end of
// its launch chain (after the voxelize and the grid update it carries)
bool prefetch_on(const gdf_engine* e) { return e->dl_prefetch && e->nframes == 1 && !e->user_stream; }
bool prefetch_fork(const gdf_engine* e) { return prefetch_on(e) && e->dl_fork; }

// parts: DL_POINTS on the slot's aux stream right after the compaction (overlaps the voxelize),
// the rest at the end of the chain
void prefetch_downloads(gdf_engine* e, hipStream_t st, uint32_t parts) {
    Slot& q = e->sl();
    if (parts & DL_MISC) q.pf_valid = false;
    if (!prefetch_on(e)) return;
    if (parts == DL_POINTS) {  // (forked: its own stream after the compaction)
        if (!q.dl_aux) {
            HIPCHK(hipStreamCreateWithFlags(&q.dl_aux, hipStreamNonBlocking));
            HIPCHK(hipEventCreateWithFlags(&q.dl_ev, hipEventDisableTiming));
        }
        HIPCHK(hipEventRecord(q.dl_ev, st));
        HIPCHK(hipStreamWaitEvent(q.dl_aux, q.dl_ev, 0));
        st = q.dl_aux;
    }
    const uint32_t cap = std::max<uint32_t>(q.n_total, 1);
    const uint32_t dcap = q.delta_valid ? (uint32_t)((mark_words(e) + 3) / 4 * 4) : 0u;
    const int set = q.mir_next();  // (never the set the caller holds)
    Slot::Mirrors& M = q.mir[set];
    // a mirror about to grow is freed first: no earlier k_download may still write it
    if (M.pts.bytes < (size_t)cap * 16 || M.coords.bytes < (size_t)cap * 4 ||
        M.vox.bytes < (size_t)cap * 16 || M.delta.bytes < (size_t)std::max<uint32_t>(dcap, 4) * 36 ||
        M.misc.bytes < kMiscWords * 4) {
        HIPCHK(hipStreamSynchronize(q.stream()));
        if (q.dl_aux) HIPCHK(hipStreamSynchronize(q.dl_aux));
    }
    DlArgs d{};
    d.misc = q.d_misc.as<uint32_t>();
    d.misc_words = kMiscWords;
    d.i_count = kCount;
    d.i_vox = kVoxCount;
    d.i_delta = kDeltaCount;
    d.pts = q.d_pts.as<uint4>();
    d.coords = q.d_coords.as<uint32_t>();
    d.vox = q.d_vox.as<uint4>();
    d.didx = q.d_didx.as<uint32_t>();
    d.ddata = q.d_ddata.as<uint4>();
    d.pts_cap = cap;
    d.vox_cap = (uint32_t)std::min<size_t>(q.d_vox.bytes / 16, cap);
    d.delta_cap = dcap;
    d.h_misc = static_cast<uint32_t*>(M.misc.ensure(kMiscWords * 4));
    d.h_pts = static_cast<uint4*>(M.pts.ensure((size_t)cap * 16));
    d.h_coords = static_cast<uint32_t*>(M.coords.ensure((size_t)cap * 4));
    d.h_vox = static_cast<uint4*>(M.vox.ensure((size_t)cap * 16));
    uint8_t* hd = static_cast<uint8_t*>(M.delta.ensure((size_t)std::max<uint32_t>(dcap, 4) * 36));
    if (!d.h_misc || !d.h_pts || !d.h_coords || !d.h_vox || !hd)
        fail(GDF_ERR_NOMEM, "pinned download mirror allocation failed");
    d.h_didx = reinterpret_cast<uint32_t*>(hd);
    d.h_ddata = reinterpret_cast<uint4*>(hd + (size_t)dcap * 4);
    d.parts = parts;
    HIPCHK(launch_download(d, st));
    if (parts & DL_MISC) {
        q.pf_valid = true;
        q.mir_pf = set;
    }
}

void run_fused_frame(gdf_engine* e, int average, uint32_t lifetime) {
    const FrameArgs a = frame_args(e, true);
    frame_launched(e, true, a.key_hist != nullptr, a.run_mode != 0);  // (the launches below follow)
    const VoxelizeArgs v = voxelize_args(e, average, (int)lifetime);
    Slot::Graphs& G = e->sl().graph;
    // (a frame without compaction kernels stores its grid ticket with a memset: not replayable)
    if (e->sl().group_marks) {  // rollbuffer frame: marks from the voxel groups, then the grid
        e->timed(GDF_KERNEL_FRAME, [&] { HIPCHK(launch_frame(a, e->s(), e->hook_ptr())); });
        e->timed(GDF_KERNEL_VOXELIZE, [&] { HIPCHK(launch_voxelize(v, e->s(), e->hook_ptr())); });
        voxelize_launched(e, -1);
        occupancy_grid(e, lifetime, e->s());
        return;
    }
    // (a prefetching frame forks its points download after the compaction: direct launches)
    // (single frames only: a multi-frame batch launches directly - its replays measured 26.8 ->
    // 25.9 Gpoints/s on the C2 line once 8 descriptors fit the argument table)
    const bool eligible = e->use_graphs && !e->profiling && !e->debug && a.ncams <= kArgCams &&
                          !e->user_stream && a.total_segs && !prefetch_fork(e) && e->nframes == 1;
    hipStream_t st = e->s();
    Slot::GraphEntry* hit = nullptr;
    if (eligible)
        for (Slot::GraphEntry& x : G.e)
            if (x.valid && same_key(a, v, x.key_a, x.key_v)) hit = &x;
    int seen = -1;
    if (eligible && !hit)
        for (int c = 0; c < Slot::kGraphCache; ++c)
            if (G.cand[c] && same_key(a, v, G.cand_a[c], G.cand_v[c])) seen = c;
    if (hit) {
        void* args[] = {const_cast<FrameArgs*>(&a)};
        for (auto& np : hit->frame_nodes) {
            hipKernelNodeParams kp = np.second;
            kp.kernelParams = args;
            HIPCHK(hipGraphExecKernelNodeSetParams(hit->x, np.first, &kp));
        }
        HIPCHK(hipGraphLaunch(hit->x, st));
        hit->used = ++G.tick;
        ++G.replays;
    } else if (seen >= 0) {
        // the arguments repeated: capture this frame's launches and replay from now on, into a
        // free entry or the least recently used one
        Slot::GraphEntry* slot = nullptr;
        for (Slot::GraphEntry& x : G.e)
            if (!x.valid) {
                slot = &x;
                break;
            }
        if (!slot) {
            slot = &G.e[0];
            for (Slot::GraphEntry& x : G.e)
                if (x.used < slot->used) slot = &x;
        }
        if (slot->valid) HIPCHK(hipStreamSynchronize(st));  // no launch of the evicted graph in flight
        slot->reset();
        HIPCHK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
        hipError_t e1 = launch_frame(a, st, nullptr);
        hipError_t e2 = e1 == hipSuccess ? launch_voxelize(v, st, nullptr) : e1;
        hipGraph_t g = nullptr;
        hipError_t e3 = hipStreamEndCapture(st, &g);
        HIPCHK(e2);
        HIPCHK(e3);
        slot->g = g;
        HIPCHK(hipGraphInstantiate(&slot->x, slot->g, nullptr, nullptr, 0));
        size_t nn = 0;
        HIPCHK(hipGraphGetNodes(slot->g, nullptr, &nn));
        std::vector<hipGraphNode_t> nodes(nn);
        HIPCHK(hipGraphGetNodes(slot->g, nodes.data(), &nn));
        const void* fk[6] = {mask_kernel(a), emit_kernel(a),
                             frame_kernel(2, a.rot45),
                             frame_kernel(3, a.rot45), frame_kernel(4, a.rot45),
                             frame_kernel(5, a.rot45)};  // (the count scans take no FrameArgs)
        slot->frame_nodes.clear();
        for (hipGraphNode_t n : nodes) {
            hipGraphNodeType t;
            HIPCHK(hipGraphNodeGetType(n, &t));
            if (t != hipGraphNodeTypeKernel) continue;
            hipKernelNodeParams kp{};
            HIPCHK(hipGraphKernelNodeGetParams(n, &kp));
            if (std::find(fk, fk + 6, kp.func) != fk + 6)
                slot->frame_nodes.emplace_back(n, kp);
        }
        if (slot->frame_nodes.empty()) fail(GDF_ERR_HIP, "frame graph: compaction kernels not found");
        graph_key(a, slot->key_a);
        slot->key_v = v;
        slot->valid = true;
        slot->used = ++G.tick;
        G.cand[seen] = false;
        ++G.captures;
        HIPCHK(hipGraphLaunch(slot->x, st));
    } else {
        if (eligible) {
            const int c = G.cand_next;
            G.cand_next = (c + 1) % Slot::kGraphCache;
            graph_key(a, G.cand_a[c]);
            G.cand_v[c] = v;
            G.cand[c] = true;
        }
        if (e->profiling) e->timed(GDF_KERNEL_EVENT_FLOOR, [] {});
        e->timed(GDF_KERNEL_FRAME, [&] { HIPCHK(launch_frame(a, st, e->hook_ptr())); });
        if (prefetch_fork(e)) prefetch_downloads(e, st, DL_POINTS);
        const VoxelizeArgs vg = gated(e, v, st);
        e->timed(GDF_KERNEL_VOXELIZE, [&] { HIPCHK(launch_voxelize(vg, st, e->hook_ptr())); });
    }
    voxelize_launched(e, (int)lifetime);
    prefetch_downloads(e, st, DL_MISC | DL_VOX | DL_DELTA | (prefetch_fork(e) ? 0u : DL_POINTS));
}

void occupancy_grid(gdf_engine* e, uint32_t lifetime, hipStream_t st) {  // fusion.cpp:1757-1823
    e->sl().pf_valid = false;
    if (!e->grid_set) fail(GDF_ERR_STATE, "voxelOccupancyGrid before computeVoxelCoords");
    widen_if_needed(e, lifetime, st);
    if (!e->sl().marks_set) {
        if (!e->sl().coords_valid) fail(GDF_ERR_STATE, "voxelOccupancyGrid needs voxel coordinates");
        HIPCHK(launch_scatter(e->sl().d_coords.as<uint32_t>(), e->sl().d_misc.as<uint32_t>() + kCount,
                              std::max<uint32_t>(e->sl().n_total, 1), marks_ptr(e), st));
    }
    ensure_misc(e);
    GridSeq q = e->grid_seq(e->grid_ticket);
    delta_args(e, q, e->grid_ticket, st == e->s());
    e->grid_ticket++;
    e->grid_gated(st, [&] {
        e->timed_on(GDF_KERNEL_GRID, st, [&] {
            if (e->grid_mode == 0)
                HIPCHK(launch_grid_u8(e->d_grid8.as<uint8_t>(), marks_ptr(e), e->ncells, lifetime, q, st));
            else
                HIPCHK(launch_grid_u32(e->d_hist32.as<uint32_t>(), marks_ptr(e),
                                       e->d_out8.as<uint8_t>(), e->ncells, lifetime, q, st));
        });
    });
    e->sl().marks_set = false;
    e->invoked_once = true;
}

const uint8_t* grid_out_ptr(const gdf_engine* e) {
    return e->grid_mode == 0 ? e->d_grid8.as<uint8_t>() : e->d_out8.as<uint8_t>();
}

template <class F>
int guarded(gdf_engine* e, F&& f) {
    try {
        if (e) HIPCHK(hipSetDevice(e->device));
        f();
        return GDF_OK;
    } catch (const GdfError& err) {
        g_last_error = err.msg;
        return err.code;
    } catch (const std::bad_alloc&) {
        g_last_error = "host allocation failed";
        return GDF_ERR_NOMEM;
    } catch (...) {
        g_last_error = "unknown error";
        return GDF_ERR_STATE;
    }
}

#define ENGINE_OR_FAIL(e)                                                   \
    do {                                                                    \
        if (!(e)) {                                                         \
            g_last_error = "null engine";                                   \
            return GDF_ERR_ARG;                                             \
        }                                                                   \
    } while (0)

// nseg > 1: buckets [depth | rollbuffer pieces] per part (a frame with selected rollbuffer points
// is cut where k_sel recorded it, kSplit0..: its depth points, then the pieces of the selection
// this rank holds; any other frame is all depth)
void partition_runs(gdf_engine* e, uint32_t nparts, float* send_pts, uint32_t* send_run_keys,
                    uint32_t* send_run_starts, uint32_t capacity, uint32_t* part_counts,
                    uint32_t nseg = 1) {
    {
        Slot& q = e->sl();
        if (!e->grid_set || !q.coords_valid) fail(GDF_ERR_STATE, "partition needs the voxel keys of a frame");
        if (nparts == 0 || nparts > kMaxParts) fail(GDF_ERR_ARG, "partition: 1..16 parts");
        if (nseg == 0 || nseg > kMaxSegs || nparts * nseg > kMaxBuckets)
            fail(GDF_ERR_ARG, "partition: 1..4 segments, parts x segments <= 32");
        if (!send_pts || !send_run_keys || !send_run_starts || !part_counts)
            fail(GDF_ERR_ARG, "partition: null buffer");
        if (capacity < q.n_total) fail(GDF_ERR_CAPACITY, "partition: send buffers smaller than the frame");
        ensure_misc(e);
        const uint32_t nmax = std::max<uint32_t>(q.n_total, 1);
        const uint32_t m = 2 * nparts * nseg * std::max<uint32_t>(part_tiles(nmax), 1u);
        const uint32_t* split = q.d_misc.as<uint32_t>() + (q.sel_frame ? kSplit0 : kCount);
        q.d_pcnt.ensure((size_t)m * 4);
        q.d_poff.ensure(seg_offsets_words(m) * 4);
        HIPCHK(launch_partition(q.d_pts.as<float4>(), q.d_coords.as<uint32_t>(),
                                q.d_misc.as<uint32_t>() + kCount, nmax, nparts, e->ncells,
                                q.d_pcnt.as<uint32_t>(), q.d_poff.as<uint32_t>(),
                                q.d_misc.as<uint32_t>() + kPartTotal,
                                reinterpret_cast<float4*>(send_pts), nullptr, part_counts, e->s(),
                                q.nframes > 1 ? q.d_fstart.as<uint32_t>() : nullptr, q.nframes,
                                q.nframes > 1 ? e->key_bits : 0u, send_run_keys, send_run_starts,
                                split, nseg - 1, q.sel_frame ? 1u : 0u));
    }
}

}  // namespace

// ==== C-ABI ============================================================================================
extern "C" {

const char* gdf_last_error(void) { return g_last_error.c_str(); }

int gdf_get_graph_stats(gdf_engine* e, uint64_t* captures, uint64_t* replays) {
    ENGINE_OR_FAIL(e);
    uint64_t c = 0, r = 0;
    for (const Slot& sl : e->slots) {
        c += sl.graph.captures;
        r += sl.graph.replays;
    }
    if (captures) *captures = c;
    if (replays) *replays = r;
    return GDF_OK;
}

int gdf_get_stream(gdf_engine* e, void** out) {
    ENGINE_OR_FAIL(e);
    if (!out) return GDF_ERR_ARG;
    *out = static_cast<void*>(e->s());
    return GDF_OK;
}

int gdf_version(int* major, int* minor) {
    if (major) *major = GDF_VERSION_MAJOR;
    if (minor) *minor = GDF_VERSION_MINOR;
    return GDF_OK;
}

int gdf_create(int device, gdf_engine** out) {
    if (!out) {
        g_last_error = "null output";
        return GDF_ERR_ARG;
    }
    *out = nullptr;
    gdf_engine* e = new (std::nothrow) gdf_engine();
    if (!e) return GDF_ERR_NOMEM;
    e->device = device;
    int rc = guarded(e, [&] {
        create_slot(e->slots[0]);
        if (const char* v = std::getenv("GDF_SORT_PT")) e->sort_pt = std::atoi(v);  // tuning knob
        // the engine's launch shapes (Tuning, gdf_device.hpp): a snapshot of the GDF_* variables
        // at creation, read by this engine's launches only
        auto knob = [](const char* name, uint32_t dflt, int lo = 0, int hi = INT32_MAX) {
            const char* v = std::getenv(name);
            return v ? (uint32_t)std::min(hi, std::max(lo, std::atoi(v))) : dflt;
        };
        const Tuning d;
        Tuning& t = e->tune;
        t.group_scan_tiles = knob("GDF_GROUP_SCAN_TILES", d.group_scan_tiles, 1);
        t.run_stage = knob("GDF_RUN_STAGE", d.run_stage, 1);  // 512 or 2048
        t.emit_px2 = knob("GDF_EMIT_PX2", d.emit_px2);
        t.mask_occ8 = knob("GDF_MASK_OCC8", d.mask_occ8);
        t.grid_wpt = knob("GDF_GRID_WPT", d.grid_wpt, 1, 8);
        t.mask_px2 = knob("GDF_MASK_PX", d.mask_px2);  // pixels per k_mask thread
        t.run_q16 = knob("GDF_RUN_Q16", d.run_q16);
        t.group_first = knob("GDF_GROUP_FIRST", d.group_first);
        t.run_wave_mode = knob("GDF_RUN_WAVE_MODE", d.run_wave_mode);
        t.run_big_occ4 = knob("GDF_RUN_BIG_OCC4", d.run_big_occ4);
        t.run_big_blocks = knob("GDF_RUN_BIG_BLOCKS", d.run_big_blocks, 1);
        t.sort_blocks = knob("GDF_SORT_BLOCKS", d.sort_blocks, 1);
        t.group_blocks = knob("GDF_GROUP_BLOCKS", d.group_blocks, 1);
        t.run_inblock = knob("GDF_RUN_INBLOCK", d.run_inblock);
        t.points_lane = knob("GDF_POINTS_LANE", d.points_lane);
        t.run_wave = knob("GDF_RUN_WAVE", d.run_wave);
        t.small_group = knob("GDF_SMALL_GROUP", d.small_group);
        if (const char* v = std::getenv("GDF_SEG_ITEMS")) {  // tuning knob
            const uint32_t si = (uint32_t)std::atoi(v);
            if (si >= 64 && si <= kSegItems && si % 64 == 0) e->seg_items = si;
        }
        if (const char* v = std::getenv("GDF_SEL_SHAPE")) {  // tuning knob: "segs,threads"
            unsigned sg = 0, th = 0;
            if (std::sscanf(v, "%u,%u", &sg, &th) == 2 && (sg == 4 || sg == 8 || sg == 16) &&
                th >= 128 && th <= 1024 && th % 64 == 0 && sg * (th / 64) <= 256) {
                e->sel_segs = sg;
                e->sel_threads = th;
                e->sel_shape_set = true;
            }
        }
        ensure_misc(e);
        HIPCHK(hipStreamSynchronize(e->s()));
        // every tuning variable this engine was created under (none changes a result; a stray
        // one must not switch kernels silently): logged once, kept for gdf_get_tuning
        for (const char* name : kTuningVars)
            if (const char* v = std::getenv(name)) e->tuning_set += std::string(name) + "=" + v + " ";
        if (!e->tuning_set.empty()) {
            e->tuning_set.pop_back();
            std::fprintf(stderr, "libgdf: engine on device %d created with tuning %s\n", device,
                         e->tuning_set.c_str());
        }
    });
    if (rc != GDF_OK) {
        delete e;
        return rc;
    }
    *out = e;
    return GDF_OK;
}

int gdf_get_tuning(gdf_engine* e, char* buf, uint32_t capacity) {
    ENGINE_OR_FAIL(e);
    if (!buf || capacity == 0) return GDF_ERR_ARG;
    if (e->tuning_set.size() + 1 > capacity) {
        g_last_error = "tuning: buffer too small";
        return GDF_ERR_CAPACITY;
    }
    std::memcpy(buf, e->tuning_set.c_str(), e->tuning_set.size() + 1);
    return GDF_OK;
}

int gdf_destroy(gdf_engine* e) {
    if (!e) return GDF_OK;
    (void)hipSetDevice(e->device);
    if (e->user_stream) (void)hipStreamSynchronize(e->user_stream);
    for (Slot& sl : e->slots)
        if (sl.stream()) (void)hipStreamSynchronize(sl.stream());
    for (auto& p : e->ev_pending) {
        (void)hipEventDestroy(p.a);
        (void)hipEventDestroy(p.b);
    }
    for (auto ev : e->ev_pool) (void)hipEventDestroy(ev);
    if (e->grid_ev) (void)hipEventDestroy(e->grid_ev);
    for (Slot& sl : e->slots) {
        sl.graph.reset();
        if (sl.dl_aux) {
            (void)hipStreamSynchronize(sl.dl_aux);
            (void)hipStreamDestroy(sl.dl_aux);
        }
        if (sl.dl_ev) (void)hipEventDestroy(sl.dl_ev);
        if (sl.h_misc) (void)hipHostFree(sl.h_misc);
        if (sl.h_stage) (void)hipHostFree(sl.h_stage);
        if (sl.h2d_done) (void)hipEventDestroy(sl.h2d_done);
        if (sl.own) (void)hipStreamDestroy(sl.own);
    }
    delete e;
    return GDF_OK;
}

int gdf_set_stream(gdf_engine* e, void* stream) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] {
        sync_all(e);
        e->user_stream = static_cast<hipStream_t>(stream);
        if (stream) {  // the caller orders frames on its own stream: one slot
            e->npipe = 1;
            e->cur = e->ring = 0;
        }
    });
}

#ifndef GDF_BUILD_INFO
#define GDF_BUILD_INFO "source_sha=unknown"
#endif
const char* gdf_build_info(void) { return GDF_BUILD_INFO; }

int gdf_get_slot(gdf_engine* e, int* slot) {
    ENGINE_OR_FAIL(e);
    if (!slot) return GDF_ERR_ARG;
    *slot = e->cur;
    return GDF_OK;
}

int gdf_select_slot(gdf_engine* e, int slot) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] {
        if (slot < 0 || slot >= e->npipe) fail(GDF_ERR_ARG, "select_slot: no such pipeline slot");
        e->cur = slot;
        e->serialized = false;
    });
}

int gdf_set_slot_streams(gdf_engine* e, void* const* streams, int n) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] {
        if (n < 0 || n > kMaxPipe || (n && !streams)) fail(GDF_ERR_ARG, "set_slot_streams: 0..4 streams");
        if (e->user_stream) fail(GDF_ERR_STATE, "set_slot_streams: the engine runs on one caller stream");
        sync_all(e);
        for (int i = 0; i < kMaxPipe; ++i) {
            create_slot(e->slots[i]);
            e->slots[i].ext = i < n ? static_cast<hipStream_t>(streams[i]) : nullptr;
        }
    });
}

int gdf_synchronize(gdf_engine* e) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] {
        sync_all(e);
        e->sync();
    });
}

int gdf_set_pipeline_depth(gdf_engine* e, int depth) {
    ENGINE_OR_FAIL(e);
    if (depth < 1 || depth > kMaxPipe) {
        g_last_error = "pipeline depth must be 1.." + std::to_string(kMaxPipe);
        return GDF_ERR_ARG;
    }
    return guarded(e, [&] {
        if (e->user_stream && depth > 1) fail(GDF_ERR_STATE, "pipelining needs the engine's own streams");
        if (depth == e->npipe) return;  // unchanged: no drain, the grid sequence continues
        sync_all(e);
        for (int i = 0; i < depth; ++i) create_slot(e->slots[i]);
        // a configuration call between frames: the next frame starts on slot 0 (a shallower
        // pipeline does not keep the results of the frame that was current)
        if (e->cur >= depth) e->cur = 0;
        e->ring = e->cur;
        if (e->grid_alloc) {  // restart the grid-update sequence (nothing in flight)
            HIPCHK(hipMemset(e->d_gridctl.p, 0, 64));
            e->grid_ticket = 0;
        }
        e->npipe = depth;
        e->serialized = false;
    });
}

int gdf_set_graphs(gdf_engine* e, int enable) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] {
        e->use_graphs = enable != 0;
        if (!e->use_graphs) {
            sync_all(e);
            for (Slot& sl : e->slots) sl.graph.reset();
        }
    });
}

int gdf_set_voxel_group_size(gdf_engine* e, int group_size) {
    ENGINE_OR_FAIL(e);
    if (group_size <= 0) {
        g_last_error = "voxel group size must be positive";
        return GDF_ERR_ARG;
    }
    e->voxel_group_size = group_size;
    return GDF_OK;
}

int gdf_clear(gdf_engine* e) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] { engine_clear(e); });
}

int gdf_add_depthmap(gdf_engine* e, const uint16_t* depth, uint32_t W, uint32_t H, float scale,
                     float fx, float fy, float cx, float cy, const float Tw[16], const float Tc[16]) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] { add_depthmap(e, depth, nullptr, W, H, scale, fx, fy, cx, cy, Tw, Tc); });
}

int gdf_add_depthmap_device(gdf_engine* e, const uint16_t* depth, uint32_t W, uint32_t H,
                            float scale, float fx, float fy, float cx, float cy, const float Tw[16],
                            const float Tc[16]) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] { add_depthmap(e, nullptr, depth, W, H, scale, fx, fy, cx, cy, Tw, Tc); });
}

int gdf_add_halo_depthmap_device(gdf_engine* e, const uint16_t* tail, uint32_t tail_pixels,
                                 uint32_t W, uint32_t H, float scale, float fx, float fy, float cx,
                                 float cy, const float Tw[16], const float Tc[16]) {
    ENGINE_OR_FAIL(e);
    return guarded(nullptr, [&] {
        if (!tail || !Tw || !Tc || W == 0 || H == 0 || tail_pixels == 0 ||
            (uint64_t)tail_pixels > (uint64_t)W * H)
            fail(GDF_ERR_ARG, "halo depth map: bad argument");
        const uint32_t fr = e->nframes - 1;  // the current frame of a batch
        if (!e->halo_cams.empty() && e->halo_cams.back().frame == fr)
            fail(GDF_ERR_STATE, "one halo camera per frame");
        if (!e->cams.empty() && e->cams.back().frame == fr)
            fail(GDF_ERR_STATE, "the halo camera comes before the frame's depth maps");
        Cam c;
        c.frame = fr;
        c.dev = tail;
        c.W = W; c.H = H; c.n = W * H;
        c.scale = scale; c.fx = fx; c.fy = fy; c.cx = cx; c.cy = cy;
        std::memcpy(c.Tw, Tw, 64);
        std::memcpy(c.Tc, Tc, 64);
        e->halo_cams.push_back(c);
        e->halo_tail.push_back(tail_pixels);
        e->depth_uploaded = false;
    });
}

int gdf_add_point_sequence(gdf_engine* e, const void* rec, uint32_t n, uint32_t step,
                           uint32_t sec, uint32_t nsec, const float Tm[16]) {
    ENGINE_OR_FAIL(e);
    return guarded(nullptr, [&] { add_point_sequence(e, rec, n, step, sec, nsec, Tm); });
}

int gdf_add_point_sequence_device(gdf_engine* e, const void* rec, uint32_t n, uint32_t step,
                                  uint32_t sec, uint32_t nsec, const float Tm[16]) {
    ENGINE_OR_FAIL(e);
    return guarded(nullptr, [&] { add_point_sequence_device(e, rec, n, step, sec, nsec, Tm); });
}

int gdf_num_collected_point_sequence_points(gdf_engine* e, uint32_t* out) {
    ENGINE_OR_FAIL(e);
    if (!out) return GDF_ERR_ARG;
    std::lock_guard<std::mutex> lk(e->ps_mutex);
    *out = e->collect->total;
    return GDF_OK;
}

int gdf_upload_point_sequences(gdf_engine* e) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] { upload_point_sequences(e); });
}

int gdf_filter_new_point_sequences(gdf_engine* e, float threshold, uint32_t filter_size) {
    ENGINE_OR_FAIL(e);
    e->ps_filter_set = true;
    e->ps_thr = threshold;
    e->ps_F = filter_size;
    return GDF_OK;
}

int gdf_insert_new_point_sequences(gdf_engine* e) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] { insert_new_point_sequences(e); });
}

int gdf_roll_rollbuffer(gdf_engine* e, uint32_t min_sec, uint32_t min_nsec) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] { roll_rollbuffer(e, min_sec, min_nsec); });
}

int gdf_select_timespan(gdf_engine* e, uint32_t mins, uint32_t minn, uint32_t maxs, uint32_t maxn) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] { select_timespan(e, mins, minn, maxs, maxn); });
}

int gdf_prepare_point_and_mask_buffers(gdf_engine* e) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] { prepare_buffers(e); });
}

int gdf_insert_selected_point_sequence(gdf_engine* e, const float Twm[16], const float Tcm[16]) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] { insert_selected(e, Twm, Tcm); });
}

int gdf_transform_point_sequence(gdf_engine* e) {
    ENGINE_OR_FAIL(e);
    if (!e->sel_inserted && e->rb.selection_point_count) {
        g_last_error = "transformPointSequence before insertSelectedPointSequence";
        return GDF_ERR_STATE;
    }
    return GDF_OK;  // fused into the compaction launch
}

int gdf_get_rollbuffer_state(gdf_engine* e, gdf_rollbuffer_state* out) {
    ENGINE_OR_FAIL(e);
    if (!out) return GDF_ERR_ARG;
    *out = e->rb;
    return GDF_OK;
}

int gdf_set_rollbuffer_shard(gdf_engine* e, uint32_t shard, uint32_t nshards, uint32_t block) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] {
        if (nshards == 0 || nshards > 16 || shard >= nshards || block == 0)
            fail(GDF_ERR_ARG, "rollbuffer shard: 0 <= shard < nshards <= 16, block >= 1");
        if (e->rb.num_seqs != 0 || !e->hdrB.empty())
            fail(GDF_ERR_STATE, "rollbuffer shard: set before the first point sequence is inserted");
        e->shard = shard;
        e->nshards = nshards;
        e->shard_block = block;
        e->seq_counter = 0;
    });
}

int gdf_get_rollbuffer_pieces(gdf_engine* e, uint32_t* owners, uint32_t capacity, uint32_t* count) {
    ENGINE_OR_FAIL(e);
    if (!count || (capacity && !owners)) return GDF_ERR_ARG;
    return guarded(e, [&] {
        const uint32_t ss = e->rb.selection_sequence_start, sc = e->rb.selection_sequence_count;
        if (sc && (uint64_t)ss + sc > e->hdrB.size()) fail(GDF_ERR_STATE, "selection exceeds rollbuffer sequences");
        uint32_t n = 0;
        int64_t cur = -1;
        for (uint32_t j = ss; j < ss + sc; ++j) {
            const Hdr& h = e->hdrB[j];
            if (!h.num_global) continue;  // (no points on any shard)
            const int64_t k = (int64_t)((h.id / e->shard_block) % e->nshards);
            if (k == cur) continue;
            if (n < capacity) owners[n] = (uint32_t)k;
            ++n;
            cur = k;
        }
        *count = n;
        if (n > capacity) fail(GDF_ERR_CAPACITY, "rollbuffer pieces: more pieces than capacity");
    });
}

int gdf_upload_depthmaps(gdf_engine* e) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] { upload_depthmaps(e); });
}

int gdf_convert_depthmaps(gdf_engine* e) {
    ENGINE_OR_FAIL(e);
    if (!e->depth_uploaded) {
        g_last_error = "convertDepthmaps before uploadDepthmaps";
        return GDF_ERR_STATE;
    }
    e->converted = true;
    return GDF_OK;
}

int gdf_filter_flying_pixels(gdf_engine* e, uint32_t filter_size, float threshold, int rot45) {
    ENGINE_OR_FAIL(e);
    e->flying_set = true;
    e->F = filter_size;
    e->thr = threshold;
    e->rot45 = rot45 ? 1 : 0;
    return GDF_OK;
}

int gdf_crop_points(gdf_engine* e, const float lower[3], const float upper[3]) {
    ENGINE_OR_FAIL(e);
    if (!lower || !upper) return GDF_ERR_ARG;
    e->crop_set = true;
    std::memcpy(e->lo, lower, 12);
    std::memcpy(e->hi, upper, 12);
    return GDF_OK;
}

int gdf_apply_point_mask(gdf_engine* e, uint32_t* out_count) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] {
        run_frame(e, false);
        if (out_count) {
            e->read_misc();
            *out_count = e->sl().h_misc[kCount];
        }
    });
}

int gdf_compute_voxel_coords(gdf_engine* e, const float lo[3], const float hi[3], const float cs[3]) {
    ENGINE_OR_FAIL(e);
    if (!lo || !hi || !cs) return GDF_ERR_ARG;
    return guarded(e, [&] { compute_voxel_coords(e, lo, hi, cs); });
}

int gdf_voxelize(gdf_engine* e, int average) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] { voxelize(e, average); });
}

int gdf_voxel_occupancy_grid(gdf_engine* e, uint32_t lifetime) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] { occupancy_grid(e, lifetime, e->s()); });
}

int gdf_get_point_count(gdf_engine* e, uint32_t* out) {
    ENGINE_OR_FAIL(e);
    if (!out) return GDF_ERR_ARG;
    return guarded(e, [&] {
        if (!e->sl().compacted) fail(GDF_ERR_STATE, "no compaction has run");
        e->read_misc();
        *out = e->sl().h_misc[kCount];
    });
}

int gdf_download_points(gdf_engine* e, float* out, uint32_t cap, uint32_t* out_count) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] {
        if (!e->sl().compacted) fail(GDF_ERR_STATE, "downloadPoints before applyPointMask");
        e->read_misc();
        const uint32_t n = e->sl().h_misc[kCount];
        if (out_count) *out_count = n;
        if (out) {
            if (cap < n) fail(GDF_ERR_CAPACITY, "downloadPoints: buffer too small");
            if (n) HIPCHK(hipMemcpy(out, e->sl().d_pts.p, (size_t)n * 16, hipMemcpyDeviceToHost));
        }
    });
}

int gdf_download_voxel_coords(gdf_engine* e, uint32_t* out, uint32_t cap, uint32_t* out_count) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] {
        if (!e->sl().coords_valid) fail(GDF_ERR_STATE, "downloadVoxelCoords before computeVoxelCoords");
        e->read_misc();
        const uint32_t n = e->sl().h_misc[kCount];
        if (out_count) *out_count = n;
        if (out) {
            if (cap < n) fail(GDF_ERR_CAPACITY, "downloadVoxelCoords: buffer too small");
            if (n) HIPCHK(hipMemcpy(out, e->sl().d_coords.p, (size_t)n * 4, hipMemcpyDeviceToHost));
        }
    });
}

int gdf_download_voxelized_points(gdf_engine* e, float* out, uint32_t cap, uint32_t* out_count) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] {
        if (!e->sl().vox_valid) fail(GDF_ERR_STATE, "no voxelize has run");
        e->read_misc();
        const uint32_t n = e->sl().h_misc[kVoxCount];
        if (out_count) *out_count = n;
        if (out) {
            if (cap < n) fail(GDF_ERR_CAPACITY, "voxelized points: buffer too small");
            if (n) HIPCHK(hipMemcpy(out, e->sl().d_vox.p, (size_t)n * 16, hipMemcpyDeviceToHost));
        }
    });
}

int gdf_download_occupancy_grid(gdf_engine* e, uint8_t* out, uint64_t cap) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] {
        if (!e->grid_set || !e->invoked_once) fail(GDF_ERR_STATE, "no voxelOccupancyGrid has run");
        if (!out || cap < e->ncells) fail(GDF_ERR_CAPACITY, "occupancy grid: buffer too small");
        sync_all(e);  // grid updates may still run on another slot's stream
        e->sync();
        HIPCHK(hipMemcpy(out, grid_out_ptr(e), e->ncells, hipMemcpyDeviceToHost));
    });
}

int gdf_download_frame(gdf_engine* e, uint32_t what, gdf_host_frame* out) {
    ENGINE_OR_FAIL(e);
    if (!out) return GDF_ERR_ARG;
    return guarded(e, [&] {
        Slot& q = e->sl();
        *out = gdf_host_frame{};
        if ((what & (GDF_DL_POINTS | GDF_DL_COORDS)) && !q.compacted)
            fail(GDF_ERR_STATE, "download_frame: no compaction has run");
        if ((what & GDF_DL_COORDS) && !q.coords_valid) fail(GDF_ERR_STATE, "download_frame: no voxel coords");
        if ((what & GDF_DL_VOXELIZED) && !q.vox_valid) fail(GDF_ERR_STATE, "download_frame: no voxelize has run");
        if ((what & GDF_DL_GRID) && (!e->grid_set || !e->invoked_once))
            fail(GDF_ERR_STATE, "download_frame: no voxelOccupancyGrid has run");
        if (what & GDF_DL_GRID) sync_all(e);  // grid updates may still run on another slot's stream
        if (q.pf_valid) {  // k_download wrote everything: the one wait (and the aux stream's)
            e->sync();
            if (q.dl_aux) HIPCHK(hipStreamSynchronize(q.dl_aux));
            q.pf_valid = false;
            Slot::Mirrors& M = q.mir[q.mir_pf];
            q.mir_out = q.mir_pf;  // (handed out: the next prefetch writes the other set)
            const uint32_t* hm = static_cast<const uint32_t*>(M.misc.p);
            if (hm[kErr]) {
                HIPCHK(hipMemsetAsync(q.d_misc.as<uint32_t>() + kErr, 0, 4, e->s()));
                fail(GDF_ERR_DEVICE, "device error flags (code " + std::to_string(hm[kErr]) + ")");
            }
            std::memcpy(q.h_misc, hm, kMiscWords * 4);
            const uint32_t n = hm[kCount], nv = hm[kVoxCount];
            if (what & GDF_DL_POINTS) {
                out->points = static_cast<const float*>(M.pts.p);
                out->num_points = n;
            }
            if (what & GDF_DL_COORDS) {
                out->voxel_coords = static_cast<const uint32_t*>(M.coords.p);
                out->num_points = n;
            }
            if (what & GDF_DL_VOXELIZED) {
                out->voxelized = static_cast<const float*>(M.vox.p);
                out->num_voxelized = nv;
            }
            if (what & GDF_DL_GRID) {
                const uint32_t latest = e->grid_ticket - 1u;
                const uint32_t nd = hm[kDeltaCount];
                const uint32_t dcap = (uint32_t)((mark_words(e) + 3) / 4 * 4);
                const bool apply = q.delta_valid && q.delta_ticket == latest && e->mirror_valid &&
                                   e->mirror_gen == e->grid_gen && e->mirror_ticket + 1u == latest &&
                                   e->grid_mode == 0 && nd <= dcap;
                const size_t padded = (size_t)mark_words(e) * 32;
                if (!e->h_mirror.ensure(padded)) fail(GDF_ERR_NOMEM, "pinned grid mirror allocation failed");
                uint8_t* mir = static_cast<uint8_t*>(e->h_mirror.p);
                if (apply) {
                    const uint8_t* hd = static_cast<const uint8_t*>(M.delta.p);
                    const uint32_t* idx = reinterpret_cast<const uint32_t*>(hd);
                    const uint8_t* data = hd + (size_t)dcap * 4;
                    for (uint32_t k = 0; k < nd; ++k)
                        std::memcpy(mir + (size_t)idx[k] * 32, data + (size_t)k * 32, 32);
                } else {
                    HIPCHK(hipMemcpyAsync(mir, grid_out_ptr(e), e->ncells, hipMemcpyDeviceToHost, e->s()));
                    e->sync();
                }
                e->mirror_valid = true;
                e->mirror_ticket = latest;
                e->mirror_gen = e->grid_gen;
                out->occupancy = mir;
                out->num_cells = e->ncells;
                if (e->grid_delta_allowed) e->grid_delta = true;
            }
            return;
        }
        e->read_misc();  // the counts (one wait)
        const uint32_t n = q.h_misc[kCount], nv = q.h_misc[kVoxCount];
        Slot::Mirrors& M = q.mir[q.mir_next()];  // (not the set the caller still holds)
        q.mir_out = q.mir_next();
        auto copy = [&](Slot::Pinned& m, const void* src, size_t bytes) -> void* {
            void* dst = m.ensure(std::max<size_t>(bytes, 64));
            if (!dst) fail(GDF_ERR_NOMEM, "pinned host mirror allocation failed");
            if (bytes) HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, e->s()));
            return dst;
        };
        if (what & GDF_DL_POINTS) {
            out->points = static_cast<const float*>(copy(M.pts, q.d_pts.p, (size_t)n * 16));
            out->num_points = n;
        }
        if (what & GDF_DL_COORDS) {
            out->voxel_coords = static_cast<const uint32_t*>(copy(M.coords, q.d_coords.p, (size_t)n * 4));
            out->num_points = n;
        }
        if (what & GDF_DL_VOXELIZED) {
            out->voxelized = static_cast<const float*>(copy(M.vox, q.d_vox.p, (size_t)nv * 16));
            out->num_voxelized = nv;
        }
        // the grid: into the engine's host mirror - only the groups the last update changed when
        // the mirror holds the grid right before it (a frame-by-frame component), else all of it
        bool apply_delta = false;
        uint32_t nd = 0;
        if (what & GDF_DL_GRID) {
            const uint32_t latest = e->grid_ticket - 1u;
            nd = q.h_misc[kDeltaCount];
            apply_delta = q.delta_valid && q.delta_ticket == latest && e->mirror_valid &&
                          e->mirror_gen == e->grid_gen && e->mirror_ticket + 1u == latest &&
                          e->grid_mode == 0;
            const size_t padded = (size_t)mark_words(e) * 32;
            if (!e->h_mirror.ensure(padded)) fail(GDF_ERR_NOMEM, "pinned grid mirror allocation failed");
            if (apply_delta) {
                uint8_t* st = static_cast<uint8_t*>(M.delta.ensure((size_t)std::max<uint32_t>(nd, 1) * 36));
                if (!st) fail(GDF_ERR_NOMEM, "pinned delta staging allocation failed");
                if (nd) {
                    HIPCHK(hipMemcpyAsync(st, q.d_didx.p, (size_t)nd * 4, hipMemcpyDeviceToHost, e->s()));
                    HIPCHK(hipMemcpyAsync(st + (size_t)nd * 4, q.d_ddata.p, (size_t)nd * 32,
                                          hipMemcpyDeviceToHost, e->s()));
                }
            } else {
                HIPCHK(hipMemcpyAsync(e->h_mirror.p, grid_out_ptr(e), e->ncells, hipMemcpyDeviceToHost,
                                      e->s()));
            }
            e->mirror_valid = true;
            e->mirror_ticket = latest;
            e->mirror_gen = e->grid_gen;
            out->occupancy = static_cast<const uint8_t*>(e->h_mirror.p);
            out->num_cells = e->ncells;
        }
        e->sync();  // every copy (the second wait)
        if (apply_delta && nd) {  // the changed groups into the mirror (32 bytes each)
            const uint8_t* st = static_cast<const uint8_t*>(M.delta.p);
            const uint32_t* idx = reinterpret_cast<const uint32_t*>(st);
            const uint8_t* data = st + (size_t)nd * 4;
            uint8_t* mir = static_cast<uint8_t*>(e->h_mirror.p);
            for (uint32_t k = 0; k < nd; ++k) std::memcpy(mir + (size_t)idx[k] * 32, data + (size_t)k * 32, 32);
        }
        if ((what & GDF_DL_GRID) && e->grid_delta_allowed) e->grid_delta = true;  // from now on
        // single frames: from now on the launch chain ends with k_download (prefetch)
        if ((what & (GDF_DL_POINTS | GDF_DL_COORDS | GDF_DL_VOXELIZED)) && q.nframes == 1 &&
            e->dl_prefetch_allowed)
            e->dl_prefetch = true;
    });
}

int gdf_get_grid_size(gdf_engine* e, uint32_t g[3], uint64_t* ncells) {
    ENGINE_OR_FAIL(e);
    if (!e->grid_set) {
        g_last_error = "no voxel grid set";
        return GDF_ERR_STATE;
    }
    if (g) std::memcpy(g, e->gs, 12);
    if (ncells) *ncells = e->ncells;
    return GDF_OK;
}

int gdf_get_device_results(gdf_engine* e, const float** pts, const uint32_t** coords,
                           const float** vox, const uint8_t** occ) {
    ENGINE_OR_FAIL(e);
    if (pts) *pts = e->sl().d_pts.as<const float>();
    if (coords) *coords = e->sl().d_coords.as<const uint32_t>();
    if (vox) *vox = e->sl().d_vox.as<const float>();
    if (occ) *occ = e->grid_set ? grid_out_ptr(e) : nullptr;
    return GDF_OK;
}

int gdf_process_frame(gdf_engine* e, const gdf_frame_params* p, gdf_frame_result* r) {
    ENGINE_OR_FAIL(e);
    if (!p) return GDF_ERR_ARG;
    // gdf_set_emit_partition arms ONE frame: disarmed on every exit, failures included (a later
    // frame must never write send lists into the caller's stale buffers)
    struct Disarm {
        gdf_engine* e;
        ~Disarm() { e->epart = gdf_engine::EmitPart{}; }
    } disarm{e};
    return guarded(e, [&] {
        gdf_frame_result res{};
        uint32_t collected;
        {
            std::lock_guard<std::mutex> lk(e->ps_mutex);
            collected = e->collect->total;
        }
        // component.cpp:150: if ((numAdded>0) || (numCollectedPointSequencePoints()>0))
        if (!(e->cams.size() > 0 || collected > 0)) {
            if (r) *r = res;
            return;
        }
        if (e->nframes > 1) {  // a multi-frame batch: depth-only frames through one launch chain
            if (collected > 0 || e->rb.num_points > 0)
                fail(GDF_ERR_STATE, "frame batches carry depth maps only (no point sequences)");
            if (e->cams.empty() || e->cams.back().frame != e->nframes - 1)
                fail(GDF_ERR_STATE, "every frame of a batch needs a depth map");
            if (p->enable_voxel_filter && !p->defer_voxelize &&
                (p->defer_occupancy_grid || p->occupancy_lifetime > 255))
                fail(GDF_ERR_STATE, "frame batches need the fused grid update (lifetime <= 255, "
                                    "not deferred)");
            if (p->enable_voxel_filter && p->defer_voxelize && !p->defer_occupancy_grid)
                fail(GDF_ERR_STATE, "a batch with deferred voxelize defers its grid update too "
                                    "(gdf_take_occupancy_marks + gdf_voxel_occupancy_grid_batch)");
            if (e->nframes > kMaxCams) fail(GDF_ERR_ARG, "at most 16 frames per batch");
        }
        res.processed = 1;
        upload_point_sequences(e);
        e->ps_filter_set = true;
        e->ps_thr = p->ps_filter_threshold;
        e->ps_F = p->ps_filter_size;
        insert_new_point_sequences(e);
        uint32_t lts = 0, ltn = 0, ets = 0, etn = 0;
        if (e->rb.last_time_sec != 0 || e->rb.last_time_nsec != 0) {
            lts = e->rb.last_time_sec;
            ltn = e->rb.last_time_nsec;
            if (!ros_time_minus(lts, ltn, (double)p->ps_timespan, &ets, &etn))
                fail(GDF_ERR_TIME, "latest time - timespan is out of ROS time range");
        }
        roll_rollbuffer(e, ets, etn);
        if (p->move_transform_available) {
            select_timespan(e, ets, etn, lts, ltn);
            prepare_buffers(e);
            insert_selected(e, p->T_world_move, p->T_crop_move);
        } else {
            prepare_buffers(e);
        }
        res.latest_time_sec = lts;
        res.latest_time_nsec = ltn;
        upload_depthmaps(e);
        e->converted = true;
        e->flying_set = true;
        e->F = p->flying_filter_size;
        e->thr = p->flying_threshold;
        e->rot45 = p->flying_rot45 ? 1 : 0;
        e->crop_set = true;
        std::memcpy(e->lo, p->crop_min, 12);
        std::memcpy(e->hi, p->crop_max, 12);
        if (p->enable_voxel_filter) {
            set_grid(e, p->voxel_min, p->voxel_max, p->voxel_size);
            if (sort_bits(e) > 32) fail(GDF_ERR_ARG, "voxel key + frame index exceed 32 bits");
            widen_if_needed(e, p->occupancy_lifetime, e->s());  // before marks are consumed
            if (p->defer_voxelize) {  // keys + marks only (multi-GPU fused cloud)
                const gdf_engine::EmitPart ep = e->epart;
                if (ep.nparts && ep.cap < e->sl().n_total)
                    fail(GDF_ERR_CAPACITY, "emit partition: send lists smaller than the frame");
                run_frame(e, true, true);
                e->epart = gdf_engine::EmitPart{};  // (one frame)
                if (ep.nparts && !e->sl().part_emitted)  // the compaction could not: a pass
                    partition_runs(e, ep.nparts, ep.pts, ep.run_keys, ep.run_starts, ep.cap, ep.counts,
                                   ep.nseg);
                if (!p->defer_occupancy_grid) occupancy_grid(e, p->occupancy_lifetime, e->s());
            } else if (!p->defer_occupancy_grid && e->grid_mode == 0) {
                run_fused_frame(e, p->voxel_average, p->occupancy_lifetime);
            } else {
                run_frame(e, true);
                voxelize(e, p->voxel_average);
                if (!p->defer_occupancy_grid) occupancy_grid(e, p->occupancy_lifetime, e->s());
            }
        } else {
            run_frame(e, false);
        }
        res.num_depth_points = e->depth_total;
        res.num_points_total = e->sl().n_total;
        if (p->synchronous) {
            e->read_misc();
            res.num_points = e->sl().h_misc[kCount];
            res.num_voxelized = p->enable_voxel_filter && !p->defer_voxelize ? e->sl().h_misc[kVoxCount] : 0;
            // what the voxelize sorted: runs of equal keys, or points
            const bool runs = e->sl().runs_valid && p->enable_voxel_filter && !p->defer_voxelize;
            e->last_sort_runs = runs;
            e->last_sort_items = runs ? e->sl().h_misc[e->sl().runs_sel ? kRunTotal : kRunCount]
                                      : res.num_points;
        }
        if (r) *r = res;
    });
}

int gdf_last_sort_items(gdf_engine* e, uint32_t* items, int* runs) {
    ENGINE_OR_FAIL(e);
    if (items) *items = e->last_sort_items;
    if (runs) *runs = e->last_sort_runs ? 1 : 0;
    return GDF_OK;
}

int gdf_mask_dilate(gdf_engine* e, const uint32_t* in, uint32_t* out, uint32_t W, uint32_t H,
                    uint32_t F, int as_written) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] {
        if ((!in || !out) && (uint64_t)W * H) fail(GDF_ERR_ARG, "mask_dilate: null mask");
        if (in == out && (uint64_t)W * H) fail(GDF_ERR_ARG, "mask_dilate: in-place is not supported");
        if (F > kDilateMaxF) fail(GDF_ERR_ARG, "mask_dilate: filter size above 16");
        HIPCHK(launch_mask_dilate(in, out, W, H, F, as_written, e->s()));
    });
}

int gdf_transform_points(gdf_engine* e, const float* in, const uint32_t* mask, float* out,
                         uint32_t n, const float T[16]) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] {
        if (!T || (n && (!in || !mask || !out))) fail(GDF_ERR_ARG, "transform_points: null argument");
        HIPCHK(launch_transform_points(reinterpret_cast<const float4*>(in), mask,
                                       reinterpret_cast<float4*>(out), n, T, e->s()));
    });
}

int gdf_partition_points(gdf_engine* e, uint32_t nparts, float* send_pts, uint32_t* send_keys,
                         uint32_t capacity, uint32_t* part_counts) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] {
        Slot& q = e->sl();
        if (!e->grid_set || !q.coords_valid) fail(GDF_ERR_STATE, "partition needs the voxel keys of a frame");
        if (nparts == 0 || nparts > kMaxParts) fail(GDF_ERR_ARG, "partition: 1..16 parts");
        if (!send_pts || !send_keys || !part_counts) fail(GDF_ERR_ARG, "partition: null buffer");
        if (capacity < q.n_total) fail(GDF_ERR_CAPACITY, "partition: send buffers smaller than the frame");
        ensure_misc(e);
        const uint32_t nmax = std::max<uint32_t>(q.n_total, 1);
        const uint32_t m = nparts * std::max<uint32_t>(part_tiles(nmax), 1u);
        q.d_pcnt.ensure((size_t)m * 4);
        q.d_poff.ensure(seg_offsets_words(m) * 4);
        HIPCHK(launch_partition(q.d_pts.as<float4>(), q.d_coords.as<uint32_t>(),
                                q.d_misc.as<uint32_t>() + kCount, nmax, nparts, e->ncells,
                                q.d_pcnt.as<uint32_t>(), q.d_poff.as<uint32_t>(),
                                q.d_misc.as<uint32_t>() + kPartTotal,
                                reinterpret_cast<float4*>(send_pts), send_keys, part_counts, e->s(),
                                q.nframes > 1 ? q.d_fstart.as<uint32_t>() : nullptr, q.nframes,
                                q.nframes > 1 ? e->key_bits : 0u));
    });
}

int gdf_set_emit_partition(gdf_engine* e, uint32_t nparts, float* send_pts, uint32_t* send_run_keys,
                           uint32_t* send_run_starts, uint32_t capacity, uint32_t* part_counts) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] {
        if (nparts > kMaxParts) fail(GDF_ERR_ARG, "emit partition: 0..16 parts");
        if (nparts && (!send_pts || !send_run_keys || !send_run_starts || !part_counts))
            fail(GDF_ERR_ARG, "emit partition: null buffer");
        e->epart.nparts = nparts;
        e->epart.cap = capacity;
        e->epart.pts = send_pts;
        e->epart.run_keys = send_run_keys;
        e->epart.run_starts = send_run_starts;
        e->epart.counts = part_counts;
    });
}

int gdf_set_partition_segments(gdf_engine* e, uint32_t nseg) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] {
        if (nseg == 0 || nseg > kMaxSegs) fail(GDF_ERR_ARG, "partition segments: 1..4");
        e->epart.nseg = nseg;
    });
}

int gdf_set_partition_marks(gdf_engine* e, int enabled) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] { e->part_marks = enabled != 0; });
}

int gdf_partition_runs(gdf_engine* e, uint32_t nparts, float* send_pts, uint32_t* send_run_keys,
                       uint32_t* send_run_starts, uint32_t capacity, uint32_t* part_counts) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] {
        partition_runs(e, nparts, send_pts, send_run_keys, send_run_starts, capacity, part_counts);
    });
}


int gdf_voxelize_runs(gdf_engine* e, const float* pts, const uint32_t* run_keys,
                      uint32_t* run_starts, uint32_t nsources, const uint32_t* point_base,
                      const uint32_t* run_base, int average) {
    return gdf_voxelize_runs_marked(e, pts, run_keys, run_starts, nsources, point_base, run_base,
                                    average, nullptr, 0);
}

namespace {
void voxelize_runs(gdf_engine* e, const float* pts, const uint32_t* run_keys, uint32_t* run_starts,
                   uint32_t nsources, const uint32_t* point_base, const uint32_t* run_base,
                   int average, uint32_t* marks, uint64_t frame_stride_words, const gdf_recv_own* own) {
    if (marks && (frame_stride_words < mark_words(e) || (e->nframes > 1 && frame_stride_words == 0)))
        fail(GDF_ERR_CAPACITY, "voxelize_runs: a frame's marks need >= the grid's mark words");
    if (!e->grid_set) fail(GDF_ERR_STATE, "voxelize_runs needs the voxel grid of a frame");
    if (nsources == 0 || nsources > kMaxSources || !point_base || !run_base)
        fail(GDF_ERR_ARG, "voxelize_runs: 1..32 sources and their bases");
    RebaseArgs rb;
    std::memset(&rb, 0, sizeof(rb));
    rb.nsrc = nsources;
    for (uint32_t k = 0; k <= nsources; ++k) {
        rb.point_base[k] = point_base[k];
        rb.run_base[k] = run_base[k];
        if (k && (point_base[k] < point_base[k - 1] || run_base[k] < run_base[k - 1]))
            fail(GDF_ERR_ARG, "voxelize_runs: bases must not decrease");
        if (k && (run_base[k] > run_base[k - 1]) != (point_base[k] > point_base[k - 1]))
            fail(GDF_ERR_ARG, "voxelize_runs: a source has points without runs or runs without points");
    }
    const uint32_t n = point_base[nsources], R = run_base[nsources];
    if (R && (!pts || !run_keys || !run_starts)) fail(GDF_ERR_ARG, "voxelize_runs: null list");
    if (!run_starts) fail(GDF_ERR_ARG, "voxelize_runs: run_starts needs R + 1 entries");
    if (own) {
        if (own->count > kMaxOwnSources) fail(GDF_ERR_ARG, "voxelize_runs: at most 4 own sources");
        rb.n_own = own->count;
        for (uint32_t k = 0; k < own->count; ++k) {
            if (own->source[k] >= nsources) fail(GDF_ERR_ARG, "voxelize_runs: own source out of range");
            for (uint32_t j = 0; j < k; ++j)
                if (own->source[j] == own->source[k]) fail(GDF_ERR_ARG, "voxelize_runs: own source twice");
            const uint32_t q = own->source[k];
            if (point_base[q + 1] > point_base[q] && (!own->points[k] || !own->run_keys[k] || !own->run_starts[k]))
                fail(GDF_ERR_ARG, "voxelize_runs: null own list");
            rb.own_src[k] = q;
            rb.own_pts[k] = reinterpret_cast<const float4*>(own->points[k]);
            rb.own_run_keys[k] = own->run_keys[k];
            rb.own_run_starts[k] = own->run_starts[k];
        }
        rb.pts = reinterpret_cast<float4*>(const_cast<float*>(pts));
        rb.run_keys = const_cast<uint32_t*>(run_keys);
        if (own->clear && own->clear_rows && own->clear_row_words) {
            if (own->clear_rows > 1 && own->clear_stride_words < own->clear_row_words)
                fail(GDF_ERR_ARG, "voxelize_runs: clear rows overlap");
            rb.zero = own->clear;
            rb.zero_row_words = own->clear_row_words;
            rb.zero_stride = own->clear_stride_words;
            rb.zero_rows = own->clear_rows;
        }
    }
    ensure_misc(e);
    if (e->sl().khist_pending) {  // the frame's compaction counted ITS keys' digits: not these
        HIPCHK(hipMemsetAsync(e->sl().d_khist.p, 0, kHistWords * 4, e->s()));
        e->sl().khist_pending = false;
    }
    e->sl().pf_valid = false;
    uint32_t* misc = e->sl().d_misc.as<uint32_t>();
    HIPCHK(launch_run_rebase(run_starts, rb, misc + kRecvCount, misc + kRecvRuns, e->s()));
    VoxSource src;
    src.pts = reinterpret_cast<const float4*>(pts);
    src.keys = run_keys;
    src.n = n;
    src.run_keys = run_keys;
    src.run_start = run_starts;
    VoxelizeArgs v = voxelize_args(e, average, -1, &src);
    if (marks) {  // every voxel's mark, frame f at f * stride (k_group_runs)
        v.group_marks = marks;
        v.group_mark_stride = frame_stride_words;
    }
    e->timed(GDF_KERNEL_VOXELIZE, [&] { HIPCHK(launch_voxelize(v, e->s(), e->hook_ptr())); });
    e->sl().vox_valid = true;
}
}  // namespace

int gdf_voxelize_runs_marked(gdf_engine* e, const float* pts, const uint32_t* run_keys,
                             uint32_t* run_starts, uint32_t nsources, const uint32_t* point_base,
                             const uint32_t* run_base, int average, uint32_t* marks,
                             uint64_t frame_stride_words) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] {
        voxelize_runs(e, pts, run_keys, run_starts, nsources, point_base, run_base, average, marks,
                      frame_stride_words, nullptr);
    });
}

int gdf_voxelize_runs_recv(gdf_engine* e, float* pts, uint32_t* run_keys, uint32_t* run_starts,
                           uint32_t nsources, const uint32_t* point_base, const uint32_t* run_base,
                           int average, uint32_t* marks, uint64_t frame_stride_words,
                           const gdf_recv_own* own) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] {
        voxelize_runs(e, pts, run_keys, run_starts, nsources, point_base, run_base, average, marks,
                      frame_stride_words, own);
    });
}

int gdf_voxelize_points(gdf_engine* e, const float* pts, const uint32_t* keys, uint32_t n,
                        int average) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] {
        if (!e->grid_set) fail(GDF_ERR_STATE, "voxelize_points needs the voxel grid of a frame");
        if (n && (!pts || !keys)) fail(GDF_ERR_ARG, "voxelize_points: null list");
        ensure_misc(e);
        if (e->sl().khist_pending) {  // the frame's compaction counted ITS keys' digits: not these
            HIPCHK(hipMemsetAsync(e->sl().d_khist.p, 0, kHistWords * 4, e->s()));
            e->sl().khist_pending = false;
        }
        e->sl().pf_valid = false;
        HIPCHK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(e->sl().d_misc.as<uint32_t>() + kRecvCount),
                                 (int)n, 1, e->s()));
        VoxSource src;
        src.pts = reinterpret_cast<const float4*>(pts);
        src.keys = keys;
        src.n = n;
        if (e->xruns && n) {  // sort the list's runs of equal keys, not its points
            Slot& q = e->sl();
            const uint32_t tiles = std::max<uint32_t>(xrun_tiles(n), 1u);
            q.d_xcnt.ensure((size_t)tiles * 4);
            q.d_xoff.ensure(seg_offsets_words(tiles) * 4);
            q.d_xrk.ensure((size_t)n * 4);
            q.d_xrs.ensure(((size_t)n + 1) * 4);
            HIPCHK(launch_xruns(keys, q.d_misc.as<uint32_t>() + kRecvCount, n, q.d_xcnt.as<uint32_t>(),
                                q.d_xoff.as<uint32_t>(), q.d_xrk.as<uint32_t>(), q.d_xrs.as<uint32_t>(),
                                q.d_misc.as<uint32_t>() + kRecvRuns, e->s()));
            src.run_keys = q.d_xrk.as<uint32_t>();
            src.run_start = q.d_xrs.as<uint32_t>();
        }
        const VoxelizeArgs v = voxelize_args(e, average, -1, &src);
        e->timed(GDF_KERNEL_VOXELIZE, [&] { HIPCHK(launch_voxelize(v, e->s(), e->hook_ptr())); });
        e->sl().khist_pending = false;
        e->sl().vox_valid = true;
    });
}

int gdf_next_frame_in_batch(gdf_engine* e) {
    ENGINE_OR_FAIL(e);
    return guarded(nullptr, [&] {
        if (e->cams.empty() || e->cams.back().frame != e->nframes - 1)
            fail(GDF_ERR_STATE, "the current frame of the batch has no depth map");
        if (e->nframes >= (uint32_t)kMaxCams) fail(GDF_ERR_ARG, "at most 16 frames per batch");
        e->nframes++;
    });
}

int gdf_get_batch_ranges(gdf_engine* e, uint32_t* point_start, uint32_t* voxel_start,
                         uint32_t capacity, uint32_t* out_frames) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] {
        Slot& q = e->sl();
        if (!q.compacted) fail(GDF_ERR_STATE, "no frame has run");
        const uint32_t nf = q.nframes;
        if (out_frames) *out_frames = nf;
        if ((point_start || voxel_start) && capacity < nf + 1)
            fail(GDF_ERR_CAPACITY, "batch ranges: need nframes + 1 entries");
        e->read_misc();  // (synchronises the frame)
        if (nf == 1) {
            if (point_start) { point_start[0] = 0; point_start[1] = q.h_misc[kCount]; }
            if (voxel_start) { voxel_start[0] = 0; voxel_start[1] = q.vox_valid ? q.h_misc[kVoxCount] : 0; }
            return;
        }
        if (point_start)
            HIPCHK(hipMemcpy(point_start, q.d_fstart.p, (nf + 1) * 4, hipMemcpyDeviceToHost));
        if (voxel_start) {
            if (q.vox_valid)
                HIPCHK(hipMemcpy(voxel_start, q.d_fvox.p, (nf + 1) * 4, hipMemcpyDeviceToHost));
            else
                std::memset(voxel_start, 0, (nf + 1) * 4);
        }
    });
}

int gdf_download_batch_occupancy_grid(gdf_engine* e, uint32_t frame, uint8_t* out, uint64_t cap) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] {
        Slot& q = e->sl();
        if (!e->grid_set || !e->invoked_once) fail(GDF_ERR_STATE, "no voxelOccupancyGrid has run");
        if (frame >= q.nframes) fail(GDF_ERR_ARG, "frame outside the batch");
        if (!out || cap < e->ncells) fail(GDF_ERR_CAPACITY, "occupancy grid: buffer too small");
        sync_all(e);
        e->sync();
        const uint8_t* src = grid_out_ptr(e);
        if (frame + 1 < q.nframes) {  // the batch's grid update kept sparse snapshots
            if (!q.snap_valid || frame + 1 >= q.snap_frames)
                fail(GDF_ERR_STATE, "the batch's grid update kept no per-frame grids (u32 history, "
                                    "or a deferred grid update that has not run)");
            e->d_snap_dense.ensure((e->ncells + 31) / 32 * 32);
            const SnapArgs sn{q.d_snap_idx.as<uint32_t>(), q.d_snap_data.as<uint4>(),
                              q.d_snap_cnt.as<uint32_t>()};
            HIPCHK(launch_snap_expand(sn, frame, q.snap_blocks, e->ncells,
                                      e->d_snap_dense.as<uint8_t>(), e->s()));
            e->sync();
            src = e->d_snap_dense.as<uint8_t>();
        }
        HIPCHK(hipMemcpy(out, src, e->ncells, hipMemcpyDeviceToHost));
    });
}

int gdf_export_occupancy_marks(gdf_engine* e, uint32_t* bits, uint64_t words) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] {
        if (!e->grid_set || !bits) fail(GDF_ERR_STATE, "no voxel grid");
        if (words < (e->ncells + 31) / 32) fail(GDF_ERR_CAPACITY, "mark bitmask too small");
        HIPCHK(launch_export_marks(marks_ptr(e), mark_words(e), bits, e->s()));
    });
}

int gdf_import_occupancy_marks(gdf_engine* e, const uint32_t* bits, uint64_t words, uint32_t nranks) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] {
        if (!e->grid_set || !bits) fail(GDF_ERR_STATE, "no voxel grid");
        if (words < (e->ncells + 31) / 32) fail(GDF_ERR_CAPACITY, "mark bitmask too small");
        HIPCHK(launch_import_marks(marks_ptr(e), mark_words(e), bits, nranks, mark_words(e), e->s()));
        e->sl().marks_set = true;
    });
}

int gdf_take_occupancy_marks(gdf_engine* e, uint32_t* bits, uint64_t words) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] {
        if (!e->grid_set || !bits) fail(GDF_ERR_STATE, "no voxel grid");
        if (words < (e->ncells + 31) / 32) fail(GDF_ERR_CAPACITY, "mark bitmask too small");
        // a batch: every frame's marks (frame f at f * mark words); taking only some would leave
        // the others' bits set for the slot's next batch
        const uint64_t nf = e->sl().nframes;
        if (nf > 1 && words < nf * mark_words(e))
            fail(GDF_ERR_CAPACITY, "take marks of a batch: the buffer must hold every frame's "
                                   "marks (nframes * mark words)");
        HIPCHK(launch_take_marks(marks_ptr(e), mark_words(e) * nf, bits, e->s()));
        e->sl().marks_set = false;
    });
}

int gdf_take_occupancy_marks_sparse(gdf_engine* e, uint32_t* bits, uint64_t words,
                                    uint32_t* pairs, uint32_t cap) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] {
        if (!e->grid_set || !bits || !pairs) fail(GDF_ERR_STATE, "no voxel grid");
        if (words < (e->ncells + 31) / 32) fail(GDF_ERR_CAPACITY, "mark bitmask too small");
        if (e->sl().nframes > 1)
            fail(GDF_ERR_STATE, "sparse take of a batch's marks: use gdf_take_occupancy_marks");
        HIPCHK(launch_take_marks_sparse(marks_ptr(e), mark_words(e), bits, pairs, cap, e->s()));
        e->sl().marks_set = false;
    });
}

int gdf_union_occupancy_pairs(gdf_engine* e, uint32_t* union_bits, uint64_t words,
                              const uint32_t* pairs, uint32_t nranks, uint32_t nframes,
                              uint32_t frames_per_rank, uint64_t record_words) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] {
        if (!e->grid_set || !union_bits || (!pairs && nranks * nframes)) fail(GDF_ERR_STATE, "no voxel grid");
        if (words < (e->ncells + 31) / 32) fail(GDF_ERR_CAPACITY, "union bitmask too small");
        if (nframes > frames_per_rank || (nframes && record_words < 3))
            fail(GDF_ERR_ARG, "union pairs: nframes > frames_per_rank or records too small");
        HIPCHK(launch_union_pairs(union_bits, mark_words(e), pairs, nranks, nframes,
                                  frames_per_rank, record_words, e->s()));
    });
}

int gdf_voxel_occupancy_grid_batch(gdf_engine* e, const uint32_t* bits, uint64_t words,
                                   uint32_t nranks, uint32_t nframes, uint64_t frame_stride_words,
                                   uint64_t rank_stride_words, uint32_t lifetime) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] {
        if (!e->grid_set || (!bits && nframes)) fail(GDF_ERR_STATE, "no voxel grid");
        if (words < (e->ncells + 31) / 32 || (nframes > 1 && frame_stride_words < words) ||
            (nranks > 1 && rank_stride_words < frame_stride_words * (nframes ? nframes : 1)))
            fail(GDF_ERR_CAPACITY, "mark bitmasks too small");
        for (int i = 0; i < e->npipe; ++i)  // a frame in flight on any slot, marks not taken
            if (e->slots[i].marks_set)
                fail(GDF_ERR_STATE, "marks of a frame are pending (take them first)");
        widen_if_needed(e, lifetime, e->s());
        e->sl().delta_valid = false;
        if (e->grid_mode == 0) {  // one pass per <= kMaxCams frames
            ensure_misc(e);
            // per-frame snapshots only for the slot's own multi-frame batch (<= kMaxCams frames,
            // downloadable with gdf_download_batch_occupancy_grid); the frames of a deferred
            // single-frame exchange (BatchedMarkExchange) can never be downloaded one by one, and
            // the kernel's per-wave snapshot counters hold kMaxCams frames
            const bool snaps = nframes > 1 && e->sl().nframes == nframes && nframes <= (uint32_t)kMaxCams;
            e->sl().snap_valid = false;
            const SnapArgs sn = snaps ? snap_args(e, batch_grid_blocks(e->ncells), nframes)
                                      : SnapArgs{nullptr, nullptr, nullptr};
            for (uint32_t f0 = 0; f0 < nframes || f0 == 0; f0 += (uint32_t)kMaxCams) {
                const uint32_t nf = std::min<uint32_t>(nframes - f0, (uint32_t)kMaxCams);
                const GridSeq q = e->grid_seq(e->grid_ticket++);
                e->grid_gated(e->s(), [&] {
                    e->timed_on(GDF_KERNEL_GRID, e->s(), [&] {
                        HIPCHK(launch_grid_u8_batch(e->d_grid8.as<uint8_t>(),
                                                    bits ? bits + (uint64_t)f0 * frame_stride_words : bits,
                                                    e->ncells, nranks, nf, frame_stride_words,
                                                    rank_stride_words, lifetime, q, sn, e->s()));
                    });
                });
                if (nframes == 0) break;
            }
        } else {  // general history: frame by frame (no per-frame grids kept)
            e->sl().snap_valid = false;
            for (uint32_t f = 0; f < nframes; ++f) {
                HIPCHK(launch_import_marks(marks_ptr(e), mark_words(e), bits + f * frame_stride_words,
                                           nranks, rank_stride_words, e->s()));
                e->sl().marks_set = true;
                occupancy_grid(e, lifetime, e->s());
            }
        }
        e->invoked_once = true;
    });
}

int gdf_import_occupancy_marks_strided(gdf_engine* e, const uint32_t* bits, uint64_t words,
                                       uint32_t nranks, uint64_t rank_stride_words) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] {
        if (!e->grid_set || !bits) fail(GDF_ERR_STATE, "no voxel grid");
        if (words < (e->ncells + 31) / 32 || rank_stride_words < words)
            fail(GDF_ERR_CAPACITY, "mark bitmask too small");
        HIPCHK(launch_import_marks(marks_ptr(e), mark_words(e), bits, nranks, rank_stride_words,
                                   e->s()));
        e->sl().marks_set = true;
    });
}

int gdf_set_profiling(gdf_engine* e, int enable) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] {
        e->resolve_events();
        e->profiling = enable != 0;
        for (int i = 0; i < GDF_KERNEL_SLOTS; ++i) {
            e->prof_ms[i] = 0.0;
            e->prof_n[i] = 0;
        }
    });
}

int gdf_get_kernel_times(gdf_engine* e, double* ms, uint64_t* n, int slots) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] {
        e->resolve_events();
        for (int i = 0; i < slots && i < GDF_KERNEL_SLOTS; ++i) {
            if (ms) ms[i] = e->prof_ms[i];
            if (n) n[i] = e->prof_n[i];
        }
    });
}

int gdf_set_debug(gdf_engine* e, int enable) {
    ENGINE_OR_FAIL(e);
    e->debug = enable != 0;
    return GDF_OK;
}

int gdf_debug_stage_masks(gdf_engine* e, uint8_t* out, uint32_t cap, uint32_t* out_count) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] {
        if (!e->debug || !e->sl().d_stage.p || !e->sl().compacted)
            fail(GDF_ERR_STATE, "stage masks need gdf_set_debug(1) before the compaction");
        if (out_count) *out_count = e->sl().dbg_count;
        if (out) {
            if (cap < e->sl().dbg_count) fail(GDF_ERR_CAPACITY, "debug masks: buffer too small");
            e->sync();
            if (e->sl().dbg_count) HIPCHK(hipMemcpy(out, e->sl().d_stage.p, e->sl().dbg_count, hipMemcpyDeviceToHost));
        }
    });
}

int gdf_debug_rollbuffer(gdf_engine* e, float* pts, uint32_t* mask, uint32_t* seq_idx,
                         uint32_t cap, uint32_t* hdr, uint32_t hdr_cap) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] {
        const uint32_t R = e->rb.num_points;
        if (cap < R || hdr_cap < e->hdrB.size()) fail(GDF_ERR_CAPACITY, "rollbuffer debug: buffer too small");
        e->sync();
        std::vector<float> tmp((size_t)R * 4);
        if (R) {
            const uint64_t first = e->ring_head % e->ring_cap;
            const uint64_t a = std::min<uint64_t>(R, e->ring_cap - first);
            HIPCHK(hipMemcpy(tmp.data(), e->d_ring.as<float4>() + first, a * 16, hipMemcpyDeviceToHost));
            if (R > a) HIPCHK(hipMemcpy(tmp.data() + 4 * a, e->d_ring.p, (R - a) * 16, hipMemcpyDeviceToHost));
        }
        for (uint32_t i = 0; i < R; ++i) {
            if (pts) {
                pts[4 * (size_t)i + 0] = tmp[4 * (size_t)i + 0];
                pts[4 * (size_t)i + 1] = tmp[4 * (size_t)i + 1];
                pts[4 * (size_t)i + 2] = tmp[4 * (size_t)i + 2];
                pts[4 * (size_t)i + 3] = 1.0f;
            }
            if (mask) mask[i] = tmp[4 * (size_t)i + 3] != 0.0f ? 1u : 0u;
        }
        if (seq_idx) {
            uint64_t pos = 0;
            for (uint32_t j = 0; j < e->hdrB.size() && pos < R; ++j)
                for (uint32_t k = 0; k < e->hdrB[j].num && pos < R; ++k) seq_idx[pos++] = j;
        }
        if (hdr)
            for (uint32_t j = 0; j < e->hdrB.size(); ++j) {
                hdr[4 * j + 0] = e->hdrB[j].sec;
                hdr[4 * j + 1] = e->hdrB[j].nsec;
                hdr[4 * j + 2] = e->hdrB[j].start;
                hdr[4 * j + 3] = e->hdrB[j].num;
            }
    });
}

int gdf_debug_historic_grid(gdf_engine* e, uint32_t* out, uint64_t cap) {
    ENGINE_OR_FAIL(e);
    return guarded(e, [&] {
        if (!e->grid_set) fail(GDF_ERR_STATE, "no voxel grid");
        if (!out || cap < e->ncells) fail(GDF_ERR_CAPACITY, "historic grid: buffer too small");
        sync_all(e);
        e->sync();
        if (e->grid_mode == 1) {
            HIPCHK(hipMemcpy(out, e->d_hist32.p, e->ncells * 4, hipMemcpyDeviceToHost));
        } else {
            std::vector<uint8_t> g(e->ncells);
            HIPCHK(hipMemcpy(g.data(), e->d_grid8.p, e->ncells, hipMemcpyDeviceToHost));
            for (uint64_t c = 0; c < e->ncells; ++c) out[c] = g[c];
        }
    });
}

}  // extern "C"
