// gdf_fused.cpp — one rank of the multi-GPU fused cloud in C++ (include/gdf_fused.h).
//
// The protocol of multi.FusedCloudRank (the reference's single-process fusion over all cameras,
// src/gpu_depthmap_fusion.cpp:1509-1581 buffer order + :1743-1756 one voxelize, cut at the
// voxel-key ranges) with no interpreter in the step: the engine calls of include/gdf.h, HIP
// copies, and RCCL collectives issued on the engine slot's stream.  RCCL is resolved at run time
// from the librccl the caller names (torch's), so the process holds one RCCL.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>  // (types and prototypes only: the functions come from dlsym)
#include <dlfcn.h>

#include <algorithm>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <vector>

#include "gdf_fused.h"

namespace gdf {
void set_last_error(const std::string& msg);
}

namespace {

struct FusedError {
    int code;
    std::string msg;
};

[[noreturn]] void fail(int code, const std::string& msg) { throw FusedError{code, msg}; }

void hipchk(hipError_t e, const char* what) {
    if (e != hipSuccess) fail(GDF_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

void gdfchk(int rc) {  // an engine call failed: its gdf_last_error stands
    if (rc != GDF_OK) throw FusedError{rc, std::string()};
}

template <class F>
int guarded(F&& f) {
    try {
        f();
        return GDF_OK;
    } catch (const FusedError& err) {
        if (!err.msg.empty()) gdf::set_last_error(err.msg);
        return err.code;
    } catch (const std::bad_alloc&) {
        gdf::set_last_error("host allocation failed");
        return GDF_ERR_NOMEM;
    }
}

// ---- RCCL, resolved from the caller's library -------------------------------------------------
struct Rccl {
    void* lib = nullptr;
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) comm_init_rank = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
};

std::mutex g_rccl_mutex;
Rccl g_rccl;

template <class T>
void sym(void* lib, T& fn, const char* name) {
    fn = reinterpret_cast<T>(dlsym(lib, name));
    if (!fn) fail(GDF_ERR_STATE, std::string("librccl lacks ") + name);
}

const Rccl& rccl(const char* path) {
    std::lock_guard<std::mutex> lk(g_rccl_mutex);
    if (g_rccl.lib) return g_rccl;
    void* lib = dlopen(path && *path ? path : "librccl.so", RTLD_NOW | RTLD_LOCAL);
    if (!lib) fail(GDF_ERR_STATE, std::string("cannot load librccl: ") + dlerror());
    Rccl r;
    r.lib = lib;
    sym(lib, r.get_unique_id, "ncclGetUniqueId");
    sym(lib, r.comm_init_rank, "ncclCommInitRank");
    sym(lib, r.comm_destroy, "ncclCommDestroy");
    sym(lib, r.all_gather, "ncclAllGather");
    sym(lib, r.send, "ncclSend");
    sym(lib, r.recv, "ncclRecv");
    sym(lib, r.group_start, "ncclGroupStart");
    sym(lib, r.group_end, "ncclGroupEnd");
    sym(lib, r.error_string, "ncclGetErrorString");
    g_rccl = r;  // (kept for the process: never dlclose'd)
    return g_rccl;
}

void ncclchk(const Rccl& r, ncclResult_t res, const char* what) {
    if (res != ncclSuccess) fail(GDF_ERR_HIP, std::string(what) + ": " + r.error_string(res));
}

// ---- per-slot exchange state ------------------------------------------------------------------
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    // grow-only; the slot's stream is drained first (its previous step may still read the buffer)
    template <class T = uint8_t>
    T* ensure(size_t bytes, hipStream_t st) {
        if (bytes > cap) {
            if (p) {
                hipchk(hipStreamSynchronize(st), "hipStreamSynchronize");
                hipchk(hipFree(p), "hipFree");
                p = nullptr;
            }
            const size_t grown = std::max(bytes, cap + cap / 2);
            hipchk(hipMalloc(&p, grown), "hipMalloc");
            cap = grown;
        }
        return static_cast<T*>(p);
    }
    template <class T = uint8_t>
    T* as() const { return static_cast<T*>(p); }
    void release() {
        if (p) hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

struct SlotX {
    DevBuf tail, tails;       // this rank's halo tails, every rank's (all-gather)
    DevBuf gathered;          // the union of the step's marks: frame f at f * W * S words, rank
                              // j's key range in words [j S, (j + 1) S) (voxelize + all-gather)
    // partitioned send lists (points, run keys, run starts), split sizes (points then runs per
    // part), every rank's split sizes
    DevBuf sp, srk, srs, cnt, cntall;
    DevBuf rp, rrk, rrs;      // received lists
    uint32_t* host = nullptr;  // pinned copy of cntall (world x 2 world)
    hipEvent_t ev = nullptr;
    bool pending = false;
    int average = 1;  // the step's voxel_average
    uint32_t nframes = 1, lifetime = 0;  // the step's batch and occupancy_lifetime
};

constexpr int kSlots = 4;  // the engine's pipeline depth is 1..4

}  // namespace

struct gdf_fused {
    gdf_engine* e = nullptr;
    const Rccl* r = nullptr;
    ncclComm_t comm_a = nullptr, comm_b = nullptr;
    int rank = 0, world = 1;
    std::vector<gdf_stream_camera> cams;
    uint32_t F = 0, Lmax = 0;
    SlotX slots[kSlots];

    ~gdf_fused() {
        if (e) {
            gdf_synchronize(e);
            gdf_set_partition_marks(e, 1);  // (the engine's default again)
        }
        for (SlotX& s : slots) {
            for (DevBuf* b : {&s.tail, &s.tails, &s.gathered, &s.sp, &s.srk, &s.srs,
                              &s.cnt, &s.cntall, &s.rp, &s.rrk, &s.rrs})
                b->release();
            if (s.host) hipHostFree(s.host);
            if (s.ev) hipEventDestroy(s.ev);
        }
        if (r) {
            if (comm_a) r->comm_destroy(comm_a);
            if (comm_b) r->comm_destroy(comm_b);
        }
    }
};

namespace {

void fused_start(gdf_fused* f, const uint16_t* const* depth, uint32_t B, const gdf_frame_params* p,
                 int* out_slot) {
    if (!depth || !p || B == 0 || B > 16) fail(GDF_ERR_ARG, "fused start: 1..16 depth maps and params");
    for (uint32_t j = 0; j < B; ++j)
        if (!depth[j]) fail(GDF_ERR_ARG, "fused start: null depth map");
    if (!p->enable_voxel_filter) fail(GDF_ERR_ARG, "fused start: the fused cloud needs the voxel filter");
    gdf_engine* e = f->e;
    const Rccl& r = *f->r;
    gdfchk(gdf_clear(e));
    int slot = 0;
    gdfchk(gdf_get_slot(e, &slot));
    if (slot < 0 || slot >= kSlots) fail(GDF_ERR_STATE, "fused start: engine slot out of range");
    void* sv = nullptr;
    gdfchk(gdf_get_stream(e, &sv));
    hipStream_t st = static_cast<hipStream_t>(sv);
    SlotX& S = f->slots[slot];
    if (S.pending) fail(GDF_ERR_STATE, "fused start: the slot's previous step is unfinished");
    const int W = f->world, R = f->rank;
    const gdf_stream_camera& c = f->cams[R];
    const size_t L2 = 2 * (size_t)f->Lmax;
    const bool halo = f->F > 0 && W > 1;
    const uint8_t* tails = nullptr;
    if (halo) {  // every rank's B tails (frame j's halo before frame j's depth map)
        uint8_t* tail = S.tail.ensure(B * L2, st);
        tails = S.tails.ensure((size_t)W * B * L2, st);
        const size_t npx = (size_t)c.width * c.height;
        for (uint32_t j = 0; j < B; ++j)
            hipchk(hipMemcpyAsync(tail + j * L2, depth[j] + (npx - f->Lmax), L2,
                                  hipMemcpyDeviceToDevice, st), "hipMemcpyAsync(tail)");
        ncclchk(r, r.all_gather(tail, S.tails.as(), B * L2, ncclUint8, f->comm_a, st),
                "ncclAllGather(tails)");
    }
    for (uint32_t j = 0; j < B; ++j) {
        if (j) gdfchk(gdf_next_frame_in_batch(e));
        if (halo && R > 0) {
            const gdf_stream_camera& pc = f->cams[R - 1];
            const uint32_t take = std::min<uint32_t>(f->Lmax, pc.width * pc.height);
            const uint8_t* t = tails + ((size_t)(R - 1) * B + j) * L2 + 2 * (size_t)(f->Lmax - take);
            gdfchk(gdf_add_halo_depthmap_device(e, reinterpret_cast<const uint16_t*>(t), take,
                                                pc.width, pc.height, pc.depth_scale, pc.fx, pc.fy,
                                                pc.cx, pc.cy, pc.T_world, pc.T_crop));
        }
        gdfchk(gdf_add_depthmap_device(e, depth[j], c.width, c.height, c.depth_scale, c.fx, c.fy,
                                       c.cx, c.cy, c.T_world, c.T_crop));
    }
    gdf_frame_params q = *p;
    q.synchronous = 0;
    q.defer_occupancy_grid = 1;
    q.defer_voxelize = 1;
    if (R != W - 1 || B > 1) q.move_transform_available = 0;  // the rollbuffer: last rank only
    // the send lists, written by the compaction itself (gdf_set_emit_partition): sized for the
    // step's pixels (+ halo) plus, on the rollbuffer rank, every point the window can select
    uint32_t* cnt = S.cnt.ensure<uint32_t>((size_t)2 * W * 4, st);
    uint32_t* cntall = S.cntall.ensure<uint32_t>((size_t)2 * W * W * 4, st);
    size_t want = (size_t)B * c.width * c.height + (halo && R > 0 ? B * (size_t)f->Lmax : 0u);
    if (R == W - 1 && B == 1 && p->move_transform_available) {  // + the window after the ingest
        gdf_rollbuffer_state rs{};
        gdfchk(gdf_get_rollbuffer_state(e, &rs));
        uint32_t col = 0;
        gdfchk(gdf_num_collected_point_sequence_points(e, &col));
        want += (size_t)rs.num_points + col;
    }
    auto arm = [&](size_t cap) {
        S.sp.ensure<float>(cap * 16, st);
        S.srk.ensure<uint32_t>(cap * 4, st);
        S.srs.ensure<uint32_t>(cap * 4, st);
        const uint32_t have = (uint32_t)std::min<size_t>({S.sp.cap / 16, S.srk.cap / 4, S.srs.cap / 4});
        gdfchk(gdf_set_emit_partition(e, W, S.sp.as<float>(), S.srk.as<uint32_t>(),
                                      S.srs.as<uint32_t>(), have, cnt));
    };
    arm(std::max<size_t>(want, 1));
    gdfchk(gdf_set_partition_marks(e, 0));
    gdf_frame_result res{};
    gdfchk(gdf_process_frame(e, &q, &res));
    // The compaction sets no marks (gdf_set_partition_marks(e, 0) before the frame): W full
    // bitmasks of B frames (3.4 MB per rank and step at VGA x 8, received W - 1 times) would travel;
    // instead the key-range voxelize of the finish marks every voxel of its range - whole mark
    // words per range - and one in-place all-gather of those slices is the union (1 / W).
    S.nframes = B;
    S.lifetime = q.occupancy_lifetime;
    // every rank's split sizes (the partition's, written with the compaction) to pinned memory
    // (no wait here)
    ncclchk(r, r.all_gather(cnt, cntall, 2 * W, ncclUint32, f->comm_a, st), "ncclAllGather(counts)");
    hipchk(hipMemcpyAsync(S.host, cntall, (size_t)2 * W * W * 4, hipMemcpyDeviceToHost, st),
           "hipMemcpyAsync(counts)");
    hipchk(hipEventRecord(S.ev, st), "hipEventRecord");
    S.average = q.voxel_average ? 1 : 0;
    S.pending = true;
    *out_slot = slot;
}

void fused_finish(gdf_fused* f, int slot, uint32_t* send_counts, uint32_t* recv_count) {
    if (slot < 0 || slot >= kSlots) fail(GDF_ERR_ARG, "fused finish: bad slot");
    gdf_engine* e = f->e;
    const Rccl& r = *f->r;
    SlotX& S = f->slots[slot];
    if (!S.pending) fail(GDF_ERR_STATE, "fused finish: no step in flight on this slot");
    gdfchk(gdf_select_slot(e, slot));
    void* sv = nullptr;
    gdfchk(gdf_get_stream(e, &sv));
    hipStream_t st = static_cast<hipStream_t>(sv);
    hipchk(hipEventSynchronize(S.ev), "hipEventSynchronize");  // (the later slots keep the GPU busy)
    const int W = f->world, R = f->rank;
    // rank q's split sizes: host[q * 2W + p] points to part p, host[q * 2W + W + p] runs
    auto pts_of = [&](int from, int to) -> uint64_t { return S.host[(size_t)from * 2 * W + to]; };
    auto runs_of = [&](int from, int to) -> uint64_t { return S.host[(size_t)from * 2 * W + W + to]; };
    uint32_t pbase[17], rbase[17];
    uint64_t n = 0, nr = 0;
    for (int q = 0; q < W; ++q) {
        pbase[q] = (uint32_t)n;
        rbase[q] = (uint32_t)nr;
        n += pts_of(q, R);
        nr += runs_of(q, R);
        if (n >= 0xFFFFFFFFull) fail(GDF_ERR_CAPACITY, "fused finish: 2^32 points received");
    }
    pbase[W] = (uint32_t)n;
    rbase[W] = (uint32_t)nr;
    float* rp = S.rp.ensure<float>(std::max<uint64_t>(n, 1) * 16, st);
    uint32_t* rrk = S.rrk.ensure<uint32_t>(std::max<uint64_t>(nr, 1) * 4, st);
    uint32_t* rrs = S.rrs.ensure<uint32_t>((nr + 1) * 4, st);
    size_t soff = 0, sroff = 0;
    for (int q = 0; q < R; ++q) {
        soff += pts_of(R, q);
        sroff += runs_of(R, q);
    }
    // the rank's own part: a device copy (an RCCL self send / recv is a slower kernel copy)
    if (const size_t c = pts_of(R, R)) {
        hipchk(hipMemcpyAsync(rp + 4 * (size_t)pbase[R], S.sp.as<float>() + 4 * soff, 16 * c,
                              hipMemcpyDeviceToDevice, st), "hipMemcpyAsync(points)");
        const size_t rc = runs_of(R, R);
        hipchk(hipMemcpyAsync(rrk + rbase[R], S.srk.as<uint32_t>() + sroff, 4 * rc,
                              hipMemcpyDeviceToDevice, st), "hipMemcpyAsync(run keys)");
        hipchk(hipMemcpyAsync(rrs + rbase[R], S.srs.as<uint32_t>() + sroff, 4 * rc,
                              hipMemcpyDeviceToDevice, st), "hipMemcpyAsync(run starts)");
    }
    if (W > 1) {
        ncclchk(r, r.group_start(), "ncclGroupStart");
        soff = sroff = 0;
        for (int q = 0; q < W; ++q) {
            const size_t sc = pts_of(R, q), sr = runs_of(R, q);
            const size_t rc = pts_of(q, R), rr = runs_of(q, R);
            if (q != R && sc) {
                ncclchk(r, r.send(S.sp.as<float>() + 4 * soff, 4 * sc, ncclFloat32, q, f->comm_b, st),
                        "ncclSend(points)");
                ncclchk(r, r.send(S.srk.as<uint32_t>() + sroff, sr, ncclUint32, q, f->comm_b, st),
                        "ncclSend(run keys)");
                ncclchk(r, r.send(S.srs.as<uint32_t>() + sroff, sr, ncclUint32, q, f->comm_b, st),
                        "ncclSend(run starts)");
            }
            if (q != R && rc) {
                ncclchk(r, r.recv(rp + 4 * (size_t)pbase[q], 4 * rc, ncclFloat32, q, f->comm_b, st),
                        "ncclRecv(points)");
                ncclchk(r, r.recv(rrk + rbase[q], rr, ncclUint32, q, f->comm_b, st), "ncclRecv(run keys)");
                ncclchk(r, r.recv(rrs + rbase[q], rr, ncclUint32, q, f->comm_b, st), "ncclRecv(run starts)");
            }
            soff += sc;
            sroff += sr;
        }
        ncclchk(r, r.group_end(), "ncclGroupEnd");
    }
    // the voxel means of this rank's key range, every voxel's mark into slice R of its frame's
    // union bitmask, the slices all-gathered in place, then the step's batched grid update
    uint32_t g[3];
    uint64_t ncells = 0;
    gdfchk(gdf_get_grid_size(e, g, &ncells));
    const uint64_t words = (ncells + 31) / 32;
    const uint64_t Sw = (words + W - 1) / W;  // = part_slice_words(W, ncells), the partition's rule
    const uint64_t stride = Sw * W;
    uint32_t* uni = S.gathered.ensure<uint32_t>(S.nframes * stride * 4, st);
    hipchk(hipMemsetAsync(uni, 0, S.nframes * stride * 4, st), "hipMemsetAsync(marks)");
    gdfchk(gdf_voxelize_runs_marked(e, rp, rrk, rrs, W, pbase, rbase, S.average, uni, stride));
    if (W > 1) {  // (on the points' communicator: the finish's collectives stay in step order,
                  // never behind the next step's start collectives on comm_a)
        ncclchk(r, r.group_start(), "ncclGroupStart");
        for (uint32_t j = 0; j < S.nframes; ++j)
            ncclchk(r, r.all_gather(uni + j * stride + (uint64_t)R * Sw, uni + j * stride, Sw, ncclUint32,
                                    f->comm_b, st), "ncclAllGather(mark slices)");
        ncclchk(r, r.group_end(), "ncclGroupEnd");
    }
    gdfchk(gdf_voxel_occupancy_grid_batch(e, uni, words, 1, S.nframes, stride, S.nframes * stride,
                                          S.lifetime));
    if (send_counts)
        for (int q = 0; q < W; ++q) send_counts[q] = (uint32_t)pts_of(R, q);
    if (recv_count) *recv_count = (uint32_t)n;
    S.pending = false;
}

}  // namespace

extern "C" {

int gdf_fused_unique_id(const char* rccl_library, uint8_t* id_out) {
    if (!id_out) return GDF_ERR_ARG;
    return guarded([&] {
        const Rccl& r = rccl(rccl_library);
        ncclUniqueId a, b;
        ncclchk(r, r.get_unique_id(&a), "ncclGetUniqueId");
        ncclchk(r, r.get_unique_id(&b), "ncclGetUniqueId");
        std::memcpy(id_out, &a, sizeof(a));
        std::memcpy(id_out + sizeof(a), &b, sizeof(b));
    });
}

int gdf_fused_create(gdf_engine* engine, const char* rccl_library, const uint8_t* id, int rank,
                     int world, const gdf_stream_camera* cams, uint32_t flying_filter_size,
                     gdf_fused** out) {
    if (!engine || !id || !cams || !out || world < 1 || world > 16 || rank < 0 || rank >= world) {
        gdf::set_last_error("fused create: engine, ids, cameras, 0 <= rank < world <= 16");
        return GDF_ERR_ARG;
    }
    *out = nullptr;
    gdf_fused* f = nullptr;
    const int rc = guarded([&] {
        const Rccl& r = rccl(rccl_library);
        f = new gdf_fused();
        f->e = engine;
        f->rank = rank;
        f->world = world;
        f->cams.assign(cams, cams + world);
        f->F = flying_filter_size;
        for (const gdf_stream_camera& c : f->cams)
            f->Lmax = std::max<uint32_t>(f->Lmax, f->F * c.width + f->F);
        for (const gdf_stream_camera& c : f->cams)
            if ((uint64_t)c.width * c.height < f->Lmax)
                fail(GDF_ERR_ARG, "fused multi-GPU frames need cameras taller than F rows");
        for (SlotX& s : f->slots) {
            hipchk(hipHostMalloc(reinterpret_cast<void**>(&s.host), (size_t)2 * world * world * 4,
                                 hipHostMallocDefault), "hipHostMalloc");
            hipchk(hipEventCreateWithFlags(&s.ev, hipEventDisableTiming), "hipEventCreate");
        }
        ncclUniqueId a, b;
        std::memcpy(&a, id, sizeof(a));
        std::memcpy(&b, id + sizeof(a), sizeof(b));
        ncclchk(r, r.comm_init_rank(&f->comm_a, world, a, rank), "ncclCommInitRank(A)");
        ncclchk(r, r.comm_init_rank(&f->comm_b, world, b, rank), "ncclCommInitRank(B)");
        f->r = &r;
    });
    if (rc != GDF_OK) {
        delete f;
        return rc;
    }
    *out = f;
    return GDF_OK;
}

int gdf_fused_destroy(gdf_fused* f) {
    delete f;
    return GDF_OK;
}

int gdf_fused_halo_pixels(gdf_fused* f, uint32_t* pixels) {
    if (!f || !pixels) return GDF_ERR_ARG;
    *pixels = f->Lmax;
    return GDF_OK;
}

int gdf_fused_start(gdf_fused* f, const uint16_t* const* depth, uint32_t nframes,
                    const gdf_frame_params* p, int* slot) {
    if (!f || !slot) return GDF_ERR_ARG;
    return guarded([&] { fused_start(f, depth, nframes, p, slot); });
}

int gdf_fused_finish(gdf_fused* f, int slot, uint32_t* send_counts, uint32_t* recv_count) {
    if (!f) return GDF_ERR_ARG;
    return guarded([&] { fused_finish(f, slot, send_counts, recv_count); });
}

int gdf_fused_run(gdf_fused* f, const gdf_stream_camera* cam, const gdf_frame_params* p,
                  uint64_t first, uint64_t steps, uint32_t batch, int depth) {
    if (!f || !cam || !p || !cam->frames || cam->ring == 0 || batch == 0 || batch > 16 ||
        depth < 1 || depth > kSlots)
        return GDF_ERR_ARG;
    return guarded([&] {
        gdfchk(gdf_set_pipeline_depth(f->e, depth));
        std::deque<int> pending;
        const uint16_t* ptrs[16];
        for (uint64_t s = 0; s < steps; ++s) {
            if ((int)pending.size() >= depth) {  // (its slot comes round again)
                fused_finish(f, pending.front(), nullptr, nullptr);
                pending.pop_front();
            }
            for (uint32_t j = 0; j < batch; ++j) ptrs[j] = cam->frames[((first + s) * batch + j) % cam->ring];
            int slot = 0;
            fused_start(f, ptrs, batch, p, &slot);
            pending.push_back(slot);
            // step s - 1 is finished once step s is queued: the GPU computes s while the host
            // waits for s - 1's split sizes
            if (depth == 1 || pending.size() > 1) {
                fused_finish(f, pending.front(), nullptr, nullptr);
                pending.pop_front();
            }
        }
        for (int k : pending) fused_finish(f, k, nullptr, nullptr);
    });
}

}  // extern "C"
