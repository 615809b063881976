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
#include <array>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
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

// ---- the step's collectives -------------------------------------------------------------------
// Everything the step exchanges goes through this interface: an all-gather of equal byte slices
// (in place when send == recv + rank * bytes), point-to-point sends / receives, and groups (the
// operations between group_start and group_end are issued as one, like ncclGroupStart/End).  Two
// communicators: kHalo (halo tails, split sizes: the start) and kPoints (points, runs, mark
// slices: the finish).  Every call is stream-ordered on `st` (the engine slot's stream).
enum Comm { kHalo = 0, kPoints = 1 };

struct Transport {
    virtual ~Transport() = default;
    virtual const char* kind() const = 0;
    virtual int ranks() const = 0;  // the rank count the communicator reports
    virtual void all_gather(const void* send, void* recv, size_t bytes, Comm c, hipStream_t st) = 0;
    virtual void group_start(Comm c) = 0;
    virtual void send(const void* buf, size_t bytes, int peer, Comm c, hipStream_t st) = 0;
    virtual void recv(void* buf, size_t bytes, int peer, Comm c, hipStream_t st) = 0;
    virtual void group_end(Comm c, hipStream_t st) = 0;
    virtual void abort() {}
};

// RCCL: two communicators of the transport's own, byte-typed transfers.
struct RcclTransport final : Transport {
    const Rccl* r = nullptr;
    ncclComm_t comm[2] = {nullptr, nullptr};
    int world = 1;
    ~RcclTransport() override {
        for (ncclComm_t c : comm)
            if (c) r->comm_destroy(c);
    }
    const char* kind() const override { return "rccl"; }
    int ranks() const override {
        int n = 0;
        using CountFn = ncclResult_t (*)(const ncclComm_t, int*);
        auto fn = reinterpret_cast<CountFn>(dlsym(r->lib, "ncclCommCount"));
        if (!fn || fn(comm[kPoints], &n) != ncclSuccess) return -1;
        return n;
    }
    void all_gather(const void* send, void* recv, size_t bytes, Comm c, hipStream_t st) override {
        ncclchk(*r, r->all_gather(send, recv, bytes, ncclUint8, comm[c], st), "ncclAllGather");
    }
    void group_start(Comm) override { ncclchk(*r, r->group_start(), "ncclGroupStart"); }
    void send(const void* buf, size_t bytes, int peer, Comm c, hipStream_t st) override {
        ncclchk(*r, r->send(buf, bytes, ncclUint8, peer, comm[c], st), "ncclSend");
    }
    void recv(void* buf, size_t bytes, int peer, Comm c, hipStream_t st) override {
        ncclchk(*r, r->recv(buf, bytes, ncclUint8, peer, comm[c], st), "ncclRecv");
    }
    void group_end(Comm, hipStream_t) override { ncclchk(*r, r->group_end(), "ncclGroupEnd"); }
};

}  // namespace

// In-process transport: `world` ranks of ONE process (one host thread and one engine each, on one
// or several devices), exchanging through device-to-device copies on the ranks' own streams.  A
// collective (or a group) is a round of its communicator; round k of communicator c is matched
// across the ranks by their k-th call, like RCCL's issue order:
//   1. each rank records `ready` on its stream (its sends are written) and posts its operations;
//   2. host barrier: every rank posted round k;
//   3. each rank checks the round's schedule (check_round: the same on every rank, so every rank
//      fails alike), copies what it receives, on ITS stream, behind the sender's `ready`;
//   4. each rank records `done` (its reads are finished); host barrier;
//   5. each rank's stream waits for every other rank's `done` before its buffers are reused.
// The host only waits for the other ranks to ISSUE (not to finish): GPU work stays queued and the
// steps stay pipelined.  A rank that fails aborts the world, so the others fail instead of waiting.
//
// The transport is as strict as RCCL is unforgiving: a schedule RCCL would hang on or corrupt
// fails here, at once and on every rank -
//   * a send no peer receives in the same round (RCCL: the sender's kernel never completes), a
//     receive without its send, sizes that differ, a bad peer;
//   * an all-gather whose send buffer overlaps its receive buffer anywhere but at recv + rank *
//     bytes (RCCL's only in-place form), all-gathers of different sizes across the ranks;
//   * the ranks issuing their collectives over the two communicators in different orders (the
//     classic two-communicator deadlock: rank 0 blocked in round k of A while rank 1 is blocked in
//     round m of B) - every rank numbers the rounds it issues over both communicators, a round's
//     number must be the same on every rank (check_round), and a rank arriving in a round checks
//     that no other rank waits in a different round under the same number (check_arrival).
namespace {
struct LocalOp {
    int kind;  // 0 all-gather, 1 send, 2 recv
    const void* src;
    void* dst;
    size_t bytes;
    int peer;
};

const char* comm_name(int c) { return c == 0 ? "halo" : "points"; }

// The schedule of one round, posts[q] = rank q's operations in its issue order, issue[q] = the
// round's number in rank q's issue order over both communicators.  Empty: the round is valid.
std::string check_round(int W, const std::vector<const std::vector<LocalOp>*>& posts,
                        const std::vector<uint64_t>& issue) {
    for (int q = 1; q < W; ++q)
        if (issue[q] != issue[0])
            return "local transport: cross-communicator issue order differs across ranks (rank 0 "
                   "issued this round as its collective #" + std::to_string(issue[0]) + ", rank " +
                   std::to_string(q) + " as #" + std::to_string(issue[q]) + ")";
    std::vector<std::vector<size_t>> ag(W);  // all-gather sizes per rank, in order
    for (int q = 0; q < W; ++q)
        for (const LocalOp& o : *posts[q]) {
            if (o.kind == 0) {
                ag[q].push_back(o.bytes);
                const uintptr_t s = (uintptr_t)o.src, d = (uintptr_t)o.dst;
                const uintptr_t se = s + o.bytes, de = d + (uintptr_t)W * o.bytes;
                if (o.bytes && s < de && d < se && s != d + (uintptr_t)q * o.bytes)
                    return "local transport: rank " + std::to_string(q) + "'s all-gather send "
                           "buffer overlaps its receive buffer other than at recv + rank * bytes";
            } else if (o.kind == 1 || o.kind == 2) {
                if (o.peer < 0 || o.peer >= W || o.peer == q)
                    return std::string("local transport: bad ") + (o.kind == 1 ? "send" : "receive") +
                           " peer " + std::to_string(o.peer) + " on rank " + std::to_string(q);
            } else {
                return "local transport: unknown operation";
            }
        }
    for (int q = 1; q < W; ++q)
        if (ag[q] != ag[0]) return "local transport: all-gather sizes differ across ranks";
    // every send s -> d matched by d's receive from s, n-th with n-th, equal sizes
    for (int s = 0; s < W; ++s)
        for (int d = 0; d < W; ++d) {
            if (s == d) continue;
            std::vector<size_t> snd, rcv;
            for (const LocalOp& o : *posts[s])
                if (o.kind == 1 && o.peer == d) snd.push_back(o.bytes);
            for (const LocalOp& o : *posts[d])
                if (o.kind == 2 && o.peer == s) rcv.push_back(o.bytes);
            const std::string pair = " (rank " + std::to_string(s) + " -> rank " + std::to_string(d) + ")";
            if (snd.size() > rcv.size()) return "local transport: a send no receive consumes" + pair;
            if (snd.size() < rcv.size()) return "local transport: a receive without its send" + pair;
            if (snd != rcv) return "local transport: send / receive sizes differ" + pair;
        }
    return std::string();
}

// Rank R arrives in round k of communicator c as its collective #issue; waiting[q] = {c, k, issue}
// of the round rank q is blocked in (c = -1: not waiting).  Empty: no crossed order.
std::string check_arrival(int W, int R, int c, uint64_t k, uint64_t issue,
                          const std::vector<std::array<int64_t, 3>>& waiting) {
    for (int q = 0; q < W; ++q) {
        if (q == R || waiting[q][0] < 0) continue;
        if ((uint64_t)waiting[q][2] == issue && (waiting[q][0] != c || (uint64_t)waiting[q][1] != k))
            return "local transport: cross-communicator issue order differs across ranks (rank " +
                   std::to_string(R) + " issued " + comm_name(c) + " round " + std::to_string(k) +
                   " as its collective #" + std::to_string(issue) + ", rank " + std::to_string(q) +
                   " waits in " + comm_name((int)waiting[q][0]) + " round " +
                   std::to_string(waiting[q][1]) + " under the same number)";
    }
    return std::string();
}
}  // namespace

struct gdf_fused_local {
    using Op = LocalOp;
    struct Post {
        std::vector<Op> ops;
        hipEvent_t ready = nullptr, done = nullptr;
        uint64_t issue = 0;
    };
    struct Round {
        std::vector<Post> posts;
        int arrived = 0, copied = 0, left = 0;
    };
    int world = 1;
    std::mutex m;
    std::condition_variable cv;
    std::map<uint64_t, Round> rounds[2];
    std::vector<std::array<int64_t, 3>> waiting;  // per rank: the round it waits in (check_arrival)
    int refs = 0;  // ranks created on this world and not destroyed
    bool aborted = false;
    std::string abort_reason;
    double timeout_s = 300.0;  // a rank that never arrives (a caller bug) ends the wait

    void abort_locked(const std::string& why) {
        if (!aborted) {
            aborted = true;
            abort_reason = why;
        }
        cv.notify_all();
    }
    template <class Pred>
    void wait(std::unique_lock<std::mutex>& lk, Pred pred, const char* what) {
        const auto until = std::chrono::steady_clock::now() +
                           std::chrono::milliseconds((long long)(timeout_s * 1e3));
        while (!pred()) {
            if (aborted) fail(GDF_ERR_STATE, std::string("local transport aborted (") + abort_reason + ")");
            if (cv.wait_until(lk, until) == std::cv_status::timeout && !pred()) {
                abort_locked(std::string("timeout at ") + what);
                fail(GDF_ERR_STATE, std::string("local transport: a rank did not reach ") + what);
            }
        }
    }
};

namespace {

struct LocalTransport final : Transport {
    gdf_fused_local* w = nullptr;
    int rank = 0;
    uint64_t seq[2] = {0, 0};
    uint64_t issued = 0;  // rounds issued over both communicators (the issue-order check)
    hipEvent_t ready[2] = {nullptr, nullptr}, done[2] = {nullptr, nullptr};
    bool grouped[2] = {false, false};
    std::vector<gdf_fused_local::Op> ops[2];

    LocalTransport(gdf_fused_local* world, int r) : w(world), rank(r) {
        for (int c = 0; c < 2; ++c) {
            hipchk(hipEventCreateWithFlags(&ready[c], hipEventDisableTiming), "hipEventCreate");
            hipchk(hipEventCreateWithFlags(&done[c], hipEventDisableTiming), "hipEventCreate");
        }
    }
    ~LocalTransport() override {
        for (int c = 0; c < 2; ++c) {
            if (ready[c]) (void)hipEventDestroy(ready[c]);
            if (done[c]) (void)hipEventDestroy(done[c]);
        }
    }
    const char* kind() const override { return "local"; }
    int ranks() const override { return w->world; }
    void abort() override {
        std::lock_guard<std::mutex> lk(w->m);
        w->abort_locked("rank " + std::to_string(rank) + " failed");
    }
    void all_gather(const void* send, void* recv, size_t bytes, Comm c, hipStream_t st) override {
        ops[c].push_back({0, send, recv, bytes, -1});
        if (!grouped[c]) run(c, st);
    }
    void group_start(Comm c) override {
        if (grouped[c]) fail(GDF_ERR_STATE, "local transport: nested group");
        grouped[c] = true;
    }
    void send(const void* buf, size_t bytes, int peer, Comm c, hipStream_t) override {
        if (!grouped[c]) fail(GDF_ERR_STATE, "local transport: send outside a group");
        ops[c].push_back({1, buf, nullptr, bytes, peer});
    }
    void recv(void* buf, size_t bytes, int peer, Comm c, hipStream_t) override {
        if (!grouped[c]) fail(GDF_ERR_STATE, "local transport: recv outside a group");
        ops[c].push_back({2, nullptr, buf, bytes, peer});
    }
    void group_end(Comm c, hipStream_t st) override {
        if (!grouped[c]) fail(GDF_ERR_STATE, "local transport: group_end without group_start");
        grouped[c] = false;
        run(c, st);
    }

  private:
    // one round (a collective, or a group of operations) of communicator c
    void run(Comm c, hipStream_t st) {
        std::vector<gdf_fused_local::Op> mine;
        mine.swap(ops[c]);
        const int W = w->world, R = rank;
        const uint64_t k = seq[c]++;
        const uint64_t issue = issued++;
        hipchk(hipEventRecord(ready[c], st), "hipEventRecord(ready)");
        gdf_fused_local::Round* rd = nullptr;
        {
            std::unique_lock<std::mutex> lk(w->m);
            if (w->waiting.size() != (size_t)W) w->waiting.assign(W, {-1, -1, -1});
            const std::string crossed = check_arrival(W, R, c, k, issue, w->waiting);
            if (!crossed.empty()) {
                w->abort_locked(crossed);
                fail(GDF_ERR_STATE, crossed);
            }
            rd = &w->rounds[c][k];
            if (rd->posts.empty()) rd->posts.resize(W);
            rd->posts[R].ops = mine;
            rd->posts[R].ready = ready[c];
            rd->posts[R].done = done[c];
            rd->posts[R].issue = issue;
            ++rd->arrived;
            w->waiting[R] = {(int64_t)c, (int64_t)k, (int64_t)issue};
            w->cv.notify_all();
            w->wait(lk, [&] { return rd->arrived == W; }, "a collective");
            w->waiting[R] = {-1, -1, -1};
        }
        // (the posts are written before the barrier and only read after it: no lock needed)
        {
            std::vector<const std::vector<LocalOp>*> posts(W);
            std::vector<uint64_t> issues(W);
            for (int q = 0; q < W; ++q) {
                posts[q] = &rd->posts[q].ops;
                issues[q] = rd->posts[q].issue;
            }
            const std::string bad = check_round(W, posts, issues);
            if (!bad.empty()) {
                std::lock_guard<std::mutex> lk(w->m);
                w->abort_locked(bad);
                fail(GDF_ERR_STATE, bad);
            }
        }
        std::vector<char> waited(W, 0);
        auto behind = [&](int q) {
            if (!waited[q]) {
                hipchk(hipStreamWaitEvent(st, rd->posts[q].ready, 0), "hipStreamWaitEvent(ready)");
                waited[q] = 1;
            }
        };
        auto copy = [&](void* dst, const void* src, size_t bytes) {
            if (bytes && dst != src)
                hipchk(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, st), "hipMemcpyAsync(local)");
        };
        int ag = 0;  // the index of this all-gather among the round's all-gathers
        std::vector<int> nrecv(W, 0);  // receives from each peer so far
        for (const gdf_fused_local::Op& op : mine) {
            if (op.kind == 0) {
                for (int q = 0; q < W; ++q) {
                    const gdf_fused_local::Op* o = nth(rd->posts[q].ops, 0, -1, ag);
                    uint8_t* dst = static_cast<uint8_t*>(op.dst) + (size_t)q * op.bytes;
                    if (q != R) behind(q);
                    copy(dst, o->src, op.bytes);  // (in place: the own slice is already there)
                }
                ++ag;
            } else if (op.kind == 2) {  // (check_round matched every receive with its send)
                const int q = op.peer;
                const gdf_fused_local::Op* o = nth(rd->posts[q].ops, 1, R, nrecv[q]++);
                behind(q);
                copy(op.dst, o->src, op.bytes);
            }
        }
        hipchk(hipEventRecord(done[c], st), "hipEventRecord(done)");
        {
            std::unique_lock<std::mutex> lk(w->m);
            ++rd->copied;
            w->cv.notify_all();
            w->wait(lk, [&] { return rd->copied == W; }, "the end of a collective");
        }
        for (int q = 0; q < W; ++q)  // (nobody writes over a buffer another rank still reads)
            if (q != R) hipchk(hipStreamWaitEvent(st, rd->posts[q].done, 0), "hipStreamWaitEvent(done)");
        std::lock_guard<std::mutex> lk(w->m);
        if (++rd->left == W) w->rounds[c].erase(k);
    }
    // the n-th operation of `kind` (to `peer`, for sends) in a rank's list
    static const gdf_fused_local::Op* nth(const std::vector<gdf_fused_local::Op>& v, int kind, int peer, int n) {
        for (const gdf_fused_local::Op& o : v)
            if (o.kind == kind && (kind != 1 || o.peer == peer) && n-- == 0) return &o;
        return nullptr;
    }
};

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

constexpr uint32_t kSegMax = 4;   // partition segments per key range (gdf_set_partition_segments)
constexpr uint32_t kSrcMax = 32;  // sources of one voxelize (gdf_voxelize_runs_marked)

struct SlotX {
    DevBuf tail, tails;       // this rank's halo tails, every rank's (all-gather)
    DevBuf gathered;          // the union of the step's marks: frame f at f * W * S words, rank
                              // j's key range in words [j S, (j + 1) S) (voxelize + all-gather)
    // partitioned send lists (points, run keys, run starts) in buckets b = nseg part + segment
    // (segment 0: the rank's depth points, 1..: the pieces of the selected window it holds, in
    // order); the split sizes record [points per bucket (nseg W) | runs per bucket (nseg W)]
    // (cnt), every rank's (cntall), and
    DevBuf sp, srk, srs, cnt, cntall;
    DevBuf rp, rrk, rrs;      // received lists
    uint32_t* host = nullptr;  // pinned copy of cntall (world x 2 nseg world)
    // the rollbuffer sources in the selection's order: (rank, segment) per piece
    uint8_t piece_rank[kSrcMax] = {}, piece_seg[kSrcMax] = {};
    uint32_t npieces = 0;
    hipEvent_t ev = nullptr;
    bool pending = false;
    int average = 1;  // the step's voxel_average
    uint32_t nframes = 1, lifetime = 0;  // the step's batch and occupancy_lifetime
};

constexpr int kSlots = 4;  // the engine's pipeline depth is 1..4

}  // namespace

struct gdf_fused {
    gdf_engine* e = nullptr;
    std::unique_ptr<Transport> x;  // RCCL, or the in-process transport of a gdf_fused_local
    gdf_fused_local* local = nullptr;
    int rank = 0, world = 1;
    std::vector<gdf_stream_camera> cams;
    uint32_t F = 0, Lmax = 0;
    uint32_t shard_block = 0;  // > 0: the rollbuffer window sharded over the ranks
    // segments per key range: [depth | up to nseg - 1 pieces of the window per rank] (W nseg <= 32
    // buckets: 4 up to 8 ranks, 2 at 16)
    uint32_t nseg = 2;
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
        x.reset();
        if (local) {
            std::lock_guard<std::mutex> lk(local->m);
            --local->refs;
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
    // frames carrying the rollbuffer run one per step (the batched launch chain has no rollbuffer
    // frame: a silent drop would lose the window's points)
    if (B > 1 && p->move_transform_available)
        fail(GDF_ERR_ARG, "fused start: a move transform (rollbuffer frame) needs nframes == 1");
    gdf_engine* e = f->e;
    Transport& x = *f->x;
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
        x.all_gather(tail, S.tails.as(), B * L2, kHalo, st);
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
    // the rollbuffer: the last rank's, or every rank's shard of the window
    const bool sharded = f->shard_block > 0;
    if (!sharded && R != W - 1) q.move_transform_available = 0;
    const bool rb = B == 1 && q.move_transform_available;
    // the send lists, written by the compaction itself (gdf_set_emit_partition): sized for the
    // step's pixels (+ halo) plus, on a rollbuffer rank, every point the window can select
    const size_t rec = (size_t)2 * f->nseg * W;  // words of a rank's split-size record
    uint32_t* cnt = S.cnt.ensure<uint32_t>(rec * 4, st);
    uint32_t* cntall = S.cntall.ensure<uint32_t>(rec * W * 4, st);
    size_t want = (size_t)B * c.width * c.height + (halo && R > 0 ? B * (size_t)f->Lmax : 0u);
    if (rb) {  // + the window after the ingest
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
        // buckets [depth | rollbuffer pieces] per part: the record's layout itself (a frame without
        // a selection: the rollbuffer segments empty, written by the compaction)
        gdfchk(gdf_set_partition_segments(e, f->nseg));
    };
    arm(std::max<size_t>(want, 1));
    gdfchk(gdf_set_partition_marks(e, 0));
    gdf_frame_result res{};
    gdfchk(gdf_process_frame(e, &q, &res));
    // the rollbuffer sources in the selection's order (the same on every rank: the headers are
    // replicated): sharded, piece i of the window is the next segment of the rank holding it;
    // unsharded, segment 1 of every rank, only the last rank's non-empty
    S.npieces = 0;
    if (sharded && rb) {
        uint32_t owners[kSrcMax], n = 0, next[16] = {};
        gdfchk(gdf_get_rollbuffer_pieces(e, owners, kSrcMax, &n));
        if ((uint64_t)W + n > kSrcMax) fail(GDF_ERR_STATE, "fused start: more window pieces than sources");
        for (uint32_t i = 0; i < n; ++i) {
            const uint32_t q = owners[i];
            if (q >= (uint32_t)W || ++next[q] >= f->nseg)
                fail(GDF_ERR_STATE, "fused start: a rank holds more window pieces than segments");
            S.piece_rank[i] = (uint8_t)q;
            S.piece_seg[i] = (uint8_t)next[q];
        }
        S.npieces = n;
    } else {
        for (int q = 0; q < W; ++q) {
            S.piece_rank[q] = (uint8_t)q;
            S.piece_seg[q] = 1;
        }
        S.npieces = (uint32_t)W;
    }
    // The compaction sets no marks (gdf_set_partition_marks(e, 0) before the frame): W full
    // bitmasks of B frames (3.4 MB per rank and step at VGA x 8, received W - 1 times) would travel;
    // instead the key-range voxelize of the finish marks every voxel of its range - whole mark
    // words per range - and one in-place all-gather of those slices is the union (1 / W).
    S.nframes = B;
    S.lifetime = q.occupancy_lifetime;
    // every rank's split sizes (the partition's, written with the compaction) to pinned memory
    // (no wait here)
    // (world 1: the all-gather is the record itself)
    if (W > 1) x.all_gather(cnt, cntall, rec * 4, kHalo, st);
    hipchk(hipMemcpyAsync(S.host, W > 1 ? cntall : cnt, rec * W * 4, hipMemcpyDeviceToHost, st),
           "hipMemcpyAsync(counts)");
    hipchk(hipEventRecord(S.ev, st), "hipEventRecord");
    S.average = q.voxel_average ? 1 : 0;
    S.pending = true;
    *out_slot = slot;
}

void fused_finish(gdf_fused* f, int slot, uint32_t* send_counts, uint32_t* recv_count) {
    if (slot < 0 || slot >= kSlots) fail(GDF_ERR_ARG, "fused finish: bad slot");
    gdf_engine* e = f->e;
    Transport& x = *f->x;
    SlotX& S = f->slots[slot];
    if (!S.pending) fail(GDF_ERR_STATE, "fused finish: no step in flight on this slot");
    gdfchk(gdf_select_slot(e, slot));
    void* sv = nullptr;
    gdfchk(gdf_get_stream(e, &sv));
    hipStream_t st = static_cast<hipStream_t>(sv);
    hipchk(hipEventSynchronize(S.ev), "hipEventSynchronize");  // (the later slots keep the GPU busy)
    const int W = f->world, R = f->rank;
    // rank q's record: host[q * rec + nseg p + s] points of bucket (part p, segment s),
    // host[q * rec + nseg W + nseg p + s] its runs
    const uint32_t NSg = f->nseg;
    const size_t rec = (size_t)2 * NSg * W;
    auto pts_of = [&](int from, int to, uint32_t sg) -> uint64_t { return S.host[(size_t)from * rec + NSg * to + sg]; };
    auto runs_of = [&](int from, int to, uint32_t sg) -> uint64_t {
        return S.host[(size_t)from * rec + (size_t)NSg * W + NSg * to + sg];
    };
    // sources in the reference's buffer order: every rank's depth points (rank order = camera
    // order), then the rollbuffer pieces in the selection's order (fusion.cpp:1509-1581)
    const int NS = W + (int)S.npieces;
    if (NS > (int)kSrcMax) fail(GDF_ERR_STATE, "fused finish: too many sources");
    int src_rank[kSrcMax], src_seg[kSrcMax];
    for (int q = 0; q < W; ++q) {
        src_rank[q] = q;
        src_seg[q] = 0;
    }
    for (uint32_t i = 0; i < S.npieces; ++i) {
        src_rank[W + i] = S.piece_rank[i];
        src_seg[W + i] = S.piece_seg[i];
    }
    uint32_t pbase[kSrcMax + 1], rbase[kSrcMax + 1];
    uint64_t n = 0, nr = 0;
    uint64_t recv_at[16][kSegMax] = {}, rrecv_at[16][kSegMax] = {};  // where rank q's segment s lands
    for (int k = 0; k < NS; ++k) {
        const int q = src_rank[k], sg = src_seg[k];
        if (q < 0 || q >= W || sg < 0 || sg >= (int)NSg) fail(GDF_ERR_STATE, "fused finish: bad rollbuffer piece");
        pbase[k] = (uint32_t)n;
        rbase[k] = (uint32_t)nr;
        recv_at[q][sg] = n;
        rrecv_at[q][sg] = nr;
        n += pts_of(q, R, sg);
        nr += runs_of(q, R, sg);
        if (n >= 0xFFFFFFFFull) fail(GDF_ERR_CAPACITY, "fused finish: 2^32 points received");
    }
    pbase[NS] = (uint32_t)n;
    rbase[NS] = (uint32_t)nr;
    // every bucket that carries points is a source (a rank's pieces are exactly its non-empty
    // rollbuffer segments)
    for (int q = 0; q < W; ++q)
        for (uint32_t sg = 1; sg < NSg; ++sg) {
            bool listed = false;
            for (int k = W; k < NS; ++k) listed |= src_rank[k] == q && src_seg[k] == (int)sg;
            if (!listed && pts_of(q, R, sg)) fail(GDF_ERR_STATE, "fused finish: a rollbuffer bucket outside the pieces");
        }
    float* rp = S.rp.ensure<float>(std::max<uint64_t>(n, 1) * 16, st);
    uint32_t* rrk = S.rrk.ensure<uint32_t>(std::max<uint64_t>(nr, 1) * 4, st);
    uint32_t* rrs = S.rrs.ensure<uint32_t>((nr + 1) * 4, st);
    // this rank's send list: bucket-major, bucket (q, s) at the sum of the buckets before it
    uint64_t send_at[16][kSegMax] = {}, rsend_at[16][kSegMax] = {};
    {
        uint64_t o = 0, ro = 0;
        for (int q = 0; q < W; ++q)
            for (uint32_t sg = 0; sg < NSg; ++sg) {
                send_at[q][sg] = o;
                rsend_at[q][sg] = ro;
                o += pts_of(R, q, sg);
                ro += runs_of(R, q, sg);
            }
    }
    // the rank's own buckets stay in its send lists: the voxelize's rebase pass reads them there
    // (gdf_voxelize_runs_recv; an RCCL self send / recv would be a kernel copy, a device copy a
    // launch each)
    gdf_recv_own own{};
    for (int k = 0; k < NS; ++k) {
        if (src_rank[k] != R) continue;
        const int sg = src_seg[k];
        if (own.count >= 4) fail(GDF_ERR_STATE, "fused finish: more than 4 own buckets");
        own.source[own.count] = (uint32_t)k;
        own.points[own.count] = S.sp.as<float>() + 4 * send_at[R][sg];
        own.run_keys[own.count] = S.srk.as<uint32_t>() + rsend_at[R][sg];
        own.run_starts[own.count] = S.srs.as<uint32_t>() + rsend_at[R][sg];
        ++own.count;
    }
    if (W > 1) {
        x.group_start(kPoints);
        for (int q = 0; q < W; ++q) {
            if (q == R) continue;
            for (uint32_t sg = 0; sg < NSg; ++sg) {  // (per peer, in the same order on both sides)
                const size_t sc = pts_of(R, q, sg), sr = runs_of(R, q, sg);
                if (sc) {
                    x.send(S.sp.as<float>() + 4 * send_at[q][sg], 16 * sc, q, kPoints, st);
                    x.send(S.srk.as<uint32_t>() + rsend_at[q][sg], 4 * sr, q, kPoints, st);
                    x.send(S.srs.as<uint32_t>() + rsend_at[q][sg], 4 * sr, q, kPoints, st);
                }
                const size_t rc = pts_of(q, R, sg), rr = runs_of(q, R, sg);
                if (rc) {
                    x.recv(rp + 4 * recv_at[q][sg], 16 * rc, q, kPoints, st);
                    x.recv(rrk + rrecv_at[q][sg], 4 * rr, q, kPoints, st);
                    x.recv(rrs + rrecv_at[q][sg], 4 * rr, q, kPoints, st);
                }
            }
        }
        x.group_end(kPoints, st);
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
    // (only slice R of each frame is cleared - by the rebase pass: the voxelize marks inside its
    // key range, the all-gather overwrites the other slices)
    own.clear = uni + (uint64_t)R * Sw;
    own.clear_row_words = Sw;
    own.clear_stride_words = stride;
    own.clear_rows = S.nframes;
    gdfchk(gdf_voxelize_runs_recv(e, rp, rrk, rrs, (uint32_t)NS, pbase, rbase, S.average, uni, stride,
                                  &own));
    if (W > 1) {  // (on the points' communicator: the finish's collectives stay in step order,
                  // never behind the next step's start collectives on the halo communicator)
        x.group_start(kPoints);
        for (uint32_t j = 0; j < S.nframes; ++j)
            x.all_gather(uni + j * stride + (uint64_t)R * Sw, uni + j * stride, Sw * 4, kPoints, st);
        x.group_end(kPoints, st);
    }
    gdfchk(gdf_voxel_occupancy_grid_batch(e, uni, words, 1, S.nframes, stride, S.nframes * stride,
                                          S.lifetime));
    if (send_counts)
        for (int q = 0; q < W; ++q) {
            uint64_t c = 0;
            for (uint32_t sg = 0; sg < NSg; ++sg) c += pts_of(R, q, sg);
            send_counts[q] = (uint32_t)c;
        }
    if (recv_count) *recv_count = (uint32_t)n;
    S.pending = false;
}

}  // namespace

namespace {

// the state every transport shares: cameras, halo size, per-slot pinned split sizes and events
gdf_fused* fused_new(gdf_engine* engine, int rank, int world, const gdf_stream_camera* cams,
                     uint32_t flying_filter_size) {
    std::unique_ptr<gdf_fused> f(new gdf_fused());
    f->rank = rank;
    f->world = world;
    f->cams.assign(cams, cams + world);
    f->F = flying_filter_size;
    f->nseg = std::max<uint32_t>(2u, std::min<uint32_t>(kSegMax, 32u / (uint32_t)world));
    for (const gdf_stream_camera& c : f->cams)
        f->Lmax = std::max<uint32_t>(f->Lmax, f->F * c.width + f->F);
    for (const gdf_stream_camera& c : f->cams)
        if ((uint64_t)c.width * c.height < f->Lmax)
            fail(GDF_ERR_ARG, "fused multi-GPU frames need cameras taller than F rows");
    for (SlotX& s : f->slots) {
        hipchk(hipHostMalloc(reinterpret_cast<void**>(&s.host), (size_t)2 * f->nseg * world * world * 4,
                             hipHostMallocDefault), "hipHostMalloc");
        hipchk(hipEventCreateWithFlags(&s.ev, hipEventDisableTiming), "hipEventCreate");
    }
    f->e = engine;  // (set last: the destructor of a half-made rank leaves the engine alone)
    return f.release();
}

bool create_args_ok(gdf_engine* engine, const gdf_stream_camera* cams, gdf_fused** out, int rank,
                    int world) {
    if (!engine || !cams || !out || world < 1 || world > 16 || rank < 0 || rank >= world) {
        gdf::set_last_error("fused create: engine, cameras, 0 <= rank < world <= 16");
        return false;
    }
    *out = nullptr;
    return true;
}

// ANY failed step aborts the in-process world, so the other ranks' threads fail at once instead of
// waiting for this rank in a collective it will never issue (an argument error on ONE rank - its
// peers already wait in the step's first round - is a failure of the world like any other; RCCL
// ranks cannot be told, and their communicators stay usable only if every rank fails alike).
template <class F>
int step_guarded(gdf_fused* f, F&& fn) {
    const int rc = guarded(fn);
    if (rc != GDF_OK && f->x) f->x->abort();
    return rc;
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
    if (!id || !create_args_ok(engine, cams, out, rank, world)) {
        if (!id) gdf::set_last_error("fused create: null communicator ids");
        return GDF_ERR_ARG;
    }
    gdf_fused* f = nullptr;
    const int rc = guarded([&] {
        const Rccl& r = rccl(rccl_library);
        f = fused_new(engine, rank, world, cams, flying_filter_size);
        std::unique_ptr<RcclTransport> t(new RcclTransport());
        t->r = &r;
        t->world = world;
        ncclUniqueId a, b;
        std::memcpy(&a, id, sizeof(a));
        std::memcpy(&b, id + sizeof(a), sizeof(b));
        ncclchk(r, r.comm_init_rank(&t->comm[kHalo], world, a, rank), "ncclCommInitRank(halo)");
        ncclchk(r, r.comm_init_rank(&t->comm[kPoints], world, b, rank), "ncclCommInitRank(points)");
        f->x = std::move(t);
    });
    if (rc != GDF_OK) {
        delete f;
        return rc;
    }
    *out = f;
    return GDF_OK;
}

int gdf_fused_local_create(int world, gdf_fused_local** out) {
    if (!out || world < 1 || world > 16) {
        gdf::set_last_error("fused local world: 1 <= world <= 16");
        return GDF_ERR_ARG;
    }
    *out = nullptr;
    return guarded([&] {
        gdf_fused_local* w = new gdf_fused_local();
        w->world = world;
        if (const char* v = std::getenv("GDF_LOCAL_TIMEOUT_S")) w->timeout_s = std::atof(v);
        *out = w;
    });
}

int gdf_fused_local_check_round(int world, const gdf_local_op* ops, const uint32_t* nops,
                                const uint64_t* issue) {
    if (world < 1 || world > 16 || !nops || !issue) {
        gdf::set_last_error("local check: 1 <= world <= 16, nops and issue");
        return GDF_ERR_ARG;
    }
    std::vector<std::vector<LocalOp>> lists(world);
    std::vector<const std::vector<LocalOp>*> posts(world);
    size_t at = 0;
    for (int q = 0; q < world; ++q) {
        for (uint32_t j = 0; j < nops[q]; ++j, ++at)
            lists[q].push_back({ops[at].kind, ops[at].src, ops[at].dst, (size_t)ops[at].bytes, ops[at].peer});
        posts[q] = &lists[q];
    }
    const std::string bad = check_round(world, posts, std::vector<uint64_t>(issue, issue + world));
    if (bad.empty()) return GDF_OK;
    gdf::set_last_error(bad);
    return GDF_ERR_STATE;
}

int gdf_fused_local_check_arrival(int world, int rank, int comm, uint64_t round, uint64_t issue,
                                  const int64_t* waiting) {
    if (world < 1 || world > 16 || rank < 0 || rank >= world || comm < 0 || comm > 1 || !waiting) {
        gdf::set_last_error("local check: 0 <= rank < world <= 16, comm 0 / 1, waiting");
        return GDF_ERR_ARG;
    }
    std::vector<std::array<int64_t, 3>> wt(world);
    for (int q = 0; q < world; ++q) wt[q] = {waiting[3 * q], waiting[3 * q + 1], waiting[3 * q + 2]};
    const std::string bad = check_arrival(world, rank, comm, round, issue, wt);
    if (bad.empty()) return GDF_OK;
    gdf::set_last_error(bad);
    return GDF_ERR_STATE;
}

int gdf_fused_local_destroy(gdf_fused_local* w) {
    if (!w) return GDF_OK;
    {
        std::lock_guard<std::mutex> lk(w->m);
        if (w->refs) {
            gdf::set_last_error("fused local world: destroy its ranks first");
            return GDF_ERR_STATE;
        }
    }
    delete w;
    return GDF_OK;
}

int gdf_fused_create_local(gdf_engine* engine, gdf_fused_local* w, int rank, int world,
                           const gdf_stream_camera* cams, uint32_t flying_filter_size,
                           gdf_fused** out) {
    if (!w || !create_args_ok(engine, cams, out, rank, world)) {
        if (!w) gdf::set_last_error("fused create: null local world");
        return GDF_ERR_ARG;
    }
    if (world != w->world) {
        gdf::set_last_error("fused create: world differs from the local world's");
        return GDF_ERR_ARG;
    }
    gdf_fused* f = nullptr;
    const int rc = guarded([&] {
        f = fused_new(engine, rank, world, cams, flying_filter_size);
        f->x.reset(new LocalTransport(w, rank));
        std::lock_guard<std::mutex> lk(w->m);
        ++w->refs;
        f->local = w;
    });
    if (rc != GDF_OK) {
        delete f;
        return rc;
    }
    *out = f;
    return GDF_OK;
}

int gdf_fused_info(gdf_fused* f, int* rank, int* world, int* transport_ranks, const char** transport) {
    if (!f) return GDF_ERR_ARG;
    if (rank) *rank = f->rank;
    if (world) *world = f->world;
    if (transport_ranks) *transport_ranks = f->x ? f->x->ranks() : -1;
    if (transport) *transport = f->x ? f->x->kind() : "none";
    return GDF_OK;
}

int gdf_fused_destroy(gdf_fused* f) {
    delete f;
    return GDF_OK;
}

int gdf_fused_set_rollbuffer_shard(gdf_fused* f, uint32_t block) {
    if (!f) return GDF_ERR_ARG;
    return guarded([&] {
        gdfchk(gdf_set_rollbuffer_shard(f->e, block ? (uint32_t)f->rank : 0u,
                                        block ? (uint32_t)f->world : 1u, block ? block : 1u));
        f->shard_block = block;
    });
}

int gdf_fused_halo_pixels(gdf_fused* f, uint32_t* pixels) {
    if (!f || !pixels) return GDF_ERR_ARG;
    *pixels = f->Lmax;
    return GDF_OK;
}

int gdf_fused_start(gdf_fused* f, const uint16_t* const* depth, uint32_t nframes,
                    const gdf_frame_params* p, int* slot) {
    if (!f || !slot) return GDF_ERR_ARG;
    return step_guarded(f, [&] { fused_start(f, depth, nframes, p, slot); });
}

int gdf_fused_finish(gdf_fused* f, int slot, uint32_t* send_counts, uint32_t* recv_count) {
    if (!f) return GDF_ERR_ARG;
    return step_guarded(f, [&] { fused_finish(f, slot, send_counts, recv_count); });
}

int gdf_fused_run(gdf_fused* f, const gdf_stream_camera* cam, const gdf_frame_params* p,
                  uint64_t first, uint64_t steps, uint32_t batch, int depth) {
    if (!f || !cam || !p || !cam->frames || cam->ring == 0 || batch == 0 || batch > 16 ||
        depth < 1 || depth > kSlots)
        return GDF_ERR_ARG;
    return step_guarded(f, [&] {
        gdfchk(gdf_set_pipeline_depth(f->e, depth));
        std::deque<int> pending;
        const uint16_t* ptrs[16];
        for (uint64_t s = 0; s < steps; ++s) {
            for (uint32_t j = 0; j < batch; ++j) ptrs[j] = cam->frames[((first + s) * batch + j) % cam->ring];
            int slot = 0;
            fused_start(f, ptrs, batch, p, &slot);
            pending.push_back(slot);
            // `depth` steps in flight: the oldest is finished once the newest is queued (the GPU
            // computes the later steps while the host waits for the oldest one's split sizes),
            // and its slot is free again before the engine hands it out
            if ((int)pending.size() >= depth) {
                fused_finish(f, pending.front(), nullptr, nullptr);
                pending.pop_front();
            }
        }
        for (int k : pending) fused_finish(f, k, nullptr, nullptr);
    });
}

}  // extern "C"
