/* gdf_fused.h — one rank of the multi-GPU fused cloud, the whole step in C++ over RCCL.
 *
 * Not a reference interface: the reference fuses every camera in ONE process
 * (GPUDepthmapFusion::processFrame over all depth maps, src/gpu_depthmap_fusion.cpp:1583-1756;
 * the buffer order [camera 0 .. camera N-1 pixels, rollbuffer points] at :1509-1581, one voxelize
 * at :1743-1756).  Here each rank (one process per GPU) holds one camera; a step is
 *   depth-tail halo all-gather (camera k reads camera k-1's last F rows + F pixels)
 *   -> the rank's compaction + voxel keys (gdf_process_frame, deferred)
 *   -> key-range partition (buckets [depth | rollbuffer] per range) -> split-size all-gather
 *   -> (finish) the points / runs all-to-all as grouped send / recv -> voxelize of the rank's key
 *      range (gdf_voxelize_runs_marked) -> mark-slice all-gather -> batched grid update,
 * with the collectives issued by this library on the engine slot's stream through RCCL
 * (dlopen'ed: the caller names the librccl it already loaded - torch's - so one RCCL serves the
 * process).  Everything runs through the public C-ABI of include/gdf.h; the Python
 * FusedCloudRank (ros_gpu_depthmap_fusion_amd/multi.py) is the same protocol with torch
 * collectives and is the one the gloo CPU tests drive.
 *
 * Two communicators: A carries the halo tails / split sizes (the start), B the points, runs and
 * mark slices (the finish).  Operations on one communicator run in issue order, so B's exchange of
 * step i never queues behind step i + 1's collectives on A (the step is pipelined: start(i + 1) is
 * issued before finish(i)).  The collectives go through a transport: RCCL (gdf_fused_create) or
 * the in-process one below (gdf_fused_create_local).
 */
#ifndef GDF_FUSED_H
#define GDF_FUSED_H

#include "gdf.h"
#include "gdf_driver.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gdf_fused gdf_fused;

#define GDF_FUSED_ID_BYTES 256 /* two ncclUniqueId (communicators A and B) */

/* Rank 0: the unique ids of the two communicators (GDF_FUSED_ID_BYTES bytes), to be broadcast to
 * every rank before gdf_fused_create.  rccl_library: path of librccl.so (NULL: the one on the
 * loader path). */
int gdf_fused_unique_id(const char* rccl_library, uint8_t* id_out);

/* Collective over the `world` ranks: creates the communicators on the engine's device and the
 * per-slot exchange state.  cams[k] = camera k's geometry (width, height, intrinsics, T_world,
 * T_crop; `frames`/`ring` unused) for k < world - this rank's camera is cams[rank].
 * flying_filter_size sets the halo (F rows + F pixels of camera k-1).  The engine keeps its own
 * slot streams and must outlive the rank (gdf_fused_destroy first). */
int gdf_fused_create(gdf_engine* engine, const char* rccl_library, const uint8_t* id, int rank,
                     int world, const gdf_stream_camera* cams, uint32_t flying_filter_size,
                     gdf_fused** out);
int gdf_fused_destroy(gdf_fused* rank);

/* In-process transport: `world` ranks of ONE process - one host thread and one engine each, on one
 * device or several - with the step's collectives as device-to-device copies on the ranks' own
 * streams (matched in issue order like RCCL's; the host only waits for every rank to ISSUE a
 * collective, never for the GPU).  The same gdf_fused_start / finish / run as the RCCL ranks: this
 * is how the multi-rank C++ step runs (and is tested) on a node with fewer GPUs than ranks, where
 * RCCL refuses two ranks on one device.  A rank whose step fails - for any reason, a bad argument
 * on that rank alone included - aborts the world: the other ranks' pending and later collectives
 * fail with GDF_ERR_STATE at once instead of waiting (so does a rank left waiting longer than
 * GDF_LOCAL_TIMEOUT_S seconds, default 300).  Every round's schedule is checked on every rank
 * before any copy (gdf_fused_local_check_round / _check_arrival below): what RCCL would hang on
 * or corrupt fails here.  Destroy every rank (gdf_fused_destroy) before the world. */
typedef struct gdf_fused_local gdf_fused_local;
int gdf_fused_local_create(int world, gdf_fused_local** out);
int gdf_fused_local_destroy(gdf_fused_local* world);
/* Diagnostics of the in-process transport's schedule checks (what a round of it verifies before
 * any copy; no device work).  gdf_fused_local_check_round: one round, rank q's operations are
 * ops[sum(nops[0..q)) .. + nops[q]) in its issue order (kind 0 all-gather: src = its send buffer,
 * dst = its receive buffer of world * bytes; 1 send to `peer` from src; 2 receive from `peer` into
 * dst), issue[q] = the round's number in rank q's issue order over both communicators.  Fails
 * (GDF_ERR_STATE, gdf_last_error names it) on a send no receive consumes, a receive without its
 * send, differing sizes, a bad peer, an all-gather send buffer overlapping its receive buffer
 * other than at recv + rank * bytes, or issue numbers that differ across the ranks.
 * gdf_fused_local_check_arrival: rank `rank` arrives in round `round` of communicator `comm`
 * (0 halo, 1 points) as its collective #issue while waiting[3q .. 3q + 2] = {comm, round, issue}
 * of the round rank q is blocked in (comm -1: not blocked); fails when another rank waits in a
 * different round under the same number (the two-communicator deadlock). */
typedef struct gdf_local_op {
    int kind;
    const void* src;
    void* dst;
    uint64_t bytes;
    int peer;
} gdf_local_op;
int gdf_fused_local_check_round(int world, const gdf_local_op* ops, const uint32_t* nops,
                                const uint64_t* issue);
int gdf_fused_local_check_arrival(int world, int rank, int comm, uint64_t round, uint64_t issue,
                                  const int64_t* waiting);
/* Not collective (no rendezvous): creates rank `rank` of the local world on `engine`; cams and
 * flying_filter_size as for gdf_fused_create. */
int gdf_fused_create_local(gdf_engine* engine, gdf_fused_local* world, int rank, int nranks,
                           const gdf_stream_camera* cams, uint32_t flying_filter_size,
                           gdf_fused** out);

/* The rank, its world, the rank count its transport reports (RCCL: ncclCommCount of the points'
 * communicator) and the transport's name ("rccl" / "local"; a static string). */
int gdf_fused_info(gdf_fused* rank, int* rank_out, int* world, int* transport_ranks,
                   const char** transport);

/* The rollbuffer window sharded over the ranks (block > 0; 0 = the last rank holds it, SURVEY
 * 8(e)): every rank is given EVERY point sequence (gdf_add_point_sequence[_device] on each
 * engine, same order) and keeps the points of the sequences k with (k / block) % world == rank
 * (gdf_set_rollbuffer_shard); a rollbuffer step (nframes == 1, move transform) then selects, on
 * every rank, its share of the window, and the exchange carries two buckets per key range - the
 * rank's depth points, then the pieces of the window it holds (a piece: a stretch of selected
 * sequences on one rank; gdf_get_rollbuffer_pieces) - which each owner places as [every rank's
 * depth points, the pieces in the selection's order] (the reference's buffer, fusion.cpp
 * :1509-1581, restricted to the key range).  A window spanning at most `world` blocks gives one
 * piece per rank (block = ceil((window - 1) / (world - 1)) sequences guarantees it); a longer one
 * (a burst of sequences) gives a rank several, up to min(3, 32 / world - 1) - beyond that the step
 * fails on every rank alike (GDF_ERR_STATE), before any rank's points move.  Call before the
 * first sequence is added. */
int gdf_fused_set_rollbuffer_shard(gdf_fused* rank, uint32_t block);

/* Depth values of the halo every rank sends (max over cameras of F * width + F). */
int gdf_fused_halo_pixels(gdf_fused* rank, uint32_t* pixels);

/* Starts a step of `nframes` frames (1..16) of this rank's camera - depth[j] = frame j's DEVICE
 * depth map - on the engine's next slot: everything up to the split sizes (queued to pinned
 * memory, no wait).  p: the frame's parameters (its defer / synchronous flags are overridden; a
 * move transform - rollbuffer rank, single frames - is honoured as by gdf_process_frame; with
 * nframes > 1 it is GDF_ERR_ARG: a batch carries no rollbuffer frame).
 * Point sequences added to the engine beforehand are ingested by this step.  *slot = the slot to
 * pass to gdf_fused_finish. */
int gdf_fused_start(gdf_fused* rank, const uint16_t* const* depth, uint32_t nframes,
                    const gdf_frame_params* p, int* slot);
/* Finishes the step started on `slot`: waits for its split sizes, runs the points all-to-all and
 * the voxelize of the rank's key range (gdf_select_slot(slot) is left selected: the rank's voxels
 * are that slot's results).  send_counts (world entries, may be NULL): points sent to each rank;
 * recv_count (may be NULL): points received. */
int gdf_fused_finish(gdf_fused* rank, int slot, uint32_t* send_counts, uint32_t* recv_count);

/* `steps` pipelined steps of `batch` frames of this rank's camera from cam->frames (step s takes
 * frames (first + s) * batch + j, modulo the ring): up to `depth` steps in flight (the engine's
 * pipeline depth is set to it) - step s - depth + 1 is finished right after step s started.  Returns
 * after the last step was finished (its work still queued: gdf_synchronize waits). */
int gdf_fused_run(gdf_fused* rank, const gdf_stream_camera* cam, const gdf_frame_params* p,
                  uint64_t first, uint64_t steps, uint32_t batch, int depth);

#ifdef __cplusplus
}
#endif

#endif /* GDF_FUSED_H */
