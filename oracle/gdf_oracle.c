/*
 * gdf_oracle.c — CPU restatement of the reference depth-fusion hot path (TEST INFRASTRUCTURE).
 *
 * See gdf_oracle.h for scope, pinning status and the floating-point contract.  Every function
 * cites the reference file:line it restates (paths relative to the reference root):
 *   fusion.cpp = src/gpu_depthmap_fusion.cpp, comp.cpp = src/gpu_depthmap_fusion_component.cpp,
 *   sh/        = shader/.
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off -fno-fast-math [-fopenmp]).
 */
#include "gdf_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

#define ORC_MAX_CAMS 64

typedef struct {
    uint32_t sec, nsec, start, num_points;
    float T_move[16];
} orc_seq; /* PointSequence, gpu_depthmap_fusion.h:178-204 (padding omitted) */

typedef struct {
    uint32_t total;
    orc_seq* seqs;
    uint32_t nseq, cap_seq;
    float* pts;
    size_t cap_pts;
} orc_psbuf; /* PointSequences, gpu_depthmap_fusion.h:206-217 */

typedef struct {
    const uint16_t* depth;
    uint32_t W, H, n;
    float scale, fx, fy, cx, cy;
    float Tw[16], Tc[16];
} orc_cam; /* DepthmapConversion, gpu_depthmap_fusion.h:163-176 */

struct orc_state {
    int nthreads;
    orc_cam cams[ORC_MAX_CAMS];
    int ncams;
    uint32_t depth_total;           /* m_depthmapsTotalElements */
    uint16_t* depth_up;             /* m_bufDepthPairs (as u16) */
    size_t cap_depth_up;
    uint32_t cam_off[ORC_MAX_CAMS];

    orc_psbuf psA, psB;
    orc_psbuf *collect, *upload;

    /* m_bufNewPointSequencesPoints / MaskA / MaskB / m_bufNewPointSequences */
    float* new_pts;
    uint32_t n_new;
    orc_seq* new_seqs;
    uint32_t s_new;
    uint32_t *new_maskA, *new_maskB;
    int new_filtered;

    /* rollbuffer A (after insert) and B (after roll), fusion.h:402-411 */
    float *hA_pts, *hB_pts;
    uint32_t *hA_mask, *hB_mask, *hA_seq, *hB_seq;
    orc_seq *hA_seqs, *hB_seqs;
    uint32_t hA_n, hA_s, hB_n, hB_s; /* logical sizes (StorageBuffer::size()) */

    uint32_t rb_pts, rb_seqs, sel_pt_start, sel_pt_count, sel_seq_start, sel_seq_count;
    uint32_t earliest_sec, earliest_nsec, last_sec, last_nsec;

    /* per-frame buffers of n = depth + selected points, fusion.h:389-395 */
    uint32_t n;
    float *A, *B, *C;
    uint32_t *maskA, *maskB;
    uint32_t* tf_idx;
    float *tfw, *tfc;

    uint32_t num_after_mask;        /* m_numItemsAfterMask */
    uint32_t* coords;               /* m_voxelCoords */
    int grid_set;
    float lb[3], ub[3], cs[3];
    uint32_t gs[3];
    uint64_t ncells;

    uint32_t *hist, *histB, *occ;   /* m_bufHistoricVoxelOccupancyA/B, m_bufVoxelOccupancyA */
    uint8_t* out8;                  /* m_bufVoxelOccupancyB / m_occupancyGrid */
    uint64_t hist_cells;
    int invoked_once;

    float* vox;                     /* m_points_voxelized */
    uint32_t nvox;
};

/* ------------------------------------------------------------------------------------------ */
static void* xrealloc(void* p, size_t bytes) {
    void* q = realloc(p, bytes ? bytes : 1);
    return q;
}

static void psbuf_clear(orc_psbuf* b) { b->total = 0; b->nseq = 0; }

orc_state* orc_create(void) {
    orc_state* s = (orc_state*)calloc(1, sizeof(orc_state));
    if (!s) return NULL;
    s->nthreads = 1;
    s->collect = &s->psA; /* fusion.cpp:19-20 */
    s->upload = &s->psB;
    return s;
}

static void psbuf_free(orc_psbuf* b) { free(b->seqs); free(b->pts); }

void orc_destroy(orc_state* s) {
    if (!s) return;
    psbuf_free(&s->psA); psbuf_free(&s->psB);
    free(s->depth_up);
    free(s->new_pts); free(s->new_seqs); free(s->new_maskA); free(s->new_maskB);
    free(s->hA_pts); free(s->hB_pts); free(s->hA_mask); free(s->hB_mask);
    free(s->hA_seq); free(s->hB_seq); free(s->hA_seqs); free(s->hB_seqs);
    free(s->A); free(s->B); free(s->C); free(s->maskA); free(s->maskB);
    free(s->tf_idx); free(s->tfw); free(s->tfc); free(s->coords);
    free(s->hist); free(s->histB); free(s->occ); free(s->out8); free(s->vox);
    free(s);
}

void orc_set_threads(orc_state* s, int nthreads) { s->nthreads = nthreads > 0 ? nthreads : 1; }

/* ---- canonical float helpers ---------------------------- */
/* out = M·p for row-major M: ((m0·x + m1·y) + m2·z) + m3·w per row (GLSL `p * M` with the
 * transpose=false upload, inc/program_uniform.h:197-209). */
static inline void mat_vec(const float* M, const float* p, float* o) {
    for (int r = 0; r < 4; ++r) {
        const float* m = M + 4 * r;
        o[r] = ((m[0] * p[0] + m[1] * p[1]) + m[2] * p[2]) + m[3] * p[3];
    }
}

/* R = A·B (row-major), ((a0·b0 + a1·b1) + a2·b2) + a3·b3 per element. */
static inline void mat_mul(const float* A, const float* B, float* R) {
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c)
            R[4 * r + c] = ((A[4 * r + 0] * B[0 * 4 + c] + A[4 * r + 1] * B[1 * 4 + c]) +
                            A[4 * r + 2] * B[2 * 4 + c]) + A[4 * r + 3] * B[3 * 4 + c];
}

static inline float dot3(const float* a, const float* b) {
    return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2];
}
static inline float length3(const float* a) { return sqrtf(dot3(a, a)); }
/* GLSL normalize(x) = x / length(x) */
static inline void normalize3(const float* a, float* o) {
    float l = length3(a);
    o[0] = a[0] / l; o[1] = a[1] / l; o[2] = a[2] / l;
}
static inline void cross3(const float* a, const float* b, float* o) {
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}

/* ---- frame inputs ------------------------------------------------------------------------ */
/* clear(), fusion.cpp:725-732 */
void orc_clear(orc_state* s) {
    s->sel_pt_count = 0;
    s->sel_seq_count = 0;
    s->depth_total = 0;
    s->ncams = 0;
}

/* addDepthmap(), fusion.cpp:798-816 (pointer borrowed until upload) */
int orc_add_depthmap(orc_state* s, const uint16_t* depth, uint32_t width, uint32_t height,
                     float depth_scale, float fx, float fy, float cx, float cy,
                     const float T_world[16], const float T_crop[16]) {
    if (s->ncams >= ORC_MAX_CAMS || !depth || !T_world || !T_crop) return -1;
    orc_cam* c = &s->cams[s->ncams++];
    c->depth = depth; c->W = width; c->H = height; c->n = width * height;
    c->scale = depth_scale; c->fx = fx; c->fy = fy; c->cx = cx; c->cy = cy;
    memcpy(c->Tw, T_world, sizeof(c->Tw));
    memcpy(c->Tc, T_crop, sizeof(c->Tc));
    s->depth_total += c->n;
    return 0;
}

/* addPointSequence(), fusion.cpp:747-796: x,y,z at byte offsets 0/4/8 of each record, w = 1 */
int orc_add_point_sequence(orc_state* s, const void* records, uint32_t num_points,
                           uint32_t point_step, uint32_t sec, uint32_t nsec,
                           const float T_move[16]) {
    orc_psbuf* b = s->collect;
    if (num_points && (!records || point_step < 12)) return -1;
    if (b->nseq == b->cap_seq) {
        b->cap_seq = b->cap_seq ? 2 * b->cap_seq : 16;
        b->seqs = (orc_seq*)xrealloc(b->seqs, b->cap_seq * sizeof(orc_seq));
    }
    orc_seq* q = &b->seqs[b->nseq++];
    q->sec = sec; q->nsec = nsec; q->start = b->total; q->num_points = num_points;
    memcpy(q->T_move, T_move, sizeof(q->T_move));
    size_t need = (size_t)(b->total + num_points) * 4;
    if (need > b->cap_pts) {
        size_t cap = b->cap_pts ? b->cap_pts : 1024;
        while (cap < need) cap *= 2;
        b->pts = (float*)xrealloc(b->pts, cap * sizeof(float));
        b->cap_pts = cap;
    }
    const uint8_t* rec = (const uint8_t*)records;
    for (uint32_t k = 0; k < num_points; ++k) {
        float* o = b->pts + 4 * ((size_t)q->start + k);
        memcpy(&o[0], rec + (size_t)k * point_step + 0, 4);
        memcpy(&o[1], rec + (size_t)k * point_step + 4, 4);
        memcpy(&o[2], rec + (size_t)k * point_step + 8, 4);
        o[3] = 1.0f;
    }
    b->total += num_points;
    return 0;
}

uint32_t orc_num_collected_point_sequence_points(orc_state* s) { return s->collect->total; }

/* ---- point-sequence chain ------------------------------------------------------------------ */
/* uploadPointSequences(), fusion.cpp:819-857 (swapPointSequencesBuffers :734-746) */
int orc_upload_point_sequences(orc_state* s) {
    if (s->collect == &s->psA) { s->upload = &s->psA; s->collect = &s->psB; }
    else { s->collect = &s->psA; s->upload = &s->psB; }
    psbuf_clear(s->collect);
    orc_psbuf* u = s->upload;
    s->n_new = u->total;
    s->s_new = u->nseq;
    s->new_pts = (float*)xrealloc(s->new_pts, (size_t)s->n_new * 4 * sizeof(float));
    if (s->n_new) memcpy(s->new_pts, u->pts, (size_t)s->n_new * 4 * sizeof(float));
    s->new_seqs = (orc_seq*)xrealloc(s->new_seqs, (size_t)s->s_new * sizeof(orc_seq));
    if (s->s_new) memcpy(s->new_seqs, u->seqs, (size_t)s->s_new * sizeof(orc_seq));
    s->new_maskA = (uint32_t*)xrealloc(s->new_maskA, (size_t)s->n_new * 4);
    s->new_maskB = (uint32_t*)xrealloc(s->new_maskB, (size_t)s->n_new * 4);
    s->new_filtered = 0;
    return 0;
}

/* sh/filter_point_sequence.glsl:49-76 (filter_flying_pixels helper) */
static int ps_neighbor_ok(const float* pts, const float* p, uint32_t other, float thr) {
    const float* q = pts + 4 * (size_t)other;
    float d[3] = {q[0] - p[0], q[1] - p[1], q[2] - p[2]};
    float dir[3], np[3], nn[3];
    normalize3(d, dir);
    normalize3(p, np);
    nn[0] = -np[0]; nn[1] = -np[1]; nn[2] = -np[2];
    float c = fabsf(dot3(dir, nn));
    if (1.0f - c < thr) return 0;
    return 1;
}

/* filterNewPointSequences(), fusion.cpp:928-976: set_uints(maskA=1) then
 * sh/filter_point_sequence.glsl:78-122 over all new points as one array */
int orc_filter_new_point_sequences(orc_state* s, float threshold, uint32_t filter_size) {
    uint32_t n = s->n_new;
    for (uint32_t i = 0; i < n; ++i) s->new_maskA[i] = 1;
    #pragma omp parallel for num_threads(s->nthreads) schedule(static)
    for (int64_t gi = 0; gi < (int64_t)n; ++gi) {
        uint32_t g = (uint32_t)gi;
        uint32_t mv = s->new_maskA[g];
        if (mv == 0) { s->new_maskB[g] = 0; continue; }
        const float* p = s->new_pts + 4 * (size_t)g;
        if (length3(p) < 1e-3f) { s->new_maskB[g] = 0; continue; }
        int invalid = 0;
        for (uint32_t i = 0; i < filter_size; ++i) {
            uint32_t j0 = g + i - 1u; /* uint arithmetic; `0 <= j` is always true */
            if (j0 < n) invalid = invalid || !ps_neighbor_ok(s->new_pts, p, j0, threshold);
            uint32_t j1 = g + i + 1u;
            if (j1 < n) invalid = invalid || !ps_neighbor_ok(s->new_pts, p, j1, threshold);
        }
        s->new_maskB[g] = invalid ? 0u : mv;
    }
    s->new_filtered = 1;
    return 0;
}

static void ensure_hist_arrays(orc_state* s, int which_a, uint32_t npts, uint32_t nseq) {
    if (which_a) {
        s->hA_pts = (float*)xrealloc(s->hA_pts, (size_t)npts * 16);
        s->hA_mask = (uint32_t*)xrealloc(s->hA_mask, (size_t)npts * 4);
        s->hA_seq = (uint32_t*)xrealloc(s->hA_seq, (size_t)npts * 4);
        s->hA_seqs = (orc_seq*)xrealloc(s->hA_seqs, (size_t)nseq * sizeof(orc_seq));
        s->hA_n = npts; s->hA_s = nseq;
    } else {
        s->hB_pts = (float*)xrealloc(s->hB_pts, (size_t)npts * 16);
        s->hB_mask = (uint32_t*)xrealloc(s->hB_mask, (size_t)npts * 4);
        s->hB_seq = (uint32_t*)xrealloc(s->hB_seq, (size_t)npts * 4);
        s->hB_seqs = (orc_seq*)xrealloc(s->hB_seqs, (size_t)nseq * sizeof(orc_seq));
        s->hB_n = npts; s->hB_s = nseq;
    }
}

/* insertNewPointSequencesInRollbuffer(), fusion.cpp:979-1087: A := B[0,R) ++ new */
int orc_insert_new_point_sequences(orc_state* s) {
    uint32_t R = s->rb_pts, S = s->rb_seqs, nn = s->n_new, sn = s->s_new;
    /* A is rewritten from B; keep B's content while resizing A */
    ensure_hist_arrays(s, 1, R + nn, S + sn);
    if (R) {
        memcpy(s->hA_pts, s->hB_pts, (size_t)R * 16);
        memcpy(s->hA_mask, s->hB_mask, (size_t)R * 4);
        memcpy(s->hA_seq, s->hB_seq, (size_t)R * 4);
    }
    if (S) memcpy(s->hA_seqs, s->hB_seqs, (size_t)S * sizeof(orc_seq));
    if (nn) {
        memcpy(s->hA_pts + 4 * (size_t)R, s->new_pts, (size_t)nn * 16);
        if (s->new_filtered) memcpy(s->hA_mask + R, s->new_maskB, (size_t)nn * 4);
        else for (uint32_t i = 0; i < nn; ++i) s->hA_mask[R + i] = 1; /* unfiltered: valid */
    }
    for (uint32_t k = 0; k < sn; ++k) {
        const orc_seq* q = &s->new_seqs[k];
        for (uint32_t i = 0; i < q->num_points; ++i) s->hA_seq[R + q->start + i] = S + k;
    }
    if (sn) memcpy(s->hA_seqs + S, s->new_seqs, (size_t)sn * sizeof(orc_seq));
    s->rb_pts = R + nn;
    s->rb_seqs = S + sn;
    if (sn > 0) {
        s->last_sec = s->new_seqs[sn - 1].sec;
        s->last_nsec = s->new_seqs[sn - 1].nsec;
    }
    return 0;
}

/* compareTime(), fusion.cpp:1089-1096 */
static int compare_time(uint32_t sa, uint32_t na, uint32_t sb, uint32_t nb) {
    if (sa < sb) return -1;
    if (sa > sb) return +1;
    if (na < nb) return -1;
    if (na > nb) return +1;
    return 0;
}

/* rollPointSequenceRollbufferCPU(), fusion.cpp:1098-1217 */
int orc_roll_rollbuffer(orc_state* s, uint32_t min_sec, uint32_t min_nsec) {
    uint32_t nseq = s->hA_s;
    uint32_t d_seqs = 0, d_pts = 0;
    for (uint32_t i = 0; i < nseq; ++i) {
        const orc_seq* q = &s->hA_seqs[i];
        if (compare_time(q->sec, q->nsec, min_sec, min_nsec) < 0) {
            d_pts += q->num_points;
        } else {
            d_seqs = i;
            break;
        }
    }
    if (nseq > d_seqs) {
        s->earliest_sec = s->hA_seqs[d_seqs].sec;
        s->earliest_nsec = s->hA_seqs[d_seqs].nsec;
    } else {
        s->earliest_sec = 0; s->earliest_nsec = 0;
        s->last_sec = 0; s->last_nsec = 0;
    }
    uint32_t R = s->rb_pts, S = s->rb_seqs;
    if (d_pts > R || d_seqs > S) return -2; /* reference would underflow (uint) here */
    uint32_t rp = R - d_pts, rs = S - d_seqs;
    ensure_hist_arrays(s, 0, rp, rs);
    if (rp) {
        memcpy(s->hB_pts, s->hA_pts + 4 * (size_t)d_pts, (size_t)rp * 16);
        memcpy(s->hB_mask, s->hA_mask + d_pts, (size_t)rp * 4);
        for (uint32_t i = 0; i < rp; ++i) s->hB_seq[i] = s->hA_seq[d_pts + i] - d_seqs;
    }
    if (rs) memcpy(s->hB_seqs, s->hA_seqs + d_seqs, (size_t)rs * sizeof(orc_seq));
    s->rb_pts = rp;
    s->rb_seqs = rs;
    return 0;
}

/* selectPointSequenceTimespanCPU(), fusion.cpp:1358-1416 (over the B headers) */
int orc_select_timespan(orc_state* s, uint32_t min_sec, uint32_t min_nsec, uint32_t max_sec,
                        uint32_t max_nsec) {
    uint32_t num_seqs = s->rb_seqs;
    int64_t start = (int64_t)num_seqs, last = 0, count = 0;
    uint32_t pcount = 0, pstart = 0;
    for (uint32_t i = 0; i < s->hB_s; ++i) {
        const orc_seq* q = &s->hB_seqs[i];
        int c0 = compare_time(min_sec, min_nsec, q->sec, q->nsec);
        int c1 = compare_time(q->sec, q->nsec, max_sec, max_nsec);
        if (c0 <= 0 && c1 <= 0) {
            if ((int64_t)i < start) start = i;
            if ((int64_t)i > last) last = i;
            pcount += q->num_points;
        }
    }
    count = (last < start) ? 0 : 1 + last - start;
    for (int64_t i = 0; i < start && i < (int64_t)s->hB_s; ++i) pstart += s->hB_seqs[i].num_points;
    s->sel_pt_start = pstart;
    s->sel_pt_count = pcount;
    s->sel_seq_start = (uint32_t)start;
    s->sel_seq_count = (uint32_t)count;
    return 0;
}

/* preparePointAndMaskBuffers(), fusion.cpp:1497-1508 */
int orc_prepare_point_and_mask_buffers(orc_state* s) {
    uint32_t n = s->depth_total + s->sel_pt_count;
    s->n = n;
    size_t m = n ? n : 1;
    free(s->A); free(s->B); free(s->C); free(s->maskA); free(s->maskB);
    s->A = (float*)calloc(m * 4, sizeof(float));
    s->B = (float*)calloc(m * 4, sizeof(float));
    s->C = (float*)calloc(m * 4, sizeof(float));
    s->maskA = (uint32_t*)calloc(m, 4);
    s->maskB = (uint32_t*)calloc(m, 4);
    return (s->A && s->B && s->C && s->maskA && s->maskB) ? 0 : -4;
}

/* insertSelectedPointSequence(), fusion.cpp:1509-1553: transfer_data (mask),
 * sh/rollbuffer_transfer_selected_transform_indices.glsl:30-42,
 * sh/rollbuffer_transfer_selected_transforms.glsl:49-66 (= T_world_move · T_move) */
int orc_insert_selected_point_sequence(orc_state* s, const float Twm[16], const float Tcm[16]) {
    uint32_t cnt = s->sel_pt_count, sc = s->sel_seq_count, ps = s->sel_pt_start;
    uint32_t P = s->depth_total;
    if (P + cnt > s->n) return -2;
    if (cnt && (uint64_t)ps + cnt > s->hB_n) return -2;
    if (sc && (uint64_t)s->sel_seq_start + sc > s->hB_s) return -2;
    s->tf_idx = (uint32_t*)xrealloc(s->tf_idx, (size_t)(cnt ? cnt : 1) * 4);
    s->tfw = (float*)xrealloc(s->tfw, (size_t)(sc ? sc : 1) * 64);
    s->tfc = (float*)xrealloc(s->tfc, (size_t)(sc ? sc : 1) * 64);
    for (uint32_t i = 0; i < cnt; ++i) {
        s->maskB[P + i] = s->hB_mask[ps + i];
        s->tf_idx[i] = s->hB_seq[ps + i] - s->hB_seq[ps];
    }
    for (uint32_t j = 0; j < sc; ++j) {
        const float* Tm = s->hB_seqs[s->sel_seq_start + j].T_move;
        mat_mul(Twm, Tm, s->tfw + 16 * (size_t)j);
        mat_mul(Tcm, Tm, s->tfc + 16 * (size_t)j);
    }
    return 0;
}

/* transformPointSequence(), fusion.cpp:1555-1581 → sh/transform_points_indirect.glsl:50-69 */
int orc_transform_point_sequence(orc_state* s) {
    uint32_t cnt = s->sel_pt_count, ps = s->sel_pt_start, P = s->depth_total;
    for (uint32_t i = 0; i < cnt; ++i) {
        if (s->hB_mask[ps + i] == 0) continue;
        const float* p = s->hB_pts + 4 * (size_t)(ps + i);
        uint32_t t = s->tf_idx[i];
        if (t >= s->sel_seq_count) return -2;
        mat_vec(s->tfw + 16 * (size_t)t, p, s->B + 4 * (size_t)(P + i));
        mat_vec(s->tfc + 16 * (size_t)t, p, s->C + 4 * (size_t)(P + i));
    }
    return 0;
}

/* ---- depth chain ---------------------------------------------------------------------------- */
/* uploadDepthmaps(), fusion.cpp:1583-1593 */
int orc_upload_depthmaps(orc_state* s) {
    size_t need = s->depth_total ? s->depth_total : 1;
    if (need > s->cap_depth_up) {
        s->depth_up = (uint16_t*)xrealloc(s->depth_up, need * 2);
        s->cap_depth_up = need;
    }
    uint32_t off = 0;
    for (int k = 0; k < s->ncams; ++k) {
        memcpy(s->depth_up + off, s->cams[k].depth, (size_t)s->cams[k].n * 2);
        s->cam_off[k] = off;
        off += s->cams[k].n;
    }
    return 0;
}

/* sh/convert_depthmap_to_points.glsl:64-73 (depthToPoint) + :75-81 (rectify: u = idx mod W,
 * v = idx / W, exact for W·H < 2^24) */
static inline void cam_point(const orc_cam* c, uint32_t idx, uint32_t d, float* p) {
    float u = (float)(idx % c->W);
    float v = (float)(idx / c->W);
    float z = (float)d * c->scale;
    float x = (u - c->cx) / c->fx;
    float y = (v - c->cy) / c->fy;
    p[0] = x * z; p[1] = y * z; p[2] = z; p[3] = 1.0f;
}

/* convertDepthmaps(), fusion.cpp:1595-1628 → sh/convert_depthmap_to_points.glsl:83-120 */
int orc_convert_depthmaps(orc_state* s) {
    if (s->n < s->depth_total) return -2;
    for (int k = 0; k < s->ncams; ++k) {
        const orc_cam* c = &s->cams[k];
        uint32_t off = s->cam_off[k];
        const uint16_t* dp = s->depth_up + off;
        #pragma omp parallel for num_threads(s->nthreads) schedule(static)
        for (int64_t ii = 0; ii < (int64_t)c->n; ++ii) {
            uint32_t idx = (uint32_t)ii, g = off + idx;
            uint32_t d = dp[idx];
            float* A = s->A + 4 * (size_t)g;
            float* B = s->B + 4 * (size_t)g;
            if (d == 0) {
                s->maskA[g] = 0;
                A[0] = A[1] = A[2] = A[3] = 0.0f;
                B[0] = B[1] = B[2] = B[3] = 0.0f;
            } else {
                float p[4];
                cam_point(c, idx, d, p);
                s->maskA[g] = 1;
                memcpy(A, p, 16);
                mat_vec(c->Tw, p, B);
                mat_vec(c->Tc, p, s->C + 4 * (size_t)g);
            }
        }
    }
    return 0;
}

/* MaskA read at a uint index that may have wrapped below 0 (out of bounds → 0, A.7) */
static inline uint32_t mask_at(const orc_state* s, int64_t gi) {
    if (gi < 0 || gi >= (int64_t)s->n) return 0;
    return s->maskA[gi];
}

/* check_at / check_at_rot45, sh/filter_flying_pixels.glsl:55-133 */
static int flying_check(const orc_state* s, int64_t g, uint32_t x, uint32_t y, uint32_t W,
                        uint32_t H, uint32_t i, int rot45, float thr) {
    if (x + i > W - 1 || y + i > H - 1) return 0;      /* x-i<0 / y-i<0 never true (uint) */
    int64_t iw = (int64_t)i * W;
    int64_t up, down, left, right, m1, m2, m3, m4;
    if (!rot45) {
        m1 = g - iw; m2 = g + iw; m3 = g - i; m4 = g + i;
        up = g - iw; down = g + iw; left = g - i; right = g + i;
    } else {
        m1 = g - iw - i; m2 = g - iw + i; m3 = g + iw - i; m4 = g + iw + i;
        up = g - iw - i; down = g + iw + i; left = g + iw - i; right = g - iw + i;
    }
    if (mask_at(s, g) == 0 || mask_at(s, m1) == 0 || mask_at(s, m2) == 0 ||
        mask_at(s, m3) == 0 || mask_at(s, m4) == 0)
        return 0;
    const float* P = s->A + 4 * (size_t)g;
    const float* pu = s->A + 4 * (size_t)up;
    const float* pd = s->A + 4 * (size_t)down;
    const float* pl = s->A + 4 * (size_t)left;
    const float* pr = s->A + 4 * (size_t)right;
    float dx[3] = {pr[0] - pl[0], pr[1] - pl[1], pr[2] - pl[2]};
    float dy[3] = {pd[0] - pu[0], pd[1] - pu[1], pd[2] - pu[2]};
    float cr[3], nrm[3], np[3], nn[3];
    cross3(dy, dx, cr);
    normalize3(cr, nrm);
    normalize3(P, np);
    nn[0] = -np[0]; nn[1] = -np[1]; nn[2] = -np[2];
    float cv = dot3(nrm, nn);
    if (cv < thr) return 0;                              /* NaN passes */
    return 1;
}

/* filterFlyingPixels(), fusion.cpp:1629-1648 → sh/filter_flying_pixels.glsl:135-165 */
int orc_filter_flying_pixels(orc_state* s, uint32_t filter_size, float threshold, int rot45) {
    const float max_distance = 10.0f; /* uniform default, never set by the host (:41) */
    for (int k = 0; k < s->ncams; ++k) {
        const orc_cam* c = &s->cams[k];
        uint32_t off = s->cam_off[k];
        #pragma omp parallel for num_threads(s->nthreads) schedule(static)
        for (int64_t ii = 0; ii < (int64_t)c->n; ++ii) {
            uint32_t idx = (uint32_t)ii;
            int64_t g = (int64_t)off + idx;
            uint32_t mv = s->maskA[g];
            if (mv == 0) { s->maskB[g] = 0; continue; }
            uint32_t out = mv;
            const float* p = s->A + 4 * (size_t)g;
            if (length3(p) > max_distance) { s->maskB[g] = 0; continue; }
            uint32_t x = idx % c->W, y = idx / c->W;
            for (uint32_t i = 0; i < filter_size; ++i) {
                if (!flying_check(s, g, x, y, c->W, c->H, i + 1, 0, threshold)) out = 0;
                if (rot45 && !flying_check(s, g, x, y, c->W, c->H, i + 1, 1, threshold)) out = 0;
            }
            s->maskB[g] = out;
        }
    }
    return 0;
}

/* cropPoints(), fusion.cpp:1649-1660 → sh/crop_points.glsl:38-67 (MaskB → MaskA over n) */
int orc_crop_points(orc_state* s, const float lo[3], const float hi[3]) {
    #pragma omp parallel for num_threads(s->nthreads) schedule(static)
    for (int64_t gi = 0; gi < (int64_t)s->n; ++gi) {
        uint32_t mv = s->maskB[gi];
        if (mv == 0) { s->maskA[gi] = 0; continue; }
        const float* p = s->C + 4 * (size_t)gi;
        if (p[0] < lo[0] || p[0] > hi[0] || p[1] < lo[1] || p[1] > hi[1] || p[2] < lo[2] ||
            p[2] > hi[2])
            s->maskA[gi] = 0;
        else
            s->maskA[gi] = mv;
    }
    return 0;
}

/* applyPointMask(), fusion.cpp:1661-1678 → sh/apply_point_mask.glsl:42-55; the reference's
 * atomicAdd order is nondeterministic, the canonical order is ascending index (A.10). */
int orc_apply_point_mask(orc_state* s, uint32_t* out_count) {
    uint32_t cnt = 0;
    for (uint32_t g = 0; g < s->n; ++g) {
        if (s->maskA[g] > 0) {
            memcpy(s->A + 4 * (size_t)cnt, s->B + 4 * (size_t)g, 16);
            ++cnt;
        }
    }
    s->num_after_mask = cnt;
    if (out_count) *out_count = cnt;
    return 0;
}

/* computeVoxelCoords(), fusion.cpp:1680-1711 → sh/compute_voxel_coords.glsl:34-55, plus the
 * VoxelGridMeta update (inc/grid_meta.h:140-158) */
int orc_compute_voxel_coords(orc_state* s, const float lo[3], const float hi[3],
                             const float cs[3]) {
    uint32_t gs[3];
    uint64_t meta_cells = 1;
    for (int a = 0; a < 3; ++a) {
        float f = (hi[a] - lo[a]) / cs[a];
        if (!(f > 0.0f) || !(f < 4294967040.0f)) return -1; /* shader grid would be 0/undefined */
        gs[a] = (uint32_t)ceilf(f);
        float l = lo[a] < hi[a] ? lo[a] : hi[a], u = lo[a] < hi[a] ? hi[a] : lo[a];
        uint32_t m = (uint32_t)ceilf((u - l) / cs[a]);
        if (m < 1) m = 1;
        if (m != gs[a]) return -1;
        meta_cells *= m;
    }
    if (meta_cells >= 0xFFFFFFFFull) return -1;
    memcpy(s->lb, lo, 12); memcpy(s->ub, hi, 12); memcpy(s->cs, cs, 12);
    memcpy(s->gs, gs, 12);
    s->ncells = meta_cells;
    s->grid_set = 1;
    uint32_t N = s->num_after_mask;
    s->coords = (uint32_t*)xrealloc(s->coords, (size_t)(N ? N : 1) * 4);
    float gmax[3] = {(float)(gs[0] - 1u), (float)(gs[1] - 1u), (float)(gs[2] - 1u)};
    #pragma omp parallel for num_threads(s->nthreads) schedule(static)
    for (int64_t ii = 0; ii < (int64_t)N; ++ii) {
        const float* p = s->A + 4 * (size_t)ii;
        uint32_t u[3];
        for (int a = 0; a < 3; ++a) {
            float f = (p[a] - lo[a]) / cs[a];
            f = fminf(fmaxf(f, 0.0f), gmax[a]); /* GLSL clamp; NaN → 0 */
            u[a] = (uint32_t)floorf(f);
        }
        s->coords[ii] = u[0] + u[1] * gs[0] + u[2] * gs[0] * gs[1];
    }
    return 0;
}

/* Stable LSD sort of u32 keys by 8-bit digits: the observable result of RadixSorter::sort
 * (inc/radix_sort.h:107-289, stable; pinned against oracle/_ref in tests). */
void orc_stable_sort_keys(const uint32_t* keys, uint32_t n, uint32_t* out_idx,
                          uint32_t* out_keys) {
    uint32_t* ti = (uint32_t*)malloc((size_t)(n ? n : 1) * 4);
    uint32_t* tk = (uint32_t*)malloc((size_t)(n ? n : 1) * 4);
    for (uint32_t i = 0; i < n; ++i) { out_idx[i] = i; out_keys[i] = keys[i]; }
    for (int d = 0; d < 4; ++d) {
        uint32_t cnt[257];
        memset(cnt, 0, sizeof(cnt));
        for (uint32_t i = 0; i < n; ++i) cnt[((out_keys[i] >> (8 * d)) & 0xFF) + 1]++;
        if (cnt[1] == n) continue;
        for (int b = 0; b < 256; ++b) cnt[b + 1] += cnt[b];
        for (uint32_t i = 0; i < n; ++i) {
            uint32_t dg = (out_keys[i] >> (8 * d)) & 0xFF;
            uint32_t t = cnt[dg]++;
            ti[t] = out_idx[i];
            tk[t] = out_keys[i];
        }
        memcpy(out_idx, ti, (size_t)n * 4);
        memcpy(out_keys, tk, (size_t)n * 4);
    }
    free(ti);
    free(tk);
}

/* voxelize(), fusion.cpp:1743-1756 → inc/voxelize.h:74-105: RadixGrouper::group
 * (inc/radix_grouper.h:22-64) then averageGridCells (voxelize.h:9-48, sum from 0 in stable
 * order, mean of x,y,z; w keeps the un-divided sum) or occupiedGridCells (voxelize.h:50-71,
 * GridMeta::worldCoord = voxel lower corner). */
int orc_voxelize(orc_state* s, int average) {
    if (!s->grid_set) return -2;
    uint32_t N = s->num_after_mask;
    uint32_t* si = (uint32_t*)malloc((size_t)(N ? N : 1) * 4);
    uint32_t* sk = (uint32_t*)malloc((size_t)(N ? N : 1) * 4);
    orc_stable_sort_keys(s->coords, N, si, sk);
    uint32_t G = 0;
    for (uint32_t i = 0; i < N; ++i) if (i == 0 || sk[i] != sk[i - 1]) ++G;
    s->vox = (float*)xrealloc(s->vox, (size_t)(G ? G : 1) * 16);
    uint32_t g = 0;
    for (uint32_t i = 0; i < N;) {
        uint32_t j = i;
        while (j < N && sk[j] == sk[i]) ++j;
        float* o = s->vox + 4 * (size_t)g;
        if (average) {
            float sum[4] = {0.0f, 0.0f, 0.0f, 0.0f};
            uint32_t count = 0;
            for (uint32_t k = i; k < j; ++k) {
                const float* p = s->A + 4 * (size_t)si[k];
                sum[0] += p[0]; sum[1] += p[1]; sum[2] += p[2]; sum[3] += p[3];
                ++count;
            }
            o[0] = sum[0] / (float)count;
            o[1] = sum[1] / (float)count;
            o[2] = sum[2] / (float)count;
            o[3] = sum[3];
        } else {
            /* GridMeta::gridCoord(cellIndex) then worldCoord (grid_meta.h:45-100) */
            uint32_t key = sk[i];
            uint32_t steps[3] = {1u, s->gs[0], s->gs[0] * s->gs[1]};
            uint32_t gc[3];
            for (int a = 0; a < 3; ++a) {
                gc[a] = (key / steps[a]) % s->gs[a];
                key -= gc[a] * steps[a];
            }
            for (int a = 0; a < 3; ++a) o[a] = (float)gc[a] * s->cs[a] + s->lb[a];
            o[3] = 0.0f;
        }
        ++g;
        i = j;
    }
    s->nvox = G;
    free(si);
    free(sk);
    return 0;
}

/* voxelOccupancyGrid(), fusion.cpp:1757-1823: zero_uints, voxel_grid_occupancy_of_points
 * (sh/:30-40), decrement_uints (sh/:31-51), max_with_uints_times_scalar (sh/:36-46),
 * uints_to_chars (sh/:31-50) */
int orc_voxel_occupancy_grid(orc_state* s, uint32_t lifetime) {
    if (!s->grid_set) return -2;
    uint64_t C = s->ncells;
    if (!s->invoked_once || s->hist_cells != C) {
        free(s->hist); free(s->histB); free(s->occ); free(s->out8);
        s->hist = (uint32_t*)calloc(C, 4);
        s->histB = (uint32_t*)calloc(C, 4);
        s->occ = (uint32_t*)calloc(C, 4);
        s->out8 = (uint8_t*)calloc(C, 1);
        if (!s->hist || !s->histB || !s->occ || !s->out8) return -4;
        s->hist_cells = C;
    }
    s->invoked_once = 1;
    memset(s->occ, 0, C * 4);
    for (uint32_t i = 0; i < s->num_after_mask; ++i) s->occ[s->coords[i]] = 1;
    #pragma omp parallel for num_threads(s->nthreads) schedule(static)
    for (int64_t c = 0; c < (int64_t)C; ++c) {
        uint32_t h = s->hist[c];
        uint32_t hb = (h >= 0u + 1u) ? h - 1u : 0u;            /* decrement=1, min_value=0 */
        uint32_t m = s->occ[c] * lifetime;                     /* u32 wrap */
        uint32_t na = hb > m ? hb : m;
        s->histB[c] = hb;
        s->hist[c] = na;
        s->out8[c] = (uint8_t)(na & 0xFFu);
    }
    return 0;
}

/* ---- ROS time (roscpp_core rostime: DurationBase::fromSec, normalizeSecNSec*) --------------- */
int orc_ros_time_minus(uint32_t sec, uint32_t nsec, double seconds, uint32_t* out_sec,
                       uint32_t* out_nsec) {
    int64_t dsec64 = (int64_t)floor(seconds);
    if (dsec64 < INT32_MIN || dsec64 > INT32_MAX) return -1;
    int32_t dsec = (int32_t)dsec64;
    int32_t dnsec = (int32_t)round((seconds - (double)dsec) * 1e9);
    int32_t rollover = (int32_t)((int64_t)dnsec / 1000000000LL);
    dsec += rollover;
    dnsec = (int32_t)((int64_t)dnsec % 1000000000LL);
    /* -Duration: normalizeSecNSecSigned(-sec, -nsec) */
    int64_t ns = -(int64_t)dnsec, ss = -(int64_t)dsec;
    int64_t np = ns % 1000000000LL, sp = ss + ns / 1000000000LL;
    if (np < 0) { np += 1000000000LL; --sp; }
    if (sp < INT32_MIN || sp > INT32_MAX) return -1;
    /* Time + Duration: normalizeSecNSecUnsigned */
    int64_t sec_sum = (int64_t)sec + sp, nsec_sum = (int64_t)nsec + np;
    int64_t np2 = nsec_sum % 1000000000LL, sp2 = sec_sum + nsec_sum / 1000000000LL;
    if (np2 < 0) { np2 += 1000000000LL; --sp2; }
    if (sp2 < 0 || sp2 > 0xFFFFFFFFLL) return -1;
    *out_sec = (uint32_t)sp2;
    *out_nsec = (uint32_t)np2;
    return 0;
}

/* GPUDepthmapFusionComponent::processDepthmaps(), comp.cpp:92-300 (engine part only: every
 * added depth map counts as numAdded; object segmentation/tracking and publishing are out of
 * scope) */
int orc_process_frame(orc_state* s, const orc_frame_params* p, int32_t* processed,
                      uint32_t* latest_sec, uint32_t* latest_nsec) {
    int rc;
    *processed = 0;
    *latest_sec = 0; *latest_nsec = 0;
    if (!(s->ncams > 0 || s->collect->total > 0)) return 0;
    *processed = 1;
    if ((rc = orc_upload_point_sequences(s))) return rc;
    if ((rc = orc_filter_new_point_sequences(s, p->ps_filter_threshold, p->ps_filter_size))) return rc;
    if ((rc = orc_insert_new_point_sequences(s))) return rc;
    uint32_t lt_s = 0, lt_ns = 0, et_s = 0, et_ns = 0;
    if (s->last_sec != 0 || s->last_nsec != 0) {
        lt_s = s->last_sec; lt_ns = s->last_nsec;
        if (orc_ros_time_minus(lt_s, lt_ns, (double)p->ps_timespan, &et_s, &et_ns)) return -6;
    }
    if ((rc = orc_roll_rollbuffer(s, et_s, et_ns))) return rc;
    if (p->move_transform_available) {
        if ((rc = orc_select_timespan(s, et_s, et_ns, lt_s, lt_ns))) return rc;
        if ((rc = orc_prepare_point_and_mask_buffers(s))) return rc;
        if ((rc = orc_insert_selected_point_sequence(s, p->T_world_move, p->T_crop_move))) return rc;
        if ((rc = orc_transform_point_sequence(s))) return rc;
    } else {
        if ((rc = orc_prepare_point_and_mask_buffers(s))) return rc;
    }
    *latest_sec = lt_s; *latest_nsec = lt_ns;
    if ((rc = orc_upload_depthmaps(s))) return rc;
    if ((rc = orc_convert_depthmaps(s))) return rc;
    if ((rc = orc_filter_flying_pixels(s, p->flying_filter_size, p->flying_threshold, p->flying_rot45))) return rc;
    if ((rc = orc_crop_points(s, p->crop_min, p->crop_max))) return rc;
    if ((rc = orc_apply_point_mask(s, NULL))) return rc;
    if (p->enable_voxel_filter) {
        if ((rc = orc_compute_voxel_coords(s, p->voxel_min, p->voxel_max, p->voxel_size))) return rc;
        if ((rc = orc_voxelize(s, p->voxel_average))) return rc;
        if ((rc = orc_voxel_occupancy_grid(s, p->occupancy_lifetime))) return rc;
    }
    return 0;
}

/* ---- accessors ----------------------------------------------------------------------------- */
uint32_t orc_num_points_total(orc_state* s) { return s->n; }
uint32_t orc_num_depth_points(orc_state* s) { return s->depth_total; }
uint32_t orc_num_points(orc_state* s) { return s->num_after_mask; }
const uint32_t* orc_mask_a(orc_state* s) { return s->maskA; }
const uint32_t* orc_mask_b(orc_state* s) { return s->maskB; }
const float* orc_points_a(orc_state* s) { return s->A; }
const float* orc_points_b(orc_state* s) { return s->B; }
const float* orc_points_c(orc_state* s) { return s->C; }
const uint32_t* orc_voxel_coords(orc_state* s) { return s->coords; }
const float* orc_voxelized(orc_state* s, uint32_t* count) { *count = s->nvox; return s->vox; }
const uint8_t* orc_occupancy(orc_state* s, uint64_t* nc) { *nc = s->hist_cells; return s->out8; }
const uint32_t* orc_historic(orc_state* s, uint64_t* nc) { *nc = s->hist_cells; return s->hist; }
void orc_grid_size(orc_state* s, uint32_t gs[3]) { memcpy(gs, s->gs, 12); }
const uint32_t* orc_new_ps_mask(orc_state* s, uint32_t* count) { *count = s->n_new; return s->new_maskB; }
void orc_rollbuffer_state(orc_state* s, uint32_t o[10]) {
    o[0] = s->rb_pts; o[1] = s->rb_seqs; o[2] = s->sel_pt_start; o[3] = s->sel_pt_count;
    o[4] = s->sel_seq_start; o[5] = s->sel_seq_count; o[6] = s->earliest_sec;
    o[7] = s->earliest_nsec; o[8] = s->last_sec; o[9] = s->last_nsec;
}
uint32_t orc_rollbuffer_b(orc_state* s, const float** pts, const uint32_t** mask,
                          const uint32_t** seq_idx, const uint32_t** headers, uint32_t* nseq) {
    static __thread uint32_t* hdr = NULL;
    static __thread uint32_t hdr_cap = 0;
    if (s->hB_s * 4 > hdr_cap) {
        hdr_cap = s->hB_s * 4;
        hdr = (uint32_t*)realloc(hdr, (size_t)hdr_cap * 4);
    }
    for (uint32_t i = 0; i < s->hB_s; ++i) {
        hdr[4 * i + 0] = s->hB_seqs[i].sec; hdr[4 * i + 1] = s->hB_seqs[i].nsec;
        hdr[4 * i + 2] = s->hB_seqs[i].start; hdr[4 * i + 3] = s->hB_seqs[i].num_points;
    }
    *pts = s->hB_pts; *mask = s->hB_mask; *seq_idx = s->hB_seq; *headers = hdr;
    *nseq = s->hB_s;
    return s->rb_pts;
}

/* ---- orphan shaders ------------------------------------------------ */
/* sh/mask_dilate.glsl:40-67, see gdf_oracle.h.  get_pixel (:33-38): x = mod(idx, width),
 * y = idx / width; the loops run dx outer, dy inner (:48-66). */
void orc_mask_dilate(const uint32_t* in_mask, uint32_t* out_mask, uint32_t W, uint32_t H,
                     uint32_t F, int as_written) {
    const int64_t f = (int64_t)F;
    for (uint32_t y = 0; y < H; ++y)
        for (uint32_t x = 0; x < W; ++x) {
            const size_t idx = (size_t)y * W + x;
            uint32_t out = as_written ? 0u : in_mask[idx];
            for (int64_t dx = -f; dx <= f && out; ++dx) {
                const uint32_t xx = x + (uint32_t)dx;  /* uint wrap: negative -> >= W */
                if (xx >= W) continue;
                for (int64_t dy = -f; dy <= f; ++dy) {
                    const uint32_t yy = y + (uint32_t)dy;
                    if (yy >= H) continue;
                    if (in_mask[(size_t)yy * W + xx] == 0) { out = 0; break; }
                }
            }
            out_mask[idx] = out;
        }
}

/* sh/transform_points.glsl:45-53 */
void orc_transform_points(const float* in, const uint32_t* mask, float* out, uint32_t n,
                          const float T[16]) {
    for (uint32_t i = 0; i < n; ++i)
        if (mask[i] != 0) mat_vec(T, in + 4 * (size_t)i, out + 4 * (size_t)i);
}
