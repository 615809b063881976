/*
 * seg_oracle.c — CPU restatement of the reference's object-segmentation FRONT END
 *  — TEST INFRASTRUCTURE ONLY (tests/ may load it; the product never does).
 *
 * Restates, per z-layer of the u8 occupancy grid (layer i = grid + i*W*H, x fastest: the
 * cv::Mat_<uint8_t>(H, W) views of downloadVoxelOccupancyGrid, src/gpu_depthmap_fusion.cpp:1824-1839):
 *   - labelVoxels (fusion.cpp:1872-2011):
 *       cv::connectedComponentsWithStats(layer, labels, stats, centroids, 8, CV_16U)  (:1918-1925)
 *       cv::findContours(layer, contours, RETR_EXTERNAL, CHAIN_APPROX_NONE)            (:1935)
 *       labelsToContours[label at contour[j][0]] = j, else -1                          (:1941-1952)
 *   - prepareLayersConnections + computeLayersConnections (fusion.cpp:2075-2151, :2200-2214,
 *     shader/layers_connections.glsl:96-122 with neighbors_size 0): for every pixel p of layers
 *     i < L-1, connection[i][label_i(p)][label_{i+1}(p)] = 1 (numA x numB u8 matrices back to back)
 *   - mergeLabelsAcrossLayers (fusion.cpp:2243-2361) with UIntGrouper (inc/uint_grouper.h:11-109):
 *     the two min-propagation passes and the merged ids in increasing order of the propagated id.
 *
 * OpenCV is a third-party dependency absent from /root/reference and from this image: its
 * behaviour is restated from its published algorithms (OpenCV 3.2-4.x, modules/imgproc/src/
 * connectedcomponents.cpp and contours.cpp), so this part is PARITY UNPINNED:
 *   - connectedComponents, 8-connectivity, default algorithm = Grana's block-based BBDT (and the
 *     block-based Spaghetti of >= 4.5.4, and the parallel stripe variant): provisional labels are
 *     created per 2x2 block in block-raster order and unions keep the smaller root, so the final
 *     label of a component is its rank by its FIRST 2x2 BLOCK in block-raster order (not by its
 *     first pixel); label 0 = background; stats rows {LEFT, TOP, WIDTH, HEIGHT, AREA} (int32) for
 *     every label incl. background, WIDTH = right - left + 1 in int arithmetic (a label without
 *     pixels keeps INT_MAX / INT_MIN init values), centroids = double(sum of x) / area;
 *   - findContours: the image binarised (nonzero -> 1), padded by one zero pixel
 *     (copyMakeBorder, offset -1), scanned in raster order (cvFindNextContour) with Suzuki-Abe
 *     border following (icvFetchContour, marks 2 / -126), RETR_EXTERNAL skipping a start whose
 *     last marked pixel `lnbd` on the row is > 0; contours returned in REVERSE discovery order
 *     (cvInsertNodeIntoTree inserts at the head of the frame's children).
 */
#include <limits.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define SEG_NONE 0xFFFFFFFFu

typedef struct {
    uint32_t W, H, L;
    uint16_t* labels;        /* [L][H][W]                                      */
    uint32_t* nlabels;       /* [L] incl. background                           */
    uint32_t* lstart;        /* [L] first label of each layer in the flat lists */
    uint32_t total_labels;
    int32_t* stats;          /* [total][5]                                     */
    double* cent;            /* [total][2]                                     */
    int32_t* l2c;            /* [total] labelsToContours                       */
    uint32_t* ncont;         /* [L] contours per layer                         */
    uint32_t total_contours;
    uint32_t* csize;         /* [total_contours] points per contour            */
    int32_t* cpts;           /* [total points][2] (x, y), layer by layer, findContours order */
    uint64_t total_points, cap_points;
    uint64_t* cstart;        /* [L-1] connection matrix starts                 */
    uint64_t conn_bytes;
    uint8_t* conn;
    uint32_t* merged;        /* [total] mergeLabelsAcrossLayers result         */
    uint32_t nobjects;
} orc_seg;

static uint32_t uf_find(uint32_t* p, uint32_t x) {
    while (p[x] != x) x = p[x];
    return x;
}
static void uf_union(uint32_t* p, uint32_t a, uint32_t b) {
    a = uf_find(p, a);
    b = uf_find(p, b);
    if (a < b) p[b] = a;
    else if (b < a) p[a] = b;
}

/* 2x2 block bits: 1 = (2bx, 2by), 2 = (2bx+1, 2by), 4 = (2bx, 2by+1), 8 = (2bx+1, 2by+1) */
static uint32_t blk_bits(const uint8_t* img, uint32_t W, uint32_t H, uint32_t bx, uint32_t by) {
    uint32_t x = 2 * bx, y = 2 * by, b = 0;
    if (img[(size_t)y * W + x]) b |= 1;
    if (x + 1 < W && img[(size_t)y * W + x + 1]) b |= 2;
    if (y + 1 < H) {
        if (img[(size_t)(y + 1) * W + x]) b |= 4;
        if (x + 1 < W && img[(size_t)(y + 1) * W + x + 1]) b |= 8;
    }
    return b;
}

/* connectedComponentsWithStats(img, labels, stats, centroids, 8, CV_16U) on one layer */
static uint32_t cc_layer(const uint8_t* img, uint32_t W, uint32_t H, uint16_t* lab) {
    const uint32_t BW = (W + 1) / 2, BH = (H + 1) / 2, NB = BW * BH;
    uint32_t* bits = (uint32_t*)malloc(sizeof(uint32_t) * NB);
    uint32_t* par = (uint32_t*)malloc(sizeof(uint32_t) * NB);
    uint32_t* bl = (uint32_t*)malloc(sizeof(uint32_t) * NB);
    for (uint32_t by = 0; by < BH; ++by)
        for (uint32_t bx = 0; bx < BW; ++bx) {
            uint32_t b = by * BW + bx;
            bits[b] = blk_bits(img, W, H, bx, by);
            par[b] = bits[b] ? b : SEG_NONE;
        }
    for (uint32_t by = 0; by < BH; ++by)
        for (uint32_t bx = 0; bx < BW; ++bx) {
            uint32_t b = by * BW + bx, m = bits[b];
            if (!m) continue;
            /* 8-adjacency of foreground pixels between neighbouring blocks */
            if (bx > 0 && (m & 5) && (bits[b - 1] & 10)) uf_union(par, b, b - 1);
            if (by > 0) {
                if ((m & 3) && (bits[b - BW] & 12)) uf_union(par, b, b - BW);
                if (bx > 0 && (m & 1) && (bits[b - BW - 1] & 8)) uf_union(par, b, b - BW - 1);
                if (bx + 1 < BW && (m & 2) && (bits[b - BW + 1] & 4)) uf_union(par, b, b - BW + 1);
            }
        }
    uint32_t next = 1;
    for (uint32_t b = 0; b < NB; ++b)
        if (bits[b] && uf_find(par, b) == b) bl[b] = next++;
    for (uint32_t y = 0; y < H; ++y)
        for (uint32_t x = 0; x < W; ++x) {
            uint32_t b = (y / 2) * BW + x / 2;
            lab[(size_t)y * W + x] = img[(size_t)y * W + x] ? (uint16_t)bl[uf_find(par, b)] : 0;
        }
    free(bits);
    free(par);
    free(bl);
    return next; /* numLabels incl. background */
}

static void cc_stats(const uint16_t* lab, uint32_t W, uint32_t H, uint32_t n, int32_t* st,
                     double* cent) {
    int32_t* mx = (int32_t*)malloc(sizeof(int32_t) * 2 * n);
    uint64_t* sum = (uint64_t*)calloc(2 * n, sizeof(uint64_t));
    for (uint32_t l = 0; l < n; ++l) {
        st[5 * l + 0] = INT_MAX; st[5 * l + 1] = INT_MAX;
        mx[2 * l] = INT_MIN; mx[2 * l + 1] = INT_MIN;
        st[5 * l + 4] = 0;
    }
    for (uint32_t y = 0; y < H; ++y)
        for (uint32_t x = 0; x < W; ++x) {
            uint32_t l = lab[(size_t)y * W + x];
            if ((int32_t)x < st[5 * l]) st[5 * l] = (int32_t)x;
            if ((int32_t)y < st[5 * l + 1]) st[5 * l + 1] = (int32_t)y;
            if ((int32_t)x > mx[2 * l]) mx[2 * l] = (int32_t)x;
            if ((int32_t)y > mx[2 * l + 1]) mx[2 * l + 1] = (int32_t)y;
            st[5 * l + 4] += 1;
            sum[2 * l] += x;
            sum[2 * l + 1] += y;
        }
    for (uint32_t l = 0; l < n; ++l) {
        /* CCStatsOp::finish: int width = right - left + 1 (wrapping for an empty label) */
        st[5 * l + 2] = (int32_t)((uint32_t)mx[2 * l] - (uint32_t)st[5 * l] + 1u);
        st[5 * l + 3] = (int32_t)((uint32_t)mx[2 * l + 1] - (uint32_t)st[5 * l + 1] + 1u);
        double area = (double)(uint32_t)st[5 * l + 4];
        cent[2 * l] = (double)sum[2 * l] / area;
        cent[2 * l + 1] = (double)sum[2 * l + 1] / area;
    }
    free(mx);
    free(sum);
}

/* ---- findContours(RETR_EXTERNAL, CHAIN_APPROX_NONE) ------------------------------------------ */
static const int kCodeDx[8] = {1, 1, 0, -1, -1, -1, 0, 1};
static const int kCodeDy[8] = {0, -1, -1, -1, 0, 1, 1, 1};

typedef struct {
    int32_t* pts;
    uint64_t n, cap;
} ptbuf;

static void pt_push(ptbuf* b, int32_t x, int32_t y) {
    if (b->n == b->cap) {
        b->cap = b->cap ? 2 * b->cap : 1024;
        b->pts = (int32_t*)realloc(b->pts, sizeof(int32_t) * 2 * b->cap);
    }
    b->pts[2 * b->n] = x;
    b->pts[2 * b->n + 1] = y;
    b->n++;
}

/* icvFetchContour for an outer border (is_hole = 0), CHAIN_APPROX_NONE; img padded, Wp wide */
static void fetch_outer(int8_t* img, int Wp, int x0, int y0, ptbuf* out) {
    int delta[16];
    const int d8[8] = {1, -Wp + 1, -Wp, -Wp - 1, -1, Wp - 1, Wp, Wp + 1};
    for (int k = 0; k < 16; ++k) delta[k] = d8[k & 7];
    const long i0 = (long)y0 * Wp + x0;
    int px = x0 - 1, py = y0 - 1; /* offset (-1, -1) of the padding */
    int s_end = 4, s = 4;
    long i1;
    do {
        s = (s - 1) & 7;
        i1 = i0 + delta[s];
    } while (img[i1] == 0 && s != s_end);
    if (s == s_end) { /* single pixel */
        img[i0] = (int8_t)(2 | -128);
        pt_push(out, px, py);
        return;
    }
    long i3 = i0, i4;
    for (;;) {
        s_end = s;
        for (;;) {
            i4 = i3 + delta[++s];
            if (img[i4] != 0) break;
        }
        s &= 7;
        if ((unsigned)(s - 1) < (unsigned)s_end) img[i3] = (int8_t)(2 | -128);
        else if (img[i3] == 1) img[i3] = 2;
        pt_push(out, px, py); /* CHAIN_APPROX_NONE writes every point */
        px += kCodeDx[s];
        py += kCodeDy[s];
        if (i4 == i0 && i3 == i1) break;
        i3 = i4;
        s = (s + 4) & 7;
    }
}

/* one layer: contours in DISCOVERY order appended to out, sizes to sz; returns their number */
static uint32_t contours_layer(const uint8_t* img, uint32_t W, uint32_t H, ptbuf* out,
                               uint32_t** sz, uint32_t* szn, uint32_t* szcap) {
    const int Wp = (int)W + 2, Hp = (int)H + 2;
    int8_t* p = (int8_t*)calloc((size_t)Wp * Hp, 1);
    for (uint32_t y = 0; y < H; ++y)
        for (uint32_t x = 0; x < W; ++x) p[(size_t)(y + 1) * Wp + x + 1] = img[(size_t)y * W + x] ? 1 : 0;
    uint32_t n = 0;
    for (int y = 1; y < Hp - 1; ++y) { /* cvFindNextContour, mode 0 */
        int8_t* row = p + (size_t)y * Wp;
        int x = 1, prev = 0, lnbd = 0;
        for (; x < Wp - 1; ++x) {
            int pv;
            for (; x < Wp - 1 && (pv = row[x]) == prev; ++x) {}
            if (x >= Wp - 1) break;
            int is_hole = 0;
            if (!(prev == 0 && pv == 1)) {
                if (pv != 0 || prev < 1) goto resume;
                if (prev & -2) lnbd = x - 1;
                is_hole = 1;
            }
            if (is_hole || row[lnbd] > 0) goto resume;
            {
                uint64_t before = out->n;
                fetch_outer(p, Wp, x, y, out);
                if (*szn == *szcap) {
                    *szcap = *szcap ? 2 * *szcap : 64;
                    *sz = (uint32_t*)realloc(*sz, sizeof(uint32_t) * *szcap);
                }
                (*sz)[(*szn)++] = (uint32_t)(out->n - before);
                ++n;
                prev = row[x]; /* the scanner resumes at x + 1 with prev = the marked start */
                continue;
            }
        resume:
            prev = pv;
            if (prev & -2) lnbd = x;
        }
    }
    free(p);
    return n;
}

/* ---- whole front end ----------------------------------------------------------------------- */
void* orc_seg_run(const uint8_t* grid, uint32_t W, uint32_t H, uint32_t L) {
    orc_seg* s = (orc_seg*)calloc(1, sizeof(orc_seg));
    s->W = W; s->H = H; s->L = L;
    const size_t LS = (size_t)W * H;
    s->labels = (uint16_t*)malloc(sizeof(uint16_t) * LS * (L ? L : 1));
    s->nlabels = (uint32_t*)calloc(L ? L : 1, sizeof(uint32_t));
    s->lstart = (uint32_t*)calloc(L ? L : 1, sizeof(uint32_t));
    for (uint32_t i = 0; i < L; ++i) {
        s->nlabels[i] = cc_layer(grid + i * LS, W, H, s->labels + i * LS);
        s->lstart[i] = s->total_labels;
        s->total_labels += s->nlabels[i];
    }
    const uint32_t T = s->total_labels ? s->total_labels : 1;
    s->stats = (int32_t*)malloc(sizeof(int32_t) * 5 * T);
    s->cent = (double*)malloc(sizeof(double) * 2 * T);
    s->l2c = (int32_t*)malloc(sizeof(int32_t) * T);
    for (uint32_t i = 0; i < L; ++i)
        cc_stats(s->labels + i * LS, W, H, s->nlabels[i], s->stats + 5 * s->lstart[i],
                 s->cent + 2 * s->lstart[i]);
    /* contours, reversed per layer into findContours order, and labelsToContours */
    s->ncont = (uint32_t*)calloc(L ? L : 1, sizeof(uint32_t));
    ptbuf all = {0, 0, 0};
    uint32_t* csz = NULL;
    uint32_t csn = 0, cscap = 0;
    for (uint32_t i = 0; i < L; ++i) {
        ptbuf lay = {0, 0, 0};
        uint32_t* sz = NULL;
        uint32_t szn = 0, szcap = 0;
        uint32_t n = contours_layer(grid + i * LS, W, H, &lay, &sz, &szn, &szcap);
        s->ncont[i] = n;
        uint64_t* off = (uint64_t*)malloc(sizeof(uint64_t) * (n + 1));
        off[0] = 0;
        for (uint32_t d = 0; d < n; ++d) off[d + 1] = off[d] + sz[d];
        int32_t* l2c = s->l2c + s->lstart[i];
        for (uint32_t k = 0; k < s->nlabels[i]; ++k) l2c[k] = -1;
        for (uint32_t j = 0; j < n; ++j) {
            uint32_t d = n - 1 - j; /* findContours order = reverse discovery */
            if (csn == cscap) {
                cscap = cscap ? 2 * cscap : 64;
                csz = (uint32_t*)realloc(csz, sizeof(uint32_t) * cscap);
            }
            csz[csn++] = sz[d];
            for (uint64_t q = off[d]; q < off[d + 1]; ++q) pt_push(&all, lay.pts[2 * q], lay.pts[2 * q + 1]);
            if (sz[d]) {
                int32_t x = lay.pts[2 * off[d]], y = lay.pts[2 * off[d] + 1];
                l2c[s->labels[i * LS + (size_t)y * W + x]] = (int32_t)j;
            }
        }
        free(off);
        free(sz);
        free(lay.pts);
        s->total_contours += n;
    }
    s->csize = csz;
    s->cpts = all.pts;
    s->total_points = all.n;
    /* layers connections */
    s->cstart = (uint64_t*)calloc(L ? L : 1, sizeof(uint64_t));
    for (uint32_t i = 0; i + 1 < L; ++i) {
        s->cstart[i] = s->conn_bytes;
        s->conn_bytes += (uint64_t)s->nlabels[i] * s->nlabels[i + 1];
    }
    s->conn = (uint8_t*)calloc(s->conn_bytes ? s->conn_bytes : 1, 1);
    for (uint32_t i = 0; i + 1 < L; ++i) {
        const uint16_t* a = s->labels + i * LS;
        const uint16_t* b = a + LS;
        uint8_t* m = s->conn + s->cstart[i];
        for (size_t q = 0; q < LS; ++q) m[(size_t)a[q] * s->nlabels[i + 1] + b[q]] = 1;
    }
    /* mergeLabelsAcrossLayers (fusion.cpp:2243-2361) */
    uint32_t* g = (uint32_t*)malloc(sizeof(uint32_t) * T);
    for (uint32_t k = 0; k < s->total_labels; ++k) g[k] = k;
    for (uint32_t i = 0; i + 1 < L; ++i) { /* bottom-up: layer_b = i + 1 takes from layer_a = i */
        uint32_t la = i, lb = i + 1, nA = s->nlabels[la], nB = s->nlabels[lb];
        const uint8_t* m = s->conn + s->cstart[i];
        for (uint32_t b = 0; b < nB; ++b) {
            uint32_t idx = s->lstart[lb] + b;
            for (uint32_t a = 0; a < nA; ++a) {
                if ((a == 0) != (b == 0)) continue; /* background only with background */
                if (!m[(size_t)a * nB + b]) continue;
                uint32_t o = s->lstart[la] + a;
                if (g[o] < g[idx]) g[idx] = g[o];
            }
        }
    }
    for (uint32_t i = 0; i + 1 < L; ++i) { /* top-down: layer_a = L-2-i takes from layer_b */
        uint32_t la = L - 2 - i, lb = L - 1 - i, nA = s->nlabels[la], nB = s->nlabels[lb];
        const uint8_t* m = s->conn + s->cstart[la];
        for (uint32_t a = 0; a < nA; ++a) {
            uint32_t idx = s->lstart[la] + a;
            for (uint32_t b = 0; b < nB; ++b) {
                if ((a == 0) != (b == 0)) continue;
                if (!m[(size_t)a * nB + b]) continue;
                uint32_t o = s->lstart[lb] + b;
                if (g[o] < g[idx]) g[idx] = g[o];
            }
        }
    }
    /* UIntGrouper over g, merged ids in increasing group number */
    uint32_t maxg = 0;
    for (uint32_t k = 0; k < s->total_labels; ++k) if (g[k] > maxg) maxg = g[k];
    uint32_t* rank = (uint32_t*)calloc((size_t)maxg + 1, sizeof(uint32_t));
    for (uint32_t k = 0; k < s->total_labels; ++k) rank[g[k]] = 1;
    uint32_t next = 0;
    for (uint32_t v = 0; v <= maxg; ++v) rank[v] = rank[v] ? next++ : SEG_NONE;
    s->merged = (uint32_t*)malloc(sizeof(uint32_t) * T);
    for (uint32_t k = 0; k < s->total_labels; ++k) s->merged[k] = rank[g[k]];
    s->nobjects = s->total_labels ? next : 0;
    free(rank);
    free(g);
    return s;
}

/* counts: [0] total labels, [1] total contours, [2] total contour points, [3] connection bytes,
 *         [4] objects */
void orc_seg_counts(const void* h, uint64_t* out) {
    const orc_seg* s = (const orc_seg*)h;
    out[0] = s->total_labels;
    out[1] = s->total_contours;
    out[2] = s->total_points;
    out[3] = s->conn_bytes;
    out[4] = s->nobjects;
}

void orc_seg_get(const void* h, uint16_t* labels, uint32_t* nlabels, int32_t* stats, double* cent,
                 int32_t* l2c, uint32_t* ncont, uint32_t* csize, int32_t* cpts, uint8_t* conn,
                 uint64_t* cstart, uint32_t* merged) {
    const orc_seg* s = (const orc_seg*)h;
    const size_t LS = (size_t)s->W * s->H;
    if (labels) memcpy(labels, s->labels, sizeof(uint16_t) * LS * s->L);
    if (nlabels) memcpy(nlabels, s->nlabels, sizeof(uint32_t) * s->L);
    if (stats) memcpy(stats, s->stats, sizeof(int32_t) * 5 * s->total_labels);
    if (cent) memcpy(cent, s->cent, sizeof(double) * 2 * s->total_labels);
    if (l2c) memcpy(l2c, s->l2c, sizeof(int32_t) * s->total_labels);
    if (ncont) memcpy(ncont, s->ncont, sizeof(uint32_t) * s->L);
    if (csize && s->total_contours) memcpy(csize, s->csize, sizeof(uint32_t) * s->total_contours);
    if (cpts && s->total_points) memcpy(cpts, s->cpts, sizeof(int32_t) * 2 * s->total_points);
    if (conn && s->conn_bytes) memcpy(conn, s->conn, s->conn_bytes);
    if (cstart && s->L > 1) memcpy(cstart, s->cstart, sizeof(uint64_t) * (s->L - 1));
    if (merged) memcpy(merged, s->merged, sizeof(uint32_t) * s->total_labels);
}

void orc_seg_free(void* h) {
    orc_seg* s = (orc_seg*)h;
    if (!s) return;
    free(s->labels); free(s->nlabels); free(s->lstart); free(s->stats); free(s->cent);
    free(s->l2c); free(s->ncont); free(s->csize); free(s->cpts); free(s->cstart); free(s->conn);
    free(s->merged);
    free(s);
}
