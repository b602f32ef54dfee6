/*
 * beam_oracle.c — CPU restatement of the reference hot path. TEST INFRASTRUCTURE ONLY
 * (see beam_oracle.h for the rules and the parity status).
 *
 * Compile with IEEE f32 and no contraction (oracle/Makefile: -ffp-contract=off, no -ffast-math,
 * no -march) so every expression rounds exactly once per operation, in the order written here,
 * which follows the reference source and glm 0.9.9.0:
 *   dot(a,b)      = (a.x*b.x + a.y*b.y) + a.z*b.z      glm/detail/func_geometric.inl:56-59
 *   cross(x,y)    = (x.y*y.z - y.y*x.z, x.z*y.x - y.z*x.x, x.x*y.y - y.x*x.y)   ibid :80-83
 *   normalize(v)  = v * (1 / sqrt(dot(v,v)))            ibid :94, func_exponential.inl:136-139
 *   mat3 * vec3   = row i: (m[0][i]*v.x + m[1][i]*v.y) + m[2][i]*v.z           type_mat3x3.inl:424-430
 */
#include "beam_oracle.h"

#include <float.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define ORC_ERR_FINE 0
#define ORC_ERR_INVALID_PARAMETER 2
#define ORC_ERR_INVALID_FORMAT 4
#define MISS_PACKED 0x0000FF00u /* 255<<8, BuildTree.cu:495 */
#define NO_TRI 0xFFFFFFFFu

/* ---- scalar helpers (reference CudaComon.cuh:71-80: ternary min/max, NaN -> 2nd arg) -------- */
static inline float rmin(float a, float b) { return a < b ? a : b; }
static inline float rmax(float a, float b) { return a > b ? a : b; }

static inline float dot3(const float* a, const float* b) { return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]; }
static inline void cross3(float* o, const float* x, const float* y) {
    o[0] = x[1] * y[2] - y[1] * x[2];
    o[1] = x[2] * y[0] - y[2] * x[0];
    o[2] = x[0] * y[1] - y[0] * x[1];
}
static inline void sub3(float* o, const float* a, const float* b) {
    o[0] = a[0] - b[0];
    o[1] = a[1] - b[1];
    o[2] = a[2] - b[2];
}

/* dir = orient * ray; orient is a glm mat3, column-major m[c][r] = o[c*3+r] (Camera.cpp:94). */
static inline void orient_dir(float* d, const float* o, const float* r) {
    d[0] = (o[0] * r[0] + o[3] * r[1]) + o[6] * r[2];
    d[1] = (o[1] * r[0] + o[4] * r[1]) + o[7] * r[2];
    d[2] = (o[2] * r[0] + o[5] * r[1]) + o[8] * r[2];
}

/* bmTriIntersect (CudaComon.cuh:117-155) with e1 = v1-v0, e2 = v2-v0 given. Returns FLT_MAX on
 * the two early rejects; otherwise t (which may be negative, inf or NaN: no det-epsilon, no t>0). */
static inline float tri_intersect_e(const float* orig, const float* dir, const float* v0,
                                   const float* e1, const float* e2, float* uo, float* vo) {
    float p[3], tv[3], q[3];
    cross3(p, dir, e2);
    float det = dot3(e1, p);
    float inv = 1.f / det;
    sub3(tv, orig, v0);
    float u = dot3(tv, p) * inv;
    if (u < 0 || u > 1) return FLT_MAX;
    cross3(q, tv, e1);
    float v = dot3(dir, q) * inv;
    if (v < 0 || v + u > 1) return FLT_MAX;
    *uo = u;
    *vo = v;
    return dot3(e2, q) * inv;
}

static inline float tri_intersect(const float* orig, const float* dir, const float* v0,
                                  const float* v1, const float* v2, float* uo, float* vo) {
    float e1[3], e2[3];
    sub3(e1, v1, v0);
    sub3(e2, v2, v0);
    return tri_intersect_e(orig, dir, v0, e1, e2, uo, vo);
}

/* bmFaceInterpolate<vec3> + normalize + pack (CudaComon.cuh:253-266, BuildTree.cu:486-492). */
static inline uint32_t shade_packed(const float* n0, const float* n1, const float* n2, float u,
                                    float v) {
    float w = 1.f - (u + v);
    float n[3];
    for (int c = 0; c < 3; ++c) n[c] = (n0[c] * w + n1[c] * u) + n2[c] * v;
    float inv = 1.f / sqrtf(dot3(n, n));
    float z = n[2] * inv;
    float r = fabsf(z * 255.f);
    uint32_t red = (r == r) ? (uint32_t)r : 0u;
    return red << 16;
}

/* ---- glm pin (tests/test_oracle_glm_pin.py): the primitives above on a batch of records --------
 * in (36 floats/record): orig[3] ray[3] orient[9, column-major] v0[3] v1[3] v2[3] n0[3] n1[3] n2[3]
 *                        su sv pad
 * out (12 floats/record): dir = orient*ray [3], 1/dir [3], bmTriIntersect t u v (t = FLT_MAX on a
 *                        reject, u = v = 0 then), packed colour of the normals interpolated at
 *                        (su, sv) (bits as f32), normalised n.z, pad.
 * oracle/glm_pin.cpp computes the same with the reference's vendored glm 0.9.9.0. */
void orc_pin_ops(uint32_t n, const float* in, float* out) {
    for (uint32_t i = 0; i < n; ++i) {
        const float* a = in + (size_t)i * 36;
        float* o = out + (size_t)i * 12;
        float d[3], u = 0.f, v = 0.f;
        orient_dir(d, a + 6, a + 3);
        for (int c = 0; c < 3; ++c) {
            o[c] = d[c];
            o[3 + c] = 1.f / d[c];
        }
        const float t = tri_intersect(a, d, a + 15, a + 18, a + 21, &u, &v);
        o[6] = t;
        o[7] = t == FLT_MAX ? 0.f : u;
        o[8] = t == FLT_MAX ? 0.f : v;
        const uint32_t packed = shade_packed(a + 24, a + 27, a + 30, a[33], a[34]);
        memcpy(&o[9], &packed, 4);
        const float w = 1.f - (a[33] + a[34]);
        float nn[3];
        for (int c = 0; c < 3; ++c) nn[c] = (a[24 + c] * w + a[27 + c] * a[33]) + a[30 + c] * a[34];
        o[10] = nn[2] * (1.f / sqrtf(dot3(nn, nn)));
        o[11] = 0.f;
    }
}

/* ---- Camera::setInitialRays (Camera.cpp:43-72) ---------------------------------------------- */
int32_t orc_camera_rays(uint32_t w, uint32_t h, float left, float right, float top, float bottom,
                        float zoom, float* out) {
    if (w == 0 || h == 0) return ORC_ERR_INVALID_PARAMETER;
    float dx = (right - left) / (float)w;
    float dy = (bottom - top) / (float)h;
    float ry = top + dy * .5f;
    float z2 = zoom * zoom;
    for (uint32_t y = 0; y < h; y++, ry += dy) {
        float rx = left + dx * .5f;
        for (uint32_t x = 0; x < w; x++, rx += dx) {
            float d = 1.f / sqrtf(z2 + rx * rx + ry * ry);
            if (isnan(d) || d <= 0.f) return ORC_ERR_INVALID_PARAMETER;
            size_t a = (size_t)y * w + x;
            out[a * 3 + 0] = rx * d;
            out[a * 3 + 1] = ry * d;
            out[a * 3 + 2] = zoom * d;
        }
    }
    return ORC_ERR_FINE;
}

/* ---- flattened triangle soup shared by both restatements ------------------------------------ */
typedef struct soup {
    uint32_t n;
    float* v;  /* n*9: v0 v1 v2 */
    float* nn; /* n*9: n0 n1 n2, or NULL when some mesh lacks normals */
} soup;

static int soup_make(soup* s, const orc_mesh* m, uint32_t nm) {
    uint64_t n = 0;
    int have_n = 1;
    for (uint32_t i = 0; i < nm; ++i) {
        n += m[i].num_idx / 3;
        if (!m[i].nrm) have_n = 0;
    }
    s->n = (uint32_t)n;
    s->v = (float*)malloc(sizeof(float) * 9 * (n ? n : 1));
    s->nn = have_n ? (float*)malloc(sizeof(float) * 9 * (n ? n : 1)) : NULL;
    uint64_t g = 0;
    for (uint32_t i = 0; i < nm; ++i) {
        for (uint32_t f = 0; f < m[i].num_idx / 3; ++f, ++g) {
            for (int k = 0; k < 3; ++k) {
                uint32_t vi = m[i].idx[f * 3 + k];
                memcpy(s->v + g * 9 + k * 3, m[i].pos + (size_t)vi * 3, 12);
                if (have_n) memcpy(s->nn + g * 9 + k * 3, m[i].nrm + (size_t)vi * 3, 12);
            }
        }
    }
    return 0;
}
static void soup_free(soup* s) {
    free(s->v);
    free(s->nn);
}

/* =============================================================================================
 * 1. Reference semantics: sparse spatial-median kd-tree (BuildTree.cu:154-256) + march (:367-499)
 * ============================================================================================= */
#define KD_MAX_DEPTH 38      /* BUILD_TREE_MAX_DEPTH, BuildTree.cuh:15 */
#define KD_LEAF_CAP 256      /* MAX_FACES_PER_BOX, BuildTree.cuh:17 */
#define KD_MIN_LEAF .03f     /* MIN_LEAF_SIZE, BuildTree.cuh:18 */

typedef struct kd_node {
    int32_t left, right; /* -1 = null */
    int32_t group;       /* index of a KD_LEAF_CAP-slot face group, -1 = null */
    uint32_t count;      /* m_faceInsertIdx (keeps counting past the cap) */
} kd_node;

struct orc_kd {
    soup s;
    float wmin, wmax;
    kd_node* nodes;
    uint32_t num_nodes, cap_nodes;
    uint32_t* groups; /* global tri ids, KD_LEAF_CAP per group */
    uint32_t num_groups, cap_groups;
    uint64_t face_refs, dropped;
};

static int32_t kd_new_node(orc_kd* kd) {
    if (kd->num_nodes == kd->cap_nodes) {
        kd->cap_nodes = kd->cap_nodes ? kd->cap_nodes * 2 : 4096;
        kd->nodes = (kd_node*)realloc(kd->nodes, sizeof(kd_node) * kd->cap_nodes);
    }
    kd_node* nd = &kd->nodes[kd->num_nodes];
    nd->left = nd->right = nd->group = -1;
    nd->count = 0;
    return (int32_t)kd->num_nodes++;
}

/* ---- Akenine-Möller triangle/box overlap, restated (BoxTriangle.cuh:57-222) ---- */
/* plane/box test (BoxTriangle.cuh:57-79) */
static int plane_box(const float* nrm, const float* vert, const float* maxbox) {
    float vmin[3], vmax[3];
    for (int q = 0; q < 3; ++q) {
        float v = vert[q];
        if (nrm[q] > 0.0f) {
            vmin[q] = -maxbox[q] - v;
            vmax[q] = maxbox[q] - v;
        } else {
            vmin[q] = maxbox[q] - v;
            vmax[q] = -maxbox[q] - v;
        }
    }
    /* DOT macro: left-to-right sum */
    if ((nrm[0] * vmin[0] + nrm[1] * vmin[1]) + nrm[2] * vmin[2] > 0.0f) return 0;
    if ((nrm[0] * vmax[0] + nrm[1] * vmax[1]) + nrm[2] * vmax[2] >= 0.0f) return 1;
    return 0;
}

/* One separating-axis test on the projection of two vertices pa, pb (already projected):
 * reject when [min,max] lies outside [-rad, rad]. The min/max selection uses the reference's
 * comparison direction (AXISTEST_* macros, BoxTriangle.cuh:83-131); it only decides which of two
 * equal values is kept, so it cannot change the outcome. */
static inline int axis_sep(float pa, float pb, float rad) {
    float mn, mx;
    if (pa < pb) { mn = pa; mx = pb; } else { mn = pb; mx = pa; }
    return (mn > rad || mx < -rad);
}

static int tri_box(const float* bc, const float* hs, const float* tv /* 9 floats */) {
    float v0[3], v1[3], v2[3], e0[3], e1[3], e2[3], nrm[3];
    sub3(v0, tv + 0, bc);
    sub3(v1, tv + 3, bc);
    sub3(v2, tv + 6, bc);
    sub3(e0, v1, v0);
    sub3(e1, v2, v1);
    sub3(e2, v0, v2);
    float fx, fy, fz, a, b, pa, pb, rad;

    /* edge e0: X01, Y02, Z12 */
    fx = fabsf(e0[0]); fy = fabsf(e0[1]); fz = fabsf(e0[2]);
    a = e0[2]; b = e0[1];                       /* X: p = a*v.y - b*v.z; rad = fz*hy + fy*hz */
    pa = a * v0[1] - b * v0[2]; pb = a * v2[1] - b * v2[2];
    rad = fz * hs[1] + fy * hs[2];
    if (axis_sep(pa, pb, rad)) return 0;
    a = e0[2]; b = e0[0];                       /* Y: p = -a*v.x + b*v.z; rad = fz*hx + fx*hz */
    pa = -a * v0[0] + b * v0[2]; pb = -a * v2[0] + b * v2[2];
    rad = fz * hs[0] + fx * hs[2];
    if (axis_sep(pa, pb, rad)) return 0;
    a = e0[1]; b = e0[0];                       /* Z: p = a*v.x - b*v.y; rad = fy*hx + fx*hy */
    pa = a * v1[0] - b * v1[1]; pb = a * v2[0] - b * v2[1];
    rad = fy * hs[0] + fx * hs[1];
    if (axis_sep(pb, pa, rad)) return 0;        /* AXISTEST_Z12 compares p2<p1 */

    /* edge e1: X01, Y02, Z0 */
    fx = fabsf(e1[0]); fy = fabsf(e1[1]); fz = fabsf(e1[2]);
    a = e1[2]; b = e1[1];
    pa = a * v0[1] - b * v0[2]; pb = a * v2[1] - b * v2[2];
    rad = fz * hs[1] + fy * hs[2];
    if (axis_sep(pa, pb, rad)) return 0;
    a = e1[2]; b = e1[0];
    pa = -a * v0[0] + b * v0[2]; pb = -a * v2[0] + b * v2[2];
    rad = fz * hs[0] + fx * hs[2];
    if (axis_sep(pa, pb, rad)) return 0;
    a = e1[1]; b = e1[0];
    pa = a * v0[0] - b * v0[1]; pb = a * v1[0] - b * v1[1];
    rad = fy * hs[0] + fx * hs[1];
    if (axis_sep(pa, pb, rad)) return 0;

    /* edge e2: X2, Y1, Z12 */
    fx = fabsf(e2[0]); fy = fabsf(e2[1]); fz = fabsf(e2[2]);
    a = e2[2]; b = e2[1];
    pa = a * v0[1] - b * v0[2]; pb = a * v1[1] - b * v1[2];
    rad = fz * hs[1] + fy * hs[2];
    if (axis_sep(pa, pb, rad)) return 0;
    a = e2[2]; b = e2[0];
    pa = -a * v0[0] + b * v0[2]; pb = -a * v1[0] + b * v1[2];
    rad = fz * hs[0] + fx * hs[2];
    if (axis_sep(pa, pb, rad)) return 0;
    a = e2[1]; b = e2[0];
    pa = a * v1[0] - b * v1[1]; pb = a * v2[0] - b * v2[1];
    rad = fy * hs[0] + fx * hs[1];
    if (axis_sep(pb, pa, rad)) return 0;

    /* triangle AABB vs box (FINDMINMAX, BoxTriangle.cuh:50-55, 198-209) */
    for (int c = 0; c < 3; ++c) {
        float mn = v0[c], mx = v0[c];
        if (v1[c] < mn) mn = v1[c];
        if (v1[c] > mx) mx = v1[c];
        if (v2[c] < mn) mn = v2[c];
        if (v2[c] > mx) mx = v2[c];
        if (mn > hs[c] || mx < -hs[c]) return 0;
    }
    /* plane of the triangle vs box (BoxTriangle.cuh:215-219); CROSS macro order */
    nrm[0] = e0[1] * e1[2] - e0[2] * e1[1];
    nrm[1] = e0[2] * e1[0] - e0[0] * e1[2];
    nrm[2] = e0[0] * e1[1] - e0[1] * e1[0];
    return plane_box(nrm, v0, hs);
}

typedef struct kd_build_entry {
    float mn[3], mx[3];
    int32_t node;
    uint32_t depth, axis;
} kd_build_entry;

/* bmTreeNode::insertFace (BuildTree.cu:36-61): lazily allocate a 256-slot group; append; drop
 * (the reference printf's) beyond the cap. */
static void kd_insert_face(orc_kd* kd, int32_t ni, uint32_t gid) {
    if (kd->nodes[ni].group < 0) {
        if (kd->num_groups == kd->cap_groups) {
            kd->cap_groups = kd->cap_groups ? kd->cap_groups * 2 : 1024;
            kd->groups = (uint32_t*)realloc(kd->groups, sizeof(uint32_t) * KD_LEAF_CAP * (size_t)kd->cap_groups);
        }
        kd->nodes[ni].group = (int32_t)kd->num_groups++;
    }
    uint32_t slot = kd->nodes[ni].count++;
    if (slot < KD_LEAF_CAP) {
        kd->groups[(size_t)kd->nodes[ni].group * KD_LEAF_CAP + slot] = gid;
        kd->face_refs++;
    } else {
        kd->dropped++;
    }
}

/* bmInsertTriangleInTree (BuildTree.cu:154-256), executed serially in launch order as the
 * reference's CPU-emulation path does (BuildTree.cu:288-306). */
static void kd_insert_tri(orc_kd* kd, uint32_t gid) {
    const float* v = kd->s.v + (size_t)gid * 9;
    kd_build_entry st[KD_MAX_DEPTH];
    int top = 0;
    for (int c = 0; c < 3; ++c) {
        st[0].mn[c] = kd->wmin;
        st[0].mx[c] = kd->wmax;
    }
    st[0].node = 0;
    st[0].depth = 0;
    st[0].axis = 0;
    do {
        kd_build_entry e = st[top--];
        float bs[3];
        sub3(bs, e.mx, e.mn);
        float dmin = rmin(bs[0], rmin(bs[1], bs[2]));
        if ((dmin < KD_MIN_LEAF) || (e.depth == KD_MAX_DEPTH - 1)) {
            kd_insert_face(kd, e.node, gid);
        } else {
            uint32_t a = e.axis, na = (a + 1) % 3, nd = e.depth + 1;
            float s = .5f * (e.mn[a] + e.mx[a]);
            float lmax[3] = {e.mx[0], e.mx[1], e.mx[2]};
            float rmn[3] = {e.mn[0], e.mn[1], e.mn[2]};
            lmax[a] = s;
            rmn[a] = s;
            float bc[3], hs[3];
            for (int c = 0; c < 3; ++c) {
                bc[c] = (lmax[c] + e.mn[c]) * .5f;
                hs[c] = (lmax[c] - e.mn[c]) * .5f;
            }
            int b1 = tri_box(bc, hs, v);
            for (int c = 0; c < 3; ++c) {
                bc[c] = (e.mx[c] + rmn[c]) * .5f;
                hs[c] = (e.mx[c] - rmn[c]) * .5f;
            }
            int b2 = tri_box(bc, hs, v);
            /* split2 (BuildTree.cu:21-34) */
            if (b1 && kd->nodes[e.node].left < 0) {
                int32_t c = kd_new_node(kd);
                kd->nodes[e.node].left = c;
            }
            if (b2 && kd->nodes[e.node].right < 0) {
                int32_t c = kd_new_node(kd);
                kd->nodes[e.node].right = c;
            }
            if (b1) {
                kd_build_entry* p = &st[++top];
                memcpy(p->mn, e.mn, 12);
                memcpy(p->mx, lmax, 12);
                p->node = kd->nodes[e.node].left;
                p->depth = nd;
                p->axis = na;
            }
            if (b2) {
                kd_build_entry* p = &st[++top];
                memcpy(p->mn, rmn, 12);
                memcpy(p->mx, e.mx, 12);
                p->node = kd->nodes[e.node].right;
                p->depth = nd;
                p->axis = na;
            }
        }
    } while (top >= 0);
}

orc_kd* orc_kd_build(const orc_mesh* meshes, uint32_t num_meshes, float wmin, float wmax) {
    orc_kd* kd = (orc_kd*)calloc(1, sizeof(orc_kd));
    soup_make(&kd->s, meshes, num_meshes);
    kd->wmin = wmin;
    kd->wmax = wmax;
    kd_new_node(kd); /* root (bmResetSceneKernel, BuildTree.cu:95-117) */
    for (uint32_t g = 0; g < kd->s.n; ++g) kd_insert_tri(kd, g);
    return kd;
}

void orc_kd_free(orc_kd* kd) {
    if (!kd) return;
    soup_free(&kd->s);
    free(kd->nodes);
    free(kd->groups);
    free(kd);
}

void orc_kd_stats(const orc_kd* kd, uint64_t stats[8]) {
    memset(stats, 0, sizeof(uint64_t) * 8);
    stats[0] = kd->num_nodes;
    stats[2] = kd->face_refs;
    stats[3] = kd->dropped;
    /* leaves, max count, max depth via a walk */
    struct { int32_t n; uint32_t d; } st[128];
    int top = 0;
    st[0].n = 0;
    st[0].d = 0;
    while (top >= 0) {
        int32_t n = st[top].n;
        uint32_t d = st[top].d;
        top--;
        const kd_node* nd = &kd->nodes[n];
        if (nd->left < 0 && nd->right < 0) {
            stats[1]++;
            if (nd->count > stats[4]) stats[4] = nd->count;
            if (d > stats[5]) stats[5] = d;
        } else {
            if (nd->left >= 0) { ++top; st[top].n = nd->left; st[top].d = d + 1; }
            if (nd->right >= 0) { ++top; st[top].n = nd->right; st[top].d = d + 1; }
        }
    }
}

/* bmBoxRayIntersect (CudaComon.cuh:158-172) */
static inline float kd_box_ray(const float* bmn, const float* bmx, const float* o, const float* inv) {
    float t0[3], t1[3];
    for (int c = 0; c < 3; ++c) {
        t0[c] = (bmn[c] - o[c]) * inv[c];
        t1[c] = (bmx[c] - o[c]) * inv[c];
    }
    float tx2[3] = {rmax(t0[0], t1[0]), rmax(t0[1], t1[1]), rmax(t0[2], t1[2])};
    float ftmax = rmin(tx2[0], rmin(tx2[1], tx2[2]));
    if (ftmax < 0.f) return FLT_MAX;
    float tn2[3] = {rmin(t0[0], t1[0]), rmin(t0[1], t1[1]), rmin(t0[2], t1[2])};
    float ftmin = rmax(tn2[0], rmax(tn2[1], tn2[2]));
    float dist = rmax(0.f, ftmin);
    return (ftmax >= ftmin ? dist : FLT_MAX);
}

typedef struct kd_march_entry {
    float mn[3], mx[3];
    int32_t node;
    uint32_t axis;
} kd_march_entry;

static int32_t kd_march_impl(const orc_kd* kd, const float* rays, uint32_t begin, uint32_t end,
                             const float eye[3], const float orient[9], uint32_t* packed, uint32_t* tri_id,
                             float* tout, uint64_t* counts) {
    if (!kd->s.nn && kd->s.n) return ORC_ERR_INVALID_FORMAT;
    for (uint32_t i = begin; i < end; ++i) {
        float dir[3], inv[3];
        orient_dir(dir, orient, rays + (size_t)i * 3);
        for (int c = 0; c < 3; ++c) inv[c] = 1.f / dir[c];
        kd_march_entry st[KD_MAX_DEPTH];
        int top = 0;
        for (int c = 0; c < 3; ++c) {
            st[0].mn[c] = kd->wmin;
            st[0].mx[c] = kd->wmax;
        }
        st[0].node = 0;
        st[0].axis = 0;
        float dclosest = FLT_MAX, tu = 0, tv = 0;
        uint32_t fclosest = NO_TRI;
        do {
            kd_march_entry e = st[top--];
            const kd_node* nd = &kd->nodes[e.node];
            float box = kd_box_ray(e.mn, e.mx, eye, inv);
            if (counts) counts[0]++;
            if (box == FLT_MAX) continue;
            if (nd->left < 0 && nd->right < 0) {
                if (nd->group >= 0) {
                    uint32_t cnt = nd->count < KD_LEAF_CAP ? nd->count : KD_LEAF_CAP;
                    if (counts) {
                        counts[1]++;
                        counts[2] += cnt;
                    }
                    const uint32_t* grp = kd->groups + (size_t)nd->group * KD_LEAF_CAP;
                    for (uint32_t k = 0; k < cnt; ++k) {
                        const float* v = kd->s.v + (size_t)grp[k] * 9;
                        float u, vv;
                        float d = tri_intersect(eye, dir, v, v + 3, v + 6, &u, &vv);
                        if (d < dclosest) {
                            dclosest = d;
                            fclosest = grp[k];
                            tu = u;
                            tv = vv;
                        }
                    }
                    if (dclosest != FLT_MAX) break; /* BuildTree.cu:427-431 */
                }
            } else {
                uint32_t a = e.axis, na = (a + 1) % 3;
                float s = .5f * (e.mx[a] + e.mn[a]);
                float p = eye[a] + box * dir[a];
                kd_march_entry* q;
                if (p < s) { /* right first, then left (popped first) */
                    if (nd->right >= 0) {
                        q = &st[++top];
                        memcpy(q->mn, e.mn, 12); memcpy(q->mx, e.mx, 12);
                        q->mn[a] = s; q->node = nd->right; q->axis = na;
                    }
                    if (nd->left >= 0) {
                        q = &st[++top];
                        memcpy(q->mn, e.mn, 12); memcpy(q->mx, e.mx, 12);
                        q->mx[a] = s; q->node = nd->left; q->axis = na;
                    }
                } else {
                    if (nd->left >= 0) {
                        q = &st[++top];
                        memcpy(q->mn, e.mn, 12); memcpy(q->mx, e.mx, 12);
                        q->mx[a] = s; q->node = nd->left; q->axis = na;
                    }
                    if (nd->right >= 0) {
                        q = &st[++top];
                        memcpy(q->mn, e.mn, 12); memcpy(q->mx, e.mx, 12);
                        q->mn[a] = s; q->node = nd->right; q->axis = na;
                    }
                }
            }
        } while (top >= 0);
        if (dclosest != FLT_MAX) {
            const float* n = kd->s.nn + (size_t)fclosest * 9;
            if (packed) packed[i] = shade_packed(n, n + 3, n + 6, tu, tv);
            if (tri_id) tri_id[i] = fclosest;
            if (tout) tout[i] = dclosest;
        } else {
            if (packed) packed[i] = MISS_PACKED;
            if (tri_id) tri_id[i] = NO_TRI;
            if (tout) tout[i] = INFINITY;
        }
    }
    return ORC_ERR_FINE;
}

int32_t orc_kd_march(const orc_kd* kd, const float* rays, uint32_t begin, uint32_t end,
                     const float eye[3], const float orient[9], uint32_t* packed, uint32_t* tri_id,
                     float* tout) {
    return kd_march_impl(kd, rays, begin, end, eye, orient, packed, tri_id, tout, NULL);
}

int32_t orc_kd_march_counts(const orc_kd* kd, const float* rays, uint32_t begin, uint32_t end,
                            const float eye[3], const float orient[9], uint64_t counts[3]) {
    counts[0] = counts[1] = counts[2] = 0;
    return kd_march_impl(kd, rays, begin, end, eye, orient, NULL, NULL, NULL, counts);
}

/* =============================================================================================
 * 1b. Reference semantics, the alternative accelerator: hashed uniform grid (Raytracer/Hash.cu,
 *     compiled by the reference only with TREE_TYPE==HASH; SceneHash.cpp:29-76). Cells of 0.03,
 *     a cell (x, y, z) lands in bucket (F16(x) + F16(y) + F16(z)) mod 65536 with F16 = Fletcher-16
 *     over the four little-endian bytes (Hash.cu:15-47); a triangle goes into every cell of its
 *     AABB that Akenine-Möller's test accepts (Hash.cu:132-178, with the insert loop's y/x indices
 *     reset per row — the reference never resets them, Hash.cu:162-164, the bug SURVEY §8(f)4 asks
 *     to fix); a bucket keeps its first 256 faces. The march (Hash.cu:235-302) walks cells from the
 *     eye, tests every face of the cell's bucket against the ray from the EYE, and stops at the
 *     first bucket with any hit (the closest of that bucket; hash collisions included), at most
 *     400 cells. Face order in a bucket: triangle id, then cell loop order (z, y, x) — the
 *     reference's serial (CPU-emulation) insertion order.
 * ============================================================================================= */
#define HG_BUCKETS 65536u  /* MAX_HASH_ELEMENTS, BuildTree.cuh:21 */
#define HG_CAP 256u        /* NUM_FACES_PER_CELL, Hash.cu:7 */
#define HG_ITERS 400       /* MAX_SEARCH_ITERS, Hash.cu:11 */
#define HG_MAX_CELLS (1u << 20) /* cells per triangle AABB this build accepts (the reference: any) */
static const float HG_CELL = 0.03f;           /* CELL_RES */
static const float HG_INV = 1.f / 0.03f;      /* INV_CELL_RES, a float constant */
static const float HG_EPS = 0.03f * 0.001f;   /* CELL_PINCH_TROUGH_EPSILON */

struct orc_hash {
    soup s;
    uint32_t* start; /* HG_BUCKETS + 1 */
    uint32_t* faces; /* bucket-major, insertion order */
    uint64_t pairs;
};

/* Fletcher-16 of a u32 (bmHash, Hash.cu:15-31) */
static inline uint32_t hg_f16(uint32_t h) {
    uint32_t s1 = 0, s2 = 0;
    for (int b = 0; b < 4; ++b) {
        s1 = (s1 + ((h >> (8 * b)) & 255u)) % 255u;
        s2 = (s2 + s1) % 255u;
    }
    return (s2 << 8) | s1;
}
static inline uint32_t hg_hash3(int32_t x, int32_t y, int32_t z) {
    return (hg_f16((uint32_t)x) + hg_f16((uint32_t)y) + hg_f16((uint32_t)z)) % HG_BUCKETS;
}
/* bmMap (Hash.cu:57-60): floor(f / cell) as i32; out-of-range saturates, NaN maps to 0 (the
 * reference's cast is undefined there; gfx950's v_cvt_i32_f32 saturates likewise) */
static inline int32_t hg_map(float f) {
    float q = floorf(f * HG_INV);
    if (q != q) return 0;
    if (q >= 2147483648.f) return INT32_MAX;
    if (q < -2147483648.f) return INT32_MIN;
    return (int32_t)q;
}

/* cells of triangle g: calls fn(hash) in insertion order; returns 0, or -1 when the AABB spans
 * more than HG_MAX_CELLS cells */
static int hg_tri_cells(const orc_hash* h, uint32_t g, uint32_t* out_hash, uint64_t* count) {
    const float* v = h->s.v + (size_t)g * 9;
    float tmin[3], tmax[3];
    for (int c = 0; c < 3; ++c) {
        tmin[c] = rmin(v[c], rmin(v[3 + c], v[6 + c]));
        tmax[c] = rmax(v[c], rmax(v[3 + c], v[6 + c]));
    }
    int64_t lo[3], hi[3], span = 1;
    for (int c = 0; c < 3; ++c) {
        lo[c] = hg_map(tmin[c]);
        hi[c] = hg_map(tmax[c]);
        span *= hi[c] >= lo[c] ? hi[c] - lo[c] + 1 : 0;
        if (span > HG_MAX_CELLS) return -1;
    }
    uint64_t k = 0;
    for (int64_t z = lo[2]; z <= hi[2]; ++z)
        for (int64_t y = lo[1]; y <= hi[1]; ++y)
            for (int64_t x = lo[0]; x <= hi[0]; ++x) {
                float bmn[3] = {(float)(int32_t)x * HG_CELL, (float)(int32_t)y * HG_CELL, (float)(int32_t)z * HG_CELL};
                float bc[3], hs[3];
                for (int c = 0; c < 3; ++c) {
                    float bmx = bmn[c] + HG_CELL;
                    bc[c] = (bmx + bmn[c]) * .5f;
                    hs[c] = (bmx - bmn[c]) * .5f;
                }
                if (tri_box(bc, hs, v)) {
                    if (out_hash) out_hash[k] = hg_hash3((int32_t)x, (int32_t)y, (int32_t)z);
                    ++k;
                }
            }
    *count = k;
    return 0;
}

orc_hash* orc_hash_build(const orc_mesh* meshes, uint32_t num_meshes) {
    orc_hash* h = (orc_hash*)calloc(1, sizeof(orc_hash));
    soup_make(&h->s, meshes, num_meshes);
    uint32_t n = h->s.n;
    uint64_t* cnt = (uint64_t*)calloc(n ? n : 1, sizeof(uint64_t));
    uint64_t total = 0;
    for (uint32_t g = 0; g < n; ++g) {
        if (hg_tri_cells(h, g, NULL, &cnt[g]) != 0) {
            free(cnt);
            orc_hash_free(h);
            return NULL;
        }
        total += cnt[g];
    }
    uint32_t* hk = (uint32_t*)malloc(sizeof(uint32_t) * (total ? total : 1));
    uint32_t* hv = (uint32_t*)malloc(sizeof(uint32_t) * (total ? total : 1));
    uint64_t o = 0;
    for (uint32_t g = 0; g < n; ++g) {
        uint64_t k;
        hg_tri_cells(h, g, hk + o, &k);
        for (uint64_t j = 0; j < k; ++j) hv[o + j] = g;
        o += k;
    }
    /* stable counting sort by bucket */
    h->start = (uint32_t*)calloc(HG_BUCKETS + 1, sizeof(uint32_t));
    for (uint64_t i = 0; i < total; ++i) h->start[hk[i] + 1]++;
    for (uint32_t b = 0; b < HG_BUCKETS; ++b) h->start[b + 1] += h->start[b];
    uint32_t* fill = (uint32_t*)malloc(sizeof(uint32_t) * HG_BUCKETS);
    memcpy(fill, h->start, sizeof(uint32_t) * HG_BUCKETS);
    h->faces = (uint32_t*)malloc(sizeof(uint32_t) * (total ? total : 1));
    for (uint64_t i = 0; i < total; ++i) h->faces[fill[hk[i]]++] = hv[i];
    h->pairs = total;
    free(fill);
    free(hk);
    free(hv);
    free(cnt);
    return h;
}

void orc_hash_free(orc_hash* h) {
    if (!h) return;
    soup_free(&h->s);
    free(h->start);
    free(h->faces);
    free(h);
}

void orc_hash_stats(const orc_hash* h, uint64_t stats[4]) {
    stats[0] = h->pairs;
    stats[1] = stats[2] = stats[3] = 0;
    for (uint32_t b = 0; b < HG_BUCKETS; ++b) {
        uint32_t c = h->start[b + 1] - h->start[b];
        if (c) stats[1]++;
        if (c > stats[2]) stats[2] = c;
        if (c > HG_CAP) stats[3] += c - HG_CAP;
    }
}

const uint32_t* orc_hash_buckets(const orc_hash* h, const uint32_t** faces) {
    if (faces) *faces = h->faces;
    return h->start;
}

/* bmBoxRayIntersectNoZero (CudaComon.cuh:176-187) */
static inline float hg_box_exit(const float* bmn, const float* bmx, const float* o, const float* inv) {
    float t0[3], t1[3], tn[3], tf[3];
    for (int c = 0; c < 3; ++c) {
        t0[c] = (bmn[c] - o[c]) * inv[c];
        t1[c] = (bmx[c] - o[c]) * inv[c];
        tn[c] = rmin(t0[c], t1[c]);
        tf[c] = rmax(t0[c], t1[c]);
    }
    float ftmin = rmax(tn[0], rmax(tn[1], tn[2]));
    float ftmax = rmin(tf[0], rmin(tf[1], tf[2]));
    return (isinf(ftmin) || ftmin < 0.f) ? ftmax : ftmin;
}

int32_t orc_hash_march(const orc_hash* h, const float* rays, uint32_t begin, uint32_t end, const float eye[3],
                       const float orient[9], uint32_t* packed, uint32_t* tri_id, float* tout) {
    if (!h->s.nn && h->s.n) return ORC_ERR_INVALID_FORMAT;
    for (uint32_t i = begin; i < end; ++i) {
        float dir[3], inv[3], pp[3];
        orient_dir(dir, orient, rays + (size_t)i * 3);
        for (int c = 0; c < 3; ++c) {
            inv[c] = 1.f / dir[c];
            pp[c] = eye[c];
        }
        float dclosest = FLT_MAX, tu = 0, tv = 0;
        uint32_t fclosest = NO_TRI;
        for (int it = 0; it < HG_ITERS; ++it) {
            int32_t cp[3] = {hg_map(pp[0]), hg_map(pp[1]), hg_map(pp[2])};
            uint32_t b = hg_hash3(cp[0], cp[1], cp[2]);
            uint32_t c0 = h->start[b], cnt = h->start[b + 1] - c0;
            if (cnt) {
                if (cnt > HG_CAP) cnt = HG_CAP;
                for (uint32_t k = 0; k < cnt; ++k) {
                    uint32_t g = h->faces[c0 + k];
                    const float* v = h->s.v + (size_t)g * 9;
                    float u, vv;
                    float d = tri_intersect(eye, dir, v, v + 3, v + 6, &u, &vv);
                    if (d < dclosest) {
                        dclosest = d;
                        fclosest = g;
                        tu = u;
                        tv = vv;
                    }
                }
                if (dclosest != FLT_MAX) break; /* Hash.cu:271 */
            }
            float bmn[3], bmx[3];
            for (int c = 0; c < 3; ++c) {
                bmn[c] = (float)cp[c] * HG_CELL;
                bmx[c] = bmn[c] + HG_CELL;
            }
            float step = hg_box_exit(bmn, bmx, pp, inv) + HG_EPS;
            for (int c = 0; c < 3; ++c) pp[c] = pp[c] + dir[c] * step;
        }
        if (dclosest != FLT_MAX) {
            const float* n = h->s.nn + (size_t)fclosest * 9;
            if (packed) packed[i] = shade_packed(n, n + 3, n + 6, tu, tv);
            if (tri_id) tri_id[i] = fclosest;
            if (tout) tout[i] = dclosest;
        } else {
            if (packed) packed[i] = MISS_PACKED;
            if (tri_id) tri_id[i] = NO_TRI;
            if (tout) tout[i] = INFINITY;
        }
    }
    return ORC_ERR_FINE;
}

/* =============================================================================================
 * 2. Closest-hit LBVH — the algorithm of raytracercuda_amd/csrc/bvh_build.hip + trace.hip.
 *    Everything here must produce bit-identical records to the HIP build (tests compare them).
 * ============================================================================================= */
#define LEAF_BIT 0x80000000u
#define EMPTY_REF 0xFFFFFFFFu
#define PAD_SCALE 0x1p-20f

struct orc_bvh {
    soup s;
    uint32_t n, leaf_size, num_records, width; /* width 2: BVH2 records, 4: BVH4 records */
    uint32_t* keys;    /* sorted */
    uint32_t* perm;    /* sorted position -> global id */
    uint32_t* records; /* num_records * orc_bvh_record_words (16 / 32 / 64) */
    uint32_t* tris;    /* n * 12, sorted order */
    uint32_t *lch, *rch, *first, *last; /* Karras tree (n-1 nodes), kept for orc_bvh_refit */
};

/* Order-independent min/max for stored bounds: compare the floats' ordered-integer images, a
 * total order in which -0 < +0 (fminf(+0,-0) vs fminf(-0,+0) differ on glibc and on the GPU).
 * Shared bit-for-bit with bm_omin/bm_omax in raytracercuda_amd/csrc/bm_common.h. */
static inline int32_t ord_i(float f) {
    int32_t i;
    memcpy(&i, &f, 4);
    return i >= 0 ? i : (i ^ 0x7FFFFFFF);
}
static inline float omin(float a, float b) { return ord_i(b) < ord_i(a) ? b : a; }
static inline float omax(float a, float b) { return ord_i(b) > ord_i(a) ? b : a; }

static inline uint32_t expand_bits10(uint32_t v) {
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}

static inline uint32_t quant10(float c, float cmin, float scale) {
    float q = (c - cmin) * scale;
    if (!(q > 0.0f)) return 0u;
    if (q >= 1023.0f) return 1023u;
    return (uint32_t)q;
}

static inline int clz32(uint32_t x) { return x ? __builtin_clz(x) : 32; }

/* Karras 2012 common-prefix length with the position tiebreak for equal keys. */
static inline int delta(const uint32_t* k, int64_t n, int64_t i, int64_t j) {
    if (j < 0 || j >= n) return -1;
    uint32_t a = k[i], b = k[j];
    if (a == b) return 32 + clz32((uint32_t)i ^ (uint32_t)j);
    return clz32(a ^ b);
}

static inline void pad_box(float* lo, float* hi, float pad) {
    for (int c = 0; c < 3; ++c) {
        lo[c] = lo[c] - (fabsf(lo[c]) * PAD_SCALE + pad);
        hi[c] = hi[c] + (fabsf(hi[c]) * PAD_SCALE + pad);
    }
}

static inline uint32_t fbits(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
}

static void write_child(uint32_t* rec, int slot, const float* lo, const float* hi, uint32_t ref) {
    for (int c = 0; c < 3; ++c) {
        rec[slot * 6 + c] = fbits(lo[c]);
        rec[slot * 6 + 3 + c] = fbits(hi[c]);
    }
    rec[12 + slot] = ref;
}

static void write_empty_child(uint32_t* rec, int slot) {
    for (int c = 0; c < 6; ++c) rec[slot * 6 + c] = 0x7FC00000u; /* quiet NaN box: never hit */
    rec[12 + slot] = EMPTY_REF;
}

/* BVH4 record (32 u32 = 128 B): child boxes SoA [0..3] lo.x [4..7] lo.y [8..11] lo.z [12..15] hi.x
 * [16..19] hi.y [20..23] hi.z, [24..27] refs, [28..31] 0; empty slot = NaN box + EMPTY_REF. */
/* Wide records, W = 4 or 8 (BVH8: 64 u32 = 256 B, [0..7] lo.x ... [40..47] hi.z, [48..55] refs,
 * [56..63] 0): plane p of child `slot` at rec[W*p + slot], refs at rec[6W + slot]. */
static void write_childw(uint32_t* rec, int W, int slot, const float* lo, const float* hi, uint32_t ref) {
    for (int c = 0; c < 3; ++c) {
        rec[W * c + slot] = fbits(lo[c]);
        rec[3 * W + W * c + slot] = fbits(hi[c]);
    }
    rec[6 * W + slot] = ref;
}

static void write_empty_childw(uint32_t* rec, int W, int slot) {
    for (int c = 0; c < 6; ++c) rec[W * c + slot] = 0x7FC00000u;
    rec[6 * W + slot] = EMPTY_REF;
}

orc_bvh* orc_bvh_build(const orc_mesh* meshes, uint32_t num_meshes, uint32_t leaf_size) {
    return orc_bvh_build_ex(meshes, num_meshes, leaf_size, 2);
}

uint32_t orc_bvh_record_words(const orc_bvh* b) { return b->width == 8 ? 64u : b->width == 4 ? 32u : 16u; }

static void bvh_make(orc_bvh* b, int refit);

orc_bvh* orc_bvh_build_ex(const orc_mesh* meshes, uint32_t num_meshes, uint32_t leaf_size, uint32_t width) {
    if (leaf_size < 1) leaf_size = 1;
    if (leaf_size > 16) leaf_size = 16;
    orc_bvh* b = (orc_bvh*)calloc(1, sizeof(orc_bvh));
    b->width = width == 8 ? 8 : width == 4 ? 4 : 2;
    soup_make(&b->s, meshes, num_meshes);
    b->n = b->s.n;
    b->leaf_size = leaf_size;
    b->num_records = b->n > 1 ? b->n - 1 : 1;
    bvh_make(b, 0);
    return b;
}

/* Refit (bm_scene_refit): new vertex positions/normals, the previous build's topology (sorted
 * order, radix tree, leaf collapse, BVH4 node set); boxes, triangle records and node records
 * recomputed exactly as a build computes them. Same triangle count required. */
int32_t orc_bvh_refit(orc_bvh* b, const orc_mesh* meshes, uint32_t num_meshes) {
    soup s;
    soup_make(&s, meshes, num_meshes);
    if (s.n != b->n) {
        soup_free(&s);
        return ORC_ERR_INVALID_PARAMETER;
    }
    soup_free(&b->s);
    b->s = s;
    free(b->tris);
    free(b->records);
    bvh_make(b, 1);
    return ORC_ERR_FINE;
}

/* Experiment hook (tools/ only): a BVH over a caller-given binary tree — perm[n] (leaf order ->
 * global id), lch/rch[n-1] (children; leaf k as k|LEAF_BIT, root = internal node 0) — packed,
 * collapsed and traversed exactly as an LBVH. Used to measure other builders' tree quality with the
 * same traversal and counters. */
orc_bvh* orc_bvh_build_tree(const orc_mesh* meshes, uint32_t num_meshes, uint32_t leaf_size, uint32_t width,
                            const uint32_t* perm, const uint32_t* lch, const uint32_t* rch) {
    orc_bvh* b = (orc_bvh*)calloc(1, sizeof(orc_bvh));
    b->width = width == 8 ? 8 : width == 4 ? 4 : 2;
    soup_make(&b->s, meshes, num_meshes);
    const uint32_t n = b->n = b->s.n;
    b->leaf_size = leaf_size < 1 ? 1 : leaf_size > 16 ? 16 : leaf_size;
    b->num_records = n > 1 ? n - 1 : 1;
    size_t nn = n ? n : 1, m = n > 1 ? n - 1 : 1;
    b->keys = (uint32_t*)calloc(nn, 4);
    b->perm = (uint32_t*)malloc(4 * nn);
    memcpy(b->perm, perm, 4 * (size_t)n);
    b->lch = (uint32_t*)malloc(4 * m);
    b->rch = (uint32_t*)malloc(4 * m);
    b->first = (uint32_t*)malloc(4 * m);
    b->last = (uint32_t*)malloc(4 * m);
    if (n > 1) {
        memcpy(b->lch, lch, 4 * (size_t)(n - 1));
        memcpy(b->rch, rch, 4 * (size_t)(n - 1));
        /* ranges bottom-up: children before parents in a post-order walk */
        uint32_t* stk = (uint32_t*)malloc(sizeof(uint32_t) * 2 * (n + 1));
        uint8_t* done = (uint8_t*)calloc(n - 1, 1);
        int64_t sp = 0;
        stk[sp++] = 0;
        while (sp > 0) {
            uint32_t i = stk[sp - 1];
            uint32_t c[2] = {b->lch[i], b->rch[i]};
            if (!done[i]) {
                done[i] = 1;
                for (int q = 0; q < 2; ++q)
                    if (!(c[q] & LEAF_BIT)) stk[sp++] = c[q];
                continue;
            }
            sp--;
            uint32_t f[2], l[2];
            for (int q = 0; q < 2; ++q) {
                uint32_t cc = c[q] & ~LEAF_BIT;
                f[q] = (c[q] & LEAF_BIT) ? cc : b->first[cc];
                l[q] = (c[q] & LEAF_BIT) ? cc : b->last[cc];
            }
            b->first[i] = f[0];
            b->last[i] = l[1];
        }
        free(stk);
        free(done);
    }
    bvh_make(b, 1);
    return b;
}

/* Geometry -> (topology unless refit) -> triangle records, refit, pack. */
static void bvh_make(orc_bvh* b, int refit) {
    const uint32_t RW = orc_bvh_record_words(b);
    const int WW = (int)b->width; /* slots of a wide record (4 or 8) */
    const uint32_t n = b->n, leaf_size = b->leaf_size;
    size_t nn = n ? n : 1;
    float* bmn = (float*)malloc(sizeof(float) * 3 * nn);
    float* bmx = (float*)malloc(sizeof(float) * 3 * nn);
    float* cen = (float*)malloc(sizeof(float) * 3 * nn);
    float smn[3] = {INFINITY, INFINITY, INFINITY}, smx[3] = {-INFINITY, -INFINITY, -INFINITY};
    float cmn[3] = {INFINITY, INFINITY, INFINITY}, cmx[3] = {-INFINITY, -INFINITY, -INFINITY};
    /* per-triangle AABB + centroid; scene and centroid bounds (bm_tri_prepare + bm_bounds) */
    for (uint32_t g = 0; g < n; ++g) {
        const float* v = b->s.v + (size_t)g * 9;
        for (int c = 0; c < 3; ++c) {
            bmn[g * 3 + c] = omin(omin(v[c], v[3 + c]), v[6 + c]);
            bmx[g * 3 + c] = omax(omax(v[c], v[3 + c]), v[6 + c]);
            cen[g * 3 + c] = (bmn[g * 3 + c] + bmx[g * 3 + c]) * 0.5f;
            smn[c] = omin(smn[c], bmn[g * 3 + c]);
            smx[c] = omax(smx[c], bmx[g * 3 + c]);
            cmn[c] = omin(cmn[c], cen[g * 3 + c]);
            cmx[c] = omax(cmx[c], cen[g * 3 + c]);
        }
    }
    if (!refit) {
    /* Morton keys (bm_morton) */
    float scale[3];
    for (int c = 0; c < 3; ++c) {
        float ext = cmx[c] - cmn[c];
        scale[c] = ext > 0.0f ? 1024.0f / ext : 0.0f;
    }
    uint32_t* key = (uint32_t*)malloc(sizeof(uint32_t) * nn);
    uint32_t* val = (uint32_t*)malloc(sizeof(uint32_t) * nn);
    uint32_t* k2 = (uint32_t*)malloc(sizeof(uint32_t) * nn);
    uint32_t* v2 = (uint32_t*)malloc(sizeof(uint32_t) * nn);
    for (uint32_t g = 0; g < n; ++g) {
        uint32_t qx = quant10(cen[g * 3 + 0], cmn[0], scale[0]);
        uint32_t qy = quant10(cen[g * 3 + 1], cmn[1], scale[1]);
        uint32_t qz = quant10(cen[g * 3 + 2], cmn[2], scale[2]);
        key[g] = (expand_bits10(qx) << 2) | (expand_bits10(qy) << 1) | expand_bits10(qz);
        val[g] = g;
    }
    /* stable LSD radix sort, 8-bit digits (bm_radix_sort) */
    for (int pass = 0; pass < 4; ++pass) {
        uint32_t cnt[257];
        memset(cnt, 0, sizeof(cnt));
        int sh = pass * 8;
        for (uint32_t i = 0; i < n; ++i) cnt[((key[i] >> sh) & 255u) + 1]++;
        for (int d = 0; d < 256; ++d) cnt[d + 1] += cnt[d];
        for (uint32_t i = 0; i < n; ++i) {
            uint32_t d = (key[i] >> sh) & 255u;
            k2[cnt[d]] = key[i];
            v2[cnt[d]] = val[i];
            cnt[d]++;
        }
        uint32_t* t = key; key = k2; k2 = t;
        t = val; val = v2; v2 = t;
    }
    free(k2);
    free(v2);
    b->keys = key;
    b->perm = val;
    }
    const uint32_t* key = b->keys;
    const uint32_t* val = b->perm;

    /* sorted triangle records: (v0, id) (e1, 0) (e2, 0) */
    b->tris = (uint32_t*)calloc(12 * nn, sizeof(uint32_t));
    for (uint32_t k = 0; k < n; ++k) {
        uint32_t g = val[k];
        const float* v = b->s.v + (size_t)g * 9;
        float e1[3], e2[3];
        sub3(e1, v + 3, v);
        sub3(e2, v + 6, v);
        uint32_t* r = b->tris + (size_t)k * 12;
        for (int c = 0; c < 3; ++c) {
            r[c] = fbits(v[c]);
            r[4 + c] = fbits(e1[c]);
            r[8 + c] = fbits(e2[c]);
        }
        r[3] = g;
    }

    float sext = omax(omax(smx[0] - smn[0], smx[1] - smn[1]), smx[2] - smn[2]);
    float pad = sext * PAD_SCALE;
    b->records = (uint32_t*)calloc(RW * (size_t)b->num_records, sizeof(uint32_t));

    if (n <= 1) {
        if (n == 1) {
            float lo[3] = {bmn[0], bmn[1], bmn[2]}, hi[3] = {bmx[0], bmx[1], bmx[2]};
            pad_box(lo, hi, pad);
            if (RW >= 32) write_childw(b->records, WW, 0, lo, hi, LEAF_BIT | 0u);
            else write_child(b->records, 0, lo, hi, LEAF_BIT | 0u);
        } else {
            if (RW >= 32) write_empty_childw(b->records, WW, 0);
            else write_empty_child(b->records, 0);
        }
        if (RW >= 32)
            for (int q = 1; q < WW; ++q) write_empty_childw(b->records, WW, q);
        else
            write_empty_child(b->records, 1);
    } else {
        const int64_t m = (int64_t)n - 1;
        if (!refit) {
            b->lch = (uint32_t*)malloc(sizeof(uint32_t) * m); /* child: leaf k -> k|LEAF_BIT */
            b->rch = (uint32_t*)malloc(sizeof(uint32_t) * m);
            b->first = (uint32_t*)malloc(sizeof(uint32_t) * m);
            b->last = (uint32_t*)malloc(sizeof(uint32_t) * m);
        }
        uint32_t *lch = b->lch, *rch = b->rch, *first = b->first, *last = b->last;
        /* Karras emit (bm_lbvh_emit) */
        for (int64_t i = 0; i < m && !refit; ++i) {
            int d = (delta(key, n, i, i + 1) - delta(key, n, i, i - 1)) >= 0 ? 1 : -1;
            int dmin = delta(key, n, i, i - d);
            int64_t lmax = 2;
            while (delta(key, n, i, i + lmax * d) > dmin) lmax *= 2;
            int64_t l = 0;
            for (int64_t t = lmax / 2; t >= 1; t /= 2)
                if (delta(key, n, i, i + (l + t) * d) > dmin) l += t;
            int64_t j = i + l * d;
            int dnode = delta(key, n, i, j);
            int64_t s = 0;
            int64_t t = l;
            do {
                t = (t + 1) / 2;
                if (delta(key, n, i, i + (s + t) * d) > dnode) s += t;
            } while (t > 1);
            int64_t gamma = i + s * d + (d < 0 ? d : 0);
            int64_t lo = i < j ? i : j, hi = i < j ? j : i;
            lch[i] = (lo == gamma) ? ((uint32_t)gamma | LEAF_BIT) : (uint32_t)gamma;
            rch[i] = (hi == gamma + 1) ? ((uint32_t)(gamma + 1) | LEAF_BIT) : (uint32_t)(gamma + 1);
            first[i] = (uint32_t)lo;
            last[i] = (uint32_t)hi;
        }
        /* refit (bm_refit): post-order over the binary radix tree */
        float* ibmn = (float*)malloc(sizeof(float) * 3 * m);
        float* ibmx = (float*)malloc(sizeof(float) * 3 * m);
        uint32_t* stk = (uint32_t*)malloc(sizeof(uint32_t) * 2 * (m + 1));
        uint8_t* done = (uint8_t*)calloc(m, 1);
        int64_t sp = 0;
        stk[sp++] = 0;
        while (sp > 0) {
            uint32_t i = stk[sp - 1];
            uint32_t c[2] = {lch[i], rch[i]};
            if (!done[i]) {
                done[i] = 1;
                for (int q = 0; q < 2; ++q)
                    if (!(c[q] & LEAF_BIT)) stk[sp++] = c[q];
                continue;
            }
            sp--;
            float lo[2][3], hi[2][3];
            for (int q = 0; q < 2; ++q) {
                uint32_t cc = c[q] & ~LEAF_BIT;
                const float* pmn = (c[q] & LEAF_BIT) ? bmn + (size_t)val[cc] * 3 : ibmn + (size_t)cc * 3;
                const float* pmx = (c[q] & LEAF_BIT) ? bmx + (size_t)val[cc] * 3 : ibmx + (size_t)cc * 3;
                memcpy(lo[q], pmn, 12);
                memcpy(hi[q], pmx, 12);
            }
            for (int a = 0; a < 3; ++a) {
                ibmn[(size_t)i * 3 + a] = omin(lo[0][a], lo[1][a]);
                ibmx[(size_t)i * 3 + a] = omax(hi[0][a], hi[1][a]);
            }
        }
        free(stk);
        free(done);
        /* pack with leaf collapse (bm_pack) */
        const uint32_t K = leaf_size;
        if (RW >= 32) {
            /* BVH4 (bm_pack4): a record for the root and every non-collapsed internal node at even
             * depth; its children are its binary children with each non-collapsed internal child
             * replaced by that child's two children (every other level collapsed). BVH8: depth a
             * multiple of 3, children the frontier three binary levels down (two levels of
             * expansion). */
            const int L = WW == 8 ? 3 : 2; /* binary levels per wide level */
            uint8_t* lvl = (uint8_t*)calloc(m, 1); /* depth mod L */
            uint32_t* dstk = (uint32_t*)malloc(sizeof(uint32_t) * (m + 1));
            int64_t dsp = 0;
            dstk[dsp++] = 0;
            while (dsp > 0) {
                uint32_t i = dstk[--dsp];
                uint32_t c[2] = {lch[i], rch[i]};
                for (int q = 0; q < 2; ++q)
                    if (!(c[q] & LEAF_BIT)) {
                        lvl[c[q]] = (uint8_t)((lvl[i] + 1) % L);
                        dstk[dsp++] = c[q];
                    }
            }
            free(dstk);
            for (int64_t i = 0; i < m; ++i) {
                uint32_t* rec = b->records + (size_t)i * RW;
                uint32_t cnt = last[i] - first[i] + 1;
                if (i != 0 && (cnt <= K || lvl[i])) continue;
                int nslot = 0;
                if (cnt <= K) { /* root is a leaf */
                    float lo[3], hi[3];
                    memcpy(lo, ibmn, 12);
                    memcpy(hi, ibmx, 12);
                    pad_box(lo, hi, pad);
                    write_childw(rec, WW, nslot++, lo, hi, LEAF_BIT | ((cnt - 1) << 27) | 0u);
                } else {
                    /* frontier: expand non-collapsed internal nodes up to L-1 times, in child order */
                    uint32_t fr[8], nf = 0, nx[8];
                    fr[nf++] = lch[i];
                    fr[nf++] = rch[i];
                    for (int e = 1; e < L; ++e) {
                        uint32_t nn = 0;
                        for (uint32_t k = 0; k < nf; ++k) {
                            uint32_t cc = fr[k] & ~LEAF_BIT;
                            if (!(fr[k] & LEAF_BIT) && (last[cc] - first[cc] + 1) > K) {
                                nx[nn++] = lch[cc];
                                nx[nn++] = rch[cc];
                            } else {
                                nx[nn++] = fr[k];
                            }
                        }
                        memcpy(fr, nx, sizeof(uint32_t) * nn);
                        nf = nn;
                    }
                    for (uint32_t k = 0; k < nf; ++k) {
                        uint32_t gc = fr[k] & ~LEAF_BIT;
                        float lo[3], hi[3];
                        uint32_t ref;
                        if (fr[k] & LEAF_BIT) {
                            memcpy(lo, bmn + (size_t)val[gc] * 3, 12);
                            memcpy(hi, bmx + (size_t)val[gc] * 3, 12);
                            ref = LEAF_BIT | gc;
                        } else {
                            uint32_t gn = last[gc] - first[gc] + 1;
                            memcpy(lo, ibmn + (size_t)gc * 3, 12);
                            memcpy(hi, ibmx + (size_t)gc * 3, 12);
                            ref = gn <= K ? (LEAF_BIT | ((gn - 1) << 27) | first[gc]) : gc;
                        }
                        pad_box(lo, hi, pad);
                        write_childw(rec, WW, nslot++, lo, hi, ref);
                    }
                }
                for (; nslot < WW; ++nslot) write_empty_childw(rec, WW, nslot);
            }
            free(lvl);
        }
        for (int64_t i = 0; i < m && RW == 16; ++i) {
            uint32_t* rec = b->records + (size_t)i * 16;
            uint32_t cnt = last[i] - first[i] + 1;
            if (i != 0 && cnt <= K) continue; /* collapsed into a leaf of its parent: zeros */
            if (i == 0 && cnt <= K) {
                float lo[3], hi[3];
                memcpy(lo, ibmn, 12);
                memcpy(hi, ibmx, 12);
                pad_box(lo, hi, pad);
                write_child(rec, 0, lo, hi, LEAF_BIT | ((cnt - 1) << 27) | 0u);
                write_empty_child(rec, 1);
                continue;
            }
            uint32_t c[2] = {lch[i], rch[i]};
            for (int q = 0; q < 2; ++q) {
                uint32_t cc = c[q] & ~LEAF_BIT;
                float lo[3], hi[3];
                uint32_t cf, cn;
                if (c[q] & LEAF_BIT) {
                    memcpy(lo, bmn + (size_t)val[cc] * 3, 12);
                    memcpy(hi, bmx + (size_t)val[cc] * 3, 12);
                    cf = cc;
                    cn = 1;
                } else {
                    memcpy(lo, ibmn + (size_t)cc * 3, 12);
                    memcpy(hi, ibmx + (size_t)cc * 3, 12);
                    cf = first[cc];
                    cn = last[cc] - first[cc] + 1;
                }
                pad_box(lo, hi, pad);
                uint32_t ref = (cn <= K) ? (LEAF_BIT | ((cn - 1) << 27) | cf) : cc;
                write_child(rec, q, lo, hi, ref);
            }
        }
        free(ibmn);
        free(ibmx);
    }
    free(bmn);
    free(bmx);
    free(cen);
}

void orc_bvh_free(orc_bvh* b) {
    if (!b) return;
    soup_free(&b->s);
    free(b->keys);
    free(b->perm);
    free(b->records);
    free(b->tris);
    free(b->lch);
    free(b->rch);
    free(b->first);
    free(b->last);
    free(b);
}

uint32_t orc_bvh_num_tris(const orc_bvh* b) { return b->n; }
uint32_t orc_bvh_num_records(const orc_bvh* b) { return b->num_records; }

void orc_bvh_export(const orc_bvh* b, uint32_t* records, uint32_t* tris, uint32_t* keys,
                    uint32_t* perm) {
    if (records) memcpy(records, b->records, sizeof(uint32_t) * orc_bvh_record_words(b) * (size_t)b->num_records);
    if (tris && b->n) memcpy(tris, b->tris, sizeof(uint32_t) * 12 * (size_t)b->n);
    if (keys && b->n) memcpy(keys, b->keys, sizeof(uint32_t) * b->n);
    if (perm && b->n) memcpy(perm, b->perm, sizeof(uint32_t) * b->n);
}

static inline float bitsf(uint32_t u) {
    float f;
    memcpy(&f, &u, 4);
    return f;
}

/* Slab test of one child box (bm_trace_primary's box test): conservative entry/exit with IEEE
 * fminf/fmaxf (a NaN slab is ignored; an all-NaN box never hits). */
static inline int child_hit(const uint32_t* rec, int slot, const float* o, const float* inv,
                            float tbest, float* tn_out) {
    float tlo[3], thi[3];
    for (int c = 0; c < 3; ++c) {
        tlo[c] = (bitsf(rec[slot * 6 + c]) - o[c]) * inv[c];
        thi[c] = (bitsf(rec[slot * 6 + 3 + c]) - o[c]) * inv[c];
    }
    float tn = fmaxf(fmaxf(fminf(tlo[0], thi[0]), fminf(tlo[1], thi[1])), fminf(tlo[2], thi[2]));
    float tf = fminf(fminf(fmaxf(tlo[0], thi[0]), fmaxf(tlo[1], thi[1])), fmaxf(tlo[2], thi[2]));
    *tn_out = tn;
    return (tn <= tf) && (tf >= 0.0f) && (tn <= tbest);
}

#define TRACE_STACK 128

static inline int child_hitw(const uint32_t* rec, int W, int slot, const float* o, const float* inv,
                             float tbest, float* tn_out) {
    float tlo[3], thi[3];
    for (int c = 0; c < 3; ++c) {
        tlo[c] = (bitsf(rec[W * c + slot]) - o[c]) * inv[c];
        thi[c] = (bitsf(rec[3 * W + W * c + slot]) - o[c]) * inv[c];
    }
    float tn = fmaxf(fmaxf(fminf(tlo[0], thi[0]), fminf(tlo[1], thi[1])), fminf(tlo[2], thi[2]));
    float tf = fminf(fminf(fmaxf(tlo[0], thi[0]), fmaxf(tlo[1], thi[1])), fmaxf(tlo[2], thi[2]));
    *tn_out = tn;
    return (tn <= tf) && (tf >= 0.0f) && (tn <= tbest);
}

/* Order key of a BVH4 child (bm_common.h order_key): the entry distance clamped at 0, as its bit
 * image with the slot in place of the last two mantissa bits — distinct per slot, so
 * one unsigned compare orders two children (nearest first, near-ties by slot). */
static inline uint32_t order_key(float tn, uint32_t slot) {
    int32_t b;
    memcpy(&b, &tn, 4);
    if (b < 0) b = 0;
    return ((uint32_t)b & ~3u) | slot;
}

/* BVH8: the same with the slot in the last three mantissa bits. */
static inline uint32_t order_key8(float tn, uint32_t slot) {
    int32_t b;
    memcpy(&b, &tn, 4);
    if (b < 0) b = 0;
    return ((uint32_t)b & ~7u) | slot;
}

/* Visit one record (bm_trace's node step): slab-test its children against [.., tmax], continue with
 * the nearest hit child and push the other hit children farthest first, so they pop nearest first.
 * Order among hit children: BVH4 by order_key, BVH8 by order_key8, BVH2 the stable sort by entry
 * distance (ties: lower slot first). Returns the next ref, or EMPTY_REF when no child is hit. */
/* per thread: the bench's CPU baseline calls orc_bvh_trace from several threads at once */
static _Thread_local int g_max_stack;
static uint32_t visit_node(const orc_bvh* b, uint32_t node, const float* o, const float* inv, float tmax,
                           uint32_t* stk_ref, float* stk_t, int* sp) {
    const int W = (int)b->width;
    const uint32_t* rec = b->records + (size_t)node * orc_bvh_record_words(b);
    float tn[8];
    int hit[8];
    uint32_t ref[8];
    for (int c = 0; c < W; ++c) {
        hit[c] = W >= 4 ? child_hitw(rec, W, c, o, inv, tmax, &tn[c]) : child_hit(rec, c, o, inv, tmax, &tn[c]);
        ref[c] = W >= 4 ? rec[6 * W + c] : rec[12 + c];
    }
    uint32_t by_ref[8], key[8];
    float by_t[8];
    int nh = 0;
    for (int c = 0; c < W; ++c)
        key[c] = !hit[c] ? 0xFFFFFFFFu : W == 8 ? order_key8(tn[c], (uint32_t)c) : order_key(tn[c], (uint32_t)c);
    for (int c = 0; c < W; ++c) {
        if (!hit[c]) continue;
        nh++;
        int r = 0;
        for (int d = 0; d < W; ++d)
            if (W >= 4 ? key[d] < key[c] : hit[d] && (tn[d] < tn[c] || (tn[d] == tn[c] && d < c))) r++;
        by_ref[r] = ref[c];
        by_t[r] = tn[c];
    }
    if (nh == 0) return EMPTY_REF;
    for (int r = nh - 1; r >= 1; --r) {
        stk_ref[*sp] = by_ref[r];
        stk_t[*sp] = by_t[r];
        (*sp)++;
    }
    if (*sp > g_max_stack) g_max_stack = *sp;
    return by_ref[0];
}

/* Optional per-ray work record (2 u32 per ray: node records, triangle tests), for the traversal
 * analysis in tools/; NULL by default. */
static uint32_t* g_ray_stats = NULL;
void orc_set_ray_stats(uint32_t* per_ray) { g_ray_stats = per_ray; g_max_stack = 0; }
int32_t orc_max_stack(void) { return g_max_stack; }

int32_t orc_bvh_trace(const orc_bvh* b, const float* rays, uint32_t begin, uint32_t end,
                      const float eye[3], const float orient[9], uint32_t* packed,
                      uint32_t* tri_id, float* tout, uint64_t counters[3]) {
    if (!b->s.nn && b->n) return ORC_ERR_INVALID_FORMAT;
    uint64_t c_nodes = 0, c_tris = 0, c_hits = 0;
    for (uint32_t i = begin; i < end; ++i) {
        float dir[3], inv[3];
        const uint64_t n0 = c_nodes, t0 = c_tris;
        orient_dir(dir, orient, rays + (size_t)i * 3);
        for (int c = 0; c < 3; ++c) inv[c] = 1.f / dir[c];
        float tbest = INFINITY, bu = 0, bv = 0;
        uint32_t ibest = NO_TRI;
        uint32_t stk_ref[TRACE_STACK];
        float stk_t[TRACE_STACK];
        int sp = 0;
        uint32_t next = 0; /* root record */
        for (;;) {
            if (next == EMPTY_REF) {
                /* pop until an entry that can still hold a closer hit */
                while (sp > 0 && stk_t[sp - 1] > tbest) sp--;
                if (sp == 0) break;
                sp--;
                next = stk_ref[sp];
            }
            if (next & LEAF_BIT) {
                uint32_t first = next & 0x07FFFFFFu, cnt = ((next >> 27) & 15u) + 1;
                for (uint32_t k = first; k < first + cnt; ++k) {
                    const uint32_t* r = b->tris + (size_t)k * 12;
                    float v0[3] = {bitsf(r[0]), bitsf(r[1]), bitsf(r[2])};
                    float e1[3] = {bitsf(r[4]), bitsf(r[5]), bitsf(r[6])};
                    float e2[3] = {bitsf(r[8]), bitsf(r[9]), bitsf(r[10])};
                    float u = 0, v = 0;
                    float t = tri_intersect_e(eye, dir, v0, e1, e2, &u, &v);
                    c_tris++;
                    if (t > 0.0f && t != FLT_MAX && (t < tbest || (t == tbest && r[3] < ibest))) {
                        tbest = t;
                        ibest = r[3];
                        bu = u;
                        bv = v;
                    }
                }
                next = EMPTY_REF;
                continue;
            }
            c_nodes++;
            next = visit_node(b, next, eye, inv, tbest, stk_ref, stk_t, &sp);
        }
        if (g_ray_stats) {
            g_ray_stats[2 * (size_t)i] = (uint32_t)(c_nodes - n0);
            g_ray_stats[2 * (size_t)i + 1] = (uint32_t)(c_tris - t0);
        }
        if (ibest != NO_TRI) {
            c_hits++;
            const float* n = b->s.nn + (size_t)ibest * 9;
            if (packed) packed[i] = shade_packed(n, n + 3, n + 6, bu, bv);
            if (tri_id) tri_id[i] = ibest;
            if (tout) tout[i] = tbest;
        } else {
            if (packed) packed[i] = MISS_PACKED;
            if (tri_id) tri_id[i] = NO_TRI;
            if (tout) tout[i] = INFINITY;
        }
    }
    if (counters) {
        counters[0] += c_nodes;
        counters[1] += c_tris;
        counters[2] += c_hits;
    }
    return ORC_ERR_FINE;
}

/* Shadow-ray origin and direction of a primary hit at distance t: the origin is
 * pulled back towards the eye by t*(1-1e-4), the direction is the unnormalised segment to the
 * light, so an occluder is any triangle with 0 < t_s < 1 along it. */
static inline void shadow_segment(const float* eye, const float* dir, float t, const float* light,
                                  float* o, float* d) {
    const float ts = t * 0.9999f;
    for (int c = 0; c < 3; ++c) {
        o[c] = eye[c] + dir[c] * ts;
        d[c] = light[c] - o[c];
    }
}

static inline int shadow_accept(float t) { return t > 0.0f && t < 1.0f; }

int32_t orc_bvh_shadow(const orc_bvh* b, const float* rays, uint32_t begin, uint32_t end,
                       const float eye[3], const float orient[9], const float light[3],
                       const uint32_t* tri_id, const float* tprim, uint8_t* shadow,
                       uint64_t counters[3]) {
    uint64_t c_nodes = 0, c_tris = 0, c_occ = 0;
    for (uint32_t i = begin; i < end; ++i) {
        if (tri_id[i] == NO_TRI) {
            shadow[i] = 0;
            continue;
        }
        float dir[3], o[3], d[3], inv[3];
        orient_dir(dir, orient, rays + (size_t)i * 3);
        shadow_segment(eye, dir, tprim[i], light, o, d);
        for (int c = 0; c < 3; ++c) inv[c] = 1.f / d[c];
        uint32_t stk[TRACE_STACK];
        float stk_t[TRACE_STACK];
        int sp = 0, occ = 0;
        uint32_t next = 0;
        for (;;) {
            if (next == EMPTY_REF) {
                if (sp == 0) break;
                next = stk[--sp];
            }
            if (next & LEAF_BIT) {
                uint32_t first = next & 0x07FFFFFFu, cnt = ((next >> 27) & 15u) + 1;
                for (uint32_t k = first; k < first + cnt && !occ; ++k) {
                    const uint32_t* r = b->tris + (size_t)k * 12;
                    float v0[3] = {bitsf(r[0]), bitsf(r[1]), bitsf(r[2])};
                    float e1[3] = {bitsf(r[4]), bitsf(r[5]), bitsf(r[6])};
                    float e2[3] = {bitsf(r[8]), bitsf(r[9]), bitsf(r[10])};
                    float u = 0, v = 0;
                    c_tris++;
                    if (shadow_accept(tri_intersect_e(o, d, v0, e1, e2, &u, &v))) occ = 1;
                }
                if (occ) break;
                next = EMPTY_REF;
                continue;
            }
            c_nodes++;
            next = visit_node(b, next, o, inv, 1.0f, stk, stk_t, &sp);
        }
        shadow[i] = (uint8_t)occ;
        c_occ += (uint64_t)occ;
    }
    if (counters) {
        counters[0] += c_nodes;
        counters[1] += c_tris;
        counters[2] += c_occ;
    }
    return ORC_ERR_FINE;
}

int32_t orc_brute_shadow(const orc_mesh* meshes, uint32_t num_meshes, const float* rays,
                         uint32_t begin, uint32_t end, const float eye[3], const float orient[9],
                         const float light[3], const uint32_t* tri_id, const float* tprim,
                         uint8_t* shadow) {
    soup s;
    soup_make(&s, meshes, num_meshes);
    for (uint32_t i = begin; i < end; ++i) {
        shadow[i] = 0;
        if (tri_id[i] == NO_TRI) continue;
        float dir[3], o[3], d[3];
        orient_dir(dir, orient, rays + (size_t)i * 3);
        shadow_segment(eye, dir, tprim[i], light, o, d);
        for (uint32_t g = 0; g < s.n; ++g) {
            const float* v = s.v + (size_t)g * 9;
            float u = 0, vv = 0;
            if (shadow_accept(tri_intersect(o, d, v, v + 3, v + 6, &u, &vv))) {
                shadow[i] = 1;
                break;
            }
        }
    }
    soup_free(&s);
    return ORC_ERR_FINE;
}

int32_t orc_brute_trace(const orc_mesh* meshes, uint32_t num_meshes, const float* rays,
                        uint32_t begin, uint32_t end, const float eye[3], const float orient[9],
                        uint32_t* packed, uint32_t* tri_id, float* tout) {
    soup s;
    soup_make(&s, meshes, num_meshes);
    if (!s.nn && s.n) {
        soup_free(&s);
        return ORC_ERR_INVALID_FORMAT;
    }
    for (uint32_t i = begin; i < end; ++i) {
        float dir[3];
        orient_dir(dir, orient, rays + (size_t)i * 3);
        float tbest = INFINITY, bu = 0, bv = 0;
        uint32_t ibest = NO_TRI;
        for (uint32_t g = 0; g < s.n; ++g) {
            const float* v = s.v + (size_t)g * 9;
            float u = 0, vv = 0;
            float t = tri_intersect(eye, dir, v, v + 3, v + 6, &u, &vv);
            if (t > 0.0f && t != FLT_MAX && t < tbest) {
                tbest = t;
                ibest = g;
                bu = u;
                bv = vv;
            }
        }
        if (ibest != NO_TRI) {
            const float* n = s.nn + (size_t)ibest * 9;
            if (packed) packed[i] = shade_packed(n, n + 3, n + 6, bu, bv);
            if (tri_id) tri_id[i] = ibest;
            if (tout) tout[i] = tbest;
        } else {
            if (packed) packed[i] = MISS_PACKED;
            if (tri_id) tri_id[i] = NO_TRI;
            if (tout) tout[i] = INFINITY;
        }
    }
    soup_free(&s);
    return ORC_ERR_FINE;
}

/* ---- OBJ reader (golden-fixture generation only) ------------------------------------------- */
typedef struct fvec { float* p; size_t n, cap; } fvec;
typedef struct uvec { uint32_t* p; size_t n, cap; } uvec;
static void fpush(fvec* v, float x) {
    if (v->n == v->cap) { v->cap = v->cap ? v->cap * 2 : 1024; v->p = (float*)realloc(v->p, v->cap * 4); }
    v->p[v->n++] = x;
}
static void upush(uvec* v, uint32_t x) {
    if (v->n == v->cap) { v->cap = v->cap ? v->cap * 2 : 1024; v->p = (uint32_t*)realloc(v->p, v->cap * 4); }
    v->p[v->n++] = x;
}

int32_t orc_obj_load(const char* path, int32_t share, orc_obj* out) {
    memset(out, 0, sizeof(*out));
    FILE* f = fopen(path, "r");
    if (!f) return -1;
    fvec P = {0}, N = {0};
    uvec FV = {0}, FN = {0}, FM = {0}; /* corner position/normal index, face mesh id */
    uint32_t cur = 0, faces_in_cur = 0;
    char line[4096];
    while (fgets(line, sizeof line, f)) {
        char* s = line;
        while (*s == ' ' || *s == '\t') s++;
        if (s[0] == 'v' && s[1] == ' ') {
            char* e = s + 2;
            for (int k = 0; k < 3; ++k) fpush(&P, strtof(e, &e));
        } else if (s[0] == 'v' && s[1] == 'n' && s[2] == ' ') {
            char* e = s + 3;
            for (int k = 0; k < 3; ++k) fpush(&N, strtof(e, &e));
        } else if (!strncmp(s, "usemtl", 6)) {
            if (faces_in_cur) { cur++; faces_in_cur = 0; }
        } else if (s[0] == 'f' && s[1] == ' ') {
            long vi[64], ni[64];
            int c = 0;
            char* e = s + 2;
            while (c < 64) {
                while (*e == ' ' || *e == '\t') e++;
                if (*e == '\0' || *e == '\n' || *e == '\r') break;
                long a = strtol(e, &e, 10), nn = 0;
                if (*e == '/') {
                    e++;
                    if (*e != '/') strtol(e, &e, 10);
                    if (*e == '/') { e++; nn = strtol(e, &e, 10); }
                }
                vi[c] = a > 0 ? a - 1 : (long)(P.n / 3) + a;
                ni[c] = nn > 0 ? nn - 1 : (nn < 0 ? (long)(N.n / 3) + nn : -1);
                c++;
                while (*e && *e != ' ' && *e != '\t' && *e != '\n' && *e != '\r') e++;
            }
            for (int k = 1; k + 1 < c; ++k) { /* fan triangulation */
                int cs[3] = {0, k, k + 1};
                for (int q = 0; q < 3; ++q) { upush(&FV, (uint32_t)vi[cs[q]]); upush(&FN, (uint32_t)ni[cs[q]]); }
                upush(&FM, cur);
                faces_in_cur++;
            }
        }
    }
    fclose(f);
    uint32_t nm = FM.n ? FM.p[FM.n - 1] + 1 : 0;
    if (nm > 16) nm = 16;
    out->num_meshes = nm;
    for (uint32_t m = 0; m < nm; ++m) {
        size_t nf = 0;
        for (size_t i = 0; i < FM.n; ++i) nf += (FM.p[i] == m);
        out->num_idx[m] = (uint32_t)(nf * 3);
        out->idx[m] = (uint32_t*)malloc(4 * nf * 3 + 4);
        int can_share = share && N.n == P.n;
        for (size_t i = 0; i < FV.n && can_share && share != 2; ++i) can_share = (FV.p[i] == FN.p[i]);
        if (can_share) {
            out->num_verts[m] = (uint32_t)(P.n / 3);
            out->pos[m] = (float*)malloc(P.n * 4);
            memcpy(out->pos[m], P.p, P.n * 4);
            out->nrm[m] = (float*)malloc(N.n * 4);
            memcpy(out->nrm[m], N.p, N.n * 4);
            size_t q = 0;
            for (size_t i = 0; i < FM.n; ++i)
                if (FM.p[i] == m) for (int k = 0; k < 3; ++k) out->idx[m][q++] = FV.p[i * 3 + k];
        } else {
            out->num_verts[m] = (uint32_t)(nf * 3);
            out->pos[m] = (float*)malloc(4 * nf * 9 + 4);
            out->nrm[m] = N.n ? (float*)malloc(4 * nf * 9 + 4) : NULL;
            size_t q = 0;
            for (size_t i = 0; i < FM.n; ++i) {
                if (FM.p[i] != m) continue;
                for (int k = 0; k < 3; ++k, ++q) {
                    memcpy(out->pos[m] + q * 3, P.p + (size_t)FV.p[i * 3 + k] * 3, 12);
                    if (out->nrm[m]) {
                        uint32_t ni = FN.p[i * 3 + k];
                        if (ni != 0xFFFFFFFFu) memcpy(out->nrm[m] + q * 3, N.p + (size_t)ni * 3, 12);
                        else memset(out->nrm[m] + q * 3, 0, 12);
                    }
                    out->idx[m][q] = (uint32_t)q;
                }
            }
        }
    }
    free(P.p); free(N.p); free(FV.p); free(FN.p); free(FM.p);
    return (int32_t)nm;
}

void orc_obj_free(orc_obj* o) {
    for (uint32_t m = 0; m < o->num_meshes; ++m) {
        free(o->pos[m]);
        free(o->nrm[m]);
        free(o->idx[m]);
    }
    memset(o, 0, sizeof(*o));
}
