// bm_kd.hip — reference mode: the reference's own acceleration structure and march on gfx950,
// for frames identical to the reference's on every pixel (the first-hit-leaf early-out included).
//
// The reference (BuildTree.cu:154-256) inserts each triangle into a sparse kd-tree over the fixed
// world box: spatial-median splits cycling x, y, z; a child is descended into when Akenine-Möller's
// triangle/box test (BoxTriangle.cuh:134-222) passes; a node becomes a leaf when its smallest edge
// is below 0.03 or at depth 37 — for the world box [-30,30]³ every leaf sits at depth 31 — and a
// leaf keeps its first 256 faces (BuildTree.cu:36-61). The march (BuildTree.cu:367-499) walks the
// tree near-first by split plane, tests every face of the first leaf that has a hit and stops there.
//
// Built here without pointers or atomics deciding anything:
//   k_kd_descend<count>  one thread per triangle repeats the reference's descent (same boxes, same
//                        SAT arithmetic) and counts the leaves it reaches;
//   exclusive scan       per-triangle output offsets (triangle id order);
//   k_kd_descend<emit>   writes (leaf path key, triangle id) pairs — a leaf is named by its 31 split
//                        decisions, so the key is the node;
//   stable sort          by key: within a leaf the faces come out in triangle-id order, the order the
//                        reference's serial (CPU) insertion gives, which decides exact-t ties and the
//                        256-face cap;
//   leaves               runs of equal keys (flags + scan);
//   radix tree           Karras over the distinct leaf keys: its internal nodes are exactly the
//                        reference's nodes with two children (depth = common prefix length); the
//                        reference's single-child nodes between them are replayed by the march (box
//                        test of every level), and nodes without leaves below cannot produce a hit.
// Bit-identical to oracle/beam_oracle.c orc_kd_build + orc_kd_march.
#include <cmath>

#include "bm_internal.h"

namespace bm {
namespace {

constexpr int BLOCK = 256;
constexpr float KD_MIN_LEAF = .03f;  // MIN_LEAF_SIZE, BuildTree.cuh:18
constexpr int KD_MAX_DEPTH = 38;     // BUILD_TREE_MAX_DEPTH, BuildTree.cuh:15
constexpr uint32_t KD_LEAF_CAP = 256;  // MAX_FACES_PER_BOX, BuildTree.cuh:17
constexpr float FLT_MAXF = 3.40282347e+38f;

__device__ __forceinline__ float rmin(float a, float b) { return a < b ? a : b; }
__device__ __forceinline__ float rmax(float a, float b) { return a > b ? a : b; }

// planeBoxOverlap (BoxTriangle.cuh:57-79)
__device__ bool plane_box(const float* nrm, const float* vert, const float* maxbox) {
    float vmin[3], vmax[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        const float v = vert[q];
        if (nrm[q] > 0.0f) {
            vmin[q] = -maxbox[q] - v;
            vmax[q] = maxbox[q] - v;
        } else {
            vmin[q] = maxbox[q] - v;
            vmax[q] = -maxbox[q] - v;
        }
    }
    if ((nrm[0] * vmin[0] + nrm[1] * vmin[1]) + nrm[2] * vmin[2] > 0.0f) return false;
    if ((nrm[0] * vmax[0] + nrm[1] * vmax[1]) + nrm[2] * vmax[2] >= 0.0f) return true;
    return false;
}

__device__ __forceinline__ bool axis_sep(float pa, float pb, float rad) {
    float mn, mx;
    if (pa < pb) {
        mn = pa;
        mx = pb;
    } else {
        mn = pb;
        mx = pa;
    }
    return (mn > rad || mx < -rad);
}

// triBoxOverlap (BoxTriangle.cuh:134-222): the nine cross-axis tests (AXISTEST_* order), the AABB
// test (FINDMINMAX) and the plane test, operation for operation.
__device__ bool tri_box(const float* bc, const float* hs, const float* tv) {
    float v0[3], v1[3], v2[3], e0[3], e1[3], e2[3], nrm[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        v0[c] = tv[c] - bc[c];
        v1[c] = tv[3 + c] - bc[c];
        v2[c] = tv[6 + c] - bc[c];
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        e0[c] = v1[c] - v0[c];
        e1[c] = v2[c] - v1[c];
        e2[c] = v0[c] - v2[c];
    }
    float fx, fy, fz, a, b, pa, pb, rad;
    fx = fabsf(e0[0]); fy = fabsf(e0[1]); fz = fabsf(e0[2]);
    a = e0[2]; b = e0[1];
    pa = a * v0[1] - b * v0[2]; pb = a * v2[1] - b * v2[2];
    rad = fz * hs[1] + fy * hs[2];
    if (axis_sep(pa, pb, rad)) return false;
    a = e0[2]; b = e0[0];
    pa = -a * v0[0] + b * v0[2]; pb = -a * v2[0] + b * v2[2];
    rad = fz * hs[0] + fx * hs[2];
    if (axis_sep(pa, pb, rad)) return false;
    a = e0[1]; b = e0[0];
    pa = a * v1[0] - b * v1[1]; pb = a * v2[0] - b * v2[1];
    rad = fy * hs[0] + fx * hs[1];
    if (axis_sep(pb, pa, rad)) return false;

    fx = fabsf(e1[0]); fy = fabsf(e1[1]); fz = fabsf(e1[2]);
    a = e1[2]; b = e1[1];
    pa = a * v0[1] - b * v0[2]; pb = a * v2[1] - b * v2[2];
    rad = fz * hs[1] + fy * hs[2];
    if (axis_sep(pa, pb, rad)) return false;
    a = e1[2]; b = e1[0];
    pa = -a * v0[0] + b * v0[2]; pb = -a * v2[0] + b * v2[2];
    rad = fz * hs[0] + fx * hs[2];
    if (axis_sep(pa, pb, rad)) return false;
    a = e1[1]; b = e1[0];
    pa = a * v0[0] - b * v0[1]; pb = a * v1[0] - b * v1[1];
    rad = fy * hs[0] + fx * hs[1];
    if (axis_sep(pa, pb, rad)) return false;

    fx = fabsf(e2[0]); fy = fabsf(e2[1]); fz = fabsf(e2[2]);
    a = e2[2]; b = e2[1];
    pa = a * v0[1] - b * v0[2]; pb = a * v1[1] - b * v1[2];
    rad = fz * hs[1] + fy * hs[2];
    if (axis_sep(pa, pb, rad)) return false;
    a = e2[2]; b = e2[0];
    pa = -a * v0[0] + b * v0[2]; pb = -a * v1[0] + b * v1[2];
    rad = fz * hs[0] + fx * hs[2];
    if (axis_sep(pa, pb, rad)) return false;
    a = e2[1]; b = e2[0];
    pa = a * v1[0] - b * v1[1]; pb = a * v2[0] - b * v2[1];
    rad = fy * hs[0] + fx * hs[1];
    if (axis_sep(pb, pa, rad)) return false;

#pragma unroll
    for (int c = 0; c < 3; ++c) {
        float mn = v0[c], mx = v0[c];
        if (v1[c] < mn) mn = v1[c];
        if (v1[c] > mx) mx = v1[c];
        if (v2[c] < mn) mn = v2[c];
        if (v2[c] > mx) mx = v2[c];
        if (mn > hs[c] || mx < -hs[c]) return false;
    }
    nrm[0] = e0[1] * e1[2] - e0[2] * e1[1];
    nrm[1] = e0[2] * e1[0] - e0[0] * e1[2];
    nrm[2] = e0[0] * e1[1] - e0[1] * e1[0];
    return plane_box(nrm, v0, hs);
}

// Box of the node reached by following `path` (bit k = right at depth k, MSB first over `depth`
// bits of a leaf_depth-bit key) from the world box, with the reference's halving arithmetic.
__device__ __forceinline__ void path_box(uint32_t key, int depth, int leaf_depth, float wmin, float wmax, float* mn,
                                         float* mx) {
    for (int c = 0; c < 3; ++c) {
        mn[c] = wmin;
        mx[c] = wmax;
    }
    for (int k = 0; k < depth; ++k) {
        const int a = k % 3;
        const float s = .5f * (mn[a] + mx[a]);
        if ((key >> (leaf_depth - 1 - k)) & 1u) mn[a] = s;
        else mx[a] = s;
    }
}

struct DescendEntry {
    uint32_t path;
    int depth;
};

// bmInsertTriangleInTree (BuildTree.cu:154-256) for one triangle: LIFO descent, left pushed before
// right as in the reference; the leaves reached are counted (EMIT=false) or written (EMIT=true).
template <bool EMIT>
__global__ __launch_bounds__(BLOCK) void k_kd_descend(const MeshDesc* __restrict__ meshes, uint32_t nm, uint32_t n,
                                                      float wmin, float wmax, int leaf_depth,
                                                      uint32_t* __restrict__ counts,
                                                      const uint32_t* __restrict__ offsets,
                                                      uint32_t* __restrict__ keys, uint32_t* __restrict__ vals) {
    const uint32_t g = blockIdx.x * BLOCK + threadIdx.x;
    if (g >= n) return;
    uint32_t a0 = 0, b0 = nm;
    while (b0 - a0 > 1) {
        const uint32_t mid = (a0 + b0) >> 1;
        if (meshes[mid].tri_offset <= g) a0 = mid;
        else b0 = mid;
    }
    const MeshDesc md = meshes[a0];
    const uint32_t f = g - md.tri_offset;
    float tv[9];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const uint32_t vi = md.idx[3 * f + k];
#pragma unroll
        for (int c = 0; c < 3; ++c) tv[3 * k + c] = md.pos[3 * vi + c];
    }
    DescendEntry st[KD_MAX_DEPTH + 2];
    int top = 0;
    st[0] = DescendEntry{0u, 0};
    uint32_t found = 0, out = EMIT ? offsets[g] : 0u;
    while (top >= 0) {
        const DescendEntry e = st[top--];
        float mn[3], mx[3];
        path_box(e.path << (leaf_depth - e.depth), e.depth, leaf_depth, wmin, wmax, mn, mx);
        const float bs[3] = {mx[0] - mn[0], mx[1] - mn[1], mx[2] - mn[2]};
        const float dmin = rmin(bs[0], rmin(bs[1], bs[2]));
        if (dmin < KD_MIN_LEAF || e.depth == KD_MAX_DEPTH - 1) {
            if (EMIT) {
                keys[out] = e.path;
                vals[out] = g;
                ++out;
            }
            ++found;
            continue;
        }
        const int ax = e.depth % 3;
        const float s = .5f * (mn[ax] + mx[ax]);
        float lmax[3] = {mx[0], mx[1], mx[2]}, rmn[3] = {mn[0], mn[1], mn[2]};
        lmax[ax] = s;
        rmn[ax] = s;
        float bc[3], hs[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            bc[c] = (lmax[c] + mn[c]) * .5f;
            hs[c] = (lmax[c] - mn[c]) * .5f;
        }
        const bool b1 = tri_box(bc, hs, tv);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            bc[c] = (mx[c] + rmn[c]) * .5f;
            hs[c] = (mx[c] - rmn[c]) * .5f;
        }
        const bool b2 = tri_box(bc, hs, tv);
        if (b1) st[++top] = DescendEntry{e.path << 1, e.depth + 1};
        if (b2) st[++top] = DescendEntry{(e.path << 1) | 1u, e.depth + 1};
    }
    if (!EMIT) counts[g] = found;
}

// ---- exclusive scan (u32): per-block scans, one workgroup over the block sums, add -------------
constexpr int SCAN_BLOCK = 1024;

__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* sh, uint32_t& total) {
    const int t = threadIdx.x;
    sh[t] = v;
    __syncthreads();
    for (int off = 1; off < SCAN_BLOCK; off <<= 1) {
        const uint32_t y = t >= off ? sh[t - off] : 0u;
        __syncthreads();
        sh[t] += y;
        __syncthreads();
    }
    total = sh[SCAN_BLOCK - 1];
    const uint32_t r = sh[t] - v;
    __syncthreads();
    return r;
}

__global__ __launch_bounds__(SCAN_BLOCK) void k_scan_local(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                            uint32_t n, uint32_t* __restrict__ sums) {
    __shared__ uint32_t sh[SCAN_BLOCK];
    const uint32_t i = blockIdx.x * SCAN_BLOCK + threadIdx.x;
    uint32_t total;
    const uint32_t r = block_exclusive_scan(i < n ? in[i] : 0u, sh, total);
    if (i < n) out[i] = r;
    if (threadIdx.x == 0) sums[blockIdx.x] = total;
}

__global__ __launch_bounds__(SCAN_BLOCK) void k_scan_sums(uint32_t* __restrict__ sums, uint32_t nb,
                                                           uint32_t* __restrict__ grand_total) {
    __shared__ uint32_t sh[SCAN_BLOCK];
    uint32_t carry = 0;
    for (uint32_t base = 0; base < nb; base += SCAN_BLOCK) {
        const uint32_t i = base + threadIdx.x;
        uint32_t total;
        const uint32_t r = block_exclusive_scan(i < nb ? sums[i] : 0u, sh, total);
        if (i < nb) sums[i] = r + carry;
        carry += total;
    }
    if (threadIdx.x == 0) *grand_total = carry;
}

__global__ __launch_bounds__(SCAN_BLOCK) void k_scan_add(uint32_t* __restrict__ out, uint32_t n,
                                                          const uint32_t* __restrict__ sums) {
    const uint32_t i = blockIdx.x * SCAN_BLOCK + threadIdx.x;
    if (i < n) out[i] += sums[blockIdx.x];
}

// 64-bit sum of u32 counts (one workgroup): guards the u32 scans of the pair counts against wrap.
__global__ __launch_bounds__(1024) void k_sum_u64(const uint32_t* __restrict__ in, uint32_t n,
                                                  unsigned long long* __restrict__ out) {
    __shared__ unsigned long long part[1024 / 64];
    unsigned long long v = 0;
    for (uint32_t i = threadIdx.x; i < n; i += 1024) v += in[i];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int k = 0; k < 1024 / 64; ++k) t += part[k];
        *out = t;
    }
}

// ---- leaves: runs of equal keys ------------------------------------------------------------------
__global__ __launch_bounds__(BLOCK) void k_kd_flags(const uint32_t* __restrict__ keys, uint32_t m,
                                                    uint32_t* __restrict__ flags) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i < m) flags[i] = (i == 0 || keys[i] != keys[i - 1]) ? 1u : 0u;
}

__global__ __launch_bounds__(BLOCK) void k_kd_leaf_count(const uint32_t* __restrict__ leaf_start, uint32_t nl,
                                                         uint32_t m, uint32_t* __restrict__ leaf_count) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i < nl) leaf_count[i] = (i + 1 < nl ? leaf_start[i + 1] : m) - leaf_start[i];
}

__global__ __launch_bounds__(BLOCK) void k_kd_leaves(const uint32_t* __restrict__ keys, uint32_t m,
                                                     const uint32_t* __restrict__ flags,
                                                     const uint32_t* __restrict__ leaf_of,
                                                     uint32_t* __restrict__ leaf_key,
                                                     uint32_t* __restrict__ leaf_start) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i < m && flags[i]) {
        leaf_key[leaf_of[i]] = keys[i];
        leaf_start[leaf_of[i]] = i;
    }
}

inline uint32_t blocks_for(uint32_t n, uint32_t per) { return (n + per - 1) / per; }

// ---- the march (bmMarchKernel, BuildTree.cu:367-499) ---------------------------------------------
// bmBoxRayIntersect (CudaComon.cuh:158-172), with the reference's _min/_max (second argument on NaN).
__device__ __forceinline__ float kd_box_ray(const float* bmn, const float* bmx, const vec3f o, const vec3f inv) {
    const float t0[3] = {(bmn[0] - o.x) * inv.x, (bmn[1] - o.y) * inv.y, (bmn[2] - o.z) * inv.z};
    const float t1[3] = {(bmx[0] - o.x) * inv.x, (bmx[1] - o.y) * inv.y, (bmx[2] - o.z) * inv.z};
    const float ftmax = rmin(rmax(t0[0], t1[0]), rmin(rmax(t0[1], t1[1]), rmax(t0[2], t1[2])));
    if (ftmax < 0.f) return FLT_MAXF;
    const float ftmin = rmax(rmin(t0[0], t1[0]), rmax(rmin(t0[1], t1[1]), rmin(t0[2], t1[2])));
    const float dist = rmax(0.f, ftmin);
    return (ftmax >= ftmin ? dist : FLT_MAXF);
}

struct KdView {
    const uint32_t* leaf_key;
    const uint32_t* leaf_start;
    const uint32_t* leaf_count;
    const uint32_t* faces;  // sorted pair values: triangle ids per leaf
    const uint32_t* lch;
    const uint32_t* rch;
    const uint32_t* first;
    const uint32_t* last;
    uint32_t num_leaves;
    int leaf_depth;
    float wmin, wmax;
};

__global__ __launch_bounds__(BLOCK) void k_kd_march(const TraceParams p, const KdView kv) {
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const uint32_t x = blockIdx.x * 16 + (w & 1) * 8 + (lane & 7);
    const uint32_t y = blockIdx.y * 16 + (w >> 1) * 8 + (lane >> 3);
    if (x >= p.width || y >= p.height) return;
    // Camera::setInitialRays for this pixel (Camera.cpp:61-66), dir = orient * ray
    const float rx = p.rx[x], ry = p.ry[y];
    const float d = 1.f / sqrtf(p.z2 + rx * rx + ry * ry);
    const vec3f r = v3(rx * d, ry * d, p.zoom * d);
    const float* m = p.orient;
    const vec3f dir = v3((m[0] * r.x + m[3] * r.y) + m[6] * r.z, (m[1] * r.x + m[4] * r.y) + m[7] * r.z,
                         (m[2] * r.x + m[5] * r.y) + m[8] * r.z);
    const vec3f inv = v3(1.f / dir.x, 1.f / dir.y, 1.f / dir.z);
    const vec3f eye = v3(p.eye[0], p.eye[1], p.eye[2]);
    const float eyea[3] = {eye.x, eye.y, eye.z}, dira[3] = {dir.x, dir.y, dir.z};

    float dclosest = FLT_MAXF, tu = 0.f, tvv = 0.f;
    uint32_t fclosest = NO_TRI;
    uint32_t st_ref[KD_MAX_DEPTH + 2];
    int st_depth[KD_MAX_DEPTH + 2];
    int top = -1;
    if (kv.num_leaves == 1) {
        st_ref[++top] = LEAF_BIT;
        st_depth[top] = 0;
    } else if (kv.num_leaves > 1) {
        st_ref[++top] = 0u;
        st_depth[top] = 0;
    }
    bool done = false;
    while (top >= 0 && !done) {
        const uint32_t ref = st_ref[top];
        int dep = st_depth[top];
        --top;
        const bool leaf = (ref & LEAF_BIT) != 0;
        const uint32_t idx = ref & ~LEAF_BIT;
        const uint32_t key = kv.leaf_key[leaf ? idx : kv.first[idx]];
        const int target = leaf ? kv.leaf_depth
                                : __clz((int)((key ^ kv.leaf_key[kv.last[idx]]) << (32 - kv.leaf_depth)));
        float mn[3], mx[3];
        path_box(key, dep, kv.leaf_depth, kv.wmin, kv.wmax, mn, mx);
        // the reference's single-child nodes between the parent's split and this node: each is
        // popped and box-tested in turn, as is this node
        float box = kd_box_ray(mn, mx, eye, inv);
        while (box != FLT_MAXF && dep < target) {
            const int a = dep % 3;
            const float s = .5f * (mx[a] + mn[a]);
            if ((key >> (kv.leaf_depth - 1 - dep)) & 1u) mn[a] = s;
            else mx[a] = s;
            ++dep;
            box = kd_box_ray(mn, mx, eye, inv);
        }
        if (box == FLT_MAXF) continue;
        if (leaf) {
            const uint32_t cnt = min(kv.leaf_count[idx], KD_LEAF_CAP);
            const uint32_t start = kv.leaf_start[idx];
            for (uint32_t k = 0; k < cnt; ++k) {
                const uint32_t gid = kv.faces[start + k];
                const float4 ta = p.tris[3 * (size_t)gid + 0], tb = p.tris[3 * (size_t)gid + 1],
                             tc = p.tris[3 * (size_t)gid + 2];
                // bmTriIntersect (CudaComon.cuh:117-155): FLT_MAX on the two rejects, else t
                const vec3f e1 = v3(tb.x, tb.y, tb.z), e2 = v3(tc.x, tc.y, tc.z);
                const vec3f pv = cross(dir, e2);
                const float det = dot(e1, pv);
                const float idet = 1.f / det;
                const vec3f tvec = sub(eye, v3(ta.x, ta.y, ta.z));
                const float u = dot(tvec, pv) * idet;
                if (u < 0 || u > 1) continue;
                const vec3f qv = cross(tvec, e1);
                const float v = dot(dir, qv) * idet;
                if (v < 0 || v + u > 1) continue;
                const float t = dot(e2, qv) * idet;
                if (t < dclosest) {
                    dclosest = t;
                    fclosest = gid;
                    tu = u;
                    tvv = v;
                }
            }
            if (dclosest != FLT_MAXF) done = true;  // first leaf with a hit ends the march (:427-431)
            continue;
        }
        // split plane of this node: near child first (popped first)
        const int a = dep % 3;
        const float s = .5f * (mx[a] + mn[a]);
        const float pp = eyea[a] + box * dira[a];
        const uint32_t lc = kv.lch[idx], rc = kv.rch[idx];
        if (pp < s) {
            st_ref[++top] = rc;
            st_depth[top] = dep + 1;
            st_ref[++top] = lc;
            st_depth[top] = dep + 1;
        } else {
            st_ref[++top] = lc;
            st_depth[top] = dep + 1;
            st_ref[++top] = rc;
            st_depth[top] = dep + 1;
        }
    }
    const size_t o = (size_t)y * p.width + x;
    uint32_t packed = MISS_PACKED;
    float nzv = 0.0f, tout = __builtin_inff();
    if (fclosest != NO_TRI) {
        const float* n = p.nrm + 9 * (size_t)fclosest;
        const float ww = 1.f - (tu + tvv);
        const vec3f nn = v3((n[0] * ww + n[3] * tu) + n[6] * tvv, (n[1] * ww + n[4] * tu) + n[7] * tvv,
                            (n[2] * ww + n[5] * tu) + n[8] * tvv);
        const float il = 1.f / sqrtf(dot(nn, nn));
        const float z = nn.z * il;
        const float rr = fabsf(z * 255.f);
        packed = ((rr == rr) ? (uint32_t)rr : 0u) << 16;
        nzv = fabsf(z);
        tout = dclosest;
    }
    p.packed[(size_t)y * p.pitch_u32 + x] = packed;
    p.tri_id[o] = fclosest;
    p.t[o] = tout;
    if (p.nz) p.nz[o] = nzv;
}

// ---- hashed uniform grid (Hash.cu, the reference's alternative accelerator) ----------------------
// Cells of 0.03; cell (x, y, z) -> bucket (F16(x) + F16(y) + F16(z)) mod 65536, F16 = Fletcher-16 of
// the four little-endian bytes (bmHash/bmHash3, Hash.cu:15-47). Built here without atomics:
//   k_hash_cells<count>  one thread per triangle visits its AABB's cells (z, y, x loops with the
//                        row indices reset, the fix of Hash.cu:162-164) and counts the cells the
//                        reference's triBoxOverlap accepts;
//   exclusive scan       per-triangle offsets;
//   k_hash_cells<emit>   writes (bucket, triangle) pairs in that order;
//   stable sort          by bucket (16-bit keys): a bucket's faces in triangle-id, then cell order —
//                        the reference's serial insertion order, which decides exact-t ties and its
//                        256-face cap (Hash.cu:82-89);
//   k_hash_ranges        bucket -> [start, end) of the sorted pairs.
// The march (bmMarchKernelSpace, Hash.cu:235-302): from the eye, cell by cell (at most 400), test
// every face of the cell's bucket (first 256) against the ray from the eye; the first bucket with a
// hit ends the march. Bit-identical to oracle/beam_oracle.c orc_hash_build + orc_hash_march.
constexpr uint32_t HG_BUCKETS = 65536;    // MAX_HASH_ELEMENTS, BuildTree.cuh:21
constexpr uint32_t HG_CAP = 256;          // NUM_FACES_PER_CELL, Hash.cu:7
constexpr int HG_ITERS = 400;             // MAX_SEARCH_ITERS, Hash.cu:11
constexpr float HG_CELL = 0.03f;          // CELL_RES
constexpr float HG_INV = 1.f / 0.03f;     // INV_CELL_RES (a float constant)
constexpr float HG_EPS = 0.03f * 0.001f;  // CELL_PINCH_TROUGH_EPSILON

__device__ __forceinline__ uint32_t hg_f16(uint32_t h) {
    uint32_t s1 = 0, s2 = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        s1 = (s1 + ((h >> (8 * b)) & 255u)) % 255u;
        s2 = (s2 + s1) % 255u;
    }
    return (s2 << 8) | s1;
}
__device__ __forceinline__ uint32_t hg_hash3(int32_t x, int32_t y, int32_t z) {
    return (hg_f16((uint32_t)x) + hg_f16((uint32_t)y) + hg_f16((uint32_t)z)) % HG_BUCKETS;
}
// bmMap (Hash.cu:57-60), saturating; NaN -> 0 (as the oracle's hg_map)
__device__ __forceinline__ int32_t hg_map(float f) {
    const float q = floorf(f * HG_INV);
    if (q != q) return 0;
    if (q >= 2147483648.f) return INT32_MAX;
    if (q < -2147483648.f) return INT32_MIN;
    return (int32_t)q;
}

template <bool EMIT>
__global__ __launch_bounds__(BLOCK) void k_hash_cells(const MeshDesc* __restrict__ meshes, uint32_t nm, uint32_t n,
                                                      uint32_t* __restrict__ counts,
                                                      const uint32_t* __restrict__ offsets,
                                                      uint32_t* __restrict__ keys, uint32_t* __restrict__ vals,
                                                      uint32_t* __restrict__ too_large) {
    const uint32_t g = blockIdx.x * BLOCK + threadIdx.x;
    if (g >= n) return;
    uint32_t a0 = 0, b0 = nm;
    while (b0 - a0 > 1) {
        const uint32_t mid = (a0 + b0) >> 1;
        if (meshes[mid].tri_offset <= g) a0 = mid;
        else b0 = mid;
    }
    const MeshDesc md = meshes[a0];
    const uint32_t f = g - md.tri_offset;
    float tv[9];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const uint32_t vi = md.idx[3 * f + k];
#pragma unroll
        for (int c = 0; c < 3; ++c) tv[3 * k + c] = md.pos[3 * vi + c];
    }
    int64_t lo[3], hi[3], span = 1;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        lo[c] = hg_map(rmin(tv[c], rmin(tv[3 + c], tv[6 + c])));
        hi[c] = hg_map(rmax(tv[c], rmax(tv[3 + c], tv[6 + c])));
        span *= hi[c] >= lo[c] ? hi[c] - lo[c] + 1 : 0;
        if (span > HG_MAX_CELLS) {  // the host fails the build (the oracle refuses the same scene)
            if (!EMIT) {
                counts[g] = 0;
                atomicOr(too_large, 1u);
            }
            return;
        }
    }
    uint32_t k = 0, out = EMIT ? offsets[g] : 0u;
    for (int64_t z = lo[2]; z <= hi[2]; ++z)
        for (int64_t y = lo[1]; y <= hi[1]; ++y)
            for (int64_t x = lo[0]; x <= hi[0]; ++x) {
                const float bmn[3] = {(float)(int32_t)x * HG_CELL, (float)(int32_t)y * HG_CELL,
                                      (float)(int32_t)z * HG_CELL};
                float bc[3], hs[3];
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    const float bmx = bmn[c] + HG_CELL;
                    bc[c] = (bmx + bmn[c]) * .5f;
                    hs[c] = (bmx - bmn[c]) * .5f;
                }
                if (tri_box(bc, hs, tv)) {
                    if (EMIT) {
                        keys[out + k] = hg_hash3((int32_t)x, (int32_t)y, (int32_t)z);
                        vals[out + k] = g;
                    }
                    ++k;
                }
            }
    if (!EMIT) counts[g] = k;
}

__global__ __launch_bounds__(BLOCK) void k_hash_ranges(const uint32_t* __restrict__ keys, uint32_t m,
                                                       uint32_t* __restrict__ bstart, uint32_t* __restrict__ bend) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= m) return;
    const uint32_t k = keys[i];
    if (i == 0 || keys[i - 1] != k) bstart[k] = i;
    if (i == m - 1 || keys[i + 1] != k) bend[k] = i + 1;
}

// bmBoxRayIntersectNoZero (CudaComon.cuh:176-187), the reference's _min/_max (second argument on NaN)
__device__ __forceinline__ float hg_box_exit(const float* bmn, const float* bmx, const vec3f o, const vec3f inv) {
    const float oa[3] = {o.x, o.y, o.z}, ia[3] = {inv.x, inv.y, inv.z};
    float tn[3], tf[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float t0 = (bmn[c] - oa[c]) * ia[c], t1 = (bmx[c] - oa[c]) * ia[c];
        tn[c] = rmin(t0, t1);
        tf[c] = rmax(t0, t1);
    }
    const float ftmin = rmax(tn[0], rmax(tn[1], tn[2]));
    const float ftmax = rmin(tf[0], rmin(tf[1], tf[2]));
    return (__builtin_isinf(ftmin) || ftmin < 0.f) ? ftmax : ftmin;
}

struct HashView {
    const uint32_t* bstart;
    const uint32_t* bend;
    const uint32_t* faces;  // sorted pair values: triangle ids per bucket
};

__global__ __launch_bounds__(BLOCK) void k_hash_march(const TraceParams p, const HashView hv) {
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const uint32_t x = blockIdx.x * 16 + (w & 1) * 8 + (lane & 7);
    const uint32_t y = blockIdx.y * 16 + (w >> 1) * 8 + (lane >> 3);
    if (x >= p.width || y >= p.height) return;
    const float rx = p.rx[x], ry = p.ry[y];
    const float d = 1.f / sqrtf(p.z2 + rx * rx + ry * ry);
    const vec3f r = v3(rx * d, ry * d, p.zoom * d);
    const float* m = p.orient;
    const vec3f dir = v3((m[0] * r.x + m[3] * r.y) + m[6] * r.z, (m[1] * r.x + m[4] * r.y) + m[7] * r.z,
                         (m[2] * r.x + m[5] * r.y) + m[8] * r.z);
    const vec3f inv = v3(1.f / dir.x, 1.f / dir.y, 1.f / dir.z);
    const vec3f eye = v3(p.eye[0], p.eye[1], p.eye[2]);
    vec3f pp = eye;
    float dclosest = FLT_MAXF, tu = 0.f, tvv = 0.f;
    uint32_t fclosest = NO_TRI;
    for (int it = 0; it < HG_ITERS; ++it) {
        const int32_t cx = hg_map(pp.x), cy = hg_map(pp.y), cz = hg_map(pp.z);
        const uint32_t b = hg_hash3(cx, cy, cz);
        const uint32_t c0 = hv.bstart[b];
        uint32_t cnt = hv.bend[b] - c0;
        if (cnt) {
            cnt = min(cnt, HG_CAP);
            for (uint32_t k = 0; k < cnt; ++k) {
                const uint32_t gid = hv.faces[c0 + k];
                const float4 ta = p.tris[3 * (size_t)gid + 0], tb = p.tris[3 * (size_t)gid + 1],
                             tc = p.tris[3 * (size_t)gid + 2];
                // bmTriIntersect (CudaComon.cuh:117-155) from the eye: FLT_MAX on the two rejects
                const vec3f e1 = v3(tb.x, tb.y, tb.z), e2 = v3(tc.x, tc.y, tc.z);
                const vec3f pv = cross(dir, e2);
                const float det = dot(e1, pv);
                const float idet = 1.f / det;
                const vec3f tvec = sub(eye, v3(ta.x, ta.y, ta.z));
                const float u = dot(tvec, pv) * idet;
                if (u < 0 || u > 1) continue;
                const vec3f qv = cross(tvec, e1);
                const float v = dot(dir, qv) * idet;
                if (v < 0 || v + u > 1) continue;
                const float t = dot(e2, qv) * idet;
                if (t < dclosest) {
                    dclosest = t;
                    fclosest = gid;
                    tu = u;
                    tvv = v;
                }
            }
            if (dclosest != FLT_MAXF) break;  // Hash.cu:271
        }
        const float bmn[3] = {(float)cx * HG_CELL, (float)cy * HG_CELL, (float)cz * HG_CELL};
        const float bmx[3] = {bmn[0] + HG_CELL, bmn[1] + HG_CELL, bmn[2] + HG_CELL};
        const float step = hg_box_exit(bmn, bmx, pp, inv) + HG_EPS;
        pp = v3(pp.x + dir.x * step, pp.y + dir.y * step, pp.z + dir.z * step);
    }
    const size_t o = (size_t)y * p.width + x;
    uint32_t packed = MISS_PACKED;
    float nzv = 0.0f, tout = __builtin_inff();
    if (fclosest != NO_TRI) {
        const float* n = p.nrm + 9 * (size_t)fclosest;
        const float ww = 1.f - (tu + tvv);
        const vec3f nn = v3((n[0] * ww + n[3] * tu) + n[6] * tvv, (n[1] * ww + n[4] * tu) + n[7] * tvv,
                            (n[2] * ww + n[5] * tu) + n[8] * tvv);
        const float il = 1.f / sqrtf(dot(nn, nn));
        const float z = nn.z * il;
        const float rr = fabsf(z * 255.f);
        packed = ((rr == rr) ? (uint32_t)rr : 0u) << 16;
        nzv = fabsf(z);
        tout = dclosest;
    }
    p.packed[(size_t)y * p.pitch_u32 + x] = packed;
    p.tri_id[o] = fclosest;
    p.t[o] = tout;
    if (p.nz) p.nz[o] = nzv;
}

}  // namespace

// Leaf depth for the world box: the reference's stop rule on its own halving arithmetic.
int kd_leaf_depth(float wmin, float wmax) {
    float mn[3] = {wmin, wmin, wmin}, mx[3] = {wmax, wmax, wmax};
    for (int d = 0; d < KD_MAX_DEPTH; ++d) {
        const float bs[3] = {mx[0] - mn[0], mx[1] - mn[1], mx[2] - mn[2]};
        const float dmin = std::fmin(bs[0], std::fmin(bs[1], bs[2]));
        if (dmin < KD_MIN_LEAF || d == KD_MAX_DEPTH - 1) return d;
        const int a = d % 3;
        mx[a] = .5f * (mn[a] + mx[a]);  // every node at depth d has the same extents
    }
    return KD_MAX_DEPTH - 1;
}

#define BM_LAUNCH_CHECK()                          \
    do {                                           \
        hipError_t e_ = hipGetLastError();         \
        if (e_ != hipSuccess) return e_;           \
    } while (0)

hipError_t launch_kd_count(const KdBuild& k, hipStream_t s) {
    if (k.n == 0) return hipSuccess;
    k_kd_descend<false><<<blocks_for(k.n, BLOCK), BLOCK, 0, s>>>(k.meshes, k.num_meshes, k.n, k.wmin, k.wmax,
                                                                 k.leaf_depth, k.counts, nullptr, nullptr, nullptr);
    BM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_exclusive_scan(const uint32_t* in, uint32_t* out, uint32_t n, uint32_t* sums,
                                 uint32_t* grand_total, hipStream_t s) {
    if (n == 0) return hipMemsetAsync(grand_total, 0, 4, s);
    const uint32_t nb = blocks_for(n, SCAN_BLOCK);
    k_scan_local<<<nb, SCAN_BLOCK, 0, s>>>(in, out, n, sums);
    BM_LAUNCH_CHECK();
    k_scan_sums<<<1, SCAN_BLOCK, 0, s>>>(sums, nb, grand_total);
    BM_LAUNCH_CHECK();
    k_scan_add<<<nb, SCAN_BLOCK, 0, s>>>(out, n, sums);
    BM_LAUNCH_CHECK();
    return hipSuccess;
}

uint32_t scan_sums_words(uint32_t n) { return blocks_for(n ? n : 1, SCAN_BLOCK); }

hipError_t launch_kd_emit(const KdBuild& k, hipStream_t s) {
    if (k.n == 0) return hipSuccess;
    k_kd_descend<true><<<blocks_for(k.n, BLOCK), BLOCK, 0, s>>>(k.meshes, k.num_meshes, k.n, k.wmin, k.wmax,
                                                                k.leaf_depth, nullptr, k.offsets, k.keys, k.vals);
    BM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_kd_flags(const uint32_t* keys, uint32_t m, uint32_t* flags, hipStream_t s) {
    if (m == 0) return hipSuccess;
    k_kd_flags<<<blocks_for(m, BLOCK), BLOCK, 0, s>>>(keys, m, flags);
    BM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_kd_leaves(const uint32_t* keys, uint32_t m, const uint32_t* flags, const uint32_t* leaf_of,
                            uint32_t* leaf_key, uint32_t* leaf_start, uint32_t* leaf_count, uint32_t nl,
                            hipStream_t s) {
    if (m == 0 || nl == 0) return hipSuccess;
    k_kd_leaves<<<blocks_for(m, BLOCK), BLOCK, 0, s>>>(keys, m, flags, leaf_of, leaf_key, leaf_start);
    BM_LAUNCH_CHECK();
    k_kd_leaf_count<<<blocks_for(nl, BLOCK), BLOCK, 0, s>>>(leaf_start, nl, m, leaf_count);
    BM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_kd_march(const TraceParams& p, const KdMarch& k, hipStream_t s) {
    if (p.width == 0 || p.height == 0) return hipSuccess;
    KdView kv{k.leaf_key, k.leaf_start, k.leaf_count, k.faces, k.lch, k.rch, k.first, k.last,
              k.num_leaves, k.leaf_depth, k.wmin, k.wmax};
    k_kd_march<<<dim3((p.width + 15) / 16, (p.height + 15) / 16), BLOCK, 0, s>>>(p, kv);
    BM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_sum_u64(const uint32_t* in, uint32_t n, unsigned long long* out, hipStream_t s) {
    k_sum_u64<<<1, 1024, 0, s>>>(in, n, out);
    BM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_hash_count(const HashBuild& h, hipStream_t s) {
    if (h.n == 0) return hipSuccess;
    k_hash_cells<false><<<blocks_for(h.n, BLOCK), BLOCK, 0, s>>>(h.meshes, h.num_meshes, h.n, h.counts, nullptr,
                                                                 nullptr, nullptr, h.too_large);
    BM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_hash_emit(const HashBuild& h, hipStream_t s) {
    if (h.n == 0) return hipSuccess;
    k_hash_cells<true><<<blocks_for(h.n, BLOCK), BLOCK, 0, s>>>(h.meshes, h.num_meshes, h.n, nullptr, h.offsets,
                                                                h.keys, h.vals, nullptr);
    BM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_hash_ranges(const uint32_t* keys, uint32_t m, uint32_t* bstart, uint32_t* bend, hipStream_t s) {
    hipError_t e;
    if ((e = hipMemsetAsync(bstart, 0, 4 * (size_t)HG_BUCKETS, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(bend, 0, 4 * (size_t)HG_BUCKETS, s)) != hipSuccess) return e;
    if (m == 0) return hipSuccess;
    k_hash_ranges<<<blocks_for(m, BLOCK), BLOCK, 0, s>>>(keys, m, bstart, bend);
    BM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_hash_march(const TraceParams& p, const uint32_t* bstart, const uint32_t* bend,
                             const uint32_t* faces, hipStream_t s) {
    if (p.width == 0 || p.height == 0) return hipSuccess;
    k_hash_march<<<dim3((p.width + 15) / 16, (p.height + 15) / 16), BLOCK, 0, s>>>(p, HashView{bstart, bend, faces});
    BM_LAUNCH_CHECK();
    return hipSuccess;
}

}  // namespace bm
