// bm_build.hip — LBVH acceleration-structure build for gfx950 (replaces the reference's
// sparse kd-tree insert, Raytracer/BuildTree.cu:95-362, and its SAT test, BoxTriangle.cuh).
//
// Pipeline (one HIP stream, no host round trips):
//   k_gather        mesh table -> per-triangle (v0,e1,e2,id) records, corner normals, AABBs;
//                   block-reduced scene/centroid bounds via ordered-int atomics
//   k_morton        30-bit Morton key of each AABB centre, value = global triangle id
//   k_radix_*  x4   stable LSD radix sort, 8-bit digits: LDS histogram, one-WG scan, wave64
//                   ballot ranking for the stable scatter
//   k_emit          Karras 2012 binary radix tree (one thread per internal node)
//   k_refit_*       bottom-up AABB refit: per-chunk in LDS, then the chunk-spanning nodes in one workgroup
//   k_pack          64-B BVH2 records with child boxes inline, leaves collapsed to <= leaf_size
//   k_sort_tris     triangle records gathered into leaf (sorted) order
// Every stored value is a deterministic function of the input (no atomics decide a value), so
// the result is bit-identical to oracle/beam_oracle.c's orc_bvh_build, which tests check.
#include <climits>

#include "bm_internal.h"

namespace bm {
namespace {

constexpr int BLOCK = 256;
constexpr int SORT_ITEMS = 16;
constexpr int SORT_TILE = BLOCK * SORT_ITEMS;
constexpr uint32_t REFIT_CHUNK_LOG2 = 10;
constexpr uint32_t REFIT_CHUNK = 1u << REFIT_CHUNK_LOG2;

__device__ __forceinline__ int wave_min(int v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = min(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = max(v, __shfl_xor(v, o));
    return v;
}

__global__ __launch_bounds__(BLOCK) void k_gather(const MeshDesc* __restrict__ meshes, uint32_t nm, uint32_t n,
                                                  float4* __restrict__ tri, float* __restrict__ nrm,
                                                  float* __restrict__ aabb, int32_t* __restrict__ bounds) {
    const uint32_t g = blockIdx.x * BLOCK + threadIdx.x;
    int lo[6], hi[6];  // ordered ints: [0..2] aabb, [3..5] centre
#pragma unroll
    for (int c = 0; c < 6; ++c) {
        lo[c] = INT_MAX;
        hi[c] = INT_MIN;
    }
    if (g < n) {
        uint32_t a = 0, b = nm;
        while (b - a > 1) {
            uint32_t mid = (a + b) >> 1;
            if (meshes[mid].tri_offset <= g) a = mid;
            else b = mid;
        }
        const MeshDesc md = meshes[a];
        const uint32_t f = g - md.tri_offset;
        const uint32_t i0 = md.idx[3 * f], i1 = md.idx[3 * f + 1], i2 = md.idx[3 * f + 2];
        const vec3f p0 = v3(md.pos[3 * i0], md.pos[3 * i0 + 1], md.pos[3 * i0 + 2]);
        const vec3f p1 = v3(md.pos[3 * i1], md.pos[3 * i1 + 1], md.pos[3 * i1 + 2]);
        const vec3f p2 = v3(md.pos[3 * i2], md.pos[3 * i2 + 1], md.pos[3 * i2 + 2]);
        const vec3f e1 = sub(p1, p0), e2 = sub(p2, p0);
        tri[3 * g + 0] = make_float4(p0.x, p0.y, p0.z, u2f(g));
        tri[3 * g + 1] = make_float4(e1.x, e1.y, e1.z, 0.0f);
        tri[3 * g + 2] = make_float4(e2.x, e2.y, e2.z, 0.0f);
        const uint32_t iv[3] = {i0, i1, i2};
#pragma unroll
        for (int k = 0; k < 3; ++k)
#pragma unroll
            for (int c = 0; c < 3; ++c) nrm[9 * g + 3 * k + c] = md.nrm[3 * iv[k] + c];
        const float pa[3] = {p0.x, p0.y, p0.z}, pb[3] = {p1.x, p1.y, p1.z}, pc[3] = {p2.x, p2.y, p2.z};
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float mn = omin(omin(pa[c], pb[c]), pc[c]);
            const float mx = omax(omax(pa[c], pb[c]), pc[c]);
            const float ce = (mn + mx) * 0.5f;
            aabb[6 * g + c] = mn;
            aabb[6 * g + 3 + c] = mx;
            lo[c] = ord(mn);
            hi[c] = ord(mx);
            lo[3 + c] = ord(ce);
            hi[3 + c] = ord(ce);
        }
    }
    __shared__ int s_lo[BLOCK / 64][6], s_hi[BLOCK / 64][6];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int c = 0; c < 6; ++c) {
        const int a = wave_min(lo[c]), b = wave_max(hi[c]);
        if (lane == 0) {
            s_lo[w][c] = a;
            s_hi[w][c] = b;
        }
    }
    __syncthreads();
    if (threadIdx.x < 6) {
        const int c = threadIdx.x;
        int a = s_lo[0][c], b = s_hi[0][c];
        for (int q = 1; q < BLOCK / 64; ++q) {
            a = min(a, s_lo[q][c]);
            b = max(b, s_hi[q][c]);
        }
        // slots: aabb min 0..2, aabb max 3..5, centre min 6..8, centre max 9..11
        const int slot_lo = c < 3 ? c : 6 + (c - 3);
        const int slot_hi = c < 3 ? 3 + c : 9 + (c - 3);
        // max slots hold ~ord (order-reversing) so one INT_MAX memset initialises every slot
        atomicMin(&bounds[slot_lo], a);
        atomicMin(&bounds[slot_hi], ~b);
    }
}

__global__ __launch_bounds__(BLOCK) void k_morton(uint32_t n, const float* __restrict__ aabb,
                                                  const int32_t* __restrict__ bounds, uint32_t* __restrict__ keys,
                                                  uint32_t* __restrict__ vals) {
    const uint32_t g = blockIdx.x * BLOCK + threadIdx.x;
    if (g >= n) return;
    uint32_t q[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float cmin = unord(bounds[6 + c]), cmax = unord(~bounds[9 + c]);
        const float ext = cmax - cmin;
        const float scale = ext > 0.0f ? 1024.0f / ext : 0.0f;
        const float ce = (aabb[6 * g + c] + aabb[6 * g + 3 + c]) * 0.5f;
        q[c] = quant10(ce, cmin, scale);
    }
    keys[g] = (expand_bits10(q[0]) << 2) | (expand_bits10(q[1]) << 1) | expand_bits10(q[2]);
    vals[g] = g;
}

// ---- stable LSD radix sort ---------------------------------------------------------------------
__global__ __launch_bounds__(BLOCK) void k_radix_hist(const uint32_t* __restrict__ keys, uint32_t n, int shift,
                                                      uint32_t* __restrict__ hist, uint32_t nblocks) {
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t base = blockIdx.x * SORT_TILE;
#pragma unroll 4
    for (int it = 0; it < SORT_ITEMS; ++it) {
        const uint32_t i = base + it * BLOCK + threadIdx.x;
        if (i < n) atomicAdd(&h[(keys[i] >> shift) & 255u], 1u);
    }
    __syncthreads();
    hist[threadIdx.x * nblocks + blockIdx.x] = h[threadIdx.x];
}

// Exclusive scan of the digit-major histogram table [256][nblocks] by one 1024-thread workgroup.
__global__ __launch_bounds__(1024) void k_radix_scan(uint32_t* __restrict__ data, uint32_t total) {
    __shared__ uint32_t sums[1024];
    const uint32_t t = threadIdx.x;
    const uint32_t per = (total + 1023) / 1024;
    const uint32_t beg = min(t * per, total), end = min(beg + per, total);
    uint32_t s = 0;
    for (uint32_t i = beg; i < end; ++i) s += data[i];
    sums[t] = s;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {
        const uint32_t v = t >= off ? sums[t - off] : 0u;
        __syncthreads();
        sums[t] += v;
        __syncthreads();
    }
    uint32_t run = sums[t] - s;
    for (uint32_t i = beg; i < end; ++i) {
        const uint32_t x = data[i];
        data[i] = run;
        run += x;
    }
}

// Stable scatter: keys are taken in input order (iteration, wave, lane); a key's rank among equal
// digits inside its wave comes from eight 64-lane ballots, across waves from per-wave counts in LDS.
__global__ __launch_bounds__(BLOCK) void k_radix_scatter(const uint32_t* __restrict__ kin,
                                                         const uint32_t* __restrict__ vin,
                                                         uint32_t* __restrict__ kout, uint32_t* __restrict__ vout,
                                                         uint32_t n, int shift, const uint32_t* __restrict__ hist,
                                                         uint32_t nblocks) {
    __shared__ uint32_t running[256];
    __shared__ uint32_t wc[BLOCK / 64][256];
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    running[t] = hist[t * nblocks + blockIdx.x];
#pragma unroll
    for (int q = 0; q < BLOCK / 64; ++q) wc[q][t] = 0;
    __syncthreads();
    const uint32_t base = blockIdx.x * SORT_TILE;
    const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    for (int it = 0; it < SORT_ITEMS; ++it) {
        if (base + it * BLOCK >= n) break;  // uniform over the block
        const uint32_t i = base + it * BLOCK + t;
        const bool valid = i < n;
        const uint32_t k = valid ? kin[i] : 0u;
        const uint32_t v = valid ? vin[i] : 0u;
        const uint32_t d = (k >> shift) & 255u;
        unsigned long long peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const bool bit = (d >> b) & 1u;
            const unsigned long long bb = __ballot(bit);
            peers &= bit ? bb : ~bb;
        }
        const uint32_t rank = __popcll(peers & lt);
        if (valid && (peers & lt) == 0ull) wc[w][d] = __popcll(peers);
        __syncthreads();
        if (valid) {
            uint32_t off = running[d] + rank;
            for (int q = 0; q < w; ++q) off += wc[q][d];
            kout[off] = k;
            vout[off] = v;
        }
        __syncthreads();
        uint32_t add = 0;
#pragma unroll
        for (int q = 0; q < BLOCK / 64; ++q) {
            add += wc[q][t];
            wc[q][t] = 0;
        }
        running[t] += add;
        __syncthreads();
    }
}

// ---- Karras 2012 radix tree ------------------------------------------------------------------
__device__ __forceinline__ int kdelta(const uint32_t* __restrict__ k, int n, int i, int j) {
    if (j < 0 || j >= n) return -1;
    const uint32_t a = k[i], b = k[j];
    if (a == b) return 32 + __clz((uint32_t)i ^ (uint32_t)j);
    return __clz(a ^ b);
}

__global__ __launch_bounds__(BLOCK) void k_emit(int n, const uint32_t* __restrict__ keys, uint32_t* __restrict__ lch,
                                                uint32_t* __restrict__ rch, uint32_t* __restrict__ first,
                                                uint32_t* __restrict__ last, uint32_t* __restrict__ parent_leaf,
                                                uint32_t* __restrict__ parent_int, uint32_t* __restrict__ cross,
                                                uint32_t* __restrict__ cross_count) {
    const int i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n - 1) return;
    const int d = (kdelta(keys, n, i, i + 1) - kdelta(keys, n, i, i - 1)) >= 0 ? 1 : -1;
    const int dmin = kdelta(keys, n, i, i - d);
    int lmax = 2;
    while (kdelta(keys, n, i, i + lmax * d) > dmin) lmax *= 2;
    int l = 0;
    for (int t = lmax / 2; t >= 1; t /= 2)
        if (kdelta(keys, n, i, i + (l + t) * d) > dmin) l += t;
    const int j = i + l * d;
    const int dnode = kdelta(keys, n, i, j);
    int s = 0, t = l;
    do {
        t = (t + 1) / 2;
        if (kdelta(keys, n, i, i + (s + t) * d) > dnode) s += t;
    } while (t > 1);
    const int gamma = i + s * d + (d < 0 ? d : 0);
    const int lo = min(i, j), hi = max(i, j);
    if (lo == gamma) {
        lch[i] = (uint32_t)gamma | LEAF_BIT;
        parent_leaf[gamma] = (uint32_t)i;
    } else {
        lch[i] = (uint32_t)gamma;
        parent_int[gamma] = (uint32_t)i;
    }
    if (hi == gamma + 1) {
        rch[i] = (uint32_t)(gamma + 1) | LEAF_BIT;
        parent_leaf[gamma + 1] = (uint32_t)i;
    } else {
        rch[i] = (uint32_t)(gamma + 1);
        parent_int[gamma + 1] = (uint32_t)i;
    }
    first[i] = (uint32_t)lo;
    last[i] = (uint32_t)hi;
    // nodes whose leaf range spans a refit chunk are refitted by k_refit_cross
    if ((lo >> REFIT_CHUNK_LOG2) != (hi >> REFIT_CHUNK_LOG2)) cross[atomicAdd(cross_count, 1u)] = (uint32_t)i;
}

__device__ __forceinline__ void child_box(uint32_t c, const uint32_t* __restrict__ perm, const float* __restrict__ aabb,
                                          const float* ibox, float* lo, float* hi) {
    const float* p = (c & LEAF_BIT) ? aabb + 6 * (size_t)perm[c & ~LEAF_BIT] : ibox + 6 * (size_t)c;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        lo[a] = p[a];
        hi[a] = p[3 + a];
    }
}

// Bottom-up refit in two phases, with no inter-workgroup hand-off inside a launch.
// Phase 1 (k_refit_chunk): one 1024-thread workgroup per chunk of 1024 sorted leaves; a thread
// climbs from its leaf through the internal nodes whose leaf range lies inside the chunk (their
// indices lie inside it too: a Karras node's index is an end of its range). Arrival counters and
// the boxes live in LDS; workgroup-scope acq_rel atomics order them. Results go to ibox.
// Phase 2 (k_refit_cross): the few nodes spanning chunks (listed by k_emit), climbed by ONE
// workgroup: the kernel boundary publishes phase 1, workgroup scope orders the rest.
// (The one-pass refit with agent-scope release/acquire per level cost ~0.26 ms at 70k triangles.)
__global__ __launch_bounds__(REFIT_CHUNK) void k_refit_chunk(uint32_t n, const uint32_t* __restrict__ lch,
                                                             const uint32_t* __restrict__ rch,
                                                             const uint32_t* __restrict__ first,
                                                             const uint32_t* __restrict__ last,
                                                             const uint32_t* __restrict__ parent_leaf,
                                                             const uint32_t* __restrict__ parent_int,
                                                             const uint32_t* __restrict__ perm,
                                                             const float* __restrict__ aabb, float* __restrict__ ibox) {
    __shared__ uint32_t s_flag[REFIT_CHUNK];
    __shared__ float s_box[REFIT_CHUNK][6];
    const uint32_t tid = threadIdx.x, c0 = blockIdx.x * REFIT_CHUNK, c1 = c0 + REFIT_CHUNK - 1;
    s_flag[tid] = 0;
    __syncthreads();
    const uint32_t k = c0 + tid;
    if (k >= n) return;
    uint32_t p = parent_leaf[k];
    for (;;) {
        if (first[p] < c0 || last[p] > c1) return;  // spans chunks: phase 2
        const uint32_t old =
            __hip_atomic_fetch_add(&s_flag[p - c0], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (old == 0u) return;
        float lo[2][3], hi[2][3];
        const uint32_t ch[2] = {lch[p], rch[p]};
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const uint32_t c = ch[q];
            if (c & LEAF_BIT) {
                const float* b = aabb + 6 * (size_t)perm[c & ~LEAF_BIT];
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    lo[q][a] = b[a];
                    hi[q][a] = b[3 + a];
                }
            } else {
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    lo[q][a] = s_box[c - c0][a];
                    hi[q][a] = s_box[c - c0][3 + a];
                }
            }
        }
        float r[6];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            r[a] = omin(lo[0][a], lo[1][a]);
            r[3 + a] = omax(hi[0][a], hi[1][a]);
        }
#pragma unroll
        for (int a = 0; a < 6; ++a) {
            s_box[p - c0][a] = r[a];
            ibox[6 * (size_t)p + a] = r[a];
        }
        if (p == 0u) return;
        p = parent_int[p];
    }
}

__device__ __forceinline__ uint32_t cross_children(uint32_t p, const uint32_t* __restrict__ lch,
                                                   const uint32_t* __restrict__ rch, const uint32_t* __restrict__ first,
                                                   const uint32_t* __restrict__ last) {
    uint32_t cnt = 0;
    const uint32_t ch[2] = {lch[p], rch[p]};
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const uint32_t c = ch[q];
        if (!(c & LEAF_BIT) && (first[c] >> REFIT_CHUNK_LOG2) != (last[c] >> REFIT_CHUNK_LOG2)) ++cnt;
    }
    return cnt;
}

__global__ __launch_bounds__(1024) void k_refit_cross(const uint32_t* __restrict__ cross,
                                                      const uint32_t* __restrict__ cross_count,
                                                      const uint32_t* __restrict__ lch, const uint32_t* __restrict__ rch,
                                                      const uint32_t* __restrict__ first,
                                                      const uint32_t* __restrict__ last,
                                                      const uint32_t* __restrict__ parent_int,
                                                      const uint32_t* __restrict__ perm, const float* __restrict__ aabb,
                                                      float* ibox, uint32_t* flags) {
    const uint32_t m = *cross_count;
    for (uint32_t j = threadIdx.x; j < m; j += blockDim.x) {
        uint32_t p = cross[j];
        if (cross_children(p, lch, rch, first, last) != 0) continue;  // reached by a climb
        for (;;) {
            float lo0[3], hi0[3], lo1[3], hi1[3];
            child_box(lch[p], perm, aabb, ibox, lo0, hi0);
            child_box(rch[p], perm, aabb, ibox, lo1, hi1);
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                ibox[6 * (size_t)p + a] = omin(lo0[a], lo1[a]);
                ibox[6 * (size_t)p + 3 + a] = omax(hi0[a], hi1[a]);
            }
            if (p == 0u) break;
            const uint32_t q = parent_int[p];
            const uint32_t need = cross_children(q, lch, rch, first, last);
            const uint32_t old =
                __hip_atomic_fetch_add(&flags[q], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (old + 1u < need) break;  // the other spanning child is not done yet
            p = q;
        }
    }
}

__device__ __forceinline__ void pad_box(float* lo, float* hi, float pad) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        lo[c] = lo[c] - (fabsf(lo[c]) * PAD_SCALE + pad);
        hi[c] = hi[c] + (fabsf(hi[c]) * PAD_SCALE + pad);
    }
}

__device__ __forceinline__ float scene_pad(const int32_t* __restrict__ bounds) {
    const float ex = unord(~bounds[3]) - unord(bounds[0]);
    const float ey = unord(~bounds[4]) - unord(bounds[1]);
    const float ez = unord(~bounds[5]) - unord(bounds[2]);
    return omax(omax(ex, ey), ez) * PAD_SCALE;
}

__device__ __forceinline__ void store_record(uint32_t* rec, const uint32_t (&r)[16]) {
    uint4* q = reinterpret_cast<uint4*>(rec);
    q[0] = make_uint4(r[0], r[1], r[2], r[3]);
    q[1] = make_uint4(r[4], r[5], r[6], r[7]);
    q[2] = make_uint4(r[8], r[9], r[10], r[11]);
    q[3] = make_uint4(r[12], r[13], r[14], r[15]);
}

__device__ __forceinline__ void set_child(uint32_t (&r)[16], int slot, const float* lo, const float* hi, uint32_t ref) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        r[slot * 6 + c] = f2u(lo[c]);
        r[slot * 6 + 3 + c] = f2u(hi[c]);
    }
    r[12 + slot] = ref;
}

__device__ __forceinline__ void set_empty(uint32_t (&r)[16], int slot) {
#pragma unroll
    for (int c = 0; c < 6; ++c) r[slot * 6 + c] = NAN_BITS;
    r[12 + slot] = EMPTY_REF;
}

__global__ __launch_bounds__(BLOCK) void k_pack(uint32_t n, uint32_t K, const uint32_t* __restrict__ lch,
                                                const uint32_t* __restrict__ rch, const uint32_t* __restrict__ first,
                                                const uint32_t* __restrict__ last, const uint32_t* __restrict__ perm,
                                                const float* __restrict__ aabb, const float* __restrict__ ibox,
                                                const int32_t* __restrict__ bounds, uint32_t* __restrict__ records) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n - 1) return;
    uint32_t r[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) r[q] = 0u;
    const uint32_t cnt = last[i] - first[i] + 1;
    if (i != 0 && cnt <= K) {  // collapsed into a leaf of its parent
        store_record(records + 16 * (size_t)i, r);
        return;
    }
    const float pad = scene_pad(bounds);
    if (i == 0 && cnt <= K) {
        float lo[3], hi[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            lo[a] = ibox[a];
            hi[a] = ibox[3 + a];
        }
        pad_box(lo, hi, pad);
        set_child(r, 0, lo, hi, LEAF_BIT | ((cnt - 1) << 27));
        set_empty(r, 1);
        store_record(records, r);
        return;
    }
    const uint32_t ch[2] = {lch[i], rch[i]};
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const uint32_t c = ch[q], cc = c & ~LEAF_BIT;
        float lo[3], hi[3];
        child_box(c, perm, aabb, ibox, lo, hi);
        uint32_t cf, cn;
        if (c & LEAF_BIT) {
            cf = cc;
            cn = 1;
        } else {
            cf = first[cc];
            cn = last[cc] - first[cc] + 1;
        }
        pad_box(lo, hi, pad);
        set_child(r, q, lo, hi, cn <= K ? (LEAF_BIT | ((cn - 1) << 27) | cf) : cc);
    }
    store_record(records + 16 * (size_t)i, r);
}

// n <= 1: a single record whose child 0 is the lone triangle (or empty).
__global__ void k_pack_small(uint32_t n, const float* __restrict__ aabb, const int32_t* __restrict__ bounds,
                             uint32_t* __restrict__ records) {
    uint32_t r[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) r[q] = 0u;
    if (n == 1) {
        float lo[3] = {aabb[0], aabb[1], aabb[2]}, hi[3] = {aabb[3], aabb[4], aabb[5]};
        pad_box(lo, hi, scene_pad(bounds));
        set_child(r, 0, lo, hi, LEAF_BIT);
    } else {
        set_empty(r, 0);
    }
    set_empty(r, 1);
    store_record(records, r);
}

__global__ __launch_bounds__(BLOCK) void k_sort_tris(uint32_t n, const uint32_t* __restrict__ perm,
                                                     const float4* __restrict__ src, float4* __restrict__ dst) {
    const uint32_t k = blockIdx.x * BLOCK + threadIdx.x;
    if (k >= n) return;
    const uint32_t g = perm[k];
    dst[3 * k + 0] = src[3 * g + 0];
    dst[3 * k + 1] = src[3 * g + 1];
    dst[3 * k + 2] = src[3 * g + 2];
}

inline uint32_t blocks_for(uint32_t n, uint32_t per) { return (n + per - 1) / per; }

}  // namespace

uint32_t radix_hist_entries(uint32_t n) { return 256u * (blocks_for(n, SORT_TILE) > 0 ? blocks_for(n, SORT_TILE) : 1u); }
uint32_t num_records(uint32_t n) { return n > 1 ? n - 1 : 1; }

#define BM_LAUNCH_CHECK()                          \
    do {                                           \
        hipError_t e_ = hipGetLastError();         \
        if (e_ != hipSuccess) return e_;           \
    } while (0)

hipError_t launch_build(const BuildBuffers& b, hipStream_t s) {
    const uint32_t n = b.n;
    hipError_t e;
    // bounds (ordered-int images; max slots store ~ord): every slot starts at INT_MAX
    if ((e = hipMemsetD32Async((hipDeviceptr_t)b.bounds, INT_MAX, BOUNDS_SLOTS, s)) != hipSuccess) return e;
    if (n == 0) {
        k_pack_small<<<1, 1, 0, s>>>(0, b.aabb, b.bounds, b.records);
        BM_LAUNCH_CHECK();
        return hipSuccess;
    }
    const uint32_t g = blocks_for(n, BLOCK);
    k_gather<<<g, BLOCK, 0, s>>>(b.meshes, b.num_meshes, n, b.tri_orig, b.nrm, b.aabb, b.bounds);
    BM_LAUNCH_CHECK();
    k_morton<<<g, BLOCK, 0, s>>>(n, b.aabb, b.bounds, b.keys, b.vals);
    BM_LAUNCH_CHECK();
    const uint32_t nb = blocks_for(n, SORT_TILE);
    uint32_t *ki = b.keys, *vi = b.vals, *ko = b.keys2, *vo = b.vals2;
    for (int pass = 0; pass < 4; ++pass) {
        const int shift = pass * 8;
        k_radix_hist<<<nb, BLOCK, 0, s>>>(ki, n, shift, b.hist, nb);
        BM_LAUNCH_CHECK();
        k_radix_scan<<<1, 1024, 0, s>>>(b.hist, 256u * nb);
        BM_LAUNCH_CHECK();
        k_radix_scatter<<<nb, BLOCK, 0, s>>>(ki, vi, ko, vo, n, shift, b.hist, nb);
        BM_LAUNCH_CHECK();
        uint32_t* tk = ki; ki = ko; ko = tk;
        uint32_t* tv = vi; vi = vo; vo = tv;
    }
    // four passes: sorted data is back in b.keys / b.vals
    if (n == 1) {
        k_pack_small<<<1, 1, 0, s>>>(1, b.aabb, b.bounds, b.records);
        BM_LAUNCH_CHECK();
    } else {
        const uint32_t gi = blocks_for(n - 1, BLOCK);
        // one memset covers the cross-node counter (word 0) and the phase-2 arrival counters
        if ((e = hipMemsetAsync(b.flags, 0, sizeof(uint32_t) * n, s)) != hipSuccess) return e;
        uint32_t* cross_count = b.flags;
        uint32_t* arrivals = b.flags + 1;
        k_emit<<<gi, BLOCK, 0, s>>>((int)n, b.keys, b.lch, b.rch, b.first, b.last, b.parent_leaf, b.parent_int,
                                    b.cross, cross_count);
        BM_LAUNCH_CHECK();
        k_refit_chunk<<<blocks_for(n, REFIT_CHUNK), REFIT_CHUNK, 0, s>>>(n, b.lch, b.rch, b.first, b.last,
                                                                       b.parent_leaf, b.parent_int, b.vals, b.aabb,
                                                                       b.ibox);
        BM_LAUNCH_CHECK();
        k_refit_cross<<<1, 1024, 0, s>>>(b.cross, cross_count, b.lch, b.rch, b.first, b.last, b.parent_int, b.vals,
                                         b.aabb, b.ibox, arrivals);
        BM_LAUNCH_CHECK();
        k_pack<<<gi, BLOCK, 0, s>>>(n, b.leaf_size, b.lch, b.rch, b.first, b.last, b.vals, b.aabb, b.ibox, b.bounds,
                                    b.records);
        BM_LAUNCH_CHECK();
    }
    k_sort_tris<<<g, BLOCK, 0, s>>>(n, b.vals, b.tri_orig, b.tris);
    BM_LAUNCH_CHECK();
    return hipSuccess;
}

}  // namespace bm
