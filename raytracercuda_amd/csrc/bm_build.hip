// bm_build.hip — LBVH acceleration-structure build for gfx950 (replaces the reference's
// sparse kd-tree insert, Raytracer/BuildTree.cu:95-362, and its SAT test, BoxTriangle.cuh).
//
// Pipeline (one HIP stream, no host round trips; 1.1M triangles in 0.29 ms on one MI355X):
//   memset          the gather's bounds replicas (the rest of the metadata block: k_gather)
//   k_gather        mesh table -> per-triangle (v0,e1,e2,id) records, corner normals, AABBs (stores
//                   staged through LDS); block-reduced scene/centroid bounds via ordered-int atomics
//                   into 64 replicas (folded by their consumers: k_morton, k_span)
//   k_morton        30-bit Morton key of each AABB centre, value = global triangle id; the digit
//                   histograms of all three sort passes
//   k_onesweep_wide x3  stable LSD radix sort, 10-bit digits, one kernel per pass: 1024-thread tiles
//                   (one digit per thread), decoupled look-back over a 32-word window, wave64 ballot
//                   ranking, the tile staged in LDS in digit order before the scatter
//   k_span          (n > 512) the radix-tree nodes whose leaf range crosses a 512-leaf chunk edge:
//                   O(1) test per index, Karras's searches 64-ary per wave; a bitmap of them
//   k_tree_chunk    per 512-leaf chunk, in LDS: the chunk-local nodes grown bottom-up (Apetrei's
//                   rule, Karras's indices) with their boxes, the triangle records in leaf order,
//                   prefix/suffix box unions at maximal-subtree ends, and (BVH4) the 128-B record of
//                   every chunk-local node above the leaf size
//   k_chunk_table   sparse table over the chunk unions (boxes of chunk-spanning ranges in O(1))
//   k_pack4_span / k_pack   BVH4 records of the spanning nodes (or all BVH2 records)
// Refit (same topology, new vertices): memset, k_gather, then k_span .. k_pack4_span as above.
// Every stored value is a deterministic function of the input (no atomics decide a value), so
// the result is bit-identical to oracle/beam_oracle.c's orc_bvh_build, which tests check.
#include <climits>

#include "bm_internal.h"

namespace bm {
namespace {

#include "bm_bdiag.h"

constexpr int BLOCK = 256;
constexpr int SORT_ITEMS = 16;  // histogram kernels; the one-sweep tile is chosen per n (onesweep_items)
constexpr int SORT_TILE = BLOCK * SORT_ITEMS;
#ifndef BM_CHUNK_DPP
#define BM_CHUNK_DPP 1  // chunk workgroups: prefix/suffix box unions by DPP rows + readlane (0: shuffles)
#endif
#ifndef BM_REFIT_CHUNK_LOG2
#define BM_REFIT_CHUNK_LOG2 9  // 512-leaf chunks: measured 2-4 % faster builds than 1024 up to 1.1M tris (256: slower at 1.1M)
#endif
constexpr uint32_t REFIT_CHUNK_LOG2 = BM_REFIT_CHUNK_LOG2;
constexpr uint32_t REFIT_CHUNK = 1u << REFIT_CHUNK_LOG2;

// Wave64 reductions on the VALU: DPP within rows of 16 (quad_perm [1,0,3,2], [2,3,0,1], row_ror 4
// and 8), then the four row results via readlane. Every lane of the wave must be active.
template <bool MAX>
__device__ __forceinline__ int wave_reduce(int v) {
    auto op = [](int a, int b) { return MAX ? max(a, b) : min(a, b); };
    v = op(v, __builtin_amdgcn_update_dpp(v, v, 0xB1, 0xF, 0xF, false));
    v = op(v, __builtin_amdgcn_update_dpp(v, v, 0x4E, 0xF, 0xF, false));
    v = op(v, __builtin_amdgcn_update_dpp(v, v, 0x124, 0xF, 0xF, false));
    v = op(v, __builtin_amdgcn_update_dpp(v, v, 0x128, 0xF, 0xF, false));
    return op(op(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
              op(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
}
__device__ __forceinline__ int wave_min(int v) { return wave_reduce<false>(v); }
__device__ __forceinline__ int wave_max(int v) { return wave_reduce<true>(v); }

// ---- build metadata block (one zero fill per build) ----------------------------------------------
//   [0, BOUNDS_SLOTS)               scene bounds (bm_common.h)
//   [META_GATHER_REPLICAS, +GATHER_REPLICAS * GATHER_REPLICA_STRIDE)  k_gather's bounds replicas
//   [META_COUNTERS, +4)             per-pass tile tickets of the one-sweep sort
//   [META_GHIST, +3*RADIX)          global digit histograms of all passes
//   [META_LOOKBACK, +3*nb*RADIX)    per-pass, per-tile, per-digit look-back words
constexpr int RADIX_BITS = 10;  // stable LSD radix sort: 3 passes of 10-bit digits over 30-bit keys
constexpr uint32_t RADIX = 1u << RADIX_BITS;
constexpr int RADIX_PASSES = 3;
constexpr uint32_t GATHER_REPLICAS = 64;
constexpr uint32_t GATHER_REPLICA_STRIDE = 32;  // 128 B apart
constexpr uint32_t META_GATHER_REPLICAS = 32;
constexpr uint32_t META_COUNTERS = META_GATHER_REPLICAS + GATHER_REPLICAS * GATHER_REPLICA_STRIDE;
constexpr uint32_t META_GATHER_CLEAR = META_COUNTERS;  // what a gather-only pass (refit, kd) zero-fills
constexpr uint32_t META_SORT_SKEW = META_COUNTERS + 3;  // buckets k_bucket_sort sorted through global memory
constexpr uint32_t META_GHIST = META_COUNTERS + 4;
constexpr uint32_t META_LOOKBACK = META_GHIST + RADIX_PASSES * RADIX;
// look-back word: flag in the top two bits, count below (counts < MAX_TRIS = 2^27)
constexpr uint32_t LB_AGG = 1u << 30;   // the tile's own digit count
constexpr uint32_t LB_PRE = 2u << 30;   // inclusive digit count over tiles 0..this
constexpr uint32_t LB_MASK = LB_AGG - 1;
// bucket plan words (bucket_plan): order, starts, skew flag
constexpr uint32_t PLAN_ORDER = 0, PLAN_START = RADIX, PLAN_FLAG = 2 * RADIX, PLAN_WORDS = 2 * RADIX + 1;
#ifndef BM_LB_WIN
#define BM_LB_WIN 8
#endif
constexpr int LB_WIN = BM_LB_WIN;       // predecessor words fetched per look-back step

// Triangles -> original-order records (v0, e1, e2 + id), corner normals, AABBs and/or AABB centres
// (each output optional), and the scene bounds of the AABBs and of their centres.
// Also zero-fills meta words [clear_begin, clear_end) — a build's: the sort's counters, histograms and
// look-back words, first used by k_morton, and the finish counters; a refit's: the finish counters —
// so that only the gather's own words need a memset.
__global__ __launch_bounds__(BLOCK) void k_gather(const MeshDesc* __restrict__ meshes, uint32_t nm, uint32_t n,
                                                  float4* __restrict__ tri, float* __restrict__ nrm,
                                                  float* __restrict__ aabb, float* __restrict__ cen,
                                                  uint32_t* __restrict__ bounds,
                                                  uint32_t clear_begin, uint32_t clear_end, int with_bounds,
                                                  int with_tri, int with_nrm) {
    BDIAG(0);
    for (uint32_t q = clear_begin + blockIdx.x * BLOCK + threadIdx.x; q < clear_end; q += gridDim.x * BLOCK)
        bounds[q] = 0u;
    // the block's records, corner normals and boxes are staged in LDS and stored as whole float4
    // runs (a lane's own 48-, 36- and 24-byte records would be strided, partial-line stores)
    __shared__ float4 s_tri[3 * BLOCK];
    __shared__ float s_nrm[9 * BLOCK];
    __shared__ float s_box[6 * BLOCK];
    __shared__ float s_cen[3 * BLOCK];
    const uint32_t g0 = blockIdx.x * BLOCK, g = g0 + threadIdx.x;
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
        if (with_tri) {
            const vec3f e1 = sub(p1, p0), e2 = sub(p2, p0);
            s_tri[3 * threadIdx.x + 0] = make_float4(p0.x, p0.y, p0.z, u2f(g));
            s_tri[3 * threadIdx.x + 1] = make_float4(e1.x, e1.y, e1.z, 0.0f);
            s_tri[3 * threadIdx.x + 2] = make_float4(e2.x, e2.y, e2.z, 0.0f);
        }
        if (with_nrm) {
            const uint32_t iv[3] = {i0, i1, i2};
#pragma unroll
            for (int k = 0; k < 3; ++k)
#pragma unroll
                for (int c = 0; c < 3; ++c) s_nrm[9 * threadIdx.x + 3 * k + c] = md.nrm[3 * iv[k] + c];
        }
        const float pa[3] = {p0.x, p0.y, p0.z}, pb[3] = {p1.x, p1.y, p1.z}, pc[3] = {p2.x, p2.y, p2.z};
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float mn = omin(omin(pa[c], pb[c]), pc[c]);
            const float mx = omax(omax(pa[c], pb[c]), pc[c]);
            const float ce = (mn + mx) * 0.5f;
            s_box[6 * threadIdx.x + c] = mn;
            s_box[6 * threadIdx.x + 3 + c] = mx;
            s_cen[3 * threadIdx.x + c] = ce;
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
    const uint32_t cnt = min(n - g0, (uint32_t)BLOCK);
    if (cnt == BLOCK) {
        if (with_tri)
            for (uint32_t q = threadIdx.x; q < 3 * BLOCK; q += BLOCK) tri[3 * (size_t)g0 + q] = s_tri[q];
        if (with_nrm) {
            float4* nd = reinterpret_cast<float4*>(nrm + 9 * (size_t)g0);
            const float4* ns = reinterpret_cast<const float4*>(s_nrm);
            for (uint32_t q = threadIdx.x; q < 9 * BLOCK / 4; q += BLOCK) nd[q] = ns[q];
        }
        if (aabb) {
            float4* bd = reinterpret_cast<float4*>(aabb + 6 * (size_t)g0);
            const float4* bs = reinterpret_cast<const float4*>(s_box);
            for (uint32_t q = threadIdx.x; q < 6 * BLOCK / 4; q += BLOCK) bd[q] = bs[q];
        }
        if (cen) {
            float4* cd = reinterpret_cast<float4*>(cen + 3 * (size_t)g0);
            const float4* cs = reinterpret_cast<const float4*>(s_cen);
            for (uint32_t q = threadIdx.x; q < 3 * BLOCK / 4; q += BLOCK) cd[q] = cs[q];
        }
    } else {
        if (with_tri)
            for (uint32_t q = threadIdx.x; q < 3 * cnt; q += BLOCK) tri[3 * (size_t)g0 + q] = s_tri[q];
        if (with_nrm)
            for (uint32_t q = threadIdx.x; q < 9 * cnt; q += BLOCK) nrm[9 * (size_t)g0 + q] = s_nrm[q];
        if (aabb)
            for (uint32_t q = threadIdx.x; q < 6 * cnt; q += BLOCK) aabb[6 * (size_t)g0 + q] = s_box[q];
        if (cen)
            for (uint32_t q = threadIdx.x; q < 3 * cnt; q += BLOCK) cen[3 * (size_t)g0 + q] = s_cen[q];
    }
    // block bounds -> replica (block % GATHER_REPLICAS) of the twelve slots, each replica on its own
    // 128-B line (fold_slot reduces them). Device atomics on one address serialise (~15 ns each),
    // so thousands of blocks updating the same twelve words would cost tens of microseconds.
    if (threadIdx.x < 6 && with_bounds) {
        const int c = threadIdx.x;
        int a = s_lo[0][c], b = s_hi[0][c];
        for (int q = 1; q < BLOCK / 64; ++q) {
            a = min(a, s_lo[q][c]);
            b = max(b, s_hi[q][c]);
        }
        // slots: aabb min 0..2, aabb max 3..5, centre min 6..8, centre max 9..11
        const int slot_lo = c < 3 ? c : 6 + (c - 3);
        const int slot_hi = c < 3 ? 3 + c : 9 + (c - 3);
        // ordered ints -> order-preserving u32; min slots complemented (see BOUNDS_SLOTS)
        uint32_t* rep = bounds + META_GATHER_REPLICAS + GATHER_REPLICA_STRIDE * (blockIdx.x % GATHER_REPLICAS);
        atomicMax(&rep[slot_lo], ~((uint32_t)a ^ 0x80000000u));
        atomicMax(&rep[slot_hi], (uint32_t)b ^ 0x80000000u);
    }
}

// ---- a triangle straight from its mesh (k_gather's operations, shared by the mesh-direct readers) -----
// Global triangle g -> its mesh (binary search over the mesh table's first ids) -> its three corners.
__device__ __forceinline__ void tri_from_mesh(const MeshDesc* __restrict__ meshes, uint32_t nm, uint32_t g,
                                              vec3f& p0, vec3f& p1, vec3f& p2) {
    uint32_t a = 0, b = nm;
    while (b - a > 1) {
        const uint32_t mid = (a + b) >> 1;
        if (meshes[mid].tri_offset <= g) a = mid;
        else b = mid;
    }
    const MeshDesc md = meshes[a];
    const uint32_t f = g - md.tri_offset;
    const uint32_t i0 = md.idx[3 * f], i1 = md.idx[3 * f + 1], i2 = md.idx[3 * f + 2];
    p0 = v3(md.pos[3 * i0], md.pos[3 * i0 + 1], md.pos[3 * i0 + 2]);
    p1 = v3(md.pos[3 * i1], md.pos[3 * i1 + 1], md.pos[3 * i1 + 2]);
    p2 = v3(md.pos[3 * i2], md.pos[3 * i2 + 1], md.pos[3 * i2 + 2]);
}
// its AABB as ordered ints (lo xyz, hi xyz): k_gather's omin/omax, so the same bits as aabb[]
__device__ __forceinline__ void tri_box_ord(const vec3f& p0, const vec3f& p1, const vec3f& p2, int32_t (&o)[6]) {
    const float pa[3] = {p0.x, p0.y, p0.z}, pb[3] = {p1.x, p1.y, p1.z}, pc[3] = {p2.x, p2.y, p2.z};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        o[c] = ord(omin(omin(pa[c], pb[c]), pc[c]));
        o[3 + c] = ord(omax(omax(pa[c], pb[c]), pc[c]));
    }
}
// its (v0 | id, e1, e2) record: k_gather's subtraction (bit-identical to bmTriIntersect's edges)
__device__ __forceinline__ void tri_record(const vec3f& p0, const vec3f& p1, const vec3f& p2, uint32_t g, float4& t0,
                                           float4& t1, float4& t2) {
    const vec3f e1 = sub(p1, p0), e2 = sub(p2, p0);
    t0 = make_float4(p0.x, p0.y, p0.z, u2f(g));
    t1 = make_float4(e1.x, e1.y, e1.z, 0.0f);
    t2 = make_float4(e2.x, e2.y, e2.z, 0.0f);
}

// Zero the gather's replica words (threads t of nthreads), after their last reader: the next LBVH
// build or refit of this buffer then needs no memset before k_gather (BuildBuffers::replicas_clean).
__device__ __forceinline__ void clear_replicas(uint32_t* __restrict__ bounds, uint32_t t, uint32_t nthreads) {
    for (uint32_t q = META_GATHER_REPLICAS + t; q < META_GATHER_CLEAR; q += nthreads) bounds[q] = 0u;
}

// Scene-bounds slot = max over the gather replicas. Folded where first needed: by k_morton (each
// block, into LDS), into bounds[0..11] by k_span's workgroup 0, k_tree_chunk (one chunk) or
// k_pack_small for the record writers.
__device__ __forceinline__ uint32_t fold_slot(const uint32_t* __restrict__ bounds, int slot) {
    uint32_t acc = 0;
#pragma unroll 16
    for (uint32_t r = 0; r < GATHER_REPLICAS; ++r)
        acc = max(acc, bounds[META_GATHER_REPLICAS + GATHER_REPLICA_STRIDE * r + slot]);
    return acc;
}

// The same fold by one wave for six consecutive slots s0..s0+5: lane r reads replica r's six words
// (three 8-B loads from one 128-B line), then a wave maximum per slot. One memory round trip instead of
// 64 dependent-free loads per slot on six lanes; every lane of the wave must be active. Returns slot
// s0 + j in lane j (j < 6).
__device__ __forceinline__ uint32_t fold6_wave(const uint32_t* __restrict__ bounds, uint32_t s0) {
    static_assert(GATHER_REPLICAS == 64, "one replica per lane");
    const uint32_t lane = threadIdx.x & 63;
    const uint2* q = reinterpret_cast<const uint2*>(bounds + META_GATHER_REPLICAS + GATHER_REPLICA_STRIDE * lane + s0);
    const uint2 a = q[0], b = q[1], c = q[2];
    uint32_t v[6] = {a.x, a.y, b.x, b.y, c.x, c.y};
    uint32_t out = 0;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        uint32_t x = v[j];
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) x = max(x, (uint32_t)__shfl_xor((int)x, o));
        out = lane == (uint32_t)j ? x : out;
    }
    return out;
}

// Morton key of each AABB centre (value = global triangle id), plus the digit histograms of all
// three sort passes (a histogram does not depend on the order the keys are in).
// 1024-thread workgroups over SORT_TILE keys (4 per thread): sixteen waves hide the loads and the
// LDS histogram atomics of a tile where four could not.
constexpr int MORTON_BLOCK = 1024;
constexpr int MORTON_ITEMS = SORT_TILE / MORTON_BLOCK;
__global__ __launch_bounds__(MORTON_BLOCK) void k_morton(uint32_t n, const float* __restrict__ cen,
                                                         uint32_t* __restrict__ meta, uint32_t* __restrict__ keys,
                                                         uint32_t* __restrict__ vals) {
    BDIAG(1);
    __shared__ uint32_t h[RADIX_PASSES * RADIX];
    __shared__ uint32_t s_cb[6];  // centre bounds slots 6..11
    // all loads first (clamped index, no branches) and before the bounds fold's barrier, so the tile
    // pays one memory latency
    const uint32_t base = blockIdx.x * SORT_TILE;
    float ce[MORTON_ITEMS][3];
#pragma unroll
    for (int it = 0; it < MORTON_ITEMS; ++it) {
        const uint32_t g = min(base + it * MORTON_BLOCK + threadIdx.x, n - 1);
        // the AABB centres k_gather computed ((lo + hi) * 0.5f per axis)
        ce[it][0] = cen[3 * (size_t)g + 0];
        ce[it][1] = cen[3 * (size_t)g + 1];
        ce[it][2] = cen[3 * (size_t)g + 2];
    }
    for (uint32_t d = threadIdx.x; d < RADIX_PASSES * RADIX; d += MORTON_BLOCK) h[d] = 0;
    if (threadIdx.x < 64) {  // wave 0: centre bounds slots 6..11
        const uint32_t v = fold6_wave(meta, 6);
        if (threadIdx.x < 6) s_cb[threadIdx.x] = v;
    }
    __syncthreads();
    float cmin[3], scale[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        cmin[c] = bounds_lo(s_cb[c]);
        const float ext = bounds_hi(s_cb[3 + c]) - cmin[c];
        scale[c] = ext > 0.0f ? 1024.0f / ext : 0.0f;
    }
#pragma unroll
    for (int it = 0; it < MORTON_ITEMS; ++it) {
        const uint32_t g = base + it * MORTON_BLOCK + threadIdx.x;
        if (g >= n) break;
        uint32_t q[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) q[c] = quant10(ce[it][c], cmin[c], scale[c]);
        const uint32_t key = (expand_bits10(q[0]) << 2) | (expand_bits10(q[1]) << 1) | expand_bits10(q[2]);
        keys[g] = key;
        vals[g] = g;
#pragma unroll
        for (int p = 0; p < RADIX_PASSES; ++p) atomicAdd(&h[p * RADIX + ((key >> (p * RADIX_BITS)) & (RADIX - 1))], 1u);
    }
    __syncthreads();
    for (uint32_t d = threadIdx.x; d < RADIX_PASSES * RADIX; d += MORTON_BLOCK)
        if (h[d]) atomicAdd(&meta[META_GHIST + d], h[d]);
}

// ---- ranked top digit (reference-mode pair sort) ------------------------------------------------------
// The reference's leaf paths are 31-bit keys: four 10-bit passes, the last over one bit. Their top 11 bits
// (the path's first 11 levels) take few values for a scene inside the reference's +-30 world — the
// (leaf, face) pairs of the bunny fall in 8 of the 2,048 — and the count pass marks the values present
// in a 2,048-bit map (`topmap`). The sort then runs three passes: bits 0-9, 10-19, and the rank of bits
// 20-30 among the values present (order-preserving, < 1,024 when at most 1,024 are present: the host
// checks). The keys themselves are not changed, so the sorted output is the four-pass one.
constexpr uint32_t TOP_BITS = 11, TOP_VALUES = 1u << TOP_BITS, TOPMAP_WORDS = TOP_VALUES / 32;
constexpr int TOP_SHIFT = 31 - (int)TOP_BITS;  // 20: the 11 bits above the two low digits of a 31-bit key
template <bool RANK>
__device__ __forceinline__ uint32_t sort_digit(uint32_t key, int shift, const uint16_t* srank) {
    return RANK ? (uint32_t)srank[key >> TOP_SHIFT] : (key >> shift) & (RADIX - 1);
}
// srank[v] = number of present values below v, from the map; one barrier inside (all threads call it)
__device__ void build_top_rank(const uint32_t* __restrict__ topmap, uint16_t* srank, uint32_t* swpre, uint32_t nthreads) {
    const uint32_t t = threadIdx.x;
    if (t < 64) {
        const uint32_t c = t < TOPMAP_WORDS ? (uint32_t)__popc(topmap[t]) : 0u;
        uint32_t incl = c;  // inclusive prefix over the wave
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)incl, o);
            if ((int)t >= o) incl += y;
        }
        swpre[t] = incl - c;
    }
    __syncthreads();
    for (uint32_t v = t; v < TOP_VALUES; v += nthreads) {
        const uint32_t w = topmap[v >> 5];
        srank[v] = (uint16_t)(swpre[v >> 5] + (uint32_t)__popc(w & ((1u << (v & 31)) - 1u)));
    }
}

// Digit histograms of every pass of a generic key sort (k_morton fuses this for the BVH build). topmap:
// the last pass (2) histograms ranked top digits (see build_top_rank).
#ifndef BM_DH_ITEMS
#define BM_DH_ITEMS 16  // keys per thread of k_digit_hist
#endif
constexpr int DH_ITEMS = BM_DH_ITEMS, DH_TILE = BLOCK * DH_ITEMS;
__global__ __launch_bounds__(BLOCK) void k_digit_hist(const uint32_t* __restrict__ keys, uint32_t n, int passes,
                                                      uint32_t* __restrict__ smeta,
                                                      const uint32_t* __restrict__ topmap) {
    __shared__ uint32_t h[4 * RADIX];
    __shared__ uint16_t srank[TOP_VALUES];
    __shared__ uint32_t swpre[64];
    for (uint32_t d = threadIdx.x; d < 4 * RADIX; d += BLOCK) h[d] = 0;
    if (topmap) build_top_rank(topmap, srank, swpre, BLOCK);
    __syncthreads();
    const uint32_t base = blockIdx.x * DH_TILE;
    uint32_t kk[DH_ITEMS];
#pragma unroll
    for (int it = 0; it < DH_ITEMS; ++it) kk[it] = keys[min(base + it * BLOCK + threadIdx.x, n - 1)];
    // A digit the whole wave shares (the high digits of spatially ordered keys: a reference-mode pair
    // list's top path bits) is one LDS add of the wave's count instead of 64 conflicting ones.
    const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
    for (int it = 0; it < DH_ITEMS; ++it) {
        const bool valid = base + it * BLOCK + threadIdx.x < n;
        const unsigned long long vm = ballot(valid);
        if (!vm) break;
        for (int p = 0; p < passes; ++p) {
            const uint32_t d = (topmap && p == 2) ? sort_digit<true>(kk[it], 0, srank)
                                                  : sort_digit<false>(kk[it], p * RADIX_BITS, nullptr);
            const uint32_t d0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)d);
            if ((ballot(d == d0) & vm) == vm) {
                if (lane == 0) atomicAdd(&h[p * RADIX + d0], (uint32_t)__popcll(vm));
            } else if (valid) {
                atomicAdd(&h[p * RADIX + d], 1u);
            }
        }
    }
    __syncthreads();
    for (uint32_t d = threadIdx.x; d < (uint32_t)passes * RADIX; d += BLOCK)
        if (h[d]) atomicAdd(&smeta[4 + d], h[d]);
}

__device__ __forceinline__ uint32_t lb_load(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lb_store(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Words handed between phases of one launch (C = true: the LSD fallback's two passes in one launch) go
// through device-coherent accesses (global_load/store sc1: written through and read past the per-XCD
// L2s), and a phase is published by its workgroup waiting for its own stores and then counting itself
// done (coh_done) — no agent-scope release fence, whose L2 write-back (buffer_wbl2) per workgroup
// serialised such hand-offs at ~0.4 us each (measured with a fused chunk + table + record kernel,
// DESIGN.md §4). C = false: plain accesses.
template <bool C, class T>
__device__ __forceinline__ T cld(const T* p) {
    static_assert(sizeof(T) == 4, "32-bit words");
    if constexpr (C) return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return *p;
}
template <bool C, class T>
__device__ __forceinline__ void cst(T* p, T v) {
    static_assert(sizeof(T) == 4, "32-bit words");
    if constexpr (C) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *p = v;
}
// Every store of this workgroup (device-coherent ones included) complete, then one count on ctr.
__device__ __forceinline__ void coh_done(uint32_t* ctr) {
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Wait for `want` counts on ctr. Only workgroups with smaller tickets are awaited (running or done).
__device__ __forceinline__ void coh_wait(const uint32_t* ctr, uint32_t want) {
    if (threadIdx.x == 0)
        while (__hip_atomic_load(const_cast<uint32_t*>(ctr), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want)
            __builtin_amdgcn_s_sleep(8);
    __syncthreads();
}

// One pass of the one-sweep stable radix sort (Adinets & Merrill 2022 style): each workgroup takes
// the next tile by ticket, publishes its digit counts, resolves its per-digit offset among earlier
// tiles by decoupled look-back, and scatters. A tile only waits on tiles with smaller tickets, which
// are already running and publish their counts without waiting, so the look-back always ends.
// Within a tile each wave ranks its own contiguous chunk (RADIX_BITS 64-lane ballots + per-wave
// running digit counts), then one pass over the digits turns the per-wave counts into offsets:
// two barriers per tile, and the sort is stable — its output is the unique stable order of the keys.
// smeta: the sort's metadata block (sort_meta_words), zero-filled: [0, 4) tickets, [4, 4 + passes *
// RADIX) digit histograms, then the per-pass look-back words.
// One tile (ticket vid) of a one-sweep pass with BLOCK lanes (four digits per thread); LDS from the
// caller (k_onesweep's own, or k_bucket_sort<256>'s when it runs the LSD fallback's last pass). lbs:
// tiles per pass in the look-back area (its stride).
template <int ITEMS>
__device__ __forceinline__ void on_tile(uint32_t* __restrict__ wc, uint32_t* __restrict__ running,
                                        uint32_t* __restrict__ wsum, const uint32_t* __restrict__ kin,
                                        const uint32_t* __restrict__ vin, uint32_t* __restrict__ kout,
                                        uint32_t* __restrict__ vout, uint32_t n, int pass, int passes,
                                        uint32_t* __restrict__ smeta, uint32_t lbs, uint32_t vid) {
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    for (uint32_t d = t; d < RADIX; d += BLOCK) {
        running[d] = 0;
#pragma unroll
        for (int q = 0; q < BLOCK / 64; ++q) wc[q * RADIX + d] = 0;
    }
    __syncthreads();
    const uint32_t base = vid * (BLOCK * ITEMS);
    const int shift = pass * RADIX_BITS;
    uint32_t k[ITEMS], v[ITEMS];
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {  // each wave: a contiguous chunk of the tile (stability)
        const uint32_t i = min(base + w * (64 * ITEMS) + it * 64 + lane, n - 1);  // branch-free: one latency
        k[it] = kin[i];
        v[it] = vin[i];
    }
#pragma unroll
    for (int it = 0; it < ITEMS; ++it)
        if (base + w * (64 * ITEMS) + it * 64 + lane < n) atomicAdd(&running[(k[it] >> shift) & (RADIX - 1)], 1u);
    __syncthreads();
    // this thread owns digits 4t..4t+3: publish the tile's counts, then resolve their offsets
    uint32_t* lb = smeta + 4 + (size_t)passes * RADIX + (size_t)pass * lbs * RADIX;
    uint32_t cnt[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        cnt[j] = running[4 * t + j];
        lb_store(&lb[(size_t)vid * RADIX + 4 * t + j], (vid == 0 ? LB_PRE : LB_AGG) | cnt[j]);
    }
    // global base of each digit: exclusive scan of this pass's digit histogram
    const uint32_t* gh = smeta + 4 + pass * RADIX;
    uint32_t g[4], s4 = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        g[j] = gh[4 * t + j];
        s4 += g[j];
    }
    uint32_t incl = wave_incl_add(s4);
    if (lane == 63) wsum[w] = incl;
    uint32_t excl[4] = {0u, 0u, 0u, 0u};
    int q[4];
    bool done[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        q[j] = (int)vid - 1;
        done[j] = vid == 0;
    }
    while (!(done[0] && done[1] && done[2] && done[3])) {
        uint32_t x[4][LB_WIN];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int m = 0; m < LB_WIN; ++m)
                x[j][m] = (!done[j] && q[j] - m >= 0) ? lb_load(&lb[(size_t)(q[j] - m) * RADIX + 4 * t + j]) : LB_PRE;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (done[j]) continue;
            int m = 0;
            for (; m < LB_WIN; ++m) {
                const uint32_t y = x[j][m];
                if (y == 0u) break;  // not published yet: poll it again
                excl[j] += y & LB_MASK;
                if (y & LB_PRE) {
                    done[j] = true;
                    break;
                }
            }
            q[j] -= m;
        }
    }
    if (vid != 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) lb_store(&lb[(size_t)vid * RADIX + 4 * t + j], LB_PRE | (excl[j] + cnt[j]));
    }
    __syncthreads();
    uint32_t gb = incl - s4;
    for (int q2 = 0; q2 < w; ++q2) gb += wsum[q2];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        running[4 * t + j] = gb + excl[j];
        gb += g[j];
    }
    __syncthreads();
    const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    // (1) rank within the wave's contiguous chunk: running per-digit counts in wc[w][*] (only this
    //     wave touches its row, and one wave's LDS operations execute in order: no barrier)
    uint32_t lrank[ITEMS];
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
        const uint32_t i = base + w * (64 * ITEMS) + it * 64 + lane;
        const bool valid = i < n;
        const uint32_t d = (k[it] >> shift) & (RADIX - 1);
        unsigned long long peers = ballot(valid);
#pragma unroll
        for (int b = 0; b < RADIX_BITS; ++b) {
            const bool bit = (d >> b) & 1u;
            const unsigned long long bb = ballot(bit);
            peers &= bit ? bb : ~bb;
        }
        const uint32_t before = valid ? wc[w * RADIX + d] : 0u;
        lrank[it] = before + __popcll(peers & lt);
        if (valid && (peers & lt) == 0ull) wc[w * RADIX + d] = before + __popcll(peers);
    }
    __syncthreads();
    // (2) per digit: wave bases = tile base of the digit + counts of the earlier waves
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t d = 4 * t + j;
        uint32_t acc = running[d];
#pragma unroll
        for (int q2 = 0; q2 < BLOCK / 64; ++q2) {
            const uint32_t c = wc[q2 * RADIX + d];
            wc[q2 * RADIX + d] = acc;
            acc += c;
        }
    }
    __syncthreads();
    // (3) scatter
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
        const uint32_t i = base + w * (64 * ITEMS) + it * 64 + lane;
        if (i < n) {
            const uint32_t off = wc[w * RADIX + ((k[it] >> shift) & (RADIX - 1))] + lrank[it];
            kout[off] = k[it];
            vout[off] = v[it];
        }
    }
}

// One pass of the one-sweep stable radix sort with 256-lane tiles (the narrow form; launch_onesweep
// uses k_onesweep_wide unless built with BM_ONESWEEP_NARROW).
template <int ITEMS>
__global__ __launch_bounds__(BLOCK) void k_onesweep(const uint32_t* __restrict__ kin,
                                                    const uint32_t* __restrict__ vin, uint32_t* __restrict__ kout,
                                                    uint32_t* __restrict__ vout, uint32_t n, int pass, int passes,
                                                    uint32_t* __restrict__ smeta, uint32_t nb) {
    __shared__ uint32_t s_vid;
    __shared__ uint32_t wsum[BLOCK / 64];
    __shared__ uint32_t running[RADIX];
    __shared__ uint32_t wc[BLOCK / 64][RADIX];
    if (threadIdx.x == 0) s_vid = atomicAdd(&smeta[pass], 1u);
    __syncthreads();
    on_tile<ITEMS>(&wc[0][0], running, wsum, kin, vin, kout, vout, n, pass, passes, smeta, nb, s_vid);
}

constexpr uint32_t OS_BLOCK_N = 1024;  // k_onesweep_wide's workgroup

// Corner normals and (j.tri set) triangle records (v0, e1, e2, id) of every triangle — what k_gather writes
// with with_nrm / with_tri set — by `nblk` workgroups of OS_BLOCK_N lanes, grid-stride, each staged through `stage`
// (12 * OS_BLOCK_N floats) for whole-float4 stores. The build reads the records only once the keys are
// sorted (the chunk kernel) and the normals never (the trace shades with them), so on the
// top-digit-first path they are gathered by extra workgroups of that pass's launch: its few dozen to ~140
// tiles leave most CUs idle while their look-back chain runs, and the gather keeps only the boxes.
struct RecJob {
    const MeshDesc* meshes;
    uint32_t nm, n, nblk;
    float4* tri;
    float* nrm;
};
// The mesh table is copied into LDS after the staging area (up to RJ_LDS_MESHES meshes), so that each
// triangle's mesh search costs LDS round trips instead of dependent global ones.
constexpr uint32_t RJ_LDS_MESHES = 256;
__device__ void gather_records(const RecJob& j, uint32_t blk, float* stage) {
    float4* st4 = reinterpret_cast<float4*>(stage);
    MeshDesc* lm = reinterpret_cast<MeshDesc*>(stage + 12 * OS_BLOCK_N);
    const bool in_lds = j.nm <= RJ_LDS_MESHES;
    if (in_lds)
        for (uint32_t t = threadIdx.x; t < j.nm; t += OS_BLOCK_N) lm[t] = j.meshes[t];
    __syncthreads();
    const MeshDesc* mt = in_lds ? lm : j.meshes;
    for (uint32_t g0 = blk * OS_BLOCK_N; g0 < j.n; g0 += j.nblk * OS_BLOCK_N) {
        const uint32_t g = g0 + threadIdx.x, cnt = min(j.n - g0, OS_BLOCK_N);
        float nv[9];
        if (g < j.n) {
            uint32_t a = 0, b = j.nm;
            while (b - a > 1) {
                const uint32_t mid = (a + b) >> 1;
                if (mt[mid].tri_offset <= g) a = mid;
                else b = mid;
            }
            const MeshDesc md = mt[a];
            const uint32_t f = g - md.tri_offset;
            const uint32_t iv[3] = {md.idx[3 * f], md.idx[3 * f + 1], md.idx[3 * f + 2]};
            // k_gather's operations
            vec3f p0 = v3(0.0f, 0.0f, 0.0f), p1 = p0, p2 = p0;
            if (j.tri) {
                p0 = v3(md.pos[3 * iv[0]], md.pos[3 * iv[0] + 1], md.pos[3 * iv[0] + 2]);
                p1 = v3(md.pos[3 * iv[1]], md.pos[3 * iv[1] + 1], md.pos[3 * iv[1] + 2]);
                p2 = v3(md.pos[3 * iv[2]], md.pos[3 * iv[2] + 1], md.pos[3 * iv[2] + 2]);
            }
#pragma unroll
            for (int k = 0; k < 3; ++k)
#pragma unroll
                for (int c = 0; c < 3; ++c) nv[3 * k + c] = md.nrm[3 * iv[k] + c];
            if (j.tri) {
                const vec3f e1 = sub(p1, p0), e2 = sub(p2, p0);
                st4[3 * threadIdx.x + 0] = make_float4(p0.x, p0.y, p0.z, u2f(g));
                st4[3 * threadIdx.x + 1] = make_float4(e1.x, e1.y, e1.z, 0.0f);
                st4[3 * threadIdx.x + 2] = make_float4(e2.x, e2.y, e2.z, 0.0f);
            }
        }
        if (j.tri) {
            __syncthreads();
            for (uint32_t q = threadIdx.x; q < 3 * cnt; q += OS_BLOCK_N) j.tri[3 * (size_t)g0 + q] = st4[q];
            __syncthreads();
        }
        if (g < j.n)
#pragma unroll
            for (int k = 0; k < 9; ++k) stage[9 * threadIdx.x + k] = nv[k];
        __syncthreads();
        if (cnt == OS_BLOCK_N) {
            float4* nd = reinterpret_cast<float4*>(j.nrm + 9 * (size_t)g0);
            for (uint32_t q = threadIdx.x; q < 9 * OS_BLOCK_N / 4; q += OS_BLOCK_N) nd[q] = st4[q];
        } else {
            for (uint32_t q = threadIdx.x; q < 9 * cnt; q += OS_BLOCK_N) j.nrm[9 * (size_t)g0 + q] = stage[q];
        }
        __syncthreads();
    }
}

// The same pass with 1024-thread workgroups: one digit per thread, so the look-back polls a window of
// OS_LB_WIN predecessor words per digit for the price of 4 x LB_WIN in k_onesweep, and 16 waves rank
// a tile in parallel. On MI355X the look-back words live beyond the per-XCD L2s (agent scope), so one
// look-back step costs a fabric round trip: with every tile resident at once a tile walks back about
// tiles / (2 x window) steps, which a 32-word window keeps to a few.
constexpr int OS_WAVES = OS_BLOCK_N / 64;
constexpr int OS_BLOCK = OS_BLOCK_N;
#ifndef BM_OS_LB_WIN
#define BM_OS_LB_WIN 32
#endif
constexpr int OS_LB_WIN = BM_OS_LB_WIN;
static_assert(OS_BLOCK == (int)RADIX, "one digit per thread");

// LDS of one wide one-sweep tile: k_onesweep_wide's own, or k_bucket_sort<1024>'s when it runs the LSD
// fallback (BsLds has the same arrays).
#ifndef BM_OW_RANK_HIST
#define BM_OW_RANK_HIST 1  // the wide tile histogram from the ranking ballots (0: one LDS atomic per key; A/B)
#endif
#ifndef BM_OS_IDENT_SKIP
#define BM_OS_IDENT_SKIP 1  // 0: no identity copy for a pass whose digit is constant (A/B)
#endif
struct OwShared {
    uint32_t* wc;       // [OS_WAVES][RADIX]: per-wave digit counts, then the tile in digit order
    uint32_t* running;  // [RADIX]
    uint32_t* wsum;     // [OS_WAVES]
    uint32_t* lsum;     // [OS_WAVES]
};

// The ranking, look-back and scatter of one wide one-sweep tile whose keys and values are in registers
// (item it of wave w, lane l: tile position w * 64 * ITEMS + it * 64 + l); running[] and wc[] zeroed and
// a barrier passed by the caller; g = digit t's global count.
template <int ITEMS, bool C, class Diag, bool RANK = false>
__device__ __forceinline__ void ow_rank(const Diag& diag, const OwShared& S, const uint32_t (&k)[ITEMS],
                                        const uint32_t (&v)[ITEMS], uint32_t g, uint32_t* __restrict__ kout,
                                        uint32_t* __restrict__ vout, uint32_t n, int pass, int passes,
                                        uint32_t* __restrict__ smeta, uint32_t lbs, uint32_t vid,
                                        const uint16_t* srank = nullptr) {
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    uint32_t* const wc = S.wc;
    uint32_t* const running = S.running;
    const uint32_t base = vid * (OS_BLOCK * ITEMS);
    const int shift = pass * RADIX_BITS;
    uint32_t* lb = smeta + 4 + (size_t)passes * RADIX + (size_t)pass * lbs * RADIX;
    int q = (int)vid - 1;
    bool done = vid == 0;
    uint32_t x[OS_LB_WIN];
    uint32_t cnt = 0;
    if (!BM_OW_RANK_HIST) {
#pragma unroll
        for (int it = 0; it < ITEMS; ++it)
            if (base + w * (64 * ITEMS) + it * 64 + lane < n) atomicAdd(&running[sort_digit<RANK>(k[it], shift, srank)], 1u);
        __syncthreads();
        diag.mark(0);
        cnt = running[t];
        lb_store(&lb[(size_t)vid * RADIX + t], (vid == 0 ? LB_PRE : LB_AGG) | cnt);
        // the first look-back window is in flight while the wave ranks its keys
#pragma unroll
        for (int m = 0; m < OS_LB_WIN; ++m)
            x[m] = (!done && q - m >= 0) ? lb_load(&lb[(size_t)(q - m) * RADIX + t]) : LB_PRE;
    }
    // (1) rank within the wave's contiguous chunk (running per-digit counts in wc[w][*]); with
    // BM_OW_RANK_HIST the tile histogram comes from the same ballots (one LDS atomic per digit run of a
    // wave instead of one per key: a tile's keys share few digits on the top pass of a coherent mesh)
    const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    uint32_t lrank[ITEMS];
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
        const uint32_t i = base + w * (64 * ITEMS) + it * 64 + lane;
        const bool valid = i < n;
        const uint32_t d = sort_digit<RANK>(k[it], shift, srank);
        unsigned long long peers = ballot(valid);
#pragma unroll
        for (int b = 0; b < RADIX_BITS; ++b) {
            const bool bit = (d >> b) & 1u;
            const unsigned long long bb = ballot(bit);
            peers &= bit ? bb : ~bb;
        }
        const uint32_t before = valid ? wc[w * RADIX + d] : 0u;
        lrank[it] = before + __popcll(peers & lt);
        if (valid && (peers & lt) == 0ull) {
            wc[w * RADIX + d] = before + __popcll(peers);
            if (BM_OW_RANK_HIST) atomicAdd(&running[d], (uint32_t)__popcll(peers));
        }
    }
    if (BM_OW_RANK_HIST) {
        __syncthreads();
        diag.mark(0);
        cnt = running[t];
        lb_store(&lb[(size_t)vid * RADIX + t], (vid == 0 ? LB_PRE : LB_AGG) | cnt);
#pragma unroll
        for (int m = 0; m < OS_LB_WIN; ++m)
            x[m] = (!done && q - m >= 0) ? lb_load(&lb[(size_t)(q - m) * RADIX + t]) : LB_PRE;
    }
    diag.mark(1);
    // inclusive scans over the digits: global histogram (digit bases in the output) and this tile's
    // counts (digit starts inside the tile)
    const uint32_t incl = wave_incl_add(g), lincl = wave_incl_add(cnt);
    if (lane == 63) {
        S.wsum[w] = incl;
        S.lsum[w] = lincl;
    }
    uint32_t excl = 0;
    while (!done) {
        int m = 0;
        for (; m < OS_LB_WIN; ++m) {
            const uint32_t y = x[m];
            if (y == 0u) break;  // not published yet: poll it again
            excl += y & LB_MASK;
            if (y & LB_PRE) {
                done = true;
                break;
            }
        }
        q -= m;
        if (!done) {
#pragma unroll
            for (int m2 = 0; m2 < OS_LB_WIN; ++m2)
                x[m2] = q - m2 >= 0 ? lb_load(&lb[(size_t)(q - m2) * RADIX + t]) : LB_PRE;
        }
    }
    if (vid != 0) lb_store(&lb[(size_t)vid * RADIX + t], LB_PRE | (excl + cnt));
    diag.mark(2);
    __syncthreads();
    uint32_t gb = incl - g, ls = lincl - cnt;
    for (int q2 = 0; q2 < w; ++q2) {
        gb += S.wsum[q2];
        ls += S.lsum[q2];
    }
    // (2) digit t: tile-local wave bases; output slot of the tile's j-th key (digit order) = running[d] + j
    {
        uint32_t acc = ls;
#pragma unroll
        for (int q2 = 0; q2 < OS_WAVES; ++q2) {
            const uint32_t c = wc[q2 * RADIX + t];
            wc[q2 * RADIX + t] = acc;
            acc += c;
        }
    }
    running[t] = gb + excl - ls;
    __syncthreads();
    uint32_t lp[ITEMS];
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) lp[it] = wc[w * RADIX + sort_digit<RANK>(k[it], shift, srank)] + lrank[it];
    __syncthreads();
    // (3) the tile in digit order through LDS (over wc), then runs of consecutive output slots
    uint32_t* s_k = wc;
    uint32_t* s_v = s_k + OS_BLOCK * ITEMS;
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
        if (base + w * (64 * ITEMS) + it * 64 + lane < n) {
            s_k[lp[it]] = k[it];
            s_v[lp[it]] = v[it];
        }
    }
    __syncthreads();
    diag.mark(3);
    const uint32_t tn = min(n - base, (uint32_t)(OS_BLOCK * ITEMS));
#pragma unroll
    for (int m = 0; m < ITEMS; ++m) {
        const uint32_t j = m * OS_BLOCK + t;
        if (j < tn) {
            const uint32_t key = s_k[j];
            const uint32_t off = running[sort_digit<RANK>(key, shift, srank)] + j;
            cst<C>(kout + off, key);
            cst<C>(vout + off, s_v[j]);
        }
    }
}

// One tile (ticket vid) of a one-sweep pass with OS_BLOCK lanes (one digit per thread). lbs: tiles per
// pass in the look-back area (its stride). wait_ctr: wait for that many (wait_for) tiles of the
// previous pass first (the LSD fallback's second pass in the same launch).
template <int ITEMS, bool C = false, class Diag, bool RANK = false>
__device__ __forceinline__ void ow_tile(const Diag& diag, const OwShared& S, const uint32_t* __restrict__ kin,
                                        const uint32_t* __restrict__ vin, uint32_t* __restrict__ kout,
                                        uint32_t* __restrict__ vout, uint32_t n, int pass, int passes,
                                        uint32_t* __restrict__ smeta, uint32_t lbs, uint32_t vid,
                                        const uint32_t* wait_ctr = nullptr, uint32_t wait_for = 0,
                                        const uint16_t* srank = nullptr) {
    static_assert(2 * OS_BLOCK * ITEMS <= OS_WAVES * RADIX, "the digit-ordered tile reuses wc");
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    uint32_t* const wc = S.wc;
    uint32_t* const running = S.running;
    const uint32_t g = cld<C>(smeta + 4 + pass * RADIX + t);  // digit t's global count
    running[t] = 0;
#pragma unroll
    for (int q = 0; q < OS_WAVES; ++q) wc[q * RADIX + t] = 0;
    if (wait_ctr) coh_wait(wait_ctr, wait_for);
    const uint32_t base = vid * (OS_BLOCK * ITEMS);
    // one digit holds every key: the stable pass is the identity, so every tile copies itself (no
    // ranking, no look-back; all tiles read the same histogram and take this branch together)
    if (__syncthreads_or(BM_OS_IDENT_SKIP && g == n)) {
#pragma unroll
        for (int it = 0; it < ITEMS; ++it) {
            const uint32_t i = base + it * OS_BLOCK + t;
            if (i < n) {
                cst<C>(kout + i, cld<C>(kin + i));
                cst<C>(vout + i, cld<C>(vin + i));
            }
        }
        return;
    }
    uint32_t k[ITEMS], v[ITEMS];
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {  // each wave: a contiguous chunk of the tile (stability)
        const uint32_t i = min(base + w * (64 * ITEMS) + it * 64 + lane, n - 1);
        k[it] = cld<C>(kin + i);
        v[it] = cld<C>(vin + i);
    }
    ow_rank<ITEMS, C, Diag, RANK>(diag, S, k, v, g, kout, vout, n, pass, passes, smeta, lbs, vid, srank);
}

struct NoDiag {
    __device__ void mark(int) const {}
};
#ifdef BM_BUILD_DIAG
#define BDIAG_OBJ bdiag_scope_
#else
#define BDIAG_OBJ NoDiag()
#endif

// The bucket plan of a top-digit-first sort, by one extra workgroup (OS_BLOCK lanes, lane t = digit t)
// of the top-digit pass's launch, beside its tiles: plan[PLAN_ORDER + i] = the i-th bucket with more
// than one key in (size class of 64 keys descending, digit) order, ~0u past them — workgroup b of
// k_bucket_sort sorts bucket b of that order, so the nonempty buckets dispatch first and the biggest in
// the first round (in digit order the 1,024-lane workgroups of empty and big buckets queued behind each
// other); plan[PLAN_START + d] = the first position of bucket d; plan[PLAN_FLAG] = some bucket holds
// skew_cap keys or more (the LSD fallback). Each bucket workgroup used to derive all of it from the
// histogram itself (~4 us of its ~9).
// C: the histogram was summed by this launch (device-coherent loads).
template <bool C = false>
__device__ void bucket_plan(const uint32_t* __restrict__ gh, uint32_t* __restrict__ plan, uint32_t skew_cap,
                            uint32_t* lds) {
    constexpr uint32_t NCLS = 128;
    const uint32_t t = threadIdx.x, w = t >> 6, lane = t & 63;
    uint32_t* cnt = lds;                    // [OS_WAVES][NCLS] per-wave class counts, then wave bases
    uint32_t* cbase = lds + OS_WAVES * NCLS;  // [NCLS] class bases
    uint32_t* wsum = cbase + NCLS;          // [OS_WAVES]
    const uint32_t c = cld<C>(gh + t);
    for (uint32_t i = t; i < OS_WAVES * NCLS; i += OS_BLOCK) cnt[i] = 0;
    // bucket starts: exclusive scan of the histogram over the digits
    uint32_t incl = wave_incl_add(c);
    if (lane == 63) wsum[w] = incl;
    const uint32_t cls = c <= 1 ? NCLS - 1 : NCLS - 2 - min(c >> 6, NCLS - 2);  // 0: the largest
    const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    unsigned long long peers = ~0ull;
#pragma unroll
    for (int b = 0; b < 7; ++b) {
        const bool bit = (cls >> b) & 1u;
        const unsigned long long bb = ballot(bit);
        peers &= bit ? bb : ~bb;
    }
    __syncthreads();  // cnt zeroed, wsum in
    uint32_t start = incl - c;
    for (uint32_t q = 0; q < w; ++q) start += wsum[q];
    plan[PLAN_START + t] = start;
    if ((peers & lt) == 0ull) cnt[w * NCLS + cls] = (uint32_t)__popcll(peers);
    __syncthreads();
    if (t < NCLS) {  // class t: its waves' bases, then the classes' exclusive scan (two waves)
        uint32_t tot = 0;
#pragma unroll
        for (int q = 0; q < OS_WAVES; ++q) {
            const uint32_t x = cnt[q * NCLS + t];
            cnt[q * NCLS + t] = tot;
            tot += x;
        }
        uint32_t ci = wave_incl_add(tot);
        cbase[t] = ci - tot;
        if (lane == 63) wsum[w] = ci;  // waves 0, 1
    }
    __syncthreads();
    const uint32_t pos = cbase[cls] + (cls >= 64 ? wsum[0] : 0u) + cnt[w * NCLS + cls] + (uint32_t)__popcll(peers & lt);
    plan[PLAN_ORDER + pos] = c > 1 ? t : ~0u;  // the single-key and empty buckets are class NCLS - 1: last
    const bool big = __syncthreads_or(c >= skew_cap);
    if (t == 0) plan[PLAN_FLAG] = big ? 1u : 0u;
}

// One pass of the sort per launch: workgroups [0, nb) take tiles by ticket, the ones past them
// gather records and normals (rj.nblk, launch_onesweep). skew_cap > 0 (the top-digit pass of a
// top-digit-first sort, launched with 2 nb tile workgroups): when k_morton's top-digit histogram has a
// bucket of skew_cap keys or more — more than k_bucket_sort's cap = skew_cap - 1 — every workgroup sees it
// and the launch runs the LSD passes 0 and 1 instead (tickets [0, nb) pass 0 keys2 -> keys, [nb, 2 nb)
// pass 1 keys -> keys2 once every pass-0 tile is done; k_bucket_sort then runs pass 2). The tile
// counter of pass 0 (the skew word) is left nonzero, which tells the host the build took that path.
template <int ITEMS, bool RANK = false>
__global__ __launch_bounds__(OS_BLOCK) void k_onesweep_wide(const uint32_t* __restrict__ kin,
                                                            const uint32_t* __restrict__ vin,
                                                            uint32_t* __restrict__ kout, uint32_t* __restrict__ vout,
                                                            uint32_t n, int pass, int passes,
                                                            uint32_t* __restrict__ smeta, uint32_t nb, uint32_t lbs,
                                                            RecJob rj, uint32_t skew_cap, uint32_t* __restrict__ plan,
                                                            const uint32_t* __restrict__ topmap = nullptr) {
    __shared__ uint32_t s_vid;
    __shared__ uint32_t wsum[OS_WAVES], lsum[OS_WAVES];
    __shared__ uint32_t running[RADIX];
    __shared__ uint32_t wc[OS_WAVES][RADIX];  // per-wave digit counts, then the tile in digit order
    static_assert(12 * OS_BLOCK + RJ_LDS_MESHES * sizeof(MeshDesc) / 4 <= OS_WAVES * RADIX,
                  "the records' staging and mesh table reuse wc");
    const uint32_t tile_wgs = skew_cap ? 2 * nb : nb;
    if (blockIdx.x >= tile_wgs) {  // workgroups past the tiles: triangle records and normals, then the plan
        if (blockIdx.x - tile_wgs < rj.nblk) gather_records(rj, blockIdx.x - tile_wgs, reinterpret_cast<float*>(&wc[0][0]));
        else bucket_plan(smeta + 4 + pass * RADIX, plan, skew_cap, &wc[0][0]);
        return;
    }
    const int t = threadIdx.x;
    const bool skew = skew_cap && __syncthreads_or(smeta[4 + pass * RADIX + t] >= skew_cap);
    if (!skew && blockIdx.x >= nb) return;
    BDIAG(2 + pass);
    if (t == 0) s_vid = atomicAdd(&smeta[skew ? 0 : pass], 1u);
    __syncthreads();
    const uint32_t vid = s_vid;
    const OwShared S{&wc[0][0], running, wsum, lsum};
    if constexpr (RANK) {  // the ranked top digit (build_top_rank): a reference-mode pair sort's last pass
        __shared__ uint16_t srank[TOP_VALUES];
        __shared__ uint32_t swpre[64];
        build_top_rank(topmap, srank, swpre, OS_BLOCK);
        __syncthreads();
        ow_tile<ITEMS, false, decltype(BDIAG_OBJ), true>(BDIAG_OBJ, S, kin, vin, kout, vout, n, pass, passes, smeta,
                                                         lbs, vid, nullptr, 0, srank);
        return;
    }
    if (!skew) {
        ow_tile<ITEMS>(BDIAG_OBJ, S, kin, vin, kout, vout, n, pass, passes, smeta, lbs, vid);
    } else if (vid < nb) {  // LSD pass 0: Morton output (kin) -> kout
        ow_tile<ITEMS, true>(BDIAG_OBJ, S, kin, vin, kout, vout, n, 0, passes, smeta, lbs, vid);
        coh_done(smeta + 3);
    } else {  // LSD pass 1: kout -> kin, after every pass-0 tile
        ow_tile<ITEMS, true>(BDIAG_OBJ, S, kout, vout, const_cast<uint32_t*>(kin), const_cast<uint32_t*>(vin), n, 1,
                             passes, smeta, lbs, vid - nb, smeta + 3, nb);
    }
}


// ---- small sorts: most significant digit first, then each bucket on its own -------------------------
// For n <= BM_MSD_MAX_N the build sorts by the top digit first (one k_onesweep_wide pass, stable) and
// then sorts each of the RADIX buckets by the two lower digits in one workgroup (k_bucket_sort), in
// place: the same stable order as three LSD passes — (top digit, lower digits, index) — in two launches
// instead of three. A bucket of at most BS_CAP keys is sorted in LDS (two 10-bit passes, ranked by
// ballots in index order as in k_onesweep_wide). When k_morton's top-digit histogram holds a larger
// bucket (a skewed scene: a far triangle stretches the scene box, and most keys share their top digit),
// the same two launches run the three LSD passes instead, decided on the device from that histogram:
// k_onesweep_wide passes 0 and 1 (the second after the first's tiles, by ticket), k_bucket_sort pass 2.
#ifndef BM_MSD_MAX_N
#define BM_MSD_MAX_N (1u << 22)  // bunny 0.080 -> 0.067 ms, armadillo 0.122 -> 0.100
#endif
#ifndef BM_MSD_WIDE_N
#define BM_MSD_WIDE_N (1u << 19)  // above: 1024-lane bucket workgroups (8,192 keys in LDS, one workgroup per CU)
#endif
#ifndef BM_MSD_MIN_N
#define BM_MSD_MIN_N (1u << 14)  // below: a few one-sweep tiles per pass are cheaper than 1024 bucket workgroups
#endif
constexpr int BS_ITEMS = 8;  // keys per lane at most: a bucket of up to BS_BLOCK * 8 keys sorts in LDS
__device__ __forceinline__ uint32_t blocks_for_dev(uint32_t n, uint32_t per) { return (n + per - 1) / per; }

template <int BS_BLOCK>
struct BsLds {
    static constexpr int BS_WAVES = BS_BLOCK / 64;
    static constexpr uint32_t BS_CAP = BS_BLOCK * BS_ITEMS;
    uint32_t wc[BS_WAVES][RADIX];  // per-wave digit counts, then output bases
    uint32_t k[BS_CAP], v[BS_CAP];
    uint32_t run[RADIX];           // LSD fallback: the one-sweep tile's running digit bases
    uint32_t wsum[BS_WAVES];
    uint32_t red[BS_WAVES];
};

// Ranks the tile's keys (wave w: items [w * 64 * ITEMS, +64 * ITEMS), lane order within an item row)
// by digit (key >> shift) & (RADIX - 1), stably: lrank = rank among equal digits of the same wave, wc[w][d]
// = the wave's count of digit d.
template <int BS_BLOCK>
__device__ __forceinline__ void bs_rank(BsLds<BS_BLOCK>& L, const uint32_t (&k)[BS_ITEMS], uint32_t (&lrank)[BS_ITEMS], int shift,
                                        uint32_t tn, int ie) {
    constexpr int BS_WAVES = BS_BLOCK / 64;
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    for (int d = t; d < BS_WAVES * (int)RADIX; d += BS_BLOCK) (&L.wc[0][0])[d] = 0;
    __syncthreads();
    const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
#pragma unroll
    for (int it = 0; it < BS_ITEMS; ++it) {
        if (it >= ie) break;
        const uint32_t i = w * (64 * ie) + it * 64 + lane;
        const bool valid = i < tn;
        const uint32_t d = (k[it] >> shift) & (RADIX - 1);
        unsigned long long peers = ballot(valid);
#pragma unroll
        for (int b = 0; b < RADIX_BITS; ++b) {
            const bool bit = (d >> b) & 1u;
            const unsigned long long bb = ballot(bit);
            peers &= bit ? bb : ~bb;
        }
        const uint32_t before = valid ? L.wc[w][d] : 0u;
        lrank[it] = before + __popcll(peers & lt);
        if (valid && (peers & lt) == 0ull) L.wc[w][d] = before + __popcll(peers);
    }
    __syncthreads();
}

// Per-wave output bases wc[w][d] = base(d) + (digit d's keys in the waves before w). LDS path (run ==
// nullptr): base(d) = exclusive scan over the digits of the tile's totals. Global path: base(d) = run[d],
// the running base of digit d over the tiles before, which then advances by the tile's count of d.
template <int BS_BLOCK>
__device__ __forceinline__ void bs_bases(BsLds<BS_BLOCK>& L, uint32_t* run) {
    constexpr int BS_WAVES = BS_BLOCK / 64;
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    constexpr int DPT = RADIX / BS_BLOCK;  // digits per thread (4)
    uint32_t tot[DPT], sum = 0;
#pragma unroll
    for (int j = 0; j < DPT; ++j) {
        const int d = t * DPT + j;
        uint32_t c = 0;
#pragma unroll
        for (int q = 0; q < BS_WAVES; ++q) c += L.wc[q][d];
        tot[j] = c;
        sum += c;
    }
    uint32_t incl = wave_incl_add(sum);
    if (lane == 63) L.wsum[w] = incl;
    __syncthreads();
    uint32_t excl = incl - sum;
    for (int q = 0; q < w; ++q) excl += L.wsum[q];
#pragma unroll
    for (int j = 0; j < DPT; ++j) {
        const int d = t * DPT + j;
        uint32_t acc = run ? run[d] : excl;
#pragma unroll
        for (int q = 0; q < BS_WAVES; ++q) {
            const uint32_t c = L.wc[q][d];
            L.wc[q][d] = acc;
            acc += c;
        }
        if (run) run[d] = acc;
        excl += tot[j];
    }
    __syncthreads();
}

// The bucket of each workgroup, its start and the skew flag come from the plan the top-digit pass's launch
// wrote (bucket_plan). Also the LSD fallback's last pass: when a top-digit bucket holds more than the LDS
// cap (the flag; k_onesweep_wide
// ran the LSD passes 0 and 1 instead of the top-digit pass, into keys2/vals2), the workgroups run the
// one-sweep pass 2 over keys2 -> keys in tiles of the top-digit pass's size (wide_items keys per lane
// of a 1,024-lane tile; 256-lane workgroups take the same tiles at 4 wide_items per lane, or half of
// one at 8 keys per lane for one-key-per-lane tiles), and no bucket is sorted.
template <int BS_BLOCK>
__global__ __launch_bounds__(BS_BLOCK) void k_bucket_sort(uint32_t* __restrict__ keys, uint32_t* __restrict__ vals,
                                                          uint32_t* __restrict__ keys2, uint32_t* __restrict__ vals2,
                                                          uint32_t* __restrict__ meta, const uint32_t* __restrict__ plan,
                                                          uint32_t n, uint32_t nb, int wide_items) {
    BDIAG(3);
    __shared__ BsLds<BS_BLOCK> L;
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    const uint32_t* gh = meta + META_GHIST + 2 * RADIX;  // top-digit histogram (k_morton)
    // the plan's skew flag: the test k_onesweep_wide made on the same histogram
    if (plan[PLAN_FLAG]) {
        uint32_t* smeta = meta + META_COUNTERS;
        __shared__ uint32_t s_vid;
        const int items = BS_BLOCK == 1024 ? 8 : wide_items == 1 ? 8 : 16;
        if (blockIdx.x >= blocks_for_dev(n, BS_BLOCK * items)) return;
        if (t == 0) s_vid = atomicAdd(&smeta[2], 1u);
        __syncthreads();
        if constexpr (BS_BLOCK == 1024) {
            const OwShared S{&L.wc[0][0], L.run, L.wsum, L.red};
            ow_tile<8>(NoDiag(), S, keys2, vals2, keys, vals, n, 2, RADIX_PASSES, smeta, nb, s_vid);
        } else if (items == 8) {
            on_tile<8>(&L.wc[0][0], L.run, L.wsum, keys2, vals2, keys, vals, n, 2, RADIX_PASSES, smeta, nb, s_vid);
        } else {
            on_tile<16>(&L.wc[0][0], L.run, L.wsum, keys2, vals2, keys, vals, n, 2, RADIX_PASSES, smeta, nb, s_vid);
        }
        return;
    }
    // workgroup b sorts the plan's b-th bucket: the nonempty ones largest first (bucket_plan)
    const uint32_t d = plan[PLAN_ORDER + blockIdx.x];
    if (d == ~0u) return;
    const uint32_t c = gh[d], start = plan[PLAN_START + d];
    uint32_t k[BS_ITEMS], v[BS_ITEMS], lrank[BS_ITEMS];
    // the bucket in LDS (c <= cap <= BS_CAP: larger buckets took the LSD fallback above): two passes,
    // one load, one store. Items per lane sized to the bucket, so that all waves share the ranking chains
    const int ie = (int)((c + BS_BLOCK - 1) / BS_BLOCK);
#pragma unroll
    for (int it = 0; it < BS_ITEMS; ++it) {
        if (it >= ie) break;
        const uint32_t i = w * (64 * ie) + it * 64 + lane;
        k[it] = i < c ? keys[start + i] : 0u;
        v[it] = i < c ? vals[start + i] : 0u;
    }
    for (int pass = 0; pass < 2; ++pass) {
        const int shift = pass * RADIX_BITS;
        BDIAG_MARK(2 * pass);
        bs_rank(L, k, lrank, shift, c, ie);
        BDIAG_MARK(2 * pass + 1);
        bs_bases(L, nullptr);
#pragma unroll
        for (int it = 0; it < BS_ITEMS; ++it) {
            if (it >= ie) break;
            const uint32_t i = w * (64 * ie) + it * 64 + lane;
            if (i < c) {
                const uint32_t o = L.wc[w][(k[it] >> shift) & (RADIX - 1)] + lrank[it];
                L.k[o] = k[it];
                L.v[o] = v[it];
            }
        }
        __syncthreads();
#pragma unroll
        for (int it = 0; it < BS_ITEMS; ++it) {
            if (it >= ie) break;
            const uint32_t i = w * (64 * ie) + it * 64 + lane;
            k[it] = i < c ? L.k[i] : 0u;
            v[it] = i < c ? L.v[i] : 0u;
        }
        __syncthreads();
    }
#pragma unroll
    for (int it = 0; it < BS_ITEMS; ++it) {
        if (it >= ie) break;
        const uint32_t i = w * (64 * ie) + it * 64 + lane;
        if (i < c) {
            keys[start + i] = k[it];
            vals[start + i] = v[it];
        }
    }
}

// ---- Karras 2012 radix tree ------------------------------------------------------------------
__device__ __forceinline__ int kdelta(const uint32_t* __restrict__ k, int n, int i, int j) {
    if (j < 0 || j >= n) return -1;
    const uint32_t a = k[i], b = k[j];
    if (a == b) return 32 + __clz((uint32_t)i ^ (uint32_t)j);
    return __clz(a ^ b);
}

// One internal node i of Karras's radix tree over n sorted keys (children, parents, covered range).
__device__ __forceinline__ void karras_node(int i, int n, const uint32_t* __restrict__ keys, uint32_t* __restrict__ lch,
                                            uint32_t* __restrict__ rch, uint32_t* __restrict__ first,
                                            uint32_t* __restrict__ last, uint32_t* __restrict__ parent_leaf,
                                            uint32_t* __restrict__ parent_int) {
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
}

// Karras radix tree over the reference-mode leaf keys (16,742 on the bunny): every
// workgroup with nodes to emit first copies all keys into LDS, so the searches' ~2 log2(n) dependent key
// reads are LDS round trips instead of global ones (13 -> ~4 us on the bunny). More keys than the LDS
// holds: the global reads. n_dev: the key count on the device (n: the capacity).
constexpr uint32_t EMIT_LDS_KEYS = 32768, EMIT_LDS_BLOCK = 1024;
__global__ __launch_bounds__(EMIT_LDS_BLOCK) void k_emit_lds(int n, const uint32_t* __restrict__ keys,
                                                             uint32_t* __restrict__ lch, uint32_t* __restrict__ rch,
                                                             uint32_t* __restrict__ first, uint32_t* __restrict__ last,
                                                             uint32_t* __restrict__ parent_leaf,
                                                             uint32_t* __restrict__ parent_int,
                                                             const uint32_t* __restrict__ n_dev) {
    __shared__ uint32_t sk[EMIT_LDS_KEYS];
    if (n_dev) n = *n_dev <= (uint32_t)n ? (int)*n_dev : 0;
    const int b0 = (int)(blockIdx.x * EMIT_LDS_BLOCK);
    if (b0 >= n - 1) return;  // the whole workgroup: no node here
    const int i = b0 + (int)threadIdx.x;
    if ((uint32_t)n <= EMIT_LDS_KEYS) {
        const int n4 = n >> 2;  // 16-B loads (the key buffer starts 16-B aligned), then the tail
        const uint4* k4 = reinterpret_cast<const uint4*>(keys);
        uint4* s4 = reinterpret_cast<uint4*>(sk);
#pragma unroll 4
        for (int q = (int)threadIdx.x; q < n4; q += (int)EMIT_LDS_BLOCK) s4[q] = k4[q];
        for (int q = 4 * n4 + (int)threadIdx.x; q < n; q += (int)EMIT_LDS_BLOCK) sk[q] = keys[q];
        __syncthreads();
        if (i < n - 1) karras_node(i, n, sk, lch, rch, first, last, parent_leaf, parent_int);
    } else if (i < n - 1) {
        karras_node(i, n, keys, lch, rch, first, last, parent_leaf, parent_int);
    }
}

__device__ __forceinline__ void child_box(uint32_t c, const uint32_t* __restrict__ perm, const float* __restrict__ aabb,
                                          const MeshDesc* __restrict__ meshes, uint32_t nm, const int32_t* ibox,
                                          float* lo, float* hi) {
    if ((c & LEAF_BIT) && !aabb) {  // mesh-direct builds keep no aabb[]: the leaf's box from its mesh
        vec3f p0, p1, p2;
        tri_from_mesh(meshes, nm, perm[c & ~LEAF_BIT], p0, p1, p2);
        int32_t o[6];
        tri_box_ord(p0, p1, p2, o);
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            lo[a] = unord(o[a]);
            hi[a] = unord(o[3 + a]);
        }
    } else if (c & LEAF_BIT) {
        const float* p = aabb + 6 * (size_t)perm[c & ~LEAF_BIT];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            lo[a] = p[a];
            hi[a] = p[3 + a];
        }
    } else {
        const int32_t* p = ibox + 6 * (size_t)c;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            lo[a] = unord(p[a]);
            hi[a] = unord(p[3 + a]);
        }
    }
}

// Refit without any inter-workgroup hand-off inside a launch. A node's box is the union of the
// leaf boxes of its sorted range [first, last] (union = ordered-int min/max: exact and
// order-independent, so equal to the oracle's recursive refit bit for bit).
// k_tree_chunk: one workgroup per chunk of 512 sorted leaves. (1) In-chunk prefix and suffix unions
// of the leaf boxes (wave scans) -> pre[], suf[]. (2) Each thread climbs from its leaf through the
// nodes whose range lies inside the chunk (their indices do too: a Karras node's index is an end of
// its range), arrival counters and boxes in LDS, workgroup-scope acq_rel atomics -> ibox[].
// k_chunk_table: sparse table of whole-chunk unions (one workgroup).
// A node spanning chunks [cf, cl] then has box = suf[first] U table(cf+1..cl-1) U pre[last]:
// k_pack4_span / k_pack evaluate that directly; no chain of dependent steps remains.
// (A one-pass refit with agent-scope release/acquire per level cost ~0.26 ms at 70k triangles,
// a second single-workgroup climb over the spanning nodes ~50 us.)
// Boxes between the leaves and the node records (in-chunk node boxes, prefix/suffix unions, the
// chunk table) live as ordered-int images (ord): a union is then one v_min_i32/v_max_i32 per
// coordinate instead of two order conversions, a compare and a select, and unord at the record
// writer restores the floats bit for bit.
__device__ __forceinline__ void box_union(int32_t* r, const int32_t* a) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        r[c] = min(r[c], a[c]);
        r[3 + c] = max(r[3 + c], a[3 + c]);
    }
}
__device__ __forceinline__ void box_identity(int32_t* r) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        r[c] = INT_MAX;
        r[3 + c] = INT_MIN;
    }
}

// ---- radix tree + chunk refit in one pass ---------------------------------------------------
// Karras's tree is the binary radix tree of the sorted keys (position tiebreak), so it can also be
// grown bottom-up (Apetrei 2014): a node [l, r] is the LEFT child of its parent iff
// delta(r, r+1) > delta(l-1, l) (ties are impossible for distinct augmented keys), its parent's
// split is then r (else l-1), and its Karras index is the end of its range facing the split (a
// left child's index is its split side r, a right child's its l). k_tree_chunk grows every node
// whose range lies in one 512-leaf chunk that way with the chunk's keys and deltas in LDS (two
// arrivals per split, workgroup-scope atomics), computing its box on the way; the nodes whose range
// crosses a chunk edge ("spanning" nodes, about ten per chunk edge: 22k at 1.1M triangles) are
// found by Karras's searches, run 64-ary by one wave each (a dozen dependent loads where the binary
// searches of a per-node Karras kernel took up to ~60). The result is karras_node's tree, bit for bit.
constexpr unsigned long long SLOT_EMPTY = ~0ull, SLOT_DONE = ~0ull - 1;  // k_tree_chunk split words

__device__ __forceinline__ int kdelta_aug(uint32_t a, uint32_t b, uint32_t i, uint32_t j) {
    return a == b ? 32 + __clz(i ^ j) : __clz(a ^ b);
}

// Largest m in [lo, hi) with pred(m), for pred monotone (true, then false) and pred(lo) true;
// one round of 64 probes per 64-fold shrink. Wave-uniform arguments, every lane active.
template <class Pred>
__device__ __forceinline__ uint32_t wave_last_true(uint32_t lo, uint32_t hi, Pred pred) {
    const uint32_t lane = threadIdx.x & 63;
    while (hi - lo > 1) {
        const uint32_t step = (hi - lo + 63) >> 6;
        const uint32_t m = lo + step * (lane + 1);
        const unsigned long long mask = ballot(m < hi && pred(m));
        if (mask) lo += step * (uint32_t)(64 - __clzll(mask));
        hi = min(hi, lo + step);
    }
    return lo;
}

// Karras node i (wave-cooperative): children and range, as karras_node writes them (parent links are
// not kept: nothing downstream reads them).
__device__ void karras_node_wave(uint32_t n, uint32_t i, const uint32_t* __restrict__ keys, uint32_t* __restrict__ lch,
                                 uint32_t* __restrict__ rch, uint32_t* __restrict__ first,
                                 uint32_t* __restrict__ last) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t ki = keys[i];
    auto delta = [&](long long j) -> int {
        if (j < 0 || j >= (long long)n) return -1;
        return kdelta_aug(ki, keys[(uint32_t)j], i, (uint32_t)j);
    };
    const int d = (delta((long long)i + 1) - delta((long long)i - 1)) >= 0 ? 1 : -1;
    const int dmin = delta((long long)i - d);
    // the other end: largest l with delta(i, i + l d) > dmin (l >= 1); exponential bracket, 64-ary refine
    const unsigned long long em = ballot(lane < 31 && delta((long long)i + (long long)d * (1ll << lane)) > dmin);
    const uint32_t a = 63 - __clzll(em);
    const uint32_t l = wave_last_true(1u << a, a >= 31 ? 0xFFFFFFFFu : (2u << a), [&](uint32_t m) {
        return delta((long long)i + (long long)d * m) > dmin;
    });
    const uint32_t j = (uint32_t)((long long)i + (long long)d * l);
    const int dnode = delta(j);
    const uint32_t sp = wave_last_true(0u, l, [&](uint32_t m) { return delta((long long)i + (long long)d * m) > dnode; });
    const uint32_t gamma = (uint32_t)((long long)i + (long long)d * sp + (d < 0 ? -1 : 0));
    if (lane != 0) return;
    const uint32_t lo = min(i, j), hi = max(i, j);
    *(lch + i) = lo == gamma ? (gamma | LEAF_BIT) : gamma;
    *(rch + i) = hi == gamma + 1 ? ((gamma + 1) | LEAF_BIT) : gamma + 1;
    *(first + i) = lo;
    *(last + i) = hi;
}

// Spanning nodes (Karras indices whose range crosses a chunk edge), one lane per index: the test is
// O(1) (delta(i, x) does not grow with the distance of x from i, so the range reaches past the chunk
// edge iff the key beyond it still shares more than dmin bits). About ten per chunk edge, clustered
// around it: a 1024-index workgroup lists its spanning indices in LDS and deals them to its 16 waves,
// which run the searches 64-ary. Each wave also stores its 64-bit ballot into span_bits (its own
// words: no atomics) for k_pack4_span; block 0 folds the scene bounds for the later kernels.
constexpr int SPAN_BLOCK = 1024;
template <int SB>
__device__ __forceinline__ void span_body(uint32_t blk, uint32_t n, const uint32_t* __restrict__ keys,
                                          uint32_t* __restrict__ lch, uint32_t* __restrict__ rch,
                                          uint32_t* __restrict__ first, uint32_t* __restrict__ last,
                                          uint32_t* __restrict__ meta, uint32_t* __restrict__ span_bits) {
    static_assert(SB % 64 == 0 && SB <= 1024, "span block: whole waves");
    __shared__ uint32_t s_list[SB];
    __shared__ uint32_t s_cnt;
    if (threadIdx.x == 0) s_cnt = 0;
    if (blk == 0 && threadIdx.x < BOUNDS_SLOTS) *(meta + threadIdx.x) = fold_slot(meta, threadIdx.x);
    const uint32_t i = blk * SB + threadIdx.x;
    const uint32_t wb = i & ~63u;  // a wave's 64 indices lie in one chunk
    const uint32_t c0 = wb & ~(REFIT_CHUNK - 1), c1 = c0 + REFIT_CHUNK - 1;
    bool sp = false;
    if (i + 1 < n) {
        const uint32_t ki = keys[i], kr = keys[i + 1];
        const int dr = kdelta_aug(ki, kr, i, i + 1);
        const int dl = i > 0 ? kdelta_aug(ki, keys[i - 1], i, i - 1) : -1;
        if (dr - dl >= 0) sp = c1 + 1 < n && kdelta_aug(ki, keys[c1 + 1], i, c1 + 1) > dl;
        else sp = c0 > 0 && kdelta_aug(ki, keys[c0 - 1], i, c0 - 1) > dr;
    }
    const unsigned long long m = ballot(sp);
    const uint32_t lane = threadIdx.x & 63;
    if (lane < 2) *(span_bits + (wb >> 5) + lane) = (uint32_t)(m >> (32 * lane));
    __syncthreads();  // s_cnt zeroed
    if (sp) s_list[atomicAdd(&s_cnt, 1u)] = i;
    __syncthreads();
    const uint32_t cnt = s_cnt;
    for (uint32_t x = threadIdx.x >> 6; x < cnt; x += SB / 64)
        karras_node_wave(n, s_list[x], keys, lch, rch, first, last);
}

__global__ __launch_bounds__(SPAN_BLOCK) void k_span(uint32_t n, const uint32_t* __restrict__ keys,
                                                     uint32_t* __restrict__ lch, uint32_t* __restrict__ rch,
                                                     uint32_t* __restrict__ first, uint32_t* __restrict__ last,
                                                     uint32_t* __restrict__ meta, uint32_t* __restrict__ span_bits) {
    BDIAG(5);
    span_body<SPAN_BLOCK>(blockIdx.x, n, keys, lch, rch, first, last, meta, span_bits);
}

__host__ __device__ __forceinline__ uint32_t floor_log2(uint32_t x) { return 31u - (uint32_t)__builtin_clz(x); }

// Sparse table of whole-chunk unions: level j, entry i = union of chunks [i, i + 2^j).
// Level 0 is the last prefix of each chunk. One workgroup; levels separated by barriers.
__global__ __launch_bounds__(1024) void k_chunk_table(uint32_t n, const int32_t* __restrict__ pre,
                                                      int32_t* __restrict__ table, uint32_t* __restrict__ bounds) {
    clear_replicas(bounds, threadIdx.x, 1024);  // the chunk kernel was their last reader
    const uint32_t nc = (n + REFIT_CHUNK - 1) >> REFIT_CHUNK_LOG2;
    for (uint32_t i = threadIdx.x; i < nc; i += blockDim.x) {
        const uint32_t end = min(n, (i + 1) << REFIT_CHUNK_LOG2) - 1;
#pragma unroll
        for (int a = 0; a < 6; ++a) table[6 * (size_t)i + a] = pre[6 * (size_t)end + a];
    }
    for (uint32_t j = 1; (1u << j) <= nc; ++j) {
        __syncthreads();  // level j-1 complete (same workgroup: workgroup-scope visibility)
        const int32_t* src = table + 6 * (size_t)(j - 1) * nc;
        int32_t* dst = table + 6 * (size_t)j * nc;
        const uint32_t half = 1u << (j - 1);
        for (uint32_t i = threadIdx.x; i + (1u << j) <= nc; i += blockDim.x) {
            int32_t r[6];
#pragma unroll
            for (int a = 0; a < 6; ++a) r[a] = src[6 * (size_t)i + a];
            box_union(r, src + 6 * (size_t)(i + half));
#pragma unroll
            for (int a = 0; a < 6; ++a) dst[6 * (size_t)i + a] = r[a];
        }
    }
}

// The same table with the levels built in LDS (ping-pong) and only written to global memory: one
// workgroup still, but each level costs an LDS round trip instead of a global one. For up to
// CT_LDS_CHUNKS chunks (1.5M triangles with 512-leaf chunks).
constexpr uint32_t CT_LDS_CHUNKS = 3072;
// Every workgroup of the grid builds the whole table in LDS (a few thousand unions per level) but
// stores only its contiguous slice of each level: one workgroup storing all of it was bound by one
// CU's store rate (0.6 MB for 2,184 chunks).
__global__ __launch_bounds__(1024) void k_chunk_table_lds(uint32_t n, const int32_t* __restrict__ pre,
                                                          int32_t* __restrict__ table, uint32_t* __restrict__ bounds) {
    if (blockIdx.x == 0) clear_replicas(bounds, threadIdx.x, 1024);  // the chunk kernel was their last reader
    BDIAG(7);
    __shared__ int32_t lv[2][CT_LDS_CHUNKS * 6];
    const uint32_t nc = (n + REFIT_CHUNK - 1) >> REFIT_CHUNK_LOG2;
    const uint32_t per = (nc + gridDim.x - 1) / gridDim.x;
    const uint32_t s0 = blockIdx.x * per, s1 = min(nc, s0 + per);  // this workgroup's slice
    for (uint32_t i = threadIdx.x; i < nc; i += blockDim.x) {
        const uint32_t end = min(n, (i + 1) << REFIT_CHUNK_LOG2) - 1;
        const bool mine = i >= s0 && i < s1;
#pragma unroll
        for (int a = 0; a < 6; ++a) {
            const int32_t v = pre[6 * (size_t)end + a];
            lv[0][6 * i + a] = v;
            if (mine) table[6 * (size_t)i + a] = v;
        }
    }
    // two levels per barrier: level j from pairs of level j-1 (global only), level j+1 from quads of
    // level j-1 (global and the other LDS buffer, the next pass's source)
    int cur = 0;
    for (uint32_t j = 1; (1u << j) <= nc; j += 2) {
        __syncthreads();
        const int32_t* src = lv[cur];
        int32_t* dst = lv[cur ^ 1];
        int32_t* g1 = table + 6 * (size_t)j * nc;
        int32_t* g2 = table + 6 * (size_t)(j + 1) * nc;
        const uint32_t h = 1u << (j - 1);
        const bool two = (1u << (j + 1)) <= nc;
        for (uint32_t i = threadIdx.x; i + 2 * h <= nc; i += blockDim.x) {
            const bool mine = i >= s0 && i < s1;
            int32_t r[6];
#pragma unroll
            for (int a = 0; a < 6; ++a) r[a] = src[6 * i + a];
            box_union(r, src + 6 * (i + h));
            if (mine)
#pragma unroll
                for (int a = 0; a < 6; ++a) g1[6 * (size_t)i + a] = r[a];
            if (two && i + 4 * h <= nc) {
                box_union(r, src + 6 * (i + 2 * h));
                box_union(r, src + 6 * (i + 3 * h));
#pragma unroll
                for (int a = 0; a < 6; ++a) {
                    dst[6 * i + a] = r[a];
                    if (mine) g2[6 * (size_t)i + a] = r[a];
                }
            }
        }
        cur ^= 1;
    }
}

// Box of an internal node from the refit products (see k_tree_chunk).
__device__ __forceinline__ void node_box(uint32_t c, const uint32_t* __restrict__ first,
                                         const uint32_t* __restrict__ last, const int32_t* __restrict__ ibox,
                                         const int32_t* __restrict__ pre, const int32_t* __restrict__ suf,
                                         const int32_t* __restrict__ table, uint32_t nc, int32_t* r);

// Same, with the node's sorted range [f, l] already loaded.
__device__ __forceinline__ void node_box_fl(uint32_t c, uint32_t f, uint32_t l, const int32_t* __restrict__ ibox,
                                            const int32_t* __restrict__ pre, const int32_t* __restrict__ suf,
                                            const int32_t* __restrict__ table, uint32_t nc, int32_t* r) {
    const uint32_t cf = f >> REFIT_CHUNK_LOG2, cl = l >> REFIT_CHUNK_LOG2;
    if (cf == cl) {
#pragma unroll
        for (int a = 0; a < 6; ++a) r[a] = ibox[6 * (size_t)c + a];
        return;
    }
#pragma unroll
    for (int a = 0; a < 6; ++a) r[a] = suf[6 * (size_t)f + a];
    box_union(r, pre + 6 * (size_t)l);
    if (cl - cf >= 2) {
        const uint32_t a0 = cf + 1, b0 = cl - 1, j = floor_log2(b0 - a0 + 1);
        const int32_t* lvl = table + 6 * (size_t)j * nc;
        box_union(r, lvl + 6 * (size_t)a0);
        box_union(r, lvl + 6 * (size_t)(b0 + 1 - (1u << j)));
    }
}

__device__ __forceinline__ void node_box(uint32_t c, const uint32_t* __restrict__ first,
                                         const uint32_t* __restrict__ last, const int32_t* __restrict__ ibox,
                                         const int32_t* __restrict__ pre, const int32_t* __restrict__ suf,
                                         const int32_t* __restrict__ table, uint32_t nc, int32_t* r) {
    node_box_fl(c, first[c], last[c], ibox, pre, suf, table, nc, r);
}

__device__ __forceinline__ void pad_box(float* lo, float* hi, float pad) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        lo[c] = lo[c] - (fabsf(lo[c]) * PAD_SCALE + pad);
        hi[c] = hi[c] + (fabsf(hi[c]) * PAD_SCALE + pad);
    }
}

__device__ __forceinline__ float scene_pad(const uint32_t* __restrict__ bounds) {
    const float ex = bounds_hi(bounds[3]) - bounds_lo(bounds[0]);
    const float ey = bounds_hi(bounds[4]) - bounds_lo(bounds[1]);
    const float ez = bounds_hi(bounds[5]) - bounds_lo(bounds[2]);
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
                                                const float* __restrict__ aabb, const MeshDesc* __restrict__ meshes,
                                                uint32_t nm, const int32_t* __restrict__ ibox,
                                                const int32_t* __restrict__ pre, const int32_t* __restrict__ suf,
                                                const int32_t* __restrict__ table, const uint32_t* __restrict__ bounds,
                                                uint32_t* __restrict__ records) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n - 1) return;
    const uint32_t nc = (n + REFIT_CHUNK - 1) >> REFIT_CHUNK_LOG2;
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
            lo[a] = unord(ibox[a]);
            hi[a] = unord(ibox[3 + a]);
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
        uint32_t cf, cn;
        if (c & LEAF_BIT) {
            child_box(c, perm, aabb, meshes, nm, ibox, lo, hi);
            cf = cc;
            cn = 1;
        } else {
            int32_t b[6];
            node_box(cc, first, last, ibox, pre, suf, table, nc, b);
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                lo[a] = unord(b[a]);
                hi[a] = unord(b[3 + a]);
            }
            cf = first[cc];
            cn = last[cc] - first[cc] + 1;
        }
        pad_box(lo, hi, pad);
        set_child(r, q, lo, hi, cn <= K ? (LEAF_BIT | ((cn - 1) << 27) | cf) : cc);
    }
    store_record(records + 16 * (size_t)i, r);
}

// ---- BVH4 records (128 B): every other level of the binary tree collapsed ---------------------
//   [0..3] lo.x of children 0..3  [4..7] lo.y  [8..11] lo.z  [12..15] hi.x  [16..19] hi.y
//   [20..23] hi.z  [24..27] child refs  [28..31] 0.  Empty slot: NaN box, EMPTY_REF.
// A record is written for the root and for every non-collapsed internal node at even depth; its
// children are its binary children with each non-collapsed internal child replaced by that child's
// two children (oracle/beam_oracle.c orc_bvh_build_ex, width 4). Other slots are left unwritten.
__device__ __forceinline__ void set_child4(uint32_t (&r)[32], int slot, const float* lo, const float* hi,
                                           uint32_t ref) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        r[4 * c + slot] = f2u(lo[c]);
        r[12 + 4 * c + slot] = f2u(hi[c]);
    }
    r[24 + slot] = ref;
}

__device__ __forceinline__ void set_empty4(uint32_t (&r)[32], int slot) {
#pragma unroll
    for (int c = 0; c < 6; ++c) r[4 * c + slot] = NAN_BITS;
    r[24 + slot] = EMPTY_REF;
}

__device__ __forceinline__ void store_record4(uint32_t* rec, const uint32_t (&r)[32]) {
    uint4* q = reinterpret_cast<uint4*>(rec);
#pragma unroll
    for (int k = 0; k < 8; ++k) q[k] = make_uint4(r[4 * k], r[4 * k + 1], r[4 * k + 2], r[4 * k + 3]);
}

// LDS of one chunk workgroup (kept under 40 KiB, four workgroups per CU: deltas as bytes, node ranges as
// chunk offsets, the keys over the node boxes, which are written only after the deltas are taken).
struct ChunkLds {
    uint32_t bnd[6];                // scene box slots 0..5 (the records' padding)
    int8_t dl[REFIT_CHUNK + 1];     // delta(j, j+1) for j = c0-1 .. c1, at j - c0 + 1 (-1 .. 64)
    int32_t leaf[REFIT_CHUNK][6];
    int32_t wtot[REFIT_CHUNK / 64][6];
    // arrivals at split gamma (at gamma - c0): the first arrival's (ref, far end of its range | side << 31)
    // exchanged in as one 64-bit word; the second arrival takes it out in the same exchange and leaves
    // SLOT_DONE, so a word still holding an arrival after the growth marks a split reached once
    unsigned long long slot[REFIT_CHUNK];
    // chunk-local internal node c0 + x: children, range, box, parent (written out coalesced at the end,
    // so the growth loop's release atomics wait on LDS traffic only; the parent only decides which)
    uint32_t ncl[REFIT_CHUNK], ncr[REFIT_CHUNK];  // children refs
    uint32_t nlr[REFIT_CHUNK];      // range: (first - c0) | (last - c0) << 16; NO_NODE: not chunk-local
    int32_t nbox[REFIT_CHUNK][6];
    // bits 0-9: chunk offset + 1 of the node's chunk-local parent (0: none); bit 16: leaf x starts a
    // maximal chunk-local subtree, bit 17: ends one
    uint32_t pe[REFIT_CHUNK];
};

// One 512-leaf chunk per workgroup: the chunk-local nodes, their boxes, the sorted triangle records.
// The scene box (for the records' padding) is folded from the gather's replicas here, so the chunk
// workgroups do not wait for k_span's fold (they may run beside k_span: k_span_chunk).
template <class Diag>
__device__ __forceinline__ void chunk_body(const Diag& diag, ChunkLds& L, uint32_t blk, uint32_t n,
                                           const uint32_t* __restrict__ keys,
                                           const uint32_t* __restrict__ perm, const float* __restrict__ aabb,
                                           const MeshDesc* __restrict__ meshes, uint32_t nm,
                                           const float4* __restrict__ tsrc, float4* __restrict__ tdst,
                                           uint32_t* __restrict__ lch, uint32_t* __restrict__ rch,
                                           uint32_t* __restrict__ first, uint32_t* __restrict__ last,
                                           int32_t* __restrict__ ibox, int32_t* __restrict__ pre,
                                           int32_t* __restrict__ suf, uint32_t* __restrict__ bounds, uint32_t K,
                                           uint32_t* __restrict__ records) {
    uint32_t* const s_bnd = L.bnd;
    if (threadIdx.x < 64) {  // wave 0
        const uint32_t v = fold6_wave(bounds, 0);
        if (threadIdx.x < 6) s_bnd[threadIdx.x] = v;
    }
    if (n <= REFIT_CHUNK && threadIdx.x < BOUNDS_SLOTS)  // one chunk: no k_span folds for the later kernels
        bounds[threadIdx.x] = fold_slot(bounds, threadIdx.x);
    int8_t* const s_dl = L.dl;
    int32_t (*const s_leaf)[6] = L.leaf;
    int32_t (*const s_wtot)[6] = L.wtot;
    unsigned long long* const s_slot = L.slot;
    uint32_t* const s_ncl = L.ncl;
    uint32_t* const s_ncr = L.ncr;
    uint32_t* const s_nlr = L.nlr;
    int32_t (*const s_nbox)[6] = L.nbox;
    uint32_t* s_key = reinterpret_cast<uint32_t*>(&s_nbox[0][0]);  // keys c0-1 .. c1+1, until the deltas
    uint32_t* const s_pe = L.pe;
    constexpr uint32_t NO_NODE = 0xFFFFFFFFu, PE_START = 1u << 16, PE_END = 1u << 17, PE_PARENT = 0x3FFu;
    const uint32_t tid = threadIdx.x, c0 = blk * REFIT_CHUNK, c1 = c0 + REFIT_CHUNK - 1;
    const uint32_t k = c0 + tid;
    const int w = tid >> 6, lane = tid & 63;
    s_slot[tid] = SLOT_EMPTY;
    s_pe[tid] = 0;
    s_nlr[tid] = NO_NODE;
    // every load issued before any is waited on: own key, the chunk's outer neighbour keys (clamped;
    // lanes 0 and 1 keep theirs), the permutation, then the box and the record it points at
    const uint32_t kc = min(k, n - 1);
    const long long jn = tid == 0 ? (long long)c0 - 1 : (long long)c1 + 1;
    const uint32_t key_own = keys[kc];
    const uint32_t key_nb = keys[(uint32_t)min(max(jn, 0ll), (long long)n - 1)];
    const uint32_t g = perm[kc];
    int32_t leaf[6];
    float4 t0, t1, t2;
    if (!tsrc) {
        // mesh-direct (the default): the sorted triangle's box and (v0, e1, e2) record straight from
        // the mesh, with k_gather's operations (tri_from_mesh): the same bits as the gathered copies,
        // without the original-order records' write and their permuted 48 + 24-B re-reads
        vec3f p0, p1, p2;
        tri_from_mesh(meshes, nm, g, p0, p1, p2);
        tri_box_ord(p0, p1, p2, leaf);
        tri_record(p0, p1, p2, g, t0, t1, t2);
    } else {
        const float2* bp = reinterpret_cast<const float2*>(aabb + 6 * (size_t)g);
        const float2 b0 = bp[0], b1 = bp[1], b2 = bp[2];
        t0 = tsrc[3 * (size_t)g + 0];
        t1 = tsrc[3 * (size_t)g + 1];
        t2 = tsrc[3 * (size_t)g + 2];
        leaf[0] = ord(b0.x);
        leaf[1] = ord(b0.y);
        leaf[2] = ord(b1.x);
        leaf[3] = ord(b1.y);
        leaf[4] = ord(b2.x);
        leaf[5] = ord(b2.y);
    }
    s_key[tid + 1] = key_own;
    if (tid < 2) s_key[tid == 0 ? 0 : REFIT_CHUNK + 1] = (jn >= 0 && jn < (long long)n) ? key_nb : 0u;
    if (k < n) {
        // triangle records into leaf (sorted) order
        tdst[3 * (size_t)k + 0] = t0;
        tdst[3 * (size_t)k + 1] = t1;
        tdst[3 * (size_t)k + 2] = t2;
    } else {
        box_identity(leaf);
    }
    __syncthreads();
    diag.mark(0);
    // adjacent deltas: entry x = delta(c0 - 1 + x, c0 + x), x in [0, 512]
    for (uint32_t x = tid; x <= REFIT_CHUNK; x += REFIT_CHUNK) {
        const long long j = (long long)c0 - 1 + x;
        s_dl[x] = (int8_t)((j < 0 || j + 1 >= (long long)n) ? -1 : kdelta_aug(s_key[x], s_key[x + 1], (uint32_t)j, (uint32_t)j + 1));
    }
    // inclusive prefix and suffix unions over the chunk
    int32_t pf[6], sf[6];
#pragma unroll
    for (int a = 0; a < 6; ++a) {
        pf[a] = leaf[a];
        sf[a] = leaf[a];
        s_leaf[tid][a] = leaf[a];
    }
#if BM_CHUNK_DPP
    // within each row of 16 lanes by DPP row shifts (lanes shifted in from outside the row keep the
    // identity), across the four rows by the rows' totals (readlane) — no LDS-crossbar round trips,
    // where the shuffle form took six dependent steps of twelve
    {
        const int row = (int)(lane >> 4);
#pragma unroll
        for (int a = 0; a < 6; ++a) {
            const int32_t id = a < 3 ? INT_MAX : INT_MIN;
            auto op = [&](int32_t x, int32_t y) { return a < 3 ? min(x, y) : max(x, y); };
            int32_t v = pf[a], u = sf[a];
            v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x111, 0xf, 0xf, false));  // row_shr:1
            v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x112, 0xf, 0xf, false));  // row_shr:2
            v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x114, 0xf, 0xf, false));  // row_shr:4
            v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x118, 0xf, 0xf, false));  // row_shr:8
            u = op(u, __builtin_amdgcn_update_dpp(id, u, 0x101, 0xf, 0xf, false));  // row_shl:1
            u = op(u, __builtin_amdgcn_update_dpp(id, u, 0x102, 0xf, 0xf, false));  // row_shl:2
            u = op(u, __builtin_amdgcn_update_dpp(id, u, 0x104, 0xf, 0xf, false));  // row_shl:4
            u = op(u, __builtin_amdgcn_update_dpp(id, u, 0x108, 0xf, 0xf, false));  // row_shl:8
            const int32_t t0 = __builtin_amdgcn_readlane(v, 15), t1 = __builtin_amdgcn_readlane(v, 31);
            const int32_t t2 = __builtin_amdgcn_readlane(v, 47), t3 = __builtin_amdgcn_readlane(v, 63);
            const int32_t p01 = op(t0, t1), s23 = op(t2, t3);
            const int32_t pre = row == 0 ? id : row == 1 ? t0 : row == 2 ? p01 : op(p01, t2);
            const int32_t suf = row == 3 ? id : row == 2 ? t3 : row == 1 ? s23 : op(t1, s23);
            pf[a] = op(v, pre);
            sf[a] = op(u, suf);
        }
    }
#else
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        int32_t up[6], dn[6];
#pragma unroll
        for (int a = 0; a < 6; ++a) {
            up[a] = __shfl_up(pf[a], off);
            dn[a] = __shfl_down(sf[a], off);
        }
        if (lane >= off) box_union(pf, up);
        if (lane + off < 64) box_union(sf, dn);
    }
#endif
    if (lane == 63) {
#pragma unroll
        for (int a = 0; a < 6; ++a) s_wtot[w][a] = pf[a];
    }
    __syncthreads();
    diag.mark(1);
    for (int q = 0; q < REFIT_CHUNK / 64; ++q) {
        if (q < w) box_union(pf, s_wtot[q]);
        if (q > w) box_union(sf, s_wtot[q]);
    }
    if (k < n) {
        // bottom-up growth from leaf k. Per level: one 64-bit exchange at the split (release: this
        // node's box is in LDS before its sibling can read it; acquire: the sibling's is), then the
        // sibling's box and the one new adjacent delta read together.
        uint32_t l = k, r = k, ref = LEAF_BIT | k, cl = 0, cr = 0;
        int32_t box[6];
#pragma unroll
        for (int a = 0; a < 6; ++a) box[a] = leaf[a];
        bool internal = false;
        int dl_r = s_dl[r - c0 + 1], dl_l = s_dl[l - c0];  // delta(r, r+1), delta(l-1, l)
        for (;;) {
            const bool root = l == 0 && r == n - 1;
            const bool right = !root && dl_r > dl_l;  // parent to the right: left child
            if (internal) {
                const uint32_t idx = root ? 0u : (right ? r : l);
                s_ncl[idx - c0] = cl;
                s_ncr[idx - c0] = cr;
                s_nlr[idx - c0] = (l - c0) | ((r - c0) << 16);
#pragma unroll
                for (int a = 0; a < 6; ++a) s_nbox[idx - c0][a] = box[a];
                if (!(cl & LEAF_BIT)) atomicOr(&s_pe[cl - c0], idx - c0 + 1);
                if (!(cr & LEAF_BIT)) atomicOr(&s_pe[cr - c0], idx - c0 + 1);
                ref = idx;
            }
            if (root || (right ? r >= c1 : l <= c0)) {  // the parent's range leaves the chunk: maximal
                atomicOr(&s_pe[l - c0], PE_START);
                atomicOr(&s_pe[r - c0], PE_END);
                break;
            }
            const uint32_t gi = (right ? r : l - 1) - c0;
            const unsigned long long mine =
                ((unsigned long long)((right ? l : r) | (right ? 0u : 0x80000000u)) << 32) | ref;
            const unsigned long long prev =
                __hip_atomic_exchange(&s_slot[gi], mine, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (prev == SLOT_EMPTY) break;  // first arrival: the sibling continues
            s_slot[gi] = SLOT_DONE;
            const uint32_t sref = (uint32_t)prev, send = (uint32_t)(prev >> 32) & 0x7FFFFFFFu;
            const int32_t* sb = (sref & LEAF_BIT) ? s_leaf[(sref & ~LEAF_BIT) - c0] : s_nbox[sref - c0];
            if (right) {
                cl = ref;
                cr = sref;
                r = send;
                dl_r = s_dl[r - c0 + 1];
            } else {
                cl = sref;
                cr = ref;
                l = send;
                dl_l = s_dl[l - c0];
            }
            box_union(box, sb);
            internal = true;
        }
    }
    __syncthreads();
    diag.mark(2);
    {  // chunk-local nodes out, coalesced (the spanning ones were written by k_span). With BVH4 records
       // written here, k_pack4_span reads only the top two levels of each maximal subtree (children
       // and grandchildren of spanning nodes); BVH2's k_pack reads every node.
        const uint32_t lr = s_nlr[tid];
        if (lr != NO_NODE) {
            const uint32_t pp = s_pe[tid] & PE_PARENT;
            if (!records || pp == 0 || (s_pe[pp - 1] & PE_PARENT) == 0) {
                *(lch + k) = s_ncl[tid];
                *(rch + k) = s_ncr[tid];
                *(first + k) = c0 + (lr & 0xFFFFu);
                *(last + k) = c0 + (lr >> 16);
#pragma unroll
                for (int a = 0; a < 6; ++a) *(ibox + 6 * (size_t)k + a) = s_nbox[tid][a];
            }
        }
    }
    // a split reached by one child only: its parent spans chunks, so that child is maximal too
    const unsigned long long once = s_slot[tid];
    if (once != SLOT_EMPTY && once != SLOT_DONE) {
        const uint32_t sd = (uint32_t)(once >> 63), far = (uint32_t)(once >> 32) & 0x7FFFFFFFu;
        atomicOr(&s_pe[sd == 0 ? far - c0 : tid + 1], PE_START);
        atomicOr(&s_pe[sd == 0 ? tid : far - c0], PE_END);
    }
    __syncthreads();
    diag.mark(3);
    // a spanning node's box is suf[its first leaf] U whole chunks U pre[its last leaf], and those leaves
    // are ends of maximal chunk-local subtrees: only there are the prefix/suffix unions needed
    if (k < n) {
        const uint32_t e = (s_pe[tid] >> 16) & 3u;
        if (e & 1u) {
#pragma unroll
            for (int a = 0; a < 6; ++a) *(suf + 6 * (size_t)k + a) = sf[a];
        }
        if (e & 2u) {
#pragma unroll
            for (int a = 0; a < 6; ++a) *(pre + 6 * (size_t)k + a) = pf[a];
        }
    }
    if (n <= REFIT_CHUNK) clear_replicas(bounds, tid, REFIT_CHUNK);  // one chunk: their last reader was above
    if (!records) return;  // BVH2: k_pack writes every record
    // BVH4 record of every chunk-local node above the leaf size (the spanning ones: k_pack4_span).
    // A traversal reaches only the records of nodes at even depth (the others are expanded into
    // their parents' records), but a node's record does not depend on its depth, so writing all of
    // them needs no depth (which only a top-down pass over the spanning nodes could supply) and
    // leaves every reachable record as the oracle's.
    const uint32_t lr = s_nlr[tid];
    if (lr == NO_NODE) return;
    const uint32_t cnt = (lr >> 16) - (lr & 0xFFFFu) + 1;
    if (cnt <= K && k != 0) return;  // inside a leaf
    const float pad = scene_pad(s_bnd);
    // slots in record order: child 0 (or its two children if expanded), then child 1 (or its two)
    uint32_t sl[4] = {EMPTY_REF, EMPTY_REF, EMPTY_REF, EMPTY_REF};
    if (cnt <= K) {  // the whole scene is one leaf: the root's own box
        sl[0] = k;
    } else {
        bool ex[2];
        uint32_t cc[2][2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const uint32_t c = q ? s_ncr[tid] : s_ncl[tid];
            const uint32_t clr = (c & LEAF_BIT) ? 0u : s_nlr[c - c0];
            ex[q] = !(c & LEAF_BIT) && (clr >> 16) - (clr & 0xFFFFu) + 1 > K;
            cc[q][0] = ex[q] ? s_ncl[c - c0] : c;
            cc[q][1] = ex[q] ? s_ncr[c - c0] : EMPTY_REF;
        }
        sl[0] = cc[0][0];
        sl[1] = ex[0] ? cc[0][1] : cc[1][0];
        sl[2] = ex[0] ? cc[1][0] : cc[1][1];
        sl[3] = ex[0] ? cc[1][1] : EMPTY_REF;
    }
    uint32_t rr[32];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t c = sl[q];
        if (c == EMPTY_REF) {
            set_empty4(rr, q);
            continue;
        }
        const int32_t* ob = (c & LEAF_BIT) ? s_leaf[(c & ~LEAF_BIT) - c0] : s_nbox[c - c0];
        float b[6];
#pragma unroll
        for (int a = 0; a < 6; ++a) b[a] = unord(ob[a]);
        uint32_t ref = c;
        if (!(c & LEAF_BIT)) {
            const uint32_t clr = s_nlr[c - c0];
            const uint32_t gn = (clr >> 16) - (clr & 0xFFFFu) + 1;
            if (gn <= K) ref = LEAF_BIT | ((gn - 1) << 27) | (c0 + (clr & 0xFFFFu));
        }
        pad_box(b, b + 3, pad);
        set_child4(rr, q, b, b + 3, ref);
    }
#pragma unroll
    for (int q = 28; q < 32; ++q) rr[q] = 0u;
    store_record4(records + 32 * (size_t)k, rr);
}

__global__ __launch_bounds__(REFIT_CHUNK) void k_tree_chunk(uint32_t n, const uint32_t* __restrict__ keys,
                                                            const uint32_t* __restrict__ perm,
                                                            const float* __restrict__ aabb,
                                                            const MeshDesc* __restrict__ meshes, uint32_t nm,
                                                            const float4* __restrict__ tsrc, float4* __restrict__ tdst,
                                                            uint32_t* __restrict__ lch, uint32_t* __restrict__ rch,
                                                            uint32_t* __restrict__ first, uint32_t* __restrict__ last,
                                                            int32_t* __restrict__ ibox,
                                                            int32_t* __restrict__ pre, int32_t* __restrict__ suf,
                                                            uint32_t* __restrict__ bounds, uint32_t K,
                                                            uint32_t* __restrict__ records) {
    BDIAG(6);
    __shared__ ChunkLds L;
    chunk_body(BDIAG_OBJ, L, blockIdx.x, n, keys, perm, aabb, meshes, nm, tsrc, tdst, lch, rch, first, last, ibox, pre,
               suf, bounds, K, records);
}

// k_span and k_tree_chunk in one launch (small scenes): workgroups [0, nchunk) grow the chunks, the
// rest find and search the spanning nodes (512 indices each). The two only read the sorted keys and
// write disjoint nodes, so they overlap instead of paying a launch boundary and k_span's span.
__global__ __launch_bounds__(REFIT_CHUNK) void k_span_chunk(uint32_t nchunk, uint32_t n, const uint32_t* __restrict__ keys,
                                                            const uint32_t* __restrict__ perm,
                                                            const float* __restrict__ aabb,
                                                            const MeshDesc* __restrict__ meshes, uint32_t nm,
                                                            const float4* __restrict__ tsrc, float4* __restrict__ tdst,
                                                            uint32_t* __restrict__ lch, uint32_t* __restrict__ rch,
                                                            uint32_t* __restrict__ first, uint32_t* __restrict__ last,
                                                            int32_t* __restrict__ ibox,
                                                            int32_t* __restrict__ pre, int32_t* __restrict__ suf,
                                                            uint32_t* __restrict__ bounds, uint32_t K,
                                                            uint32_t* __restrict__ records, uint32_t* __restrict__ span_bits) {
    __shared__ ChunkLds L;
    if (blockIdx.x < nchunk) {
        BDIAG(6);
        chunk_body(BDIAG_OBJ, L, blockIdx.x, n, keys, perm, aabb, meshes, nm, tsrc, tdst, lch, rch, first, last, ibox,
                   pre, suf, bounds, K, records);
    } else {
        BDIAG(5);
        span_body<REFIT_CHUNK>(blockIdx.x - nchunk, n, keys, lch, rch, first, last, bounds, span_bits);
    }
}

// BVH4 records of the spanning nodes (k_span's bitmap: about ten per chunk edge), four lanes per
// record, lane c building slot c. A record is latency-bound — children, their ranges and children,
// the slot nodes' ranges or triangle ids, then up to four boxes per slot (a spanning slot: suffix,
// prefix, two table entries) — so the lanes of a record run those rounds side by side instead of one
// lane running all four slots (about 3,000 instructions: 15 us per record at one wave per CU).
// One 256-thread workgroup per 1024 indices (32 bitmap words): records dealt 64 per round.
constexpr uint32_t PACK4_IDX = 1024;
// The records of window `win` (PACK4_IDX indices) by BLOCK threads, tid = 0 .. BLOCK - 1 (whole waves).
__device__ __forceinline__ void pack4_body(uint32_t win, uint32_t tid, uint32_t n, uint32_t K,
                                           const uint32_t* __restrict__ span_bits, const uint32_t* __restrict__ lch,
                                           const uint32_t* __restrict__ rch, const uint32_t* __restrict__ first,
                                           const uint32_t* __restrict__ last, const uint32_t* __restrict__ perm,
                                           const float* __restrict__ aabb, const MeshDesc* __restrict__ meshes,
                                           uint32_t nm, const int32_t* __restrict__ ibox,
                                           const int32_t* __restrict__ pre, const int32_t* __restrict__ suf,
                                           const int32_t* __restrict__ table, const uint32_t* __restrict__ bounds,
                                           uint32_t* __restrict__ records) {
    const uint32_t lane = tid & 63, c = tid & 3;
    // every wave: the workgroup's 32 bitmap words in lanes 0..31 and their inclusive popcount prefix
    const uint32_t q = win * (PACK4_IDX / 32) + lane;
    const uint32_t nw = (n - 1 + 31) >> 5;
    const uint32_t word = (lane < PACK4_IDX / 32 && q < nw) ? *(span_bits + q) : 0u;
    const uint32_t pc = __popc(word);
    const uint32_t incl = wave_incl_add(pc);  // (lanes 32..63 hold no words: their sums are the total)
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 31);
    const uint32_t nc = (n + REFIT_CHUNK - 1) >> REFIT_CHUNK_LOG2;
    const float pad = scene_pad(bounds);
    for (uint32_t r0 = 0; r0 < total; r0 += BLOCK / 4) {
        const uint32_t want = r0 + (tid >> 2);  // this lane's record: the want-th set bit
        uint32_t lo = 0;  // word holding it: the first lane whose inclusive count exceeds want
#pragma unroll
        for (uint32_t step = 16; step >= 1; step >>= 1) {
            const uint32_t v = __shfl(incl, lo + step - 1);
            if (v <= want) lo += step;
        }
        const uint32_t wq = __shfl(word, lo), before = __shfl(incl, lo) - __shfl(pc, lo);
        if (want >= total) continue;
        uint32_t bits = wq;
        for (uint32_t skip = want - before; skip; --skip) bits &= bits - 1;
        const uint32_t i = win * PACK4_IDX + 32 * lo + (uint32_t)__ffs(bits) - 1;
        // round 1-2: the node's children, then each internal child's range and children (a spanning
        // node holds more than 512 > K triangles: never a leaf, always a record)
        const uint32_t ch0 = *(lch + i), ch1 = *(rch + i);
        const uint32_t c0 = (ch0 & LEAF_BIT) ? 0u : ch0, c1 = (ch1 & LEAF_BIT) ? 0u : ch1;
        const uint32_t f0 = *(first + c0), l0 = *(last + c0), g0l = *(lch + c0), g0r = *(rch + c0);
        const uint32_t f1 = *(first + c1), l1 = *(last + c1), g1l = *(lch + c1), g1r = *(rch + c1);
        const bool ex0 = !(ch0 & LEAF_BIT) && l0 - f0 + 1 > K, ex1 = !(ch1 & LEAF_BIT) && l1 - f1 + 1 > K;
        // slots in record order: child 0 (or its two children), then child 1 (or its two)
        const uint32_t n0 = ex0 ? 2u : 1u, used = n0 + (ex1 ? 2u : 1u);
        uint32_t cand = EMPTY_REF;
        if (c < n0) cand = ex0 ? (c == 0 ? g0l : g0r) : ch0;
        else if (c < used) cand = ex1 ? (c == n0 ? g1l : g1r) : ch1;
        // round 3: a triangle slot's sorted position -> id; a node slot's range
        const bool use = cand != EMPTY_REF, leaf = use && (cand & LEAF_BIT);
        const uint32_t gc = cand & ~LEAF_BIT;
        const uint32_t pm = perm[leaf ? gc : 0u];
        const uint32_t nd = (use && !leaf) ? gc : 0u;
        const uint32_t f = *(first + nd), l = *(last + nd);
        // round 4: the slot's boxes, all issued before any is used
        const int32_t* src[4] = {nullptr, nullptr, nullptr, nullptr};
        int parts = 0;
        int32_t bx[4][6];
        const bool mesh_leaf = leaf && !aabb;  // the slot's box from its mesh (mesh-direct builds: no aabb[])
        if (mesh_leaf) {  // as float bits, straight into bx[0] (no pointer to a local array: no scratch)
            vec3f p0, p1, p2;
            tri_from_mesh(meshes, nm, pm, p0, p1, p2);
            tri_box_ord(p0, p1, p2, bx[0]);
#pragma unroll
            for (int a = 0; a < 6; ++a) bx[0][a] = f2i(unord(bx[0][a]));
            parts = 1;
        } else if (leaf) {
            src[0] = reinterpret_cast<const int32_t*>(aabb + 6 * (size_t)pm);
            parts = 1;
        } else if (use) {
            const uint32_t k0 = f >> REFIT_CHUNK_LOG2, k1 = l >> REFIT_CHUNK_LOG2;
            if (k0 == k1) {
                src[0] = ibox + 6 * (size_t)gc;
                parts = 1;
            } else {
                src[0] = suf + 6 * (size_t)f;
                src[1] = pre + 6 * (size_t)l;
                parts = 2;
                if (k1 - k0 >= 2) {
                    const uint32_t a0 = k0 + 1, b0 = k1 - 1, j = floor_log2(b0 - a0 + 1);
                    const int32_t* lvl = table + 6 * (size_t)j * nc;
                    src[2] = lvl + 6 * (size_t)a0;
                    src[3] = lvl + 6 * (size_t)(b0 + 1 - (1u << j));
                    parts = 4;
                }
            }
        }
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            if (m < parts && !(m == 0 && mesh_leaf)) {
                const int2 x0 = *reinterpret_cast<const int2*>(src[m]), x1 = *reinterpret_cast<const int2*>(src[m] + 2), x2 = *reinterpret_cast<const int2*>(src[m] + 4);
                bx[m][0] = x0.x;
                bx[m][1] = x0.y;
                bx[m][2] = x1.x;
                bx[m][3] = x1.y;
                bx[m][4] = x2.x;
                bx[m][5] = x2.y;
            }
        }
        uint32_t out[7];
        if (use) {
            int32_t ob[6];
#pragma unroll
            for (int a = 0; a < 6; ++a) ob[a] = bx[0][a];
#pragma unroll
            for (int m = 1; m < 4; ++m)
                if (m < parts) box_union(ob, bx[m]);
            float b[6];
#pragma unroll
            for (int a = 0; a < 6; ++a) b[a] = leaf ? i2f(ob[a]) : unord(ob[a]);
            const uint32_t gn = l - f + 1;
            pad_box(b, b + 3, pad);
#pragma unroll
            for (int a = 0; a < 6; ++a) out[a] = f2u(b[a]);
            out[6] = leaf ? (LEAF_BIT | gc) : gn <= K ? (LEAF_BIT | ((gn - 1) << 27) | f) : gc;
        } else {
#pragma unroll
            for (int a = 0; a < 6; ++a) out[a] = NAN_BITS;
            out[6] = EMPTY_REF;
        }
        // lane c owns dword c of each 16-B plane: lo.x lo.y lo.z hi.x hi.y hi.z refs 0
        uint32_t* rec = records + 32 * (size_t)i + c;
#pragma unroll
        for (int a = 0; a < 7; ++a) rec[4 * a] = out[a];
        rec[28] = 0u;
    }
}

__global__ __launch_bounds__(BLOCK) void k_pack4_span(uint32_t n, uint32_t K, const uint32_t* __restrict__ span_bits,
                                                      const uint32_t* __restrict__ lch, const uint32_t* __restrict__ rch,
                                                      const uint32_t* __restrict__ first,
                                                      const uint32_t* __restrict__ last,
                                                      const uint32_t* __restrict__ perm, const float* __restrict__ aabb,
                                                       const MeshDesc* __restrict__ meshes, uint32_t nm,
                                                      const int32_t* __restrict__ ibox, const int32_t* __restrict__ pre,
                                                      const int32_t* __restrict__ suf, const int32_t* __restrict__ table,
                                                      const uint32_t* __restrict__ bounds,
                                                      uint32_t* __restrict__ records) {
    BDIAG(8);
    pack4_body(blockIdx.x, threadIdx.x, n, K, span_bits, lch, rch, first, last, perm, aabb, meshes, nm, ibox, pre, suf,
               table, bounds, records);
}

// Up to BM_PACK_TABLE_CHUNKS chunks (BVH4): no chunk-table launch — each k_pack4_table workgroup builds
// the sparse table of chunk unions (k_chunk_table's levels, same unions in the same order) in its own
// LDS, ~1 us for the bunny's 136 chunks, and answers its spanning records' range queries from there;
// workgroup 0 clears the gather replicas (the chunk kernel was their last reader).
#ifndef BM_PACK_TABLE_CHUNKS
#define BM_PACK_TABLE_CHUNKS 256u
#endif
constexpr uint32_t PT_MAX_CHUNKS = 256, PT_LEVELS = 9;  // levels j with 2^j <= 256
__global__ __launch_bounds__(BLOCK) void k_pack4_table(uint32_t n, uint32_t K, const uint32_t* __restrict__ span_bits,
                                                       const uint32_t* __restrict__ lch, const uint32_t* __restrict__ rch,
                                                       const uint32_t* __restrict__ first,
                                                       const uint32_t* __restrict__ last,
                                                       const uint32_t* __restrict__ perm, const float* __restrict__ aabb,
                                                       const MeshDesc* __restrict__ meshes, uint32_t nm,
                                                       const int32_t* __restrict__ ibox, const int32_t* __restrict__ pre,
                                                       const int32_t* __restrict__ suf, uint32_t* __restrict__ bounds,
                                                       uint32_t* __restrict__ records) {
    BDIAG(8);
    __shared__ int32_t lt[PT_LEVELS * PT_MAX_CHUNKS * 6];
    if (blockIdx.x == 0) clear_replicas(bounds, threadIdx.x, BLOCK);
    const uint32_t nc = (n + REFIT_CHUNK - 1) >> REFIT_CHUNK_LOG2;
    for (uint32_t i = threadIdx.x; i < nc; i += BLOCK) {
        const uint32_t end = min(n, (i + 1) << REFIT_CHUNK_LOG2) - 1;
#pragma unroll
        for (int a = 0; a < 6; ++a) lt[6 * i + a] = pre[6 * (size_t)end + a];
    }
    for (uint32_t j = 1; (1u << j) <= nc; ++j) {
        __syncthreads();
        const int32_t* src = lt + 6 * (j - 1) * nc;
        int32_t* dst = lt + 6 * j * nc;
        const uint32_t h = 1u << (j - 1);
        for (uint32_t i = threadIdx.x; i + (1u << j) <= nc; i += BLOCK) {
            int32_t r[6];
#pragma unroll
            for (int a = 0; a < 6; ++a) r[a] = src[6 * i + a];
            box_union(r, src + 6 * (i + h));
#pragma unroll
            for (int a = 0; a < 6; ++a) dst[6 * i + a] = r[a];
        }
    }
    __syncthreads();
    pack4_body(blockIdx.x, threadIdx.x, n, K, span_bits, lch, rch, first, last, perm, aabb, meshes, nm, ibox, pre, suf,
               lt, bounds, records);
}

// n <= 1: a single record whose child 0 is the lone triangle (or empty).
__global__ void k_pack_small(uint32_t n, uint32_t width, const float* __restrict__ aabb,
                             uint32_t* __restrict__ bounds, uint32_t* __restrict__ records) {
    for (int t = 0; t < BOUNDS_SLOTS; ++t) bounds[t] = fold_slot(bounds, t);
    clear_replicas(bounds, 0, 1);
    float lo[3] = {0.f, 0.f, 0.f}, hi[3] = {0.f, 0.f, 0.f};
    if (n == 1) {
        for (int a = 0; a < 3; ++a) {
            lo[a] = aabb[a];
            hi[a] = aabb[3 + a];
        }
        pad_box(lo, hi, scene_pad(bounds));
    }
    if (width == 4) {
        uint32_t r[32];
        for (int q = 0; q < 32; ++q) r[q] = 0u;
        if (n == 1) set_child4(r, 0, lo, hi, LEAF_BIT);
        else set_empty4(r, 0);
        for (int q = 1; q < 4; ++q) set_empty4(r, q);
        store_record4(records, r);
        return;
    }
    uint32_t r[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) r[q] = 0u;
    if (n == 1) set_child(r, 0, lo, hi, LEAF_BIT);
    else set_empty(r, 0);
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

// BVH8 records (256 B: lo.x[8] lo.y[8] lo.z[8] hi.x[8] hi.y[8] hi.z[8] refs[8] 0[8]) collapsed from
// the BVH2 records: record i lists the frontier three binary levels below node i — its children,
// each non-collapsed internal one replaced by its children, twice — in child order, with the padded
// boxes and refs of the BVH2 records (oracle/beam_oracle.c, width 8). Written for every node (a
// traversal reaches those at depths divisible by three; the others are never read); a BVH2 record
// of zeros (a node collapsed into its parent's leaf) gives zeros.
__global__ __launch_bounds__(BLOCK) void k_pack8(uint32_t nrec, const uint32_t* __restrict__ rec2,
                                                 uint32_t* __restrict__ rec8) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= nrec) return;
    const uint32_t* r = rec2 + 16 * (size_t)i;
    uint32_t* o = rec8 + 64 * (size_t)i;
    uint32_t out[64];
#pragma unroll
    for (int q = 0; q < 64; ++q) out[q] = 0u;
    const bool zero = r[12] == 0u && r[13] == 0u && r[0] == 0u && r[6] == 0u;
    if (!zero) {
        // frontier entries: (BVH2 record holding the entry, its slot there)
        uint32_t frec[8], fslot[8], nf = 0;
        for (uint32_t q = 0; q < 2; ++q)
            if (r[12 + q] != EMPTY_REF) {
                frec[nf] = i;
                fslot[nf++] = q;
            }
        for (int e = 0; e < 2; ++e) {
            uint32_t nrec_[8], nslot_[8], nn = 0;
            for (uint32_t k = 0; k < nf; ++k) {
                const uint32_t ref = rec2[16 * (size_t)frec[k] + 12 + fslot[k]];
                if (!(ref & LEAF_BIT)) {  // a non-collapsed internal node: its two children
                    nrec_[nn] = ref;
                    nslot_[nn++] = 0;
                    nrec_[nn] = ref;
                    nslot_[nn++] = 1;
                } else {
                    nrec_[nn] = frec[k];
                    nslot_[nn++] = fslot[k];
                }
            }
            for (uint32_t k = 0; k < nn; ++k) {
                frec[k] = nrec_[k];
                fslot[k] = nslot_[k];
            }
            nf = nn;
        }
        for (uint32_t k = 0; k < 8; ++k) {
            if (k < nf) {
                const uint32_t* c = rec2 + 16 * (size_t)frec[k];
                const uint32_t q = fslot[k];
                for (int a = 0; a < 3; ++a) {
                    out[8 * a + k] = c[6 * q + a];
                    out[24 + 8 * a + k] = c[6 * q + 3 + a];
                }
                out[48 + k] = c[12 + q];
            } else {
                for (int a = 0; a < 6; ++a) out[8 * a + k] = NAN_BITS;
                out[48 + k] = EMPTY_REF;
            }
        }
    }
    uint4* o4 = reinterpret_cast<uint4*>(o);
#pragma unroll
    for (int q = 0; q < 16; ++q) o4[q] = make_uint4(out[4 * q], out[4 * q + 1], out[4 * q + 2], out[4 * q + 3]);
}

inline uint32_t blocks_for(uint32_t n, uint32_t per) { return (n + per - 1) / per; }

// Up to this many triangles k_span and k_tree_chunk run as one launch (k_span_chunk): measured faster
// at every size (bunny 0.089 -> 0.080 ms, armadillo proxy 0.131 -> 0.122, 1.1M merged 0.270 -> 0.264);
// -DBM_SPAN_FUSE_MAX_N=0 restores the two launches for A/B builds.
#ifndef BM_SPAN_FUSE_MAX_N
#define BM_SPAN_FUSE_MAX_N 0xFFFFFFFFu
#endif

// One-sweep tile: small sorts are latency-bound (a few dozen tiles, each a serial chain of load,
// look-back, rank, scatter), so they take short tiles; big ones take long tiles, which halve the
// look-back work per key. Measured on MI355X (tools/build_bench.py): 8 items win up to ~0.5M keys.
#ifndef BM_ONESWEEP_SMALL_N
#define BM_ONESWEEP_SMALL_N (1u << 16)  // up to this many keys: 2048-key tiles; above, 4096 (armadillo build -6 %)
#endif
#ifndef BM_ONESWEEP_BIG_ITEMS
#define BM_ONESWEEP_BIG_ITEMS 16
#endif
#ifndef BM_ONESWEEP_HUGE_N
#define BM_ONESWEEP_HUGE_N (1u << 19)  // above this many keys: 8192-key tiles (1.1M-triangle build -3 %)
#endif
#ifndef BM_OSW_SMALL_N
#define BM_OSW_SMALL_N (1u << 17)  // up to this many keys (above BM_OSW_TINY_N): 2048-key tiles (2 per thread)
#endif
#ifndef BM_OSW_MID_N
#define BM_OSW_MID_N (1u << 19)    // up to this many keys: 4096-key tiles; above, 8192
#endif
#ifdef BM_ONESWEEP_NARROW
inline int onesweep_items(uint32_t n) {
    return n <= BM_ONESWEEP_SMALL_N ? 8 : n <= BM_ONESWEEP_HUGE_N ? BM_ONESWEEP_BIG_ITEMS : 32;
}
inline uint32_t onesweep_tiles(uint32_t n) { return n ? blocks_for(n, BLOCK * onesweep_items(n)) : 1u; }

void launch_onesweep(const uint32_t* ki, const uint32_t* vi, uint32_t* ko, uint32_t* vo, uint32_t n, int pass,
                     int passes, uint32_t* smeta, hipStream_t s, RecJob = RecJob{}) {  // (no records job here)
    const uint32_t nb = onesweep_tiles(n);
    if (onesweep_items(n) == 8)
        k_onesweep<8><<<nb, BLOCK, 0, s>>>(ki, vi, ko, vo, n, pass, passes, smeta, nb);
    else if (onesweep_items(n) == 32)
        k_onesweep<32><<<nb, BLOCK, 0, s>>>(ki, vi, ko, vo, n, pass, passes, smeta, nb);
    else
        k_onesweep<BM_ONESWEEP_BIG_ITEMS><<<nb, BLOCK, 0, s>>>(ki, vi, ko, vo, n, pass, passes, smeta, nb);
}
#else
#ifndef BM_OSW_TINY_N
#define BM_OSW_TINY_N (1u << 17)  // up to this many keys: 1024-key tiles (1 per thread; bunny build 0.114 -> 0.110 ms)
#endif
inline int onesweep_items(uint32_t n) {
    return n <= BM_OSW_TINY_N ? 1 : n <= BM_OSW_SMALL_N ? 2 : n <= BM_OSW_MID_N ? 4 : 8;
}
inline uint32_t onesweep_tiles(uint32_t n) { return n ? blocks_for(n, OS_BLOCK * onesweep_items(n)) : 1u; }

// rj.nblk > 0: that many more workgroups gather the triangle records and corner normals (gather_records).
// skew_cap > 0: the top-digit pass of a top-digit-first sort, with the LSD fallback's second set of tiles
// skew_cap > 0: the top-digit pass of a top-digit-first sort, with the LSD fallback's second set of tiles
// and one more workgroup for the bucket plan (written to `plan`)
void launch_onesweep(const uint32_t* ki, const uint32_t* vi, uint32_t* ko, uint32_t* vo, uint32_t n, int pass,
                     int passes, uint32_t* smeta, hipStream_t s, RecJob rj = RecJob{}, uint32_t skew_cap = 0,
                     uint32_t* plan = nullptr, const uint32_t* topmap = nullptr) {
    const uint32_t nb = onesweep_tiles(n), grid = (skew_cap ? 2 * nb + 1 : nb) + rj.nblk;
    if (topmap) {  // ranked top digit (no records job, no skew fallback on this path)
        switch (onesweep_items(n)) {
            case 1: k_onesweep_wide<1, true><<<nb, OS_BLOCK, 0, s>>>(ki, vi, ko, vo, n, pass, passes, smeta, nb, nb, rj, 0, nullptr, topmap); break;
            case 2: k_onesweep_wide<2, true><<<nb, OS_BLOCK, 0, s>>>(ki, vi, ko, vo, n, pass, passes, smeta, nb, nb, rj, 0, nullptr, topmap); break;
            case 4: k_onesweep_wide<4, true><<<nb, OS_BLOCK, 0, s>>>(ki, vi, ko, vo, n, pass, passes, smeta, nb, nb, rj, 0, nullptr, topmap); break;
            default: k_onesweep_wide<8, true><<<nb, OS_BLOCK, 0, s>>>(ki, vi, ko, vo, n, pass, passes, smeta, nb, nb, rj, 0, nullptr, topmap); break;
        }
        return;
    }
    switch (onesweep_items(n)) {
        case 1: k_onesweep_wide<1><<<grid, OS_BLOCK, 0, s>>>(ki, vi, ko, vo, n, pass, passes, smeta, nb, nb, rj, skew_cap, plan); break;
        case 2: k_onesweep_wide<2><<<grid, OS_BLOCK, 0, s>>>(ki, vi, ko, vo, n, pass, passes, smeta, nb, nb, rj, skew_cap, plan); break;
        case 4: k_onesweep_wide<4><<<grid, OS_BLOCK, 0, s>>>(ki, vi, ko, vo, n, pass, passes, smeta, nb, nb, rj, skew_cap, plan); break;
        default: k_onesweep_wide<8><<<grid, OS_BLOCK, 0, s>>>(ki, vi, ko, vo, n, pass, passes, smeta, nb, nb, rj, skew_cap, plan); break;
    }
}
#endif

}  // namespace


// The bucket plan (bucket_plan) follows the look-back words, outside the block k_gather zero-fills (it is
// written whole before k_bucket_sort reads it).
static size_t plan_offset(uint32_t n) { return META_LOOKBACK + (size_t)RADIX_PASSES * onesweep_tiles(n) * RADIX; }
size_t build_meta_words(uint32_t n) { return plan_offset(n) + PLAN_WORDS; }

// triangles -> original-order records, AABBs and scene bounds (needs META_GATHER_CLEAR zeroed words);
// zero-fills meta words [clear_begin, clear_end)
static void launch_gather_kernel(const BuildBuffers& b, hipStream_t s, uint32_t clear_begin = 0, uint32_t clear_end = 0,
                                 bool with_bounds = true, bool with_tri = true, bool with_nrm = true,
                                 bool with_aabb = true, bool with_cen = false) {
    k_gather<<<blocks_for(b.n, BLOCK), BLOCK, 0, s>>>(b.meshes, b.num_meshes, b.n, b.tri_orig, b.nrm,
                                                     with_aabb ? b.aabb : nullptr, with_cen ? b.cen : nullptr,
                                                     b.bounds, clear_begin, clear_end, with_bounds ? 1 : 0,
                                                     with_tri ? 1 : 0, with_nrm ? 1 : 0);
}
uint32_t num_records(uint32_t n) { return n > 1 ? n - 1 : 1; }

size_t sort_meta_words(uint32_t n, int key_bits) {
    const int passes = (key_bits + RADIX_BITS - 1) / RADIX_BITS;
    const uint32_t nb = onesweep_tiles(n);
    return 4 + (size_t)passes * RADIX + (size_t)passes * nb * RADIX;
}
size_t chunk_table_floats(uint32_t n) {
    const uint32_t nc = n ? (n + REFIT_CHUNK - 1) >> REFIT_CHUNK_LOG2 : 1;
    return (size_t)6 * nc * (floor_log2(nc) + 1);
}

#define BM_LAUNCH_CHECK()                          \
    do {                                           \
        hipError_t e_ = hipGetLastError();         \
        if (e_ != hipSuccess) return e_;           \
    } while (0)

// Shared by build and refit: bottom-up boxes over the current topology, node records, sorted
// triangle records. Needs gather (aabb, bounds, tri_orig) and the topology (vals, tree arrays).
// the refit products (ibox, pre, suf, table) hold ordered-int box images (see box_union)
inline int32_t* ob(float* p) { return reinterpret_cast<int32_t*>(p); }

#ifndef BM_CHUNK_MESH
#define BM_CHUNK_MESH 1  // the chunk kernel reads each sorted triangle from its mesh (no original-order records)
#endif
// What the chunk kernel reads its triangles from: nullptr = the meshes (mesh-direct), else the
// original-order records of the gather
static const float4* chunk_tsrc(const BuildBuffers& b) { return BM_CHUNK_MESH ? nullptr : b.tri_orig; }
// Whether this build must leave the original-order records in tri_orig: a multi-device root reshades
// from them (launch_reshade), the one-triangle path sorts them (k_sort_tris), and without the
// mesh-direct chunk kernel they are its source.
static bool need_orig(const BuildBuffers& b) { return b.orig_records || b.n == 1 || !BM_CHUNK_MESH; }
// Whether the build keeps per-triangle AABBs (aabb[]): only the one-triangle path (k_pack_small) and the
// non-mesh-direct chunk kernel read them; mesh-direct record writers take a leaf's box from its mesh and
// the Morton keys come from the gather's AABB centres (cen[], 12 B instead of 24).
static bool need_aabb(const BuildBuffers& b) { return b.n == 1 || !BM_CHUNK_MESH; }
static const float* finish_aabb(const BuildBuffers& b) { return need_aabb(b) ? b.aabb : nullptr; }

// BVH8: the BVH2 records (into records2), then k_pack8 collapses them into records.
static hipError_t launch_pack8(const BuildBuffers& b, hipStream_t s) {
    const uint32_t nrec = b.n > 1 ? b.n - 1 : 1;
    k_pack8<<<blocks_for(nrec, BLOCK), BLOCK, 0, s>>>(nrec, b.records2, b.records);
    BM_LAUNCH_CHECK();
    return hipSuccess;
}

#ifndef BM_CT_SPLIT_CHUNKS
#define BM_CT_SPLIT_CHUNKS 512  // from this many chunks the LDS table's stores are split over 8 workgroups
#endif
static hipError_t launch_finish(const BuildBuffers& b, hipStream_t s) {
    const uint32_t n = b.n;
    const bool w8 = b.width == 8;
    uint32_t* rec2 = w8 ? b.records2 : b.records;  // where the BVH2 (or small-scene) records go
    if (n == 1) {
        k_pack_small<<<1, 1, 0, s>>>(1, w8 ? 2u : b.width, b.aabb, b.bounds, rec2);
        BM_LAUNCH_CHECK();
        k_sort_tris<<<1, BLOCK, 0, s>>>(n, b.vals, b.tri_orig, b.tris);
        BM_LAUNCH_CHECK();
        return w8 ? launch_pack8(b, s) : hipSuccess;
    }
    // the sort's scratch is free again: vals2 holds the spanning bitmap
    uint32_t* span_bits = b.vals2;
    const bool w4 = b.width == 4;
    const uint32_t nchunk = blocks_for(n, REFIT_CHUNK);
    if (n > REFIT_CHUNK && n <= BM_SPAN_FUSE_MAX_N) {
        k_span_chunk<<<nchunk + blocks_for(n - 1, REFIT_CHUNK), REFIT_CHUNK, 0, s>>>(
            nchunk, n, b.keys, b.vals, finish_aabb(b), b.meshes, b.num_meshes, chunk_tsrc(b), b.tris, b.lch, b.rch, b.first,
            b.last, ob(b.ibox), ob(b.pre),
            ob(b.suf), b.bounds, b.leaf_size, w4 ? b.records : nullptr, span_bits);
        BM_LAUNCH_CHECK();
    } else {
        if (n > REFIT_CHUNK) {
            k_span<<<blocks_for(n - 1, SPAN_BLOCK), SPAN_BLOCK, 0, s>>>(n, b.keys, b.lch, b.rch, b.first, b.last,
                                                                       b.bounds, span_bits);
            BM_LAUNCH_CHECK();
        }
        k_tree_chunk<<<nchunk, REFIT_CHUNK, 0, s>>>(n, b.keys, b.vals, finish_aabb(b), b.meshes, b.num_meshes, chunk_tsrc(b),
                                                    b.tris, b.lch, b.rch, b.first,
                                                    b.last, ob(b.ibox), ob(b.pre), ob(b.suf), b.bounds, b.leaf_size,
                                                    w4 ? b.records : nullptr);
        BM_LAUNCH_CHECK();
    }
    if (n > REFIT_CHUNK && w4 && nchunk <= std::min(BM_PACK_TABLE_CHUNKS, PT_MAX_CHUNKS)) {
        k_pack4_table<<<blocks_for(n - 1, PACK4_IDX), BLOCK, 0, s>>>(n, b.leaf_size, span_bits, b.lch, b.rch, b.first,
                                                                    b.last, b.vals, finish_aabb(b), b.meshes,
                                                                    b.num_meshes, ob(b.ibox), ob(b.pre),
                                                                    ob(b.suf), b.bounds, b.records);
        BM_LAUNCH_CHECK();
    } else if (n > REFIT_CHUNK) {
        if (((n + REFIT_CHUNK - 1) >> REFIT_CHUNK_LOG2) <= CT_LDS_CHUNKS)
            k_chunk_table_lds<<<nchunk >= BM_CT_SPLIT_CHUNKS ? 8 : 1, 1024, 0, s>>>(n, ob(b.pre), ob(b.table), b.bounds);
        else
            k_chunk_table<<<1, 1024, 0, s>>>(n, ob(b.pre), ob(b.table), b.bounds);
        BM_LAUNCH_CHECK();
        if (w4) {
            k_pack4_span<<<blocks_for(n - 1, PACK4_IDX), BLOCK, 0, s>>>(n, b.leaf_size, span_bits, b.lch, b.rch,
                                                                   b.first, b.last, b.vals, finish_aabb(b), b.meshes,
                                                                   b.num_meshes, ob(b.ibox),
                                                                   ob(b.pre), ob(b.suf), ob(b.table), b.bounds,
                                                                   b.records);
            BM_LAUNCH_CHECK();
        }
    }
    if (!w4) {
        k_pack<<<blocks_for(n - 1, BLOCK), BLOCK, 0, s>>>(n, b.leaf_size, b.lch, b.rch, b.first, b.last, b.vals,
                                                         finish_aabb(b), b.meshes, b.num_meshes, ob(b.ibox), ob(b.pre), ob(b.suf), ob(b.table), b.bounds,
                                                         rec2);
        BM_LAUNCH_CHECK();
    }
    return w8 ? launch_pack8(b, s) : hipSuccess;
}

#ifndef BM_NRM_BLOCKS
#define BM_NRM_BLOCKS 448u  // normal-gathering workgroups beside the top-digit pass's tiles (merged: 128 -> 0.260 ms, 256 -> 0.249, 448 -> 0.244)
#endif

#ifndef BM_REC_DEFER_MAX_N
#define BM_REC_DEFER_MAX_N (1u << 19)  // bunny 0.068 -> 0.067 ms, armadillo 0.100 -> 0.099; merged 0.244 -> 0.250
#endif

bool msd_sort(uint32_t n, const Tuning& t) {
    static_assert(BM_MSD_MAX_N <= MSD_MAX_N_CAP, "the LSD fallback inside k_bucket_sort covers at most RADIX tiles");
    return (int64_t)n <= std::min<int64_t>(t.get(BM_PARAM_MSD_MAX_N, BM_MSD_MAX_N), MSD_MAX_N_CAP) && n >= BM_MSD_MIN_N;
}
uint32_t build_sort_skew_word() { return META_SORT_SKEW; }

hipError_t launch_build(const BuildBuffers& b, hipStream_t s) {
    const uint32_t n = b.n;
    hipError_t e;
    // bounds, sort tickets, digit histograms and look-back words all start at zero: the gather's own
    // words here (unless the previous build of this buffer cleared them), the rest by k_gather itself
    if (!(n && b.replicas_clean) &&
        (e = hipMemsetD32Async((hipDeviceptr_t)b.bounds, 0, n ? META_GATHER_CLEAR : build_meta_words(n), s)) !=
            hipSuccess)
        return e;
    if (n == 0) {
        k_pack_small<<<1, 1, 0, s>>>(0, b.width == 8 ? 2u : b.width, b.aabb, b.bounds,
                                     b.width == 8 ? b.records2 : b.records);
        BM_LAUNCH_CHECK();
        return b.width == 8 ? launch_pack8(b, s) : hipSuccess;
    }
    static const Tuning dflt;
    const Tuning& tune = b.tune ? *b.tune : dflt;
    const bool msd = msd_sort(n, tune);
    // top-digit-first sorts: the triangle records and corner normals ride on the top-digit pass
    // (BM_PARAM_NRM_DEFER 0: in the gather)
#ifdef BM_ONESWEEP_NARROW
    constexpr bool nrm_defer = false;
#else
    const bool nrm_defer = tune.get(BM_PARAM_NRM_DEFER, 1) != 0;
#endif
    const bool defer = msd && nrm_defer;
    const bool orig = need_orig(b);
    if (b.orig_written) *b.orig_written = orig;
    // the records too up to BM_REC_DEFER_MAX_N triangles (above, the pass's extra workgroups outlast its
    // tiles), when this build writes them at all
    const bool defer_tri = defer && orig && n <= BM_REC_DEFER_MAX_N;
    launch_gather_kernel(b, s, META_GATHER_CLEAR, (uint32_t)plan_offset(n), true, orig && !defer_tri, !defer,
                         need_aabb(b), true);
    BM_LAUNCH_CHECK();
    // an odd number of passes: start in the scratch pair so the sorted data ends in keys/vals
    k_morton<<<blocks_for(n, SORT_TILE), MORTON_BLOCK, 0, s>>>(n, b.cen, b.bounds, b.keys2, b.vals2);
    BM_LAUNCH_CHECK();
    if (msd) {  // top digit (keys2 -> keys), then each bucket in place; or the LSD fallback (skew)
        // 256-lane bucket workgroups up to 2^19 keys at most (their fallback tiles must not outnumber the
        // top-digit pass's, whose count sizes the look-back area); the parameter can only lower that
        const bool wide = (int64_t)n > std::min<int64_t>(tune.get(BM_PARAM_MSD_WIDE_N, BM_MSD_WIDE_N), BM_MSD_WIDE_N);
        // buckets above this take the LSD fallback: the kernel's LDS capacity, or below it
        // BM_PARAM_BUCKET_LDS_CAP (tests force the fallback with 0)
        const uint32_t cap = (uint32_t)std::min<int64_t>(tune.get(BM_PARAM_BUCKET_LDS_CAP, 0xFFFFFFFFll),
                                                         (wide ? 1024 : 256) * BS_ITEMS);
#ifdef BM_NO_NRM_PROBE  // A/B probe only (wrong colours): the build's cost without any corner-normal gather
        const RecJob rj{b.meshes, b.num_meshes, n, 0u, nullptr, b.nrm};
#else
        const RecJob rj{b.meshes, b.num_meshes, n, defer ? std::min<uint32_t>(BM_NRM_BLOCKS, blocks_for(n, OS_BLOCK_N)) : 0u,
                        defer_tri ? b.tri_orig : nullptr, b.nrm};
#endif
        uint32_t* smeta = b.bounds + META_COUNTERS;
        uint32_t* plan = b.bounds + plan_offset(n);
        const uint32_t nb = onesweep_tiles(n);
        const int wi = onesweep_items(n);
        launch_onesweep(b.keys2, b.vals2, b.keys, b.vals, n, RADIX_PASSES - 1, RADIX_PASSES, smeta, s, rj, cap + 1, plan);
        BM_LAUNCH_CHECK();
        if (wide)
            k_bucket_sort<1024><<<RADIX, 1024, 0, s>>>(b.keys, b.vals, b.keys2, b.vals2, b.bounds, plan, n, nb, wi);
        else
            k_bucket_sort<256><<<RADIX, 256, 0, s>>>(b.keys, b.vals, b.keys2, b.vals2, b.bounds, plan, n, nb, wi);
        BM_LAUNCH_CHECK();
        return launch_finish(b, s);
    }
    uint32_t *ki = b.keys2, *vi = b.vals2, *ko = b.keys, *vo = b.vals;
    static_assert(RADIX_PASSES % 2 == 1, "sorted output must land in keys/vals");
    for (int pass = 0; pass < RADIX_PASSES; ++pass) {
        launch_onesweep(ki, vi, ko, vo, n, pass, RADIX_PASSES, b.bounds + META_COUNTERS, s);
        BM_LAUNCH_CHECK();
        uint32_t* tk = ki; ki = ko; ko = tk;
        uint32_t* tv = vi; vi = vo; vo = tv;
    }
    // sorted data is in b.keys / b.vals: tree, boxes and sorted triangle records in one pass
    return launch_finish(b, s);
}

#ifdef BM_BUILD_DIAG
hipError_t build_diag(unsigned long long* out) { return bdiag_io((const void*)&g_bdiag, out, 0, 9); }
#endif

hipError_t launch_gather(const BuildBuffers& b, hipStream_t s) {  // reference modes: no scene bounds needed
    if (b.n == 0) return hipSuccess;
    // zeroes bounds words 0-2 and the map after them: the reference-mode build's queue count, overflow
    // flag, top-bit count and top-bit map (KdBuild::qcount, topcount, topmap)
    launch_gather_kernel(b, s, 0, 3 + KD_TOPMAP_WORDS, false);
    BM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_orig_records(const BuildBuffers& b, hipStream_t s) {  // tri_orig only (no boxes, normals, bounds)
    if (b.n == 0) return hipSuccess;
    k_gather<<<blocks_for(b.n, BLOCK), BLOCK, 0, s>>>(b.meshes, b.num_meshes, b.n, b.tri_orig, nullptr, nullptr,
                                                     nullptr, b.bounds, 0, 0, 0, 1, 0);
    BM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_sort_pairs(uint32_t* keys, uint32_t* vals, uint32_t* keys2, uint32_t* vals2, uint32_t n,
                             int key_bits, uint32_t* smeta, hipStream_t s, bool* in_scratch, bool meta_zeroed,
                             const uint32_t* topmap) {
    if (topmap && key_bits != 31) return hipErrorInvalidValue;  // the ranked top digit is bits 20-30
    const int passes = topmap ? 3 : (key_bits + RADIX_BITS - 1) / RADIX_BITS;
    if (passes < 1 || passes > 4) return hipErrorInvalidValue;
    hipError_t e;
    if (!meta_zeroed &&
        (e = hipMemsetD32Async((hipDeviceptr_t)smeta, 0, sort_meta_words(n, key_bits), s)) != hipSuccess)
        return e;
    *in_scratch = false;
    if (n == 0) return hipSuccess;
    k_digit_hist<<<blocks_for(n, DH_TILE), BLOCK, 0, s>>>(keys, n, passes, smeta, topmap);
    BM_LAUNCH_CHECK();
    uint32_t *ki = keys, *vi = vals, *ko = keys2, *vo = vals2;
    for (int pass = 0; pass < passes; ++pass) {
        launch_onesweep(ki, vi, ko, vo, n, pass, passes, smeta, s, RecJob{}, 0, nullptr,
                        topmap && pass == 2 ? topmap : nullptr);
        BM_LAUNCH_CHECK();
        uint32_t* tk = ki; ki = ko; ko = tk;
        uint32_t* tv = vi; vi = vo; vo = tv;
    }
    *in_scratch = (passes % 2) == 1;
    return hipSuccess;
}

hipError_t launch_radix_tree(const uint32_t* keys, uint32_t n, uint32_t* lch, uint32_t* rch, uint32_t* first,
                             uint32_t* last, uint32_t* parent_leaf, uint32_t* parent_int, hipStream_t s,
                             const uint32_t* n_dev) {
    if (n < 2) return hipSuccess;
    k_emit_lds<<<blocks_for(n - 1, EMIT_LDS_BLOCK), EMIT_LDS_BLOCK, 0, s>>>((int)n, keys, lch, rch, first, last,
                                                                          parent_leaf, parent_int, n_dev);
    BM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_refit(const BuildBuffers& b, hipStream_t s) {
    const uint32_t n = b.n;
    hipError_t e;
    if (!(n && b.replicas_clean) && (e = hipMemsetD32Async((hipDeviceptr_t)b.bounds, 0, META_GATHER_CLEAR, s)) != hipSuccess)
        return e;
    if (n == 0) {
        k_pack_small<<<1, 1, 0, s>>>(0, b.width == 8 ? 2u : b.width, b.aabb, b.bounds,
                                     b.width == 8 ? b.records2 : b.records);
        BM_LAUNCH_CHECK();
        return b.width == 8 ? launch_pack8(b, s) : hipSuccess;
    }
    const bool orig = need_orig(b);
    if (b.orig_written) *b.orig_written = orig;
    launch_gather_kernel(b, s, 0, 0, true, orig, true, need_aabb(b));
    BM_LAUNCH_CHECK();
    return launch_finish(b, s);
}

}  // namespace bm
