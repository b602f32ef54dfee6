// bm_common.h — layouts and bit-exact scalar math shared by the gfx950 kernels.
//
// Every translation unit that includes this is compiled with -ffp-contract=off and IEEE f32
// division/sqrt (see build.py), so each expression rounds once per operation in the order written:
// the order of glm 0.9.9.0 as the reference compiles it (dot = (x*x'+y*y')+z*z', cross, mat3*vec3
// row sums) and of Raytracer/CudaComon.cuh. That is what makes hit ids, packed colours and t
// bit-identical to the CPU oracle.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bm {

// ---- BVH2 node record: 16 x u32 = 64 B, one per Karras internal node slot --------------------
//   [0..5]  child0 box lo.xyz hi.xyz     [6..11] child1 box lo.xyz hi.xyz
//   [12]    child0 ref                   [13]    child1 ref            [14,15] 0
// ref: internal node index (< 2^31), or LEAF_BIT | (count-1)<<27 | first (sorted triangle index),
// or EMPTY_REF (its box is all-NaN, which no slab test accepts).
constexpr uint32_t LEAF_BIT = 0x80000000u;
constexpr uint32_t EMPTY_REF = 0xFFFFFFFFu;
constexpr uint32_t NAN_BITS = 0x7FC00000u;
constexpr uint32_t FIRST_MASK = 0x07FFFFFFu;
constexpr uint32_t MAX_TRIS = 1u << 27;
constexpr float PAD_SCALE = 0x1p-20f;  // box inflation: |x|*2^-20 + extent*2^-20

// ---- triangle record: 3 x float4 = 48 B, sorted (leaf) order ---------------------------------
//   (v0.xyz, bits(global id)) (e1 = v1-v0, 0) (e2 = v2-v0, 0)

constexpr uint32_t MISS_PACKED = 0x0000FF00u;  // 255<<8, BuildTree.cu:495
constexpr uint32_t NO_TRI = 0xFFFFFFFFu;

__host__ __device__ __forceinline__ int32_t f2i(float f) { return __builtin_bit_cast(int32_t, f); }
__host__ __device__ __forceinline__ float i2f(int32_t i) { return __builtin_bit_cast(float, i); }
__host__ __device__ __forceinline__ uint32_t f2u(float f) { return __builtin_bit_cast(uint32_t, f); }
__host__ __device__ __forceinline__ float u2f(uint32_t u) { return __builtin_bit_cast(float, u); }

// Ordered-integer image of a float: a total order with -0 < +0, so min/max of stored bounds do
// not depend on evaluation order (and atomicMin/atomicMax on it reduce floats exactly).
__host__ __device__ __forceinline__ int32_t ord(float f) {
    int32_t i = f2i(f);
    return i >= 0 ? i : (i ^ 0x7FFFFFFF);
}
__host__ __device__ __forceinline__ float unord(int32_t o) { return i2f(o >= 0 ? o : (o ^ 0x7FFFFFFF)); }
__host__ __device__ __forceinline__ float omin(float a, float b) { return ord(b) < ord(a) ? b : a; }
__host__ __device__ __forceinline__ float omax(float a, float b) { return ord(b) > ord(a) ? b : a; }

__host__ __device__ __forceinline__ uint32_t expand_bits10(uint32_t v) {
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}

__host__ __device__ __forceinline__ uint32_t quant10(float c, float cmin, float scale) {
    float q = (c - cmin) * scale;
    if (!(q > 0.0f)) return 0u;
    if (q >= 1023.0f) return 1023u;
    return (uint32_t)q;
}

// Order key of a BVH4 child hit by a ray at entry distance tn: tn clamped at 0 (a box around the
// origin enters at 0) as its bit image (monotone for non-negative floats) with the child's slot in
// place of the last two mantissa bits. Keys of distinct slots differ, so one unsigned
// compare orders two children: nearest first, (near-)ties by slot. The traversal visits the hit
// children in key order; oracle/beam_oracle.c (visit_node) uses the same key, so the COUNT
// build's counters match it step for step. The order decides work, never the closest hit.
__host__ __device__ __forceinline__ uint32_t order_key(float tn, uint32_t slot) {
    const int32_t b = f2i(tn) > 0 ? f2i(tn) : 0;  // negative tn and -0 -> 0; +inf keeps its place (above all finite)
    return ((uint32_t)b & ~3u) | slot;
}

struct vec3f {
    float x, y, z;
};
__host__ __device__ __forceinline__ vec3f v3(float x, float y, float z) { return vec3f{x, y, z}; }
__host__ __device__ __forceinline__ vec3f sub(vec3f a, vec3f b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
__host__ __device__ __forceinline__ float dot(vec3f a, vec3f b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
__host__ __device__ __forceinline__ vec3f cross(vec3f x, vec3f y) {
    return v3(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y);
}

// Möller-Trumbore (bmTriIntersect, CudaComon.cuh:117-155) against one 48-B triangle record, e1/e2
// precomputed bit-identically. Returns false on the reference's two early rejects; otherwise t
// (which may be negative, inf or NaN: no det-epsilon) and u, v.
// The exact-safe early reject uses the 1-ulp hardware reciprocal: when the approximate u or v lies
// outside [0,1] by 2^-10 the correctly rounded value does too (their relative difference is
// < 2^-21); NaN never rejects there. Only candidates pay the correctly rounded division the
// reference's arithmetic requires. (|det| >= 2^-100 keeps the reciprocal away from denormal and
// overflow ranges.)
__device__ __forceinline__ bool tri_test(const float4 a, const float4 b, const float4 c, const vec3f orig,
                                         const vec3f dir, float& t, float& u, float& v) {
    const vec3f e1 = v3(b.x, b.y, b.z), e2 = v3(c.x, c.y, c.z);
    const vec3f pv = cross(dir, e2);
    const float det = dot(e1, pv);
    const vec3f tv = sub(orig, v3(a.x, a.y, a.z));
    const float un = dot(tv, pv);
    const vec3f qv = cross(tv, e1);
    const float vn = dot(dir, qv);
    const float ra = __builtin_amdgcn_rcpf(det);
    const float ua = un * ra, va = vn * ra;
    const bool far_out = fabsf(det) >= 0x1p-100f &&
                         (ua < -0x1p-10f || ua > 1.0f + 0x1p-10f || va < -0x1p-10f || va + ua > 1.0f + 0x1p-9f);
    bool in = false;
    if (!far_out) {
        const float idet = 1.f / det;
        u = un * idet;
        v = vn * idet;
        if (!(u < 0 || u > 1) && !(v < 0 || v + u > 1)) {
            t = dot(e2, qv) * idet;
            in = true;
        }
    }
    return in;
}

// Wave64 ballot of a bool: the compare mask itself. HIP's __ballot takes an int predicate, so a bool
// argument costs a select to 0/1 and a compare back per call (BM_BOOL_BALLOT 0 restores it for A/B).
#ifndef BM_BOOL_BALLOT
#define BM_BOOL_BALLOT 1
#endif
__device__ __forceinline__ unsigned long long ballot(bool b) {
#if BM_BOOL_BALLOT
    return __builtin_amdgcn_ballot_w64(b);
#else
    return __ballot(b);
#endif
}

// Inclusive prefix sum over the wave's 64 lanes in six DPP steps: shifts by 1, 2, 4, 8 within each row
// of 16 (lanes shifted in from outside the row read 0), then row 15's total into rows 1 and 3 and
// lane 31's into rows 2 and 3 — no LDS round trip, where a shuffle scan takes six.
__device__ __forceinline__ uint32_t wave_incl_add(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return v;
}

// Mesh table entry for the gather kernel (one per scene mesh, in scene order).
struct MeshDesc {
    const float* pos;     // 3 floats / vertex
    const float* nrm;     // 3 floats / vertex
    const uint32_t* idx;  // 3 per face
    uint32_t tri_offset;  // first global triangle id of this mesh
    uint32_t num_tris;
};

// Scene-bounds slots, all reduced with unsigned atomicMax from a zero fill (so they share the one
// memset of the build's metadata block): [0..2] min xyz and [3..5] max xyz of the triangle AABBs,
// [6..8] min and [9..11] max of the AABB centres. A value is stored as its order-preserving u32
// image (bkey); min slots store its complement, so every slot's identity is 0.
constexpr int BOUNDS_SLOTS = 12;
__host__ __device__ __forceinline__ uint32_t bkey(float f) { return (uint32_t)ord(f) ^ 0x80000000u; }
__host__ __device__ __forceinline__ uint32_t bkey_lo(float f) { return ~bkey(f); }
__host__ __device__ __forceinline__ float bounds_lo(uint32_t v) { return unord((int32_t)(~v ^ 0x80000000u)); }
__host__ __device__ __forceinline__ float bounds_hi(uint32_t v) { return unord((int32_t)(v ^ 0x80000000u)); }

}  // namespace bm
