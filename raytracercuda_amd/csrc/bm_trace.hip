// bm_trace.hip — per-pixel primary-ray trace for gfx950 (replaces bmMarchKernel,
// Raytracer/BuildTree.cu:367-499; Trace.cu and Trace2.cu carry no live semantics).
//
// One thread per pixel, 256-thread workgroups covering a 16x16 pixel tile, each wave64 an 8x8
// sub-tile (coherent rays share BVH nodes). The ray direction is rebuilt on the device from the
// camera's column/row tables with the reference's exact arithmetic (Camera.cpp:51-66), so no
// 12-byte-per-pixel ray table is read. Traversal is near-first over 64-byte BVH2 records (both
// child boxes inline: one record = four 16-B loads per visit), with the short traversal stack in
// LDS (LDS_STACK entries per lane, [depth][lane] so every access is bank-conflict free) spilling
// to scratch beyond that. Triangles are 48-byte (v0,id | e1 | e2) records in leaf order.
//
// Semantics: closest hit with t > 0; equal t resolved to the lowest global triangle id (the order
// the reference's serial leaf lists give, BuildTree.cu:419-425); Möller-Trumbore and shading in
// the reference's operation order (CudaComon.cuh:117-155, 253-266). Bit-identical to
// oracle/beam_oracle.c orc_bvh_trace, including the node/triangle counters of the COUNT build.
#include "bm_internal.h"

namespace bm {
namespace {

constexpr int TILE = 16;
constexpr int BLOCK = TILE * TILE;
constexpr int LDS_STACK = 16;
constexpr int MAX_STACK = 64;  // >= BVH depth: a Karras tree over 30-bit keys + 32-bit tiebreak

__device__ __forceinline__ bool child_hit(const float* lo, const float* hi, const vec3f o, const vec3f inv,
                                          float tbest, float& tn_out) {
    const float tlx = (lo[0] - o.x) * inv.x, thx = (hi[0] - o.x) * inv.x;
    const float tly = (lo[1] - o.y) * inv.y, thy = (hi[1] - o.y) * inv.y;
    const float tlz = (lo[2] - o.z) * inv.z, thz = (hi[2] - o.z) * inv.z;
    const float tn = fmaxf(fmaxf(fminf(tlx, thx), fminf(tly, thy)), fminf(tlz, thz));
    const float tf = fminf(fminf(fmaxf(tlx, thx), fmaxf(tly, thy)), fmaxf(tlz, thz));
    tn_out = tn;
    return (tn <= tf) && (tf >= 0.0f) && (tn <= tbest);
}

template <bool COUNT>
__global__ __launch_bounds__(BLOCK) void k_trace_primary(const TraceParams p) {
    __shared__ uint32_t s_ref[LDS_STACK][BLOCK];
    __shared__ float s_t[LDS_STACK][BLOCK];
    uint32_t x_ref[MAX_STACK - LDS_STACK];
    float x_t[MAX_STACK - LDS_STACK];

    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const uint32_t x = blockIdx.x * TILE + (w & 1) * 8 + (lane & 7);
    const uint32_t lr = blockIdx.y * TILE + (w >> 1) * 8 + (lane >> 3);
    const uint32_t gy = ((lr / p.band_h) * p.band_step + p.band_first) * p.band_h + lr % p.band_h;
    if (x >= p.width || lr >= p.local_rows || gy >= p.height) return;

    // Camera::setInitialRays (Camera.cpp:61-66) for this pixel, then dir = orient * ray.
    const float rx = p.rx[x], ry = p.ry[gy];
    const float d = 1.f / sqrtf(p.z2 + rx * rx + ry * ry);
    const vec3f r = v3(rx * d, ry * d, p.zoom * d);
    const float* m = p.orient;
    const vec3f dir = v3((m[0] * r.x + m[3] * r.y) + m[6] * r.z, (m[1] * r.x + m[4] * r.y) + m[7] * r.z,
                         (m[2] * r.x + m[5] * r.y) + m[8] * r.z);
    const vec3f inv = v3(1.f / dir.x, 1.f / dir.y, 1.f / dir.z);
    const vec3f eye = v3(p.eye[0], p.eye[1], p.eye[2]);

    float tbest = __builtin_inff(), bu = 0.f, bv = 0.f;
    uint32_t ibest = NO_TRI;
    unsigned long long c_nodes = 0, c_tris = 0;
    int sp = 0;
    uint32_t next = p.num_tris ? 0u : EMPTY_REF;

    for (;;) {
        if (next == EMPTY_REF) {
            // pop until an entry that can still hold a closer hit
            bool found = false;
            while (sp > 0) {
                --sp;
                uint32_t ref;
                float tt;
                if (sp < LDS_STACK) {
                    ref = s_ref[sp][tid];
                    tt = s_t[sp][tid];
                } else {
                    ref = x_ref[sp - LDS_STACK];
                    tt = x_t[sp - LDS_STACK];
                }
                if (!(tt > tbest)) {
                    next = ref;
                    found = true;
                    break;
                }
            }
            if (!found) break;
        }
        if (next & LEAF_BIT) {
            const uint32_t first = next & FIRST_MASK, cnt = ((next >> 27) & 15u) + 1u;
            for (uint32_t k = first; k < first + cnt; ++k) {
                const float4 a = p.tris[3 * k + 0];
                const float4 b = p.tris[3 * k + 1];
                const float4 c = p.tris[3 * k + 2];
                if (COUNT) ++c_tris;
                // bmTriIntersect (CudaComon.cuh:117-155), e1/e2 precomputed bit-identically
                const vec3f e1 = v3(b.x, b.y, b.z), e2 = v3(c.x, c.y, c.z);
                const vec3f pv = cross(dir, e2);
                const float det = dot(e1, pv);
                const float idet = 1.f / det;
                const vec3f tv = sub(eye, v3(a.x, a.y, a.z));
                const float u = dot(tv, pv) * idet;
                if (u < 0 || u > 1) continue;
                const vec3f qv = cross(tv, e1);
                const float v = dot(dir, qv) * idet;
                if (v < 0 || v + u > 1) continue;
                const float t = dot(e2, qv) * idet;
                const uint32_t id = f2u(a.w);
                if (t > 0.0f && t != 3.40282347e+38f && (t < tbest || (t == tbest && id < ibest))) {
                    tbest = t;
                    ibest = id;
                    bu = u;
                    bv = v;
                }
            }
            next = EMPTY_REF;
            continue;
        }
        const uint4* nd = p.nodes + 4 * (size_t)next;
        const uint4 q0 = nd[0], q1 = nd[1], q2 = nd[2], q3 = nd[3];
        if (COUNT) ++c_nodes;
        const float lo0[3] = {u2f(q0.x), u2f(q0.y), u2f(q0.z)}, hi0[3] = {u2f(q0.w), u2f(q1.x), u2f(q1.y)};
        const float lo1[3] = {u2f(q1.z), u2f(q1.w), u2f(q2.x)}, hi1[3] = {u2f(q2.y), u2f(q2.z), u2f(q2.w)};
        float tn0, tn1;
        const bool h0 = child_hit(lo0, hi0, eye, inv, tbest, tn0);
        const bool h1 = child_hit(lo1, hi1, eye, inv, tbest, tn1);
        if (h0 && h1) {
            uint32_t near_ref, far_ref;
            float far_t;
            if (tn1 < tn0) {
                near_ref = q3.y;
                far_ref = q3.x;
                far_t = tn0;
            } else {
                near_ref = q3.x;
                far_ref = q3.y;
                far_t = tn1;
            }
            if (sp < LDS_STACK) {
                s_ref[sp][tid] = far_ref;
                s_t[sp][tid] = far_t;
            } else {
                x_ref[sp - LDS_STACK] = far_ref;
                x_t[sp - LDS_STACK] = far_t;
            }
            ++sp;
            next = near_ref;
        } else if (h0) {
            next = q3.x;
        } else if (h1) {
            next = q3.y;
        } else {
            next = EMPTY_REF;
        }
    }

    const size_t o = (size_t)lr * p.width + x;
    uint32_t packed = MISS_PACKED;
    float nzv = 0.0f;
    if (ibest != NO_TRI) {
        // bmFaceInterpolate<vec3> + normalize + pack (CudaComon.cuh:253-266, BuildTree.cu:489-491)
        const float* n = p.nrm + 9 * (size_t)ibest;
        const float ww = 1.f - (bu + bv);
        const vec3f nn = v3((n[0] * ww + n[3] * bu) + n[6] * bv, (n[1] * ww + n[4] * bu) + n[7] * bv,
                            (n[2] * ww + n[5] * bu) + n[8] * bv);
        const float il = 1.f / sqrtf(dot(nn, nn));
        const float z = nn.z * il;
        const float rr = fabsf(z * 255.f);
        packed = ((rr == rr) ? (uint32_t)rr : 0u) << 16;
        nzv = fabsf(z);
    }
    p.packed[(size_t)lr * p.pitch_u32 + x] = packed;
    p.tri_id[o] = ibest;
    p.t[o] = tbest;
    if (p.nz) p.nz[o] = nzv;
    if (COUNT) {
        atomicAdd(&p.counters[0], c_nodes);
        atomicAdd(&p.counters[1], c_tris);
        if (ibest != NO_TRI) atomicAdd(&p.counters[2], 1ull);
    }
}

__global__ __launch_bounds__(256) void k_clear(uint32_t* buf, uint32_t pitch_u32, uint32_t width, uint32_t height,
                                               uint32_t value) {
    const uint32_t x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
    if (x < width && y < height) buf[(size_t)y * pitch_u32 + x] = value;
}

}  // namespace

hipError_t launch_trace(const TraceParams& p, bool count, hipStream_t s) {
    if (p.width == 0 || p.local_rows == 0) return hipSuccess;
    const dim3 grid((p.width + TILE - 1) / TILE, (p.local_rows + TILE - 1) / TILE);
    if (count) k_trace_primary<true><<<grid, BLOCK, 0, s>>>(p);
    else k_trace_primary<false><<<grid, BLOCK, 0, s>>>(p);
    return hipGetLastError();
}

hipError_t launch_clear(uint32_t* buf, uint32_t pitch_u32, uint32_t width, uint32_t height, uint32_t value,
                        hipStream_t s) {
    if (width == 0 || height == 0) return hipSuccess;
    k_clear<<<dim3((width + 255) / 256, height), 256, 0, s>>>(buf, pitch_u32, width, height, value);
    return hipGetLastError();
}

}  // namespace bm
