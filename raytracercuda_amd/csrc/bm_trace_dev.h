// bm_trace_dev.h — device code of the primary-ray trace, shared by bm_trace.hip (the product
// kernels and their launchers) and bm_trace_ab.hip (trace variants measured slower and kept for A/B
// builds only, -DBM_TRACE_AB=1). Everything here lives in an anonymous namespace:
// each translation unit instantiates the templates it launches.
//
// Semantics: closest hit with t > 0; equal t resolved to the lowest global triangle id (the order
// the reference's serial leaf lists give, BuildTree.cu:419-425); Möller-Trumbore and shading in
// the reference's operation order (CudaComon.cuh:117-155, 253-266). Bit-identical to
// oracle/beam_oracle.c orc_bvh_trace, including the node/triangle counters of the COUNT build.
#pragma once
#include <mutex>
#include <unordered_map>

#include "bm_internal.h"

namespace bm {
namespace {


// Blocks of one kernel the device keeps resident at once (its occupancy x CUs), cached per kernel.
template <typename K>
uint32_t resident_blocks(K kernel, uint32_t block) {
    static std::mutex mu;
    static std::unordered_map<const void*, uint32_t> cache;
    std::lock_guard<std::mutex> lock(mu);
    const void* key = reinterpret_cast<const void*>(kernel);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    int dev = 0, per_cu = 0;
    hipDeviceProp_t prop;
    uint32_t n = 1024;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess &&
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, block, 0) == hipSuccess && per_cu > 0)
        n = (uint32_t)per_cu * (uint32_t)prop.multiProcessorCount;
    cache.emplace(key, n);
    return n;
}

constexpr int BLOCK = 256;
constexpr int WAVES = BLOCK / 64;

// Occupancy knob of the persistent trace kernels (A/B builds: -DBM_TRACE_WAVES_PER_EU=n asks the
// compiler to fit n waves per SIMD).
#ifndef BM_TRACE_WAVES_PER_EU
#define BM_TRACE_WAVES_PER_EU 0
#endif
#if BM_TRACE_WAVES_PER_EU > 0
#define BM_TRACE_OCCUPANCY __attribute__((amdgpu_waves_per_eu(BM_TRACE_WAVES_PER_EU)))
#else
#define BM_TRACE_OCCUPANCY
#endif

typedef float f32x2 __attribute__((ext_vector_type(2)));

enum Ovf { OVF_NONE = 0, OVF_SCRATCH = 1, OVF_GLOBAL = 2 };

// Slab test of one child box, t = (box - o) * inv per plane (the reference's formulation,
// CudaComon.cuh:158-172; an FMA form box*inv - o*inv loses conservativeness for axis-parallel
// rays, inf - inf). A NaN plane (box plane through the eye, parallel ray) leaves that axis
// unconstrained; an all-NaN box never hits.
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

// A global load the compiler cannot merge with an LDS load (see QStack::get); rare path: it waits
// for all of the wave's vector memory operations.
__device__ __forceinline__ uint32_t ovf_load(const uint32_t* ptr) {
    uint32_t v;
    asm volatile("global_load_dword %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(ptr) : "memory");
    return v;
}

template <int LDS_N, int OVF>
struct Stack {
    uint32_t (*s_ref)[BLOCK];
    float (*s_t)[BLOCK];
    int tid;
    // overflow: global [depth][slot] (OVF_GLOBAL) or private (OVF_SCRATCH)
    uint32_t* g_ref;
    float* g_t;
    uint32_t stride;
    uint32_t x_ref[OVF == OVF_SCRATCH ? MAX_STACK - LDS_N : 1];
    float x_t[OVF == OVF_SCRATCH ? MAX_STACK - LDS_N : 1];

    __device__ __forceinline__ void put(int sp, uint32_t ref, float t) {
        if (OVF == OVF_NONE && sp >= LDS_N) return;  // experiment-only variant: drops (never faults)
        if (OVF == OVF_NONE || sp < LDS_N) {
            s_ref[sp][tid] = ref;
            s_t[sp][tid] = t;
        } else if (OVF == OVF_SCRATCH) {
            x_ref[sp - LDS_N] = ref;
            x_t[sp - LDS_N] = t;
        } else {
            g_ref[(size_t)(sp - LDS_N) * stride] = ref;
            g_t[(size_t)(sp - LDS_N) * stride] = t;
        }
    }
    __device__ __forceinline__ void get(int sp, uint32_t& ref, float& t) const {
        if (OVF == OVF_NONE && sp >= LDS_N) {
            ref = EMPTY_REF;
            t = __builtin_inff();
            return;
        }
        if (OVF == OVF_NONE || sp < LDS_N) {
            ref = s_ref[sp][tid];
            t = s_t[sp][tid];
        } else if (OVF == OVF_SCRATCH) {
            ref = x_ref[sp - LDS_N];
            t = x_t[sp - LDS_N];
        } else {
            ref = ovf_load(&g_ref[(size_t)(sp - LDS_N) * stride]);  // not mergeable into a flat load
            t = u2f(ovf_load(reinterpret_cast<const uint32_t*>(&g_t[(size_t)(sp - LDS_N) * stride])));
        }
    }
};

// orient * ray with a glm mat3 (column-major m[c*3+r]; type_mat3x3.inl:427-429 row sums).
__device__ __forceinline__ vec3f orient_mul(const float* m, const vec3f r) {
    return v3((m[0] * r.x + m[3] * r.y) + m[6] * r.z, (m[1] * r.x + m[4] * r.y) + m[7] * r.z,
              (m[2] * r.x + m[5] * r.y) + m[8] * r.z);
}

// Camera::setInitialRays (Camera.cpp:61-66) for pixel (x, gy), then dir = orient * ray.
__device__ __forceinline__ vec3f primary_dir(const TraceParams& p, uint32_t x, uint32_t gy) {
    const float rx = p.rx[x], ry = p.ry[gy];
    const float d = 1.f / sqrtf(p.z2 + rx * rx + ry * ry);
    return orient_mul(p.orient, v3(rx * d, ry * d, p.zoom * d));
}

// Raises the wave's issue priority once it has run `after` traversal steps (wave-uniform count).
// Waves still traversing then hold the frame's critical path (grazing silhouette rays).
// The level is fixed (2): levels 1-3 measured alike, and a runtime level costs a
// chain of scalar compares and branches in every traversal step.
template <uint32_t PRIO_AFTER>
__device__ __forceinline__ void prio_boost(const TraceParams& p, uint32_t& iter) {
    if (PRIO_AFTER) {
        iter = __builtin_amdgcn_readfirstlane(iter) + 1u;
        if (iter == p.prio_after) __builtin_amdgcn_s_setprio(2);
    }
}

// tri_test (Möller-Trumbore with the exact-safe early reject): bm_common.h

// BVH4 node step (128-B record, SoA child boxes): slab-test the four children against [.., tmax],
// return the nearest hit child and push the other hit children farthest first, so they pop nearest
// first. The order is that of the children's order keys (bm_common.h), as in the oracle's
// visit_node, so the traversal (and the COUNT build's counters) match it step for step.
template <typename STACK>
__device__ __forceinline__ uint32_t visit4(const TraceParams& p, uint32_t node, const vec3f o, const vec3f inv,
                                           float tmax, STACK& st, int& sp) {
    const uint4* nd = p.nodes + 8 * (size_t)node;
    const uint4 lx = nd[0], ly = nd[1], lz = nd[2], hx = nd[3], hy = nd[4], hz = nd[5], rf = nd[6];
    const uint32_t LX[4] = {lx.x, lx.y, lx.z, lx.w}, LY[4] = {ly.x, ly.y, ly.z, ly.w}, LZ[4] = {lz.x, lz.y, lz.z, lz.w};
    const uint32_t HX[4] = {hx.x, hx.y, hx.z, hx.w}, HY[4] = {hy.x, hy.y, hy.z, hy.w}, HZ[4] = {hz.x, hz.y, hz.z, hz.w};
    const uint32_t R[4] = {rf.x, rf.y, rf.z, rf.w};
    // branch-free: every test below is a compare + mask, no short-circuit control flow
    // slab distances two children at a time: float2 lanes map onto gfx950's packed f32 add/mul
    // (v_pk_add_f32, v_pk_mul_f32), each element still one IEEE operation
    float tn[4];
    bool h[4];
    const f32x2 ox = {o.x, o.x}, oy = {o.y, o.y}, oz = {o.z, o.z};
    const f32x2 ix = {inv.x, inv.x}, iy = {inv.y, inv.y}, iz = {inv.z, inv.z};
#pragma unroll
    for (int c = 0; c < 4; c += 2) {
        const f32x2 tlx = (f32x2{u2f(LX[c]), u2f(LX[c + 1])} - ox) * ix, thx = (f32x2{u2f(HX[c]), u2f(HX[c + 1])} - ox) * ix;
        const f32x2 tly = (f32x2{u2f(LY[c]), u2f(LY[c + 1])} - oy) * iy, thy = (f32x2{u2f(HY[c]), u2f(HY[c + 1])} - oy) * iy;
        const f32x2 tlz = (f32x2{u2f(LZ[c]), u2f(LZ[c + 1])} - oz) * iz, thz = (f32x2{u2f(HZ[c]), u2f(HZ[c + 1])} - oz) * iz;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            tn[c + k] = fmaxf(fmaxf(fminf(tlx[k], thx[k]), fminf(tly[k], thy[k])), fminf(tlz[k], thz[k]));
            const float tf = fminf(fminf(fmaxf(tlx[k], thx[k]), fmaxf(tly[k], thy[k])), fmaxf(tlz[k], thz[k]));
            h[c + k] = (tn[c + k] <= tf) & (tf >= 0.0f) & (tn[c + k] <= tmax);
        }
    }
    // rank = position in the order of the hit children's keys (order_key; a miss is ~0u)
    uint32_t key[4], rank[4], nh = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        key[c] = h[c] ? order_key(tn[c], (uint32_t)c) : ~0u;
        nh += h[c] ? 1u : 0u;
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        uint32_t r = 0;
#pragma unroll
        for (int d = 0; d < 4; ++d)
            if (d != c) r += key[d] < key[c] ? 1u : 0u;
        rank[c] = r;
    }
#pragma unroll
    for (uint32_t r = 3; r >= 1; --r) {
        uint32_t ref = EMPTY_REF;
        float t = 0.0f;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const bool sel = h[c] & (rank[c] == r);
            ref = sel ? R[c] : ref;
            t = sel ? tn[c] : t;
        }
        if (r < nh) {
            st.put(sp, ref, t);
            ++sp;
        }
    }
    uint32_t next = EMPTY_REF;
#pragma unroll
    for (int c = 0; c < 4; ++c) next = (h[c] & (rank[c] == 0)) ? R[c] : next;
    return next;
}

// Any-hit shadow segment o + s*d, 0 < s < 1 (oracle/beam_oracle.c orc_bvh_shadow, same traversal
// order, so the COUNT build's counters match). Boxes are culled beyond s = 1.
template <bool COUNT, typename STACK, uint32_t PRIO_AFTER, int W>
__device__ __forceinline__ bool shadow_ray(const TraceParams& p, STACK& st, const vec3f o, const vec3f d,
                                           unsigned long long& c_nodes, unsigned long long& c_tris) {
    const vec3f inv = v3(1.f / d.x, 1.f / d.y, 1.f / d.z);
    int sp = 0;
    uint32_t next = 0, iter = 0;
    for (;;) {
        prio_boost<PRIO_AFTER>(p, iter);
        if (next == EMPTY_REF) {
            if (sp == 0) return false;
            --sp;
            float tt;
            st.get(sp, next, tt);
        }
        if (next & LEAF_BIT) {
            const uint32_t first = next & FIRST_MASK, last = first + ((next >> 27) & 15u);
            float4 a = p.tris[3 * first + 0], b = p.tris[3 * first + 1], c = p.tris[3 * first + 2];
            for (uint32_t k = first;; ++k) {
                float4 na = a, nb = b, nc = c;
                if (k < last) {
                    na = p.tris[3 * k + 3];
                    nb = p.tris[3 * k + 4];
                    nc = p.tris[3 * k + 5];
                }
                if (COUNT) ++c_tris;
                float t, u, v;
                if (tri_test(a, b, c, o, d, t, u, v) && t > 0.0f && t < 1.0f) return true;
                if (k >= last) break;
                a = na;
                b = nb;
                c = nc;
            }
            next = EMPTY_REF;
            continue;
        }
        if (COUNT) ++c_nodes;
        if constexpr (W == 4) {
            next = visit4(p, next, o, inv, 1.0f, st, sp);
            continue;
        }
        const uint4* nd = p.nodes + 4 * (size_t)next;
        const uint4 q0 = nd[0], q1 = nd[1], q2 = nd[2], q3 = nd[3];
        const float lo0[3] = {u2f(q0.x), u2f(q0.y), u2f(q0.z)}, hi0[3] = {u2f(q0.w), u2f(q1.x), u2f(q1.y)};
        const float lo1[3] = {u2f(q1.z), u2f(q1.w), u2f(q2.x)}, hi1[3] = {u2f(q2.y), u2f(q2.z), u2f(q2.w)};
        float tn0, tn1;
        const bool h0 = child_hit(lo0, hi0, o, inv, 1.0f, tn0);
        const bool h1 = child_hit(lo1, hi1, o, inv, 1.0f, tn1);
        if (h0 && h1) {
            const bool swap = tn1 < tn0;
            st.put(sp, swap ? q3.x : q3.y, 0.0f);
            ++sp;
            next = swap ? q3.y : q3.x;
        } else if (h0) {
            next = q3.x;
        } else if (h1) {
            next = q3.y;
        } else {
            next = EMPTY_REF;
        }
    }
}

__device__ __forceinline__ uint32_t global_row(const TraceParams& p, uint32_t lr) {
    if (p.band_step == 1 && p.band_first == 0) return lr;  // whole frame: no integer division
    return ((lr / p.band_h) * p.band_step + p.band_first) * p.band_h + lr % p.band_h;
}

template <bool COUNT>
__device__ __forceinline__ void flush_counters(const TraceParams& p, unsigned long long n, unsigned long long t,
                                               unsigned long long h, const unsigned long long (&sh)[3]) {
    if (COUNT) {
        atomicAdd(&p.counters[0], n);
        atomicAdd(&p.counters[1], t);
        atomicAdd(&p.counters[2], h);
        if (p.shadow_counters)
            for (int k = 0; k < 3; ++k) atomicAdd(&p.shadow_counters[k], sh[k]);
    }
}

// Trace one pixel (x, local row lr, global row gy) and write its framebuffer entries; returns hit.
// Shadow modes of the primary kernels: none, fused (the pixel's own thread traces its shadow ray
// right after the primary hit, so shadow work interleaves with primary work over the whole
// persistent grid) or queue (hit pixels compacted for k_shadow_persistent, the wavefront form).
enum ShadowMode { SH_NONE = 0, SH_FUSED = 1, SH_QUEUE = 2 };

// Shadow segment of a primary hit at distance t: origin pulled back towards the eye by
// t * (1 - 1e-4), direction to the light (unnormalised).
__device__ __forceinline__ void shadow_segment(const TraceParams& p, const vec3f eye, const vec3f dir, float t,
                                               vec3f& o, vec3f& d) {
    const float ts = t * 0.9999f;
    o = v3(eye.x + dir.x * ts, eye.y + dir.y * ts, eye.z + dir.z * ts);
    d = v3(p.light[0] - o.x, p.light[1] - o.y, p.light[2] - o.z);
}

template <bool COUNT, typename STACK, uint32_t PRIO_AFTER = 0, int SH = SH_NONE, int W = 2>
__device__ __forceinline__ bool trace_pixel(const TraceParams& p, STACK& st, uint32_t x, uint32_t lr, uint32_t gy,
                                            unsigned long long& c_nodes, unsigned long long& c_tris,
                                            unsigned long long& c_hits, unsigned long long (&c_sh)[3]) {
    const vec3f dir = primary_dir(p, x, gy);
    const vec3f inv = v3(1.f / dir.x, 1.f / dir.y, 1.f / dir.z);
    const vec3f eye = v3(p.eye[0], p.eye[1], p.eye[2]);

    float tbest = __builtin_inff(), bu = 0.f, bv = 0.f;
    uint32_t ibest = NO_TRI;
    int sp = 0;
    uint32_t next = p.num_tris ? 0u : EMPTY_REF;
    uint32_t iter = 0;

    for (;;) {
        prio_boost<PRIO_AFTER>(p, iter);
        if (next == EMPTY_REF) {
            // pop until an entry that can still hold a closer hit
            bool found = false;
            while (sp > 0) {
                --sp;
                uint32_t ref;
                float tt;
                st.get(sp, ref, tt);
                if (!(tt > tbest)) {
                    next = ref;
                    found = true;
                    break;
                }
            }
            if (!found) break;
        }
        if (next & LEAF_BIT) {
            const uint32_t first = next & FIRST_MASK, last = first + ((next >> 27) & 15u);
            // software-pipelined: the next triangle's record is in flight while this one is tested
            float4 a = p.tris[3 * first + 0], b = p.tris[3 * first + 1], c = p.tris[3 * first + 2];
            for (uint32_t k = first;; ++k) {
                float4 na = a, nb = b, nc = c;
                if (k < last) {
                    na = p.tris[3 * k + 3];
                    nb = p.tris[3 * k + 4];
                    nc = p.tris[3 * k + 5];
                }
                if (COUNT) ++c_tris;
                // bmTriIntersect as in tri_test, written out: this form schedules better here
                const vec3f e1 = v3(b.x, b.y, b.z), e2 = v3(c.x, c.y, c.z);
                const vec3f pv = cross(dir, e2);
                const float det = dot(e1, pv);
                const vec3f tv = sub(eye, v3(a.x, a.y, a.z));
                const float un = dot(tv, pv);
                const vec3f qv = cross(tv, e1);
                const float vn = dot(dir, qv);
                const float ra = __builtin_amdgcn_rcpf(det);
                const float ua = un * ra, va = vn * ra;
                const bool far_out =
                    fabsf(det) >= 0x1p-100f &&
                    (ua < -0x1p-10f || ua > 1.0f + 0x1p-10f || va < -0x1p-10f || va + ua > 1.0f + 0x1p-9f);
                if (!far_out) {
                    const float idet = 1.f / det;
                    const float u = un * idet;
                    const float v = vn * idet;
                    if (!(u < 0 || u > 1) && !(v < 0 || v + u > 1)) {
                        const float t = dot(e2, qv) * idet;
                        const uint32_t id = f2u(a.w);
                        if (t > 0.0f && t != 3.40282347e+38f && (t < tbest || (t == tbest && id < ibest))) {
                            tbest = t;
                            ibest = id;
                            bu = u;
                            bv = v;
                        }
                    }
                }
                if (k >= last) break;
                a = na;
                b = nb;
                c = nc;
            }
            next = EMPTY_REF;
            continue;
        }
        if constexpr (W == 4) {
            if (COUNT) ++c_nodes;
            next = visit4(p, next, eye, inv, tbest, st, sp);
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
            const bool swap = tn1 < tn0;
            st.put(sp, swap ? q3.x : q3.y, swap ? tn0 : tn1);
            ++sp;
            next = swap ? q3.y : q3.x;
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
        if (COUNT) ++c_hits;
    }
    p.packed[(size_t)lr * p.pitch_u32 + x] = packed;
    p.tri_id[o] = ibest;
    p.t[o] = tbest;
    if (p.nz) p.nz[o] = nzv;
    if (SH == SH_QUEUE) p.shadow[o] = 0;
    if (SH == SH_FUSED) {
        bool occ = false;
        if (ibest != NO_TRI) {
            vec3f so, sd;
            shadow_segment(p, eye, dir, tbest, so, sd);
            occ = shadow_ray<COUNT, STACK, PRIO_AFTER, W>(p, st, so, sd, c_sh[0], c_sh[1]);
            if (COUNT) c_sh[2] += occ;
        }
        p.shadow[o] = occ ? 1 : 0;
    }
    return ibest != NO_TRI;
}

// Shadow pass input: the hit pixels of a wave are appended to the queue with one atomic per wave
// (ballot + popcount ranks). Queue order varies run to run; each entry's result does not.
__device__ __forceinline__ void enqueue_hit(const TraceParams& p, bool hit, uint32_t pix) {
    const unsigned long long hits = ballot(hit);
    if (!hits) return;
    const int leader = __ffsll((long long)ballot(1)) - 1;
    const uint32_t lane = __lane_id();
    uint32_t base = 0;
    if ((int)lane == leader) base = atomicAdd(p.queue_count, (uint32_t)__popcll(hits));
    base = __shfl(base, leader);
    if (hit) p.queue[base + __popcll(hits & ((1ull << lane) - 1ull))] = pix;
}

// Persistent grid: wave g traces 8x8 tiles g, g + G, g + 2G, ... (G = waves in the grid).
// Dynamic tile scheduling: the wave's next 8x8 tile from the context's ticket counter (one atomic
// per tile). Tickets past the frame's tiles end the wave, so a launch consumes exactly
// tiles + waves tickets and the host advances tile_base by that much.
__device__ __forceinline__ uint32_t next_tile(const TraceParams& p) {
    uint32_t t = 0;
    if (__lane_id() == 0) t = (uint32_t)(atomicAdd(p.tile_ctr, 1ull) - p.tile_base);
    return __builtin_amdgcn_readfirstlane(t);
}

// DIAG (bm_camera_trace_profile, never timed): per wave, s_memrealtime (100 MHz) at start and end,
// (XCC id << 32 | HW_ID) and the sum over its tiles of the tile's longest per-lane work (node
// records + triangle tests; needs COUNT).
template <bool COUNT, int LDS_N, int OVF, uint32_t PRIO = 0, int SH = SH_NONE, int W = 2, bool DYN = false,
          bool DIAG = false>
__global__ __launch_bounds__(BLOCK) BM_TRACE_OCCUPANCY void k_trace_persistent(const TraceParams p) {
    static_assert(!DIAG || COUNT, "the diagnostic build counts work");
    const uint64_t t_start = DIAG ? __builtin_amdgcn_s_memrealtime() : 0;
    uint32_t diag_work = 0;
    __shared__ uint32_t s_ref[LDS_N][BLOCK];
    __shared__ float s_t[LDS_N][BLOCK];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    Stack<LDS_N, OVF> st;
    st.s_ref = s_ref;
    st.s_t = s_t;
    st.tid = tid;
    const uint32_t slot = blockIdx.x * BLOCK + tid;
    st.g_ref = p.ovf_ref + slot;
    st.g_t = p.ovf_t + slot;
    st.stride = p.ovf_stride;
    const uint32_t tiles_x = (p.width + 7) / 8, tiles_y = (p.local_rows + 7) / 8;
    const uint32_t ntiles = tiles_x * tiles_y;
    const uint32_t nwaves = gridDim.x * WAVES;
    unsigned long long cn = 0, ct = 0, ch = 0, csh[3] = {0, 0, 0};
    for (uint32_t i = DYN ? next_tile(p) : blockIdx.x * WAVES + w; i < ntiles;
         i = DYN ? next_tile(p) : i + nwaves) {
        // scramble: tile = i * P mod ntiles (P prime > ntiles: a bijection) spreads the costly
        // tiles of a compact subject evenly over waves, SIMDs and CUs
        const uint32_t t = p.scramble ? (uint32_t)(((uint64_t)i * 2654435761ull) % ntiles) : i;
        const uint32_t x = (t % tiles_x) * 8 + (lane & 7);
        const uint32_t lr = (t / tiles_x) * 8 + (lane >> 3);
        const uint32_t gy = lr < p.local_rows ? global_row(p, lr) : p.height;
        const unsigned long long before = cn + ct;
        if (x < p.width && gy < p.height) {
            __builtin_amdgcn_s_setprio(0);
            const bool hit = trace_pixel<COUNT, decltype(st), PRIO, SH, W>(p, st, x, lr, gy, cn, ct, ch, csh);
            if (SH == SH_QUEUE) enqueue_hit(p, hit, lr * p.width + x);
        }
        if (DIAG) {
            uint32_t wl = (uint32_t)(cn + ct - before);
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) wl = max(wl, (uint32_t)__shfl_xor((int)wl, o));
            diag_work += wl;
        }
    }
    flush_counters<COUNT>(p, cn, ct, ch, csh);
    if (DIAG) {
        const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
        if (lane == 0) {
            // HW_REG_HW_ID (id 4, all 32 bits) and HW_REG_XCC_ID (id 20, bits 3:0)
            const uint32_t hwid = __builtin_amdgcn_s_getreg((31 << 11) | 4);
            const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);
            const size_t wv = (size_t)blockIdx.x * WAVES + w;
            p.diag[4 * wv + 0] = t_start;
            p.diag[4 * wv + 1] = t_end;
            p.diag[4 * wv + 2] = ((uint64_t)xcc << 32) | hwid;
            p.diag[4 * wv + 3] = diag_work;
        }
    }
}

// bmFaceInterpolate<vec3> + normalize + pack (CudaComon.cuh:253-266, BuildTree.cu:489-491): the
// packed framebuffer entry of a hit (red = trunc(|n.z| * 255)); nzv receives |n.z|.
// bmFaceInterpolate<vec3> + normalize + pack (CudaComon.cuh:253-266, BuildTree.cu:489-491) of the
// corner normals n[9] at (bu, bv): the packed colour, z = the normalised n.z.
__device__ __forceinline__ uint32_t shade_normals(const float* n, float bu, float bv, float& z) {
    const float ww = 1.f - (bu + bv);
    const vec3f nn = v3((n[0] * ww + n[3] * bu) + n[6] * bv, (n[1] * ww + n[4] * bu) + n[7] * bv,
                        (n[2] * ww + n[5] * bu) + n[8] * bv);
    const float il = 1.f / sqrtf(dot(nn, nn));
    z = nn.z * il;
    const float rr = fabsf(z * 255.f);
    return ((rr == rr) ? (uint32_t)rr : 0u) << 16;
}

__device__ __forceinline__ uint32_t shade_hit(const TraceParams& p, uint32_t id, float bu, float bv, float& nzv) {
    float z;
    const uint32_t packed = shade_normals(p.nrm + 9 * (size_t)id, bu, bv, z);
    nzv = fabsf(z);
    return packed;
}

// ---- ray quads: four lanes per ray over the BVH4 --------------------------------------------------
// A wave traces a 4x4 pixel tile: lane 4q+c works for ray q. At a node lane c slab-tests child c
// (one dword of each SoA plane: the quad's four loads hit one 16-B segment); at a leaf lane c tests
// triangles first+c, first+c+4, ... Ranks, the nearest child and the closest hit are combined
// across the quad with DPP quad permutations, so every lane of a quad holds the same ray state
// (next, sp, tbest, ibest, u, v) and the quad's control flow is uniform. Per ray a node step costs
// about a third of the single-lane step's instructions and a leaf of up to four triangles one
// triangle test, so the grazing rays that set the frame time (SURVEY §8(a) a4's hot loop, the
// critical path of the heaviest 8x8 tiles) finish in a fraction of the dependent steps. The
// traversal order (stable nearest-first child order, pop-skip of entries beyond tbest) and
// therefore the COUNT build's counters are exactly those of trace_pixel / orc_bvh_trace.
constexpr int QRAYS = BLOCK / 4;  // rays per workgroup
constexpr uint32_t LPT_MAX = 128;  // tiles of one workgroup's share the cost-ordered schedule sorts
// Cost-ordered scheduling needs every share (tiles b, b + B, ... in the XCD-aware order) to fit LPT_MAX.
__host__ __device__ __forceinline__ bool lpt_share_fits(uint32_t ntiles, uint32_t blocks) {
    return blocks >= 8 && (blocks & 7u) == 0 && (ntiles + blocks - 1) / blocks + 8 <= LPT_MAX;
}

#ifndef BM_QUAD_WAVES
#define BM_QUAD_WAVES 7  // waves per SIMD the quad kernels' registers must allow (72 VGPRs; 8 measured slower)
#endif
#ifndef BM_QUAD_WAVES_FUSED
#define BM_QUAD_WAVES_FUSED 7  // with fused shadow rays (6 waves: 80 VGPRs, measured 6-10 % slower)
#endif
// Pixel tile of one wave of the quad kernel (16 rays): QTW x QTH. 4x4 (default) writes each plane
// row as 16-B pieces that L2 merges only partly (WRITE_SIZE 1.58x the planes' bytes); 8x2 writes
// 32-B pieces (1.26x) but its rays are less coherent: 4-14 % slower.
#ifndef BM_QUAD_TW
#define BM_QUAD_TW 4
#endif
// Cost-ordered schedule keyed by run cost (1): a run (8 horizontally adjacent tiles, one 128-B line
// per row of each 4-B plane) is dealt to 8 workgroups of one XCD, tile j to the j-th; when each of
// them orders its share by its own tiles' costs (0), a run's tiles complete at different times and the
// L2 writes its lines back in pieces (WRITE_SIZE 1.56x the planes' bytes on C2). Keyed by the run's
// summed cost, the 8 workgroups order their shares alike and a run's tiles complete together.
#ifndef BM_QUAD_RUN_COST
#define BM_QUAD_RUN_COST 1
#endif
#ifndef BM_QUAD_RUN_BLOCK
#define BM_QUAD_RUN_BLOCK 0
#endif
constexpr uint32_t QTW = BM_QUAD_TW, QTH = 16 / BM_QUAD_TW;
static_assert(QTW * QTH == 16, "a wave traces 16 rays");
#ifndef BM_QUAD_LDS
#define BM_QUAD_LDS 24
#endif
constexpr int QUAD_LDS = BM_QUAD_LDS;      // LDS stack entries per ray (>= the fallback's 12: the overflow area fits both)
// LDS-staged leaf triangle tiles (A/B experiment, -DBM_QUAD_LEAF_LDS=1): the quad loads the up to four
// triangle records of a leaf group as twelve contiguous 16-B pieces (lane c: pieces c, c+4, c+8, so
// each load instruction reads one contiguous 64-B run per quad), stages them in LDS and reads back its
// own triangle's three pieces. Measured against per-lane record loads in DESIGN.md §5.
#ifndef BM_QUAD_VISITS
#define BM_QUAD_VISITS 2  // quad_closest: node visits per loop iteration while the nearest child is internal (3, 4: within 1 % in flight, single frame 1-2 % slower)
#endif
#ifndef BM_QUAD_LEAF_LDS
#define BM_QUAD_LEAF_LDS 0
#endif

template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return i2f(__builtin_amdgcn_mov_dpp(f2i(v), CTRL, 0xF, 0xF, true));
}
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
}
constexpr int QP_X1 = 0xB1;  // quad_perm [1,0,3,2]: lane c reads lane c^1
constexpr int QP_X2 = 0x4E;  // quad_perm [2,3,0,1]: lane c^2
constexpr int QP_X3 = 0x1B;  // quad_perm [3,2,1,0]: lane c^3

// Lexicographic (t, id) minimum of the quad's candidates; u, v travel with the winner.
template <int CTRL>
__device__ __forceinline__ void quad_min_step(float& t, uint32_t& id, float& u, float& v) {
    const float ot = dpp_f<CTRL>(t), ou = dpp_f<CTRL>(u), ov = dpp_f<CTRL>(v);
    const uint32_t oid = dpp_u<CTRL>(id);
    const bool take = ot < t || (ot == t && oid < id);
    t = take ? ot : t;
    id = take ? oid : id;
    u = take ? ou : u;
    v = take ? ov : v;
}
__device__ __forceinline__ void quad_min_hit(float& t, uint32_t& id, float& u, float& v) {
    quad_min_step<QP_X1>(t, id, u, v);
    quad_min_step<QP_X2>(t, id, u, v);
}

// Per-ray stack of a quad: LDS [depth][ray] of (ref, t) pairs below LDS_N (one 8-B read or write
// per entry), the global overflow area beyond. All four lanes pop the same entry (an LDS
// broadcast); a push is written by the lane that owns the child.
template <int LDS_N, int RAYS = QRAYS>
struct QStack {
    uint2 (*s)[RAYS];
    int ray;
    uint32_t* g_ref;  // overflow area bases (wave-uniform: kept in SGPRs) ...
    float* g_t;
    uint32_t slot;    // ... and this ray's slot in them (one VGPR instead of two 64-bit pointers)
    uint32_t stride;
#if BM_QUAD_LEAF_LDS
    float4* lt;       // this ray's 12-piece leaf tile in LDS (BM_QUAD_LEAF_LDS)
#endif
    __device__ __forceinline__ void put(int sp, uint32_t ref, float t) const {
        if (sp < LDS_N) {
            s[sp][ray] = make_uint2(ref, f2u(t));
        } else {
            g_ref[(size_t)(sp - LDS_N) * stride + slot] = ref;
            g_t[(size_t)(sp - LDS_N) * stride + slot] = t;
        }
    }
    // The overflow side reads through an opaque global load (ovf_load): with plain loads the
    // compiler merges the two sides into one flat load through a selected pointer, and a flat load
    // waits on vmcnt(0) and lgkmcnt(0) — every pop would wait for all of the wave's outstanding
    // global memory traffic instead of one LDS read.
    __device__ __forceinline__ void get(int sp, uint32_t& ref, float& t) const {
        if (sp < LDS_N) {
            const uint2 e = s[sp][ray];
            ref = e.x;
            t = u2f(e.y);
        } else {
            ref = ovf_load(&g_ref[(size_t)(sp - LDS_N) * stride + slot]);
            t = u2f(ovf_load(reinterpret_cast<const uint32_t*>(&g_t[(size_t)(sp - LDS_N) * stride + slot])));
        }
    }
};

// Quad node step: lane c slab-tests child c of the 128-B record against [.., tmax]; the hit
// children are ranked by their order keys (order_key: entry distance, then slot), ranks 1..nh-1
// pushed farthest first (rank r at sp + nh-1-r) with push_t(tn) as their stack key, and the rank-0
// child returned to all four lanes (EMPTY_REF when nothing is hit) — visit4's order exactly.
// VALU economy (the quad kernels are issue-bound): the record is addressed by a
// 32-bit offset from the node base (one shift), the lo/hi planes of an axis go through packed f32
// subtract/multiply (each element one IEEE operation, as in the scalar form), a rank is three
// unsigned compares of DPP-exchanged keys, and the quad's hit count is the minimum over the quad of
// (hit ? 4 : rank) — a missing child's key ~0u ranks after every hit, so its rank is the hit count.
template <typename QS>
__device__ __forceinline__ uint32_t quad_visit(const TraceParams& p, uint32_t node, int c,
                                               const vec3f o, const vec3f inv, float tmax, bool key_t, const QS& st,
                                               int& sp) {
    const uint32_t* nd = reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(p.nodes) +
                                                           ((node << 7) | ((uint32_t)c << 2)));
    const f32x2 bx = {u2f(nd[0]), u2f(nd[12])}, by = {u2f(nd[4]), u2f(nd[16])}, bz = {u2f(nd[8]), u2f(nd[20])};
    const uint32_t ref = nd[24];
    const f32x2 tx = (bx - f32x2{o.x, o.x}) * f32x2{inv.x, inv.x};
    const f32x2 ty = (by - f32x2{o.y, o.y}) * f32x2{inv.y, inv.y};
    const f32x2 tz = (bz - f32x2{o.z, o.z}) * f32x2{inv.z, inv.z};
    const float tn = fmaxf(fmaxf(fminf(tx.x, tx.y), fminf(ty.x, ty.y)), fminf(tz.x, tz.y));
    const float tf = fminf(fminf(fmaxf(tx.x, tx.y), fmaxf(ty.x, ty.y)), fmaxf(tz.x, tz.y));
    const bool h = (tn <= tf) & (tf >= 0.0f) & (tn <= tmax);
    const uint32_t key = h ? order_key(tn, (uint32_t)c) : ~0u;
    const uint32_t k1 = dpp_u<QP_X1>(key), k2 = dpp_u<QP_X2>(key), k3 = dpp_u<QP_X3>(key);
    const uint32_t rank = (uint32_t)(k1 < key) + (uint32_t)(k2 < key) + (uint32_t)(k3 < key);
    uint32_t nh = h ? 4u : rank;
    nh = min(nh, dpp_u<QP_X1>(nh));
    nh = min(nh, dpp_u<QP_X2>(nh));
    if (h && rank > 0) st.put(sp + (int)(nh - 1u - rank), ref, key_t ? tn : 0.0f);
    sp += max((int)nh - 1, 0);
    uint32_t nx = (h && rank == 0) ? ref : EMPTY_REF;
    nx = min(nx, dpp_u<QP_X1>(nx));
    nx = min(nx, dpp_u<QP_X2>(nx));
    return nx;
}

// BVH8 quad node step (256-B records, oracle width 8): lane c holds children 2c and 2c+1 — adjacent
// dwords of every SoA plane, one 8-B load per plane, the two slabs in packed f32 — and ranks each
// among all eight by order_key8 (the three partners' two keys by DPP). Positions, hit count and the
// next child as in quad_visit.
__device__ __forceinline__ uint32_t order_key8(float tn, uint32_t slot) {
    const int32_t b = f2i(tn) > 0 ? f2i(tn) : 0;
    return ((uint32_t)b & ~7u) | slot;
}

template <typename QS>
__device__ __forceinline__ uint32_t quad_visit8(const TraceParams& p, uint32_t node, int c, const vec3f o,
                                                const vec3f inv, float tmax, bool key_t, const QS& st, int& sp) {
    const uint2* nd = reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(p.nodes) + ((size_t)node << 8)) + c;
    const uint2 lxp = nd[0], lyp = nd[4], lzp = nd[8], hxp = nd[12], hyp = nd[16], hzp = nd[20], rp = nd[24];
    const f32x2 ox = {o.x, o.x}, oy = {o.y, o.y}, oz = {o.z, o.z};
    const f32x2 ix = {inv.x, inv.x}, iy = {inv.y, inv.y}, iz = {inv.z, inv.z};
    const f32x2 tlx = (f32x2{u2f(lxp.x), u2f(lxp.y)} - ox) * ix, thx = (f32x2{u2f(hxp.x), u2f(hxp.y)} - ox) * ix;
    const f32x2 tly = (f32x2{u2f(lyp.x), u2f(lyp.y)} - oy) * iy, thy = (f32x2{u2f(hyp.x), u2f(hyp.y)} - oy) * iy;
    const f32x2 tlz = (f32x2{u2f(lzp.x), u2f(lzp.y)} - oz) * iz, thz = (f32x2{u2f(hzp.x), u2f(hzp.y)} - oz) * iz;
    const float tna = fmaxf(fmaxf(fminf(tlx.x, thx.x), fminf(tly.x, thy.x)), fminf(tlz.x, thz.x));
    const float tfa = fminf(fminf(fmaxf(tlx.x, thx.x), fmaxf(tly.x, thy.x)), fmaxf(tlz.x, thz.x));
    const float tnb = fmaxf(fmaxf(fminf(tlx.y, thx.y), fminf(tly.y, thy.y)), fminf(tlz.y, thz.y));
    const float tfb = fminf(fminf(fmaxf(tlx.y, thx.y), fmaxf(tly.y, thy.y)), fmaxf(tlz.y, thz.y));
    const bool ha = (tna <= tfa) & (tfa >= 0.0f) & (tna <= tmax);
    const bool hb = (tnb <= tfb) & (tfb >= 0.0f) & (tnb <= tmax);
    const uint32_t ka = ha ? order_key8(tna, 2u * (uint32_t)c) : ~0u;
    const uint32_t kb = hb ? order_key8(tnb, 2u * (uint32_t)c + 1u) : ~0u;
    const uint32_t a1 = dpp_u<QP_X1>(ka), a2 = dpp_u<QP_X2>(ka), a3 = dpp_u<QP_X3>(ka);
    const uint32_t b1 = dpp_u<QP_X1>(kb), b2 = dpp_u<QP_X2>(kb), b3 = dpp_u<QP_X3>(kb);
    const uint32_t ra = (uint32_t)(kb < ka) + (uint32_t)(a1 < ka) + (uint32_t)(a2 < ka) + (uint32_t)(a3 < ka) +
                        (uint32_t)(b1 < ka) + (uint32_t)(b2 < ka) + (uint32_t)(b3 < ka);
    const uint32_t rb = (uint32_t)(ka < kb) + (uint32_t)(a1 < kb) + (uint32_t)(a2 < kb) + (uint32_t)(a3 < kb) +
                        (uint32_t)(b1 < kb) + (uint32_t)(b2 < kb) + (uint32_t)(b3 < kb);
    // hit count: a missing child's key ~0u ranks after every hit, so its rank is the hit count
    uint32_t nh = min(ha ? 8u : ra, hb ? 8u : rb);
    nh = min(nh, dpp_u<QP_X1>(nh));
    nh = min(nh, dpp_u<QP_X2>(nh));
    if (ha && ra > 0) st.put(sp + (int)(nh - 1u - ra), rp.x, key_t ? tna : 0.0f);
    if (hb && rb > 0) st.put(sp + (int)(nh - 1u - rb), rp.y, key_t ? tnb : 0.0f);
    sp += max((int)nh - 1, 0);
    uint32_t nx = (ha && ra == 0) ? rp.x : ((hb && rb == 0) ? rp.y : EMPTY_REF);
    nx = min(nx, dpp_u<QP_X1>(nx));
    nx = min(nx, dpp_u<QP_X2>(nx));
    return nx;
}

template <int BW, typename QS>
__device__ __forceinline__ uint32_t quad_visit_w(const TraceParams& p, uint32_t node, int c, const vec3f o,
                                                 const vec3f inv, float tmax, bool key_t, const QS& st, int& sp) {
    if constexpr (BW == 8) return quad_visit8(p, node, c, o, inv, tmax, key_t, st, sp);
    else return quad_visit(p, node, c, o, inv, tmax, key_t, st, sp);
}

// Closest hit of one ray over the quad (trace_pixel's loop): t > 0, ties to the lowest id.
template <bool COUNT, uint32_t PRIO, typename QS, int BW = 4>
__device__ __forceinline__ void quad_closest(const TraceParams& p, const QS& st, int c,
                                             const vec3f eye, const vec3f dir, const vec3f inv, float& tbest,
                                             uint32_t& ibest, float& bu, float& bv, unsigned long long& cn,
                                             unsigned long long& ct) {
    // One iteration: the pending leaf (if any), then the pop that follows it, then the node visit —
    // a leaf and the next node share an iteration (one loop overhead and one divergent pass fewer
    // per leaf); the per-ray sequence of leaf tests, pops and node visits is trace_pixel's.
    int sp = 0;
    uint32_t next = p.num_tris ? 0u : EMPTY_REF;
    uint32_t iter = 0;
    for (;;) {
        prio_boost<PRIO>(p, iter);
        if (next != EMPTY_REF && (next & LEAF_BIT)) {
            const uint32_t first = next & FIRST_MASK, cnt = ((next >> 27) & 15u) + 1u;
            for (uint32_t k0 = 0; k0 < cnt; k0 += 4) {
                const uint32_t k = first + k0 + c;
                float t = __builtin_inff(), u = 0.f, v = 0.f;
                uint32_t id = NO_TRI;
#if BM_QUAD_LEAF_LDS
                {  // the group's pieces, contiguous per load instruction, through this ray's LDS tile
                    const uint32_t np = 3 * min(4u, cnt - k0);
                    const float4* src = p.tris + 3 * (size_t)(first + k0);
#pragma unroll
                    for (uint32_t j = 0; j < 3; ++j)
                        if (4 * j + c < np) st.lt[4 * j + c] = src[4 * j + c];
                }
#endif
                if (k0 + c < cnt) {
#if BM_QUAD_LEAF_LDS
                    const float4 a = st.lt[3 * c + 0], b = st.lt[3 * c + 1], cc = st.lt[3 * c + 2];
#else
                    const float4 a = p.tris[3 * k + 0], b = p.tris[3 * k + 1], cc = p.tris[3 * k + 2];
#endif
                    float tt, uu, vv;
                    if (tri_test(a, b, cc, eye, dir, tt, uu, vv) && tt > 0.0f && tt != 3.40282347e+38f) {
                        t = tt;
                        id = f2u(a.w);
                        u = uu;
                        v = vv;
                    }
                }
                quad_min_hit(t, id, u, v);
                if (t < tbest || (t == tbest && id < ibest)) {
                    tbest = t;
                    ibest = id;
                    bu = u;
                    bv = v;
                }
            }
            if (COUNT && c == 0) ct += cnt;
            next = EMPTY_REF;
        }
        if (next == EMPTY_REF) {
            bool found = false;
            while (sp > 0) {
                --sp;
                uint32_t ref;
                float tt;
                st.get(sp, ref, tt);
                if (!(tt > tbest)) {
                    next = ref;
                    found = true;
                    break;
                }
            }
            if (!found) break;
            if (next & LEAF_BIT) continue;  // a popped leaf: tested at the top of the next iteration
        }
        if (COUNT && c == 0) ++cn;
        next = quad_visit_w<BW>(p, next, c, eye, inv, tbest, true, st, sp);
        // more node visits in the same iteration while the nearest child is internal (same
        // sequence; a second visit halved the loop overhead on descents: armadillo proxy -3 %, merged
        // proxy -9 %)
#pragma unroll
        for (int extra = 1; extra < BM_QUAD_VISITS; ++extra) {
            if (next == EMPTY_REF || (next & LEAF_BIT)) break;
            if (COUNT && c == 0) ++cn;
            next = quad_visit_w<BW>(p, next, c, eye, inv, tbest, true, st, sp);
        }
    }
}

// Any-hit segment o + s*d, 0 < s < 1 (shadow_ray's loop). Within a leaf the triangles are tested
// four at a time; the counter takes the tests up to the first occluder in leaf order, as the
// sequential loop of orc_bvh_shadow stops there.
template <bool COUNT, uint32_t PRIO, typename QS, int BW = 4>
__device__ __forceinline__ bool quad_anyhit(const TraceParams& p, const QS& st, int c,
                                            const vec3f o, const vec3f d, unsigned long long& cn,
                                            unsigned long long& ct) {
    const vec3f inv = v3(1.f / d.x, 1.f / d.y, 1.f / d.z);
    int sp = 0;
    uint32_t next = 0, iter = 0;
    for (;;) {  // leaf, pop, node visit in one iteration, as in quad_closest
        prio_boost<PRIO>(p, iter);
        if (next != EMPTY_REF && (next & LEAF_BIT)) {
            const uint32_t first = next & FIRST_MASK, cnt = ((next >> 27) & 15u) + 1u;
            for (uint32_t k0 = 0; k0 < cnt; k0 += 4) {
                const uint32_t k = first + k0 + c;
                uint32_t occ_at = 4;  // slot of the first occluder in this group of four
                if (k0 + c < cnt) {
                    float t, u, v;
                    if (tri_test(p.tris[3 * k + 0], p.tris[3 * k + 1], p.tris[3 * k + 2], o, d, t, u, v) &&
                        t > 0.0f && t < 1.0f)
                        occ_at = (uint32_t)c;
                }
                occ_at = min(occ_at, dpp_u<QP_X1>(occ_at));
                occ_at = min(occ_at, dpp_u<QP_X2>(occ_at));
                if (occ_at < 4) {
                    if (COUNT && c == 0) ct += occ_at + 1;
                    return true;
                }
                if (COUNT && c == 0) ct += min(4u, cnt - k0);
            }
            next = EMPTY_REF;
        }
        if (next == EMPTY_REF) {
            if (sp == 0) return false;
            --sp;
            float tt;
            st.get(sp, next, tt);
            if (next & LEAF_BIT) continue;  // a popped leaf: tested at the top of the next iteration
        }
        if (COUNT && c == 0) ++cn;
        next = quad_visit_w<BW>(p, next, c, o, inv, 1.0f, false, st, sp);
        if (next != EMPTY_REF && !(next & LEAF_BIT)) {  // second node visit, as in quad_closest
            if (COUNT && c == 0) ++cn;
            next = quad_visit_w<BW>(p, next, c, o, inv, 1.0f, false, st, sp);
        }
    }
}

template <bool COUNT, int LDS_N, uint32_t PRIO, int SH, bool DIAG = false, int BW = 4>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(COUNT ? 1 : SH == SH_FUSED ? BM_QUAD_WAVES_FUSED
                                                                                               : BM_QUAD_WAVES))) void
k_trace_quad(const TraceParams p) {
    static_assert(SH == SH_NONE || SH == SH_FUSED, "quad kernel: primary or fused shadow rays");
    static_assert(!DIAG || COUNT, "the diagnostic build counts work");
    const uint64_t t_start = DIAG ? __builtin_amdgcn_s_memrealtime() : 0;
    uint64_t diag_work = 0;
    __shared__ uint2 s_stk[LDS_N][QRAYS];
#if BM_QUAD_LEAF_LDS
    __shared__ float4 s_lt[QRAYS][12];
#endif
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int c = lane & 3, q = lane >> 2;
    QStack<LDS_N> st;
    st.s = s_stk;
#if BM_QUAD_LEAF_LDS
    st.lt = s_lt[w * 16 + q];
#endif
    st.ray = w * 16 + q;
    const uint32_t slot = blockIdx.x * QRAYS + st.ray;
    st.g_ref = p.ovf_ref;
    st.g_t = p.ovf_t;
    st.slot = slot;
    st.stride = p.ovf_stride;
    const uint32_t tiles_x = (p.width + QTW - 1) / QTW, tiles_y = (p.local_rows + QTH - 1) / QTH;
    const uint32_t ntiles = tiles_x * tiles_y;
    const uint32_t nwaves = gridDim.x * WAVES;
    const vec3f eye = v3(p.eye[0], p.eye[1], p.eye[2]);
    unsigned long long cn = 0, ct = 0, ch = 0, csh[3] = {0, 0, 0};
    // Tile order. Static: wave g of the grid takes tiles g, g + G, ... (G = waves in the grid).
    // Block-dynamic (p.sched == 1): the block's share of the frame — tiles b, b + B, b + 2B, ...
    // (B = blocks), in screen order — is handed to its four waves one tile at a time from an LDS
    // ticket, so a wave that drew a heavy (silhouette) tile does not also own its fixed share of
    // the rest: list scheduling inside the CU, no global atomics.
    // XCD-aware: with a grid that is a multiple of 8 blocks (blocks are placed on the 8 XCDs round
    // robin, block b on XCD b % 8) runs of 8 horizontally adjacent tiles (32 pixels = one 128-B line
    // per row of each 4-B plane) belong to one XCD, so partial lines merge in that XCD's L2 before
    // they are written back; the XCD's runs are dealt to its blocks tile by tile.
    // Cost-ordered (p.sched == 2, p.tile_cost): the block's share is handed out longest first, by
    // the time each tile took in the previous trace of this render target (LPT list scheduling;
    // tile_cost holds it, in 10-ns s_memrealtime ticks, rewritten as the tiles complete). The heavy
    // silhouette tiles then start first instead of whenever screen order reaches them. First trace
    // (all costs zero): screen order. Frames do not depend on the order.
    __shared__ uint32_t s_ticket;
    __shared__ uint32_t s_order[LPT_MAX];
    const bool dyn = p.sched >= 1;
    const bool xcd_map = dyn && (gridDim.x & 7u) == 0;
    const uint32_t xcd = blockIdx.x & 7u, xj = blockIdx.x >> 3, xblocks = gridDim.x >> 3;
    auto tile_of = [&](uint32_t k) -> uint32_t {
        if (!xcd_map) return blockIdx.x + k * gridDim.x;
        // this XCD's local tile: tile by tile over its blocks, or (BM_QUAD_RUN_BLOCK = G) G adjacent tiles
        // to one block's four waves (G = 8: a run, whose lines one CU then writes within about two tiles' time)
        constexpr uint32_t G = BM_QUAD_RUN_BLOCK;  // tiles per group dealt to one block (8: a run)
        const uint32_t l = G ? G * (xj + (k / G) * xblocks) + (k % G) : xj + k * xblocks;
        return 8u * (xcd + 8u * (l >> 3)) + (l & 7u);
    };
    const bool lpt = p.sched == 2 && p.tile_cost != nullptr && lpt_share_fits(ntiles, gridDim.x);
    if (lpt) {  // sort the share by descending cost (bitonic, in LDS; key = cost << 9 | (511 - k))
        // run-cost keys need the 8 workgroups of a run to share their share indices (xblocks % 8 == 0)
        const bool run_cost = BM_QUAD_RUN_COST && (BM_QUAD_RUN_BLOCK || (xblocks & 7u) == 0);
        for (uint32_t k = tid; k < LPT_MAX; k += BLOCK) {
            const uint32_t tk = tile_of(k);
            uint32_t cst = 0u;
            if (tk < ntiles) {
                if (run_cost) {  // the run's tiles: tk & ~7 .. (tk | 7), those inside the frame
                    for (uint32_t j = tk & ~7u; j <= (tk | 7u) && j < ntiles; ++j) cst += min(p.tile_cost[j], (1u << 18) - 1u);
                    cst = min(cst, (1u << 22) - 2u) + 1u;
                } else {
                    cst = min(p.tile_cost[tk], (1u << 22) - 1u) + 1u;
                }
            }
            s_order[k] = (cst << 9) | (LPT_MAX - 1u - k);
        }
        __syncthreads();
        for (uint32_t size = 2; size <= LPT_MAX; size <<= 1)
            for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
                for (uint32_t k = tid; k < LPT_MAX; k += BLOCK) {
                    const uint32_t o = k ^ stride;
                    if (o > k) {
                        const uint32_t a = s_order[k], b = s_order[o];
                        const bool desc = (k & size) == 0;  // descending runs first: final order descending
                        if (desc ? a < b : a > b) {
                            s_order[k] = b;
                            s_order[o] = a;
                        }
                    }
                }
                __syncthreads();
            }
        for (uint32_t k = tid; k < LPT_MAX; k += BLOCK) s_order[k] = LPT_MAX - 1u - (s_order[k] & (LPT_MAX - 1u));
    }
    auto pick = [&](uint32_t r) -> uint32_t { return tile_of(lpt ? (r < LPT_MAX ? s_order[r] : LPT_MAX) : r); };
    if (tid == 0) s_ticket = WAVES;
    __syncthreads();
    for (uint32_t i = dyn ? pick((uint32_t)w) : blockIdx.x * WAVES + w; i < ntiles;) {
        uint32_t knext = 0;
        if (dyn) {
            if (lane == 0) knext = atomicAdd(&s_ticket, 1u);
            knext = __builtin_amdgcn_readfirstlane(knext);
        }
        const uint32_t tile = i;
        const uint32_t x = (i % tiles_x) * QTW + (q % QTW);
        const uint32_t lr = (i / tiles_x) * QTH + (q / QTW);
        const uint32_t gy = lr < p.local_rows ? global_row(p, lr) : p.height;
        i = dyn ? pick(knext) : i + nwaves;
        if (x >= p.width || gy >= p.height) continue;  // whole quads only
        const uint64_t tile_t0 = lpt ? __builtin_amdgcn_s_memrealtime() : 0;
        __builtin_amdgcn_s_setprio(0);
        const vec3f dir = primary_dir(p, x, gy);
        float tbest = __builtin_inff(), bu = 0.f, bv = 0.f;
        uint32_t ibest = NO_TRI;
        const vec3f inv = v3(1.f / dir.x, 1.f / dir.y, 1.f / dir.z);
        const unsigned long long before_work = cn + ct;
        quad_closest<COUNT, PRIO, QStack<LDS_N>, BW>(p, st, c, eye, dir, inv, tbest, ibest, bu, bv, cn, ct);
        if (DIAG) {  // the tile's longest ray (node records + triangle tests), summed per wave
            uint32_t wl = (uint32_t)(cn + ct - before_work);
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) wl = max(wl, (uint32_t)__shfl_xor((int)wl, o));
            diag_work += wl;
        }
        // 32-bit pixel offset (planes hold < 2^32 pixels): one VGPR live across the fused shadow ray
        const uint32_t o32 = lr * p.width + x;
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
            if (COUNT && c == 0) ++ch;
        }
        // one plane per lane of the quad
        if (c == 0) p.packed[(size_t)lr * p.pitch_u32 + x] = packed;
        else if (c == 1) p.tri_id[o32] = ibest;
        else if (c == 2) p.t[o32] = tbest;
        else if (p.nz) p.nz[o32] = nzv;
        if (SH == SH_FUSED) {
            bool occ = false;
            if (ibest != NO_TRI) {
                vec3f so, sd;
                shadow_segment(p, eye, dir, tbest, so, sd);
                occ = quad_anyhit<COUNT, PRIO, QStack<LDS_N>, BW>(p, st, c, so, sd, csh[0], csh[1]);
                if (COUNT && c == 0) csh[2] += occ;
            }
            // one byte per quad (measured, round 4: the tile row's four flags as one aligned 4-B store
            // cost three VGPR spills at 7 waves per SIMD, and the scratch traffic outweighed the stores
            // it saved — WRITE_SIZE 61.4 -> 73.2 MB per C5 frame, the same with no shadow store at all)
            if (c == 0) p.shadow[o32] = occ ? 1 : 0;
        }
        if (lpt && lane == 0) p.tile_cost[tile] = (uint32_t)(__builtin_amdgcn_s_memrealtime() - tile_t0);
    }
    flush_counters<COUNT>(p, cn, ct, ch, csh);
    if (DIAG) {
        const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
        if (lane == 0) {
            const uint32_t hwid = __builtin_amdgcn_s_getreg((31 << 11) | 4);
            const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);
            const size_t wv = (size_t)blockIdx.x * WAVES + w;
            p.diag[4 * wv + 0] = t_start;
            p.diag[4 * wv + 1] = t_end;
            p.diag[4 * wv + 2] = ((uint64_t)xcc << 32) | hwid;
            p.diag[4 * wv + 3] = diag_work;
        }
    }
}

// Compacted ray quads (TRACE_COMPACT, two launches). k_cull runs one lane per pixel over 8x8 tiles:
// the ray setup and a conservative slab test against the root record's four child boxes (inflated,
// see k_cull). A ray that misses all of them is finished exactly as the quad traversal would finish
// it (no child pushed, empty stack): its own lane writes its miss entries. The others are appended
// to their region of the ray queue (a region = a run of consecutive tiles owned by one workgroup;
// wave ballot + popcount rank and one LDS atomic per wave, no global atomics), and the region's
// count is published. k_trace_rays is persistent: each workgroup scans the region counts in LDS,
// and wave w traces the survivors 16 at a time as ray quads (quad_closest, from the root), batches
// w, w + G, w + 2G, ... of the concatenated queue, so quads are only spent on rays that enter the
// scene and the hard rays are spread over every wave. Frames and COUNT counters are those of
// k_trace_quad / orc_bvh_trace (a culled ray counts the one root record the quad traversal visits).
// Measured: on par with k_trace_quad — the survivors' traversal steps, not the
// culled rays, set the frame time.
constexpr int CULL_TILE = 8;
#ifndef BM_CULL_MAX_REGIONS
#define BM_CULL_MAX_REGIONS 1024  // 1024 vs 2048: shorter prefix scan, C2/C3 in flight +1-2 %
#endif
constexpr uint32_t CULL_MAX_REGIONS = BM_CULL_MAX_REGIONS;  // LDS prefix table of k_trace_rays (4 B each)
#ifndef BM_RAYS_SEARCH64
#define BM_RAYS_SEARCH64 1  // k_trace_rays: a batch's region by a two-level 64-ary ballot search (0: binary)
#endif

template <bool COUNT, int SH>
__global__ __launch_bounds__(BLOCK) void k_cull(const TraceParams p) {
    __shared__ uint32_t s_n;
    const int tid = threadIdx.x, w = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    if (tid == 0) s_n = 0;
    __syncthreads();
    const uint32_t tiles_x = (p.width + CULL_TILE - 1) / CULL_TILE;
    const uint32_t ntiles = tiles_x * ((p.local_rows + CULL_TILE - 1) / CULL_TILE);
    const uint32_t t0 = blockIdx.x * p.rayq_tpr, t1 = min(t0 + p.rayq_tpr, ntiles);
    uint32_t* region = p.rayq + (size_t)blockIdx.x * p.rayq_region;
    const vec3f eye = v3(p.eye[0], p.eye[1], p.eye[2]);
    // Conservative root cull: the root's four child boxes, each inflated by m = 2^-12 x the
    // scene-and-eye scale, against the exact ray direction with the hardware reciprocal (1 ulp)
    // for 1/d. Its slab distances deviate from the exact test's by ~1e-7 of |box - eye| <= 2 x
    // scale, far inside m, so a culled ray misses every child under the exact test (BuildTree.cu
    // semantics as in quad_visit); rays near the margin just take the exact traversal. Empty
    // children are all-NaN and never pass. Near-axis directions (|d| < 2^-100: reciprocal
    // overflow, 0 x inf) are never culled.
    const uint4* rn = p.nodes;
    const uint4 rlx = rn[0], rly = rn[1], rlz = rn[2], rhx = rn[3], rhy = rn[4], rhz = rn[5];
    const uint32_t LX[4] = {rlx.x, rlx.y, rlx.z, rlx.w}, LY[4] = {rly.x, rly.y, rly.z, rly.w};
    const uint32_t LZ[4] = {rlz.x, rlz.y, rlz.z, rlz.w}, HX[4] = {rhx.x, rhx.y, rhx.z, rhx.w};
    const uint32_t HY[4] = {rhy.x, rhy.y, rhy.z, rhy.w}, HZ[4] = {rhz.x, rhz.y, rhz.z, rhz.w};
    float scale = fmaxf(fabsf(eye.x), fmaxf(fabsf(eye.y), fabsf(eye.z)));
#pragma unroll
    for (int k = 0; k < 4; ++k)
        scale = fmaxf(scale, fmaxf(fmaxf(fmaxf(fabsf(u2f(LX[k])), fabsf(u2f(LY[k]))), fabsf(u2f(LZ[k]))),
                                   fmaxf(fmaxf(fabsf(u2f(HX[k])), fabsf(u2f(HY[k]))), fabsf(u2f(HZ[k])))));
    const float margin = scale * 0x1p-12f;
    float cb[4][6], ub[6] = {__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""),
                             __builtin_nanf(""), __builtin_nanf("")};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        cb[k][0] = u2f(LX[k]) - margin, cb[k][1] = u2f(LY[k]) - margin, cb[k][2] = u2f(LZ[k]) - margin;
        cb[k][3] = u2f(HX[k]) + margin, cb[k][4] = u2f(HY[k]) + margin, cb[k][5] = u2f(HZ[k]) + margin;
#pragma unroll
        for (int a = 0; a < 3; ++a) ub[a] = fminf(ub[a], cb[k][a]), ub[3 + a] = fmaxf(ub[3 + a], cb[k][3 + a]);
    }
    const bool any_tris = p.num_tris != 0;
    unsigned long long cn = 0;
    const unsigned long long below = (1ull << lane) - 1ull;
    // Four tiles per step with their camera-table loads issued together (the only dependent loads
    // of a ray's setup), so a wave waits for one load latency per four tiles.
    constexpr int UNR = 4;
    for (uint32_t i0 = t0 + w; i0 < t1; i0 += UNR * WAVES) {
        float crx[UNR], cry[UNR];
        uint32_t cx[UNR], clr[UNR];
        bool cval[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const uint32_t i = i0 + u * WAVES;
            cx[u] = (i % tiles_x) * CULL_TILE + (lane & 7);
            clr[u] = (i / tiles_x) * CULL_TILE + (lane >> 3);
            const uint32_t gy = clr[u] < p.local_rows ? global_row(p, clr[u]) : p.height;
            cval[u] = i < t1 && cx[u] < p.width && gy < p.height;
            crx[u] = cval[u] ? p.rx[cx[u]] : 0.f;
            cry[u] = cval[u] ? p.ry[gy] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            if (i0 + u * WAVES >= t1) break;
            const uint32_t x = cx[u], lr = clr[u];
            bool enter = false;
            if (cval[u]) {
                if (any_tris) {
                    const float rx = crx[u], ry = cry[u];
                    // primary_dir from the preloaded tables; with a near-orthonormal orient (host
                    // check, p.fast_cull) the cull may use the 1-ulp reciprocal square root: the
                    // direction then deviates by ~2^-21 relative, inside the margin m
                    const float q2 = p.z2 + rx * rx + ry * ry;
                    const float d = p.fast_cull ? __builtin_amdgcn_rsqf(q2) : 1.f / sqrtf(q2);
                    const vec3f r = v3(rx * d, ry * d, p.zoom * d);
                    const float* om = p.orient;
                    const vec3f dir = v3((om[0] * r.x + om[3] * r.y) + om[6] * r.z, (om[1] * r.x + om[4] * r.y) + om[7] * r.z,
                                         (om[2] * r.x + om[5] * r.y) + om[8] * r.z);
                    const bool tiny = !(fabsf(dir.x) >= 0x1p-100f && fabsf(dir.y) >= 0x1p-100f && fabsf(dir.z) >= 0x1p-100f);
                    const vec3f inv = v3(__builtin_amdgcn_rcpf(dir.x), __builtin_amdgcn_rcpf(dir.y), __builtin_amdgcn_rcpf(dir.z));
                    // union of the inflated children first (monotone slab distances: a child hit is a
                    // union hit), then the children themselves
                    float tn;
                    enter = tiny;
                    if (!tiny && child_hit(&ub[0], &ub[3], eye, inv, __builtin_inff(), tn)) {
#pragma unroll
                        for (int k = 0; k < 4; ++k) enter |= child_hit(&cb[k][0], &cb[k][3], eye, inv, __builtin_inff(), tn);
                    }
                    if (COUNT && !enter) ++cn;  // the root record the quad traversal would visit
                }
                if (!enter) {
                    const size_t o = (size_t)lr * p.width + x;
                    p.packed[(size_t)lr * p.pitch_u32 + x] = MISS_PACKED;
                    p.tri_id[o] = NO_TRI;
                    p.t[o] = __builtin_inff();
                    if (p.nz) p.nz[o] = 0.0f;
                    if (SH == SH_FUSED) p.shadow[o] = 0;
                }
            }
            const unsigned long long mask = ballot(enter);
            if (mask) {
                uint32_t base = 0;
                if (lane == 0) base = atomicAdd(&s_n, (uint32_t)__popcll(mask));
                base = __builtin_amdgcn_readfirstlane(base);
                if (enter) region[base + (uint32_t)__popcll(mask & below)] = x | (lr << 16);
            }
        }
    }
    __syncthreads();
    if (tid == 0) p.rayq_count[blockIdx.x] = s_n;
    if (COUNT) atomicAdd(&p.counters[0], cn);
}

template <bool COUNT, int LDS_N, uint32_t PRIO, int SH, bool DIAG = false>
__global__ __launch_bounds__(BLOCK) void k_trace_rays(const TraceParams p) {
    static_assert(SH == SH_NONE || SH == SH_FUSED, "compact kernels: primary or fused shadow rays");
    static_assert(!DIAG || COUNT, "the diagnostic build counts work");
    const uint64_t t_start = DIAG ? __builtin_amdgcn_s_memrealtime() : 0;
    uint64_t diag_work = 0;
    __shared__ uint2 s_stk[LDS_N][QRAYS];
#if BM_QUAD_LEAF_LDS
    __shared__ float4 s_lt[QRAYS][12];
#endif
    __shared__ uint32_t s_pre[CULL_MAX_REGIONS];  // inclusive prefix of the region counts
    __shared__ uint32_t s_wsum[WAVES];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int c = lane & 3, q = lane >> 2;
    // ---- inclusive scan of the region counts (every workgroup, into LDS) ----
    const uint32_t nreg = p.rayq_regions;
    constexpr uint32_t PER = CULL_MAX_REGIONS / BLOCK;
    uint32_t v[PER], run = 0;
#pragma unroll
    for (uint32_t k = 0; k < PER; ++k) {
        const uint32_t r = tid * PER + k;
        run += r < nreg ? p.rayq_count[r] : 0u;
        v[k] = run;
    }
    const uint32_t incl = wave_incl_add(run);  // wave-inclusive scan of the per-thread totals
    if (lane == 63) s_wsum[w] = incl;
    __syncthreads();
    uint32_t off = incl - run;
    for (int k = 0; k < w; ++k) off += s_wsum[k];
#pragma unroll
    for (uint32_t k = 0; k < PER; ++k) s_pre[tid * PER + k] = v[k] + off;
    __syncthreads();
    const uint32_t total = s_wsum[0] + s_wsum[1] + s_wsum[2] + s_wsum[3];
    QStack<LDS_N> st;
    st.s = s_stk;
#if BM_QUAD_LEAF_LDS
    st.lt = s_lt[w * 16 + q];
#endif
    st.ray = w * 16 + q;
    const uint32_t slot = blockIdx.x * QRAYS + st.ray;
    st.g_ref = p.ovf_ref;
    st.g_t = p.ovf_t;
    st.slot = slot;
    st.stride = p.ovf_stride;
    const vec3f eye = v3(p.eye[0], p.eye[1], p.eye[2]);
    unsigned long long cn = 0, ct = 0, ch = 0, csh[3] = {0, 0, 0};
    const uint32_t nbatch = (total + 15) / 16, nwaves = gridDim.x * WAVES;
    const uint32_t last = nreg ? nreg - 1 : 0;
    for (uint32_t b = blockIdx.x * WAVES + w; b < nbatch; b += nwaves) {
        const uint32_t sidx = b * 16 + (uint32_t)q;
        const unsigned long long before_work = cn + ct;
#if BM_RAYS_SEARCH64
        // region of the batch's first survivor (the first r with s_pre[r] > 16 b) by a 64-ary search —
        // each lane reads one segment end, a ballot picks the segment, then its 16 entries the same
        // way: two LDS reads where a binary search over 1,024 regions took ten dependent ones; each ray
        // then steps forward over the (rare) region ends inside its batch
        static_assert(CULL_MAX_REGIONS <= 1024, "64 segments of 16 regions");
        uint32_t lo;
        {
            const uint32_t s0 = b * 16;
            const unsigned long long m1 = ballot(s_pre[min(16u * (uint32_t)lane + 15u, last)] > s0);
            const uint32_t seg = m1 ? (uint32_t)__ffsll((long long)m1) - 1u : 63u;
            const unsigned long long m2 = ballot(s_pre[min(seg * 16u + ((uint32_t)lane & 15u), last)] > s0) & 0xFFFFull;
            lo = min(seg * 16u + (m2 ? (uint32_t)__ffsll((long long)m2) - 1u : 15u), last);
        }
        if (sidx < total) {  // whole quads only
            while (lo < last && s_pre[lo] <= sidx) ++lo;
#else
        if (sidx < total) {  // whole quads only
            // region of survivor sidx: the first r with s_pre[r] > sidx
            uint32_t lo = 0, hi = last;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (s_pre[mid] > sidx) hi = mid;
                else lo = mid + 1;
            }
#endif
            const uint32_t before = lo ? s_pre[lo - 1] : 0u;
            const uint32_t pix = p.rayq[(size_t)lo * p.rayq_region + (sidx - before)];
            const uint32_t x = pix & 0xFFFFu, lr = pix >> 16;
            __builtin_amdgcn_s_setprio(0);
            const vec3f dir = primary_dir(p, x, global_row(p, lr));
            const vec3f inv = v3(1.f / dir.x, 1.f / dir.y, 1.f / dir.z);
            float tbest = __builtin_inff(), bu = 0.f, bv = 0.f;
            uint32_t ibest = NO_TRI;
            quad_closest<COUNT, PRIO>(p, st, c, eye, dir, inv, tbest, ibest, bu, bv, cn, ct);
            const size_t o = (size_t)lr * p.width + x;
            uint32_t packed = MISS_PACKED;
            float nzv = 0.0f;
            if (ibest != NO_TRI) {
                packed = shade_hit(p, ibest, bu, bv, nzv);
                if (COUNT && c == 0) ++ch;
            }
            if (c == 0) p.packed[(size_t)lr * p.pitch_u32 + x] = packed;
            else if (c == 1) p.tri_id[o] = ibest;
            else if (c == 2) p.t[o] = tbest;
            else if (p.nz) p.nz[o] = nzv;
            if (SH == SH_FUSED) {
                bool occ = false;
                if (ibest != NO_TRI) {
                    vec3f so, sd;
                    shadow_segment(p, eye, dir, tbest, so, sd);
                    occ = quad_anyhit<COUNT, PRIO>(p, st, c, so, sd, csh[0], csh[1]);
                    if (COUNT && c == 0) csh[2] += occ;
                }
                if (c == 0) p.shadow[o] = occ ? 1 : 0;
            }
        }
        if (DIAG) {
            uint32_t wl = (uint32_t)(cn + ct - before_work);
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) wl = max(wl, (uint32_t)__shfl_xor((int)wl, o));
            diag_work += wl;
        }
    }
    flush_counters<COUNT>(p, cn, ct, ch, csh);
    if (DIAG) {
        const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
        if (lane == 0) {
            const uint32_t hwid = __builtin_amdgcn_s_getreg((31 << 11) | 4);
            const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);
            const size_t wv = (size_t)blockIdx.x * WAVES + w;
            p.diag[4 * wv + 0] = t_start;
            p.diag[4 * wv + 1] = t_end;
            p.diag[4 * wv + 2] = ((uint64_t)xcc << 32) | hwid;
            p.diag[4 * wv + 3] = diag_work;
        }
    }
}

// ---- wave packets: one 8x8 tile of coherent primary rays per wave over the BVH4 (TRACE_PACKET) ------
// the quad step is bound by its dependent chain (LDS pop -> seven per-lane record loads ->
// slab tests -> DPP ranking -> LDS push, ~1,800 cycles) and the filled view takes ~16.6 of them per ray.
// Here the traversal state is the wave's, not the lane's: one node record per wave step, read by
// scalar loads (the record address is wave-uniform: the constant address space makes the compiler
// issue s_load into SGPRs), each lane slab-tests the four children against its own ray, a ballot per
// child gives the lanes that descend, and the wave walks one shared stack in LDS whose entries carry
// (child box, child ref, lane mask). A popped entry's lanes re-test its box against their current
// closest hit, so a subtree is entered only by lanes whose own traversal would enter it; every lane
// keeps its own (t, id) closest hit with lowest-id ties, which does not depend on the order the
// subtrees are visited in — the frame equals the oracle's (the visit order and the COUNT counters do
// not, so counting traces keep the quad kernel). Children are ordered by the entry distances of the
// packet's first lane (children that lane misses after).
// Stack bound: the BVH4 levels of a < 64-level Karras tree are < 32, a packet step pushes <= 3
// siblings, and the stack holds siblings of the current path only: PK_DEPTH = MAX_STACK entries.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(4))) const u32x4 cuint4;   // scalar (SMEM) loads of uniform records
typedef __attribute__((address_space(4))) const uint32_t cuint;
typedef unsigned long long u64x4 __attribute__((ext_vector_type(4)));
constexpr int PK_DEPTH = MAX_STACK;
#ifndef BM_PACKET_WAVES
#define BM_PACKET_WAVES 8  // waves per SIMD the packet kernel's registers must allow (6 / 7: 1-2 % slower, r06_v11)
#endif
#ifndef BM_PK_POP_SLOAD
#define BM_PK_POP_SLOAD 1  // 1: 16-B entries, a pop re-loads the child's box from its parent's record by scalar
                           // loads (filled view 333 -> 314 us); 0: the box in LDS beside the entry
#endif
#ifndef BM_PK_SORTNET
#define BM_PK_SORTNET 1  // rank the children by a scalar sorting network (0: per-child compare counts, 4-5 % slower in flight)
#endif
#ifndef BM_PK_ORDER
#define BM_PK_ORDER 1  // children order: 1 by the packet's first lane's entry distances, 2 by the tile's centre
                       // lane's (first lane when it is out), 0 slot order
#endif
#ifndef BM_PK_LEAF_BATCH
#define BM_PK_LEAF_BATCH 1  // leaf triangle records loaded per batch before their tests
#endif
#ifndef BM_PK_PICK_VEC
#define BM_PK_PICK_VEC 1  // children picked by slot from SGPR vectors
#endif
#ifndef BM_PK_NODE_SGPR
#define BM_PK_NODE_SGPR 1  // no readfirstlane of the node at the loop head (every assignment is uniform)
#endif
#ifndef BM_PK_ORIGIN_VGPR
#define BM_PK_ORIGIN_VGPR 1
#endif
#ifndef BM_PK_VKEYS
#define BM_PK_VKEYS 1  // children's order keys per lane by VALU, the lead lane's read (scalar key forms cost SALU)
#endif
// BM_PK_PUSH_M: a pushed child carries its parent node's lanes M instead of the child's own mask B and
// no ref (read from the parent's record at the pop). The pop re-tests the child's box for the lanes it
// carries against their closest hit then (t_pop <= t_push): M & test(t_pop) = B & test(t_pop), since B =
// M & test(t_push) and the box terms are the same arithmetic on the same operands. No per-push picks.
#ifndef BM_PK_PUSH_M
#define BM_PK_PUSH_M 1
#endif
#ifndef BM_PK_MASKS
#define BM_PK_MASKS 1  // child and pop masks as ANDs of per-compare ballots (scalar), lead keys on the scalar side
#endif
#ifndef BM_PK_PRIO_AFTER
#define BM_PK_PRIO_AFTER 0  // > 0: a packet raises its issue priority after that many node steps (the tail's waves)
#endif

// Slab planes by direction sign (BM_PK_SIGNS). When every ray of the tile has finite, nonzero inverse
// direction components of one sign per axis (all tiles but those on the image's sign-change lines),
// the entry plane of each axis is the same for all of them: lo for a positive component, hi for a
// negative one. Then min(t_lo, t_hi) is t_near exactly — (b - o) * inv is monotone in b for a finite
// inv of fixed sign, so t_lo <= t_hi or the reverse, ties included (a signed zero only ties) — and
// t_far likewise, and NaN-box (empty) slots give NaN either way: tn = max3 of the near values and
// tf = min3 of the far ones, bit-identical to the min/max form, two operations per child instead of
// eight. The walk is instantiated per sign combination (SG = x | y << 1 | z << 2 negative), SG = 8 the
// general form for the other tiles.
#ifndef BM_PK_SIGNS
#define BM_PK_SIGNS 1
#endif

struct PkHit {
    float t, u, v;
    uint32_t id;
};

// One 8x8 tile's walk by one wave (all 64 lanes, wave-uniform control flow). s_e: the wave's stack (PK_DEPTH).
template <bool DIAG, int SG>
__device__ __forceinline__ void packet_walk(const TraceParams& p, int lane, uint4* __restrict__ s_e,
                                            uint4* __restrict__ s_h, uint32_t* __restrict__ s_mh,
                                            unsigned long long* __restrict__ dslot, uint64_t t_start, bool valid,
                                            const vec3f eye, const vec3f dir, const vec3f inv, PkHit& hit) {
    uint32_t d_nodes = 0, d_leaves = 0, d_tris = 0, d_lanes = 0;
    (void)s_h, (void)s_mh, (void)dslot;
    uint32_t steps = 0;
    constexpr bool NX = SG & 1, NY = SG & 2, NZ = SG & 4;  // (SG < 8) axes whose entry plane is hi
#if BM_PK_ORIGIN_VGPR  // the eye pairs held in VGPRs (a packed op takes one SGPR operand: the record's)
    f32x2 ox = {eye.x, eye.x}, oy = {eye.y, eye.y}, oz = {eye.z, eye.z};
    asm volatile("" : "+v"(ox), "+v"(oy), "+v"(oz));
#else
    const f32x2 ox = {eye.x, eye.x}, oy = {eye.y, eye.y}, oz = {eye.z, eye.z};
#endif
    const f32x2 ix = {inv.x, inv.x}, iy = {inv.y, inv.y}, iz = {inv.z, inv.z};
    float tbest = __builtin_inff(), bu = 0.f, bv = 0.f;
    uint32_t ibest = NO_TRI;
    unsigned long long M = ballot(valid);  // lanes of the current node
    uint32_t node = p.num_tris && M ? 0u : EMPTY_REF;
    int sp = 0;
    cuint4* const nodes = (cuint4*)(p.nodes);  // generic -> constant address space (a C cast)
    cuint4* const tris = (cuint4*)(p.tris);
    for (;;) {
#if !BM_PK_NODE_SGPR
        node = __builtin_amdgcn_readfirstlane(node);
#endif
        if (node != EMPTY_REF) {
            const bool act = (M >> lane) & 1ull;
            if (node & LEAF_BIT) {
                const uint32_t first = node & FIRST_MASK, cnt = ((node >> 27) & 15u) + 1u;
                if (DIAG) ++d_leaves, d_tris += cnt;
                constexpr uint32_t LB = BM_PK_LEAF_BATCH;
                for (uint32_t k0 = 0; k0 < cnt; k0 += LB) {  // LB records in flight, then their tests
                    u32x4 r[LB][3];
#pragma unroll
                    for (uint32_t j = 0; j < LB; ++j) {
                        cuint4* tr = tris + 3 * (size_t)(first + min(k0 + j, cnt - 1u));
                        r[j][0] = tr[0], r[j][1] = tr[1], r[j][2] = tr[2];
                    }
#pragma unroll
                    for (uint32_t j = 0; j < LB; ++j) {
                        if (k0 + j < cnt && act) {
                            float tt, uu, vv;
                            const float4 a = make_float4(u2f(r[j][0].x), u2f(r[j][0].y), u2f(r[j][0].z), 0.f);
                            const float4 b = make_float4(u2f(r[j][1].x), u2f(r[j][1].y), u2f(r[j][1].z), 0.f);
                            const float4 c = make_float4(u2f(r[j][2].x), u2f(r[j][2].y), u2f(r[j][2].z), 0.f);
                            if (tri_test(a, b, c, eye, dir, tt, uu, vv) && tt > 0.0f && tt != 3.40282347e+38f) {
                                const uint32_t id = r[j][0].w;
                                if (tt < tbest || (tt == tbest && id < ibest)) {
                                    tbest = tt;
                                    ibest = id;
                                    bu = uu;
                                    bv = vv;
                                }
                            }
                        }
                    }
                }
                node = EMPTY_REF;
            } else {
                if (DIAG) ++d_nodes, d_lanes += (uint32_t)__popcll(M);
                if (BM_PK_PRIO_AFTER && ++steps == BM_PK_PRIO_AFTER) __builtin_amdgcn_s_setprio(2);
                cuint4* nd = nodes + 8 * (size_t)node;
                const u32x4 lx = nd[0], ly = nd[1], lz = nd[2], hx = nd[3], hy = nd[4], hz = nd[5], rf = nd[6];
                const uint32_t LX[4] = {lx.x, lx.y, lx.z, lx.w}, LY[4] = {ly.x, ly.y, ly.z, ly.w};
                const uint32_t LZ[4] = {lz.x, lz.y, lz.z, lz.w}, HX[4] = {hx.x, hx.y, hx.z, hx.w};
                const uint32_t HY[4] = {hy.x, hy.y, hy.z, hy.w}, HZ[4] = {hz.x, hz.y, hz.z, hz.w};
                const uint32_t R[4] = {rf.x, rf.y, rf.z, rf.w};
                // slab tests two children at a time (adjacent SGPRs feed the packed f32 operations)
                unsigned long long B[4];
#if BM_PK_MASKS && !BM_PK_VKEYS
                float tnl[4];  // this lane's entry distance of each child
#else
                uint32_t kl[4];  // this lane's order key of each child (its misses after its hits)
#endif
#pragma unroll
                for (int c = 0; c < 4; c += 2) {
                    const f32x2 tlx = (f32x2{u2f(LX[c]), u2f(LX[c + 1])} - ox) * ix;
                    const f32x2 thx = (f32x2{u2f(HX[c]), u2f(HX[c + 1])} - ox) * ix;
                    const f32x2 tly = (f32x2{u2f(LY[c]), u2f(LY[c + 1])} - oy) * iy;
                    const f32x2 thy = (f32x2{u2f(HY[c]), u2f(HY[c + 1])} - oy) * iy;
                    const f32x2 tlz = (f32x2{u2f(LZ[c]), u2f(LZ[c + 1])} - oz) * iz;
                    const f32x2 thz = (f32x2{u2f(HZ[c]), u2f(HZ[c + 1])} - oz) * iz;
#pragma unroll
                    for (int k = 0; k < 2; ++k) {
                        float tn, tf;
                        if constexpr (SG < 8) {  // entry / exit planes known per axis (BM_PK_SIGNS)
                            tn = fmaxf(fmaxf(NX ? thx[k] : tlx[k], NY ? thy[k] : tly[k]), NZ ? thz[k] : tlz[k]);
                            tf = fminf(fminf(NX ? tlx[k] : thx[k], NY ? tly[k] : thy[k]), NZ ? tlz[k] : thz[k]);
                        } else {
                            tn = fmaxf(fmaxf(fminf(tlx[k], thx[k]), fminf(tly[k], thy[k])), fminf(tlz[k], thz[k]));
                            tf = fminf(fminf(fmaxf(tlx[k], thx[k]), fmaxf(tly[k], thy[k])), fmaxf(tlz[k], thz[k]));
                        }
#if BM_PK_MASKS
                        // each compare's ballot is its own SGPR mask; the node's lanes and the AND are scalar
                        const bool c1 = tn <= tf, c2 = tf >= 0.0f, c3 = tn <= tbest;
                        B[c + k] = ballot(c1) & ballot(c2) & ballot(c3) & M;
#if BM_PK_VKEYS  // every lane's key by VALU (the lead lane's is read below): fewer scalar operations
                        kl[c + k] = (c1 & c2 & c3) ? order_key(tn, (uint32_t)(c + k)) : (0xFFFFFFF0u | (uint32_t)(c + k));
#else
                        tnl[c + k] = tn;
#endif
#else
                        const bool h = act & (tn <= tf) & (tf >= 0.0f) & (tn <= tbest);
                        B[c + k] = ballot(h);
                        kl[c + k] = h ? order_key(tn, (uint32_t)(c + k)) : (0xFFFFFFF0u | (uint32_t)(c + k));
#endif
                    }
                }
                // order by the packet's first lane; a child no lane enters ranks last (key ~0)
#if BM_PK_ORDER == 2
                const int lead = ((M >> 27) & 1ull) ? 27 : __builtin_ctzll(M);  // the tile's centre lane (3, 3)
#else
                const int lead = __builtin_ctzll(M);
#endif
                uint32_t K[4], nh = 0;
#pragma unroll
                for (int c = 0; c < 4; ++c) {
#if BM_PK_ORDER == 0
                    K[c] = B[c] ? (uint32_t)c : ~0u;  // slot order (A/B: what the ordering buys)
                    (void)lead;
#elif BM_PK_MASKS && BM_PK_VKEYS
                    // sortable as they are: a child no lane enters is 0xFFFFFFFC | slot
                    K[c] = B[c] ? (uint32_t)__builtin_amdgcn_readlane((int)kl[c], lead) : (0xFFFFFFFCu | (uint32_t)c);
#elif BM_PK_MASKS
                    // the lead lane's key, formed on the scalar side: its entry distance when it enters the
                    // child, else after every child it enters (the same keys as the per-lane form)
                    const uint32_t tb = (uint32_t)__builtin_amdgcn_readlane(__float_as_int(tnl[c]), lead);
                    K[c] = B[c] ? (((B[c] >> lead) & 1ull) ? order_key(__int_as_float((int)tb), (uint32_t)c)
                                                            : (0xFFFFFFF0u | (uint32_t)c))
                                : ~0u;
#else
                    K[c] = B[c] ? (uint32_t)__builtin_amdgcn_readlane((int)kl[c], lead) : ~0u;
#endif
                    nh += B[c] ? 1u : 0u;
                }
                node = EMPTY_REF;
                unsigned long long Mn = 0;
#if BM_PK_SORTNET && BM_PK_POP_SLOAD
                {  // keys sorted by a five-exchange network (scalar min/max; a key's low two bits are its slot,
                   // a child no lane enters sorts last as ~0 - 3 + slot), then the children by rank
#if BM_PK_MASKS && BM_PK_VKEYS && BM_PK_ORDER != 0
                    uint32_t k0 = K[0], k1 = K[1], k2 = K[2], k3 = K[3];
#else
                    uint32_t k0 = K[0] == ~0u ? 0xFFFFFFFCu : K[0], k1 = K[1] == ~0u ? 0xFFFFFFFDu : K[1];
                    uint32_t k2 = K[2] == ~0u ? 0xFFFFFFFEu : K[2], k3 = K[3];
#endif
                    auto cx = [](uint32_t& x, uint32_t& y) {
                        const uint32_t lo = min(x, y), hi = max(x, y);
                        x = lo, y = hi;
                    };
                    cx(k0, k1), cx(k2, k3), cx(k0, k2), cx(k1, k3), cx(k1, k2);
                    const uint32_t ks[4] = {k0, k1, k2, k3};
                    const uint32_t pcs = (uint32_t)((nd - nodes) >> 3) << 2;
#if BM_PK_PICK_VEC  // dynamic element of an SGPR vector (s_movrels) instead of a branch chain
                    const u64x4 BV = {B[0], B[1], B[2], B[3]};
                    auto pick_r = [&](uint32_t sl) { return rf[sl & 3u]; };
                    auto pick_b = [&](uint32_t sl) { return BV[sl & 3u]; };
#else
                    auto pick_r = [&](uint32_t sl) { return sl == 0 ? R[0] : sl == 1 ? R[1] : sl == 2 ? R[2] : R[3]; };
                    auto pick_b = [&](uint32_t sl) { return sl == 0 ? B[0] : sl == 1 ? B[1] : sl == 2 ? B[2] : B[3]; };
#endif
                    // a key below 0xFFFFFFFC is a child some lane enters (no count of them needed: the
                    // pushes go farthest first, each on top of the last, so they pop nearest first)
                    if (k0 < 0xFFFFFFFCu) {
                        node = pick_r(k0 & 3u);
                        Mn = pick_b(k0 & 3u);
                    }
#pragma unroll
                    for (int r = 3; r >= 1; --r) {
                        if (ks[r] < 0xFFFFFFFCu) {
                            const uint32_t sl = ks[r] & 3u;
#if BM_PK_PUSH_M  // the node's lanes: the pop's re-test leaves exactly the child's (see BM_PK_PUSH_M)
                            const int at = __builtin_amdgcn_readfirstlane(min(sp, PK_DEPTH - 1));
                            if (lane == 0) s_e[at] = make_uint4(0u, (uint32_t)M, (uint32_t)(M >> 32), pcs | sl);
#else
                            const unsigned long long bm = pick_b(sl);
                            if (lane == 0)
                                s_e[min(sp, PK_DEPTH - 1)] =
                                    make_uint4(pick_r(sl), (uint32_t)bm, (uint32_t)(bm >> 32), pcs | sl);
#endif
                            sp = __builtin_amdgcn_readfirstlane(min(sp + 1, PK_DEPTH));
                        }
                    }
                    sp = __builtin_amdgcn_readfirstlane(sp);  // uniform (the lane-0 stores must not make it look divergent)
                }
#else
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    uint32_t r = 0;
#pragma unroll
                    for (int d = 0; d < 4; ++d)
                        if (d != c) r += K[d] < K[c] ? 1u : 0u;
                    if (B[c] && r == 0) {
                        node = R[c];
                        Mn = B[c];
                    } else if (B[c]) {  // pushed farthest deepest, so they pop nearest first
                        const int at = min(sp + (int)(nh - 1u - r), PK_DEPTH - 1);
                        if (lane == 0) {
#if BM_PK_POP_SLOAD
                            s_e[at] = make_uint4(R[c], (uint32_t)B[c], (uint32_t)(B[c] >> 32),
                                                    (uint32_t)((nd - nodes) >> 3) << 2 | (uint32_t)c);
#else
                            s_e[at] = make_uint4(LX[c], LY[c], LZ[c], R[c]);
                            s_h[at] = make_uint4(HX[c], HY[c], HZ[c], (uint32_t)B[c]);
                            s_mh[at] = (uint32_t)(B[c] >> 32);
#endif
                        }
                    }
                }
                sp = min(sp + max((int)nh - 1, 0), PK_DEPTH);
#endif
                M = Mn;
                continue;
            }
        }
        // pop: the next entry some lane still enters (its box re-tested against the lane's closest hit)
        bool found = false;
        while (sp > 0) {
            --sp;
            const uint4 e = s_e[sp];
#if BM_PK_POP_SLOAD
            const uint32_t pcs = __builtin_amdgcn_readfirstlane(e.w);
            const unsigned long long em = ((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane(e.z) << 32) |
                                          (uint32_t)__builtin_amdgcn_readfirstlane(e.y);
            cuint* pr = (cuint*)(p.nodes) + 32 * (size_t)(pcs >> 2) + (pcs & 3u);
            const float blx = u2f(pr[0]), bly = u2f(pr[4]), blz = u2f(pr[8]);
            const float bhx = u2f(pr[12]), bhy = u2f(pr[16]), bhz = u2f(pr[20]);
#if BM_PK_PUSH_M
            const uint32_t eref = pr[24];  // the child's ref from its parent's record
#else
            const uint32_t eref = e.x;
#endif
#else
            const uint4 h = s_h[sp];
            const unsigned long long em = ((unsigned long long)s_mh[sp] << 32) | h.w;
            const float blx = u2f(e.x), bly = u2f(e.y), blz = u2f(e.z);
            const float bhx = u2f(h.x), bhy = u2f(h.y), bhz = u2f(h.z);
            const uint32_t eref = e.w;
#endif
            const f32x2 tx = (f32x2{blx, bhx} - ox) * ix, ty = (f32x2{bly, bhy} - oy) * iy, tz = (f32x2{blz, bhz} - oz) * iz;
            float tn, tf;
            if constexpr (SG < 8) {
                tn = fmaxf(fmaxf(NX ? tx.y : tx.x, NY ? ty.y : ty.x), NZ ? tz.y : tz.x);
                tf = fminf(fminf(NX ? tx.x : tx.y, NY ? ty.x : ty.y), NZ ? tz.x : tz.y);
            } else {
                tn = fmaxf(fmaxf(fminf(tx.x, tx.y), fminf(ty.x, ty.y)), fminf(tz.x, tz.y));
                tf = fminf(fminf(fmaxf(tx.x, tx.y), fmaxf(ty.x, ty.y)), fmaxf(tz.x, tz.y));
            }
#if BM_PK_MASKS
            M = em & ballot(tn <= tf) & ballot(tf >= 0.0f) & ballot(tn <= tbest);
#else
            const bool a = ((em >> lane) & 1ull) && (tn <= tf) && (tf >= 0.0f) && (tn <= tbest);
            M = ballot(a);
#endif
            if (M) {
                node = __builtin_amdgcn_readfirstlane(eref);
                found = true;
                break;
            }
        }
        if (!found) break;
    }
    if (DIAG && lane == 0) {  // per tile: start, end, (leaf << 32 | node steps), (tri tests << 32 | lanes)
        dslot[0] = t_start;
        dslot[1] = __builtin_amdgcn_s_memrealtime();
        dslot[2] = ((uint64_t)d_leaves << 32) | d_nodes;
        dslot[3] = ((uint64_t)d_tris << 32) | d_lanes;
    }
    hit = PkHit{tbest, bu, bv, ibest};
}

template <bool DIAG>
__device__ __forceinline__ void packet_tile(const TraceParams& p, uint32_t tile, uint32_t tiles_x, int lane,
                                            uint4* __restrict__ s_e, uint4* __restrict__ s_h,
                                            uint32_t* __restrict__ s_mh, unsigned long long* __restrict__ dslot) {
    const uint64_t t_start = DIAG ? __builtin_amdgcn_s_memrealtime() : 0;
    const uint32_t x = (tile % tiles_x) * 8 + (lane & 7);
    const uint32_t lr = (tile / tiles_x) * 8 + (lane >> 3);
    const uint32_t gy = lr < p.local_rows ? global_row(p, lr) : p.height;
    const bool valid = x < p.width && gy < p.height;
    const vec3f eye = v3(p.eye[0], p.eye[1], p.eye[2]);
    vec3f dir = v3(0.f, 0.f, 1.f), inv = v3(0.f, 0.f, 1.f);
    if (valid) {
        dir = primary_dir(p, x, gy);
        inv = v3(1.f / dir.x, 1.f / dir.y, 1.f / dir.z);
    }
    PkHit hit;
#if BM_PK_SIGNS
    // the tile's sign combination when its rays' inverse components are finite and of one sign per axis
    const unsigned long long V = ballot(valid);
    const bool fin = __builtin_isfinite(inv.x) && __builtin_isfinite(inv.y) && __builtin_isfinite(inv.z);
    const unsigned long long bad = V & ~ballot(fin);
    const unsigned long long nx = ballot(valid && inv.x < 0.f), ny = ballot(valid && inv.y < 0.f),
                             nz = ballot(valid && inv.z < 0.f);
    const bool uni = !bad && (nx == 0 || nx == V) && (ny == 0 || ny == V) && (nz == 0 || nz == V);
    const int sg = uni ? (nx ? 1 : 0) | (ny ? 2 : 0) | (nz ? 4 : 0) : 8;
    switch (sg) {
        case 0: packet_walk<DIAG, 0>(p, lane, s_e, s_h, s_mh, dslot, t_start, valid, eye, dir, inv, hit); break;
        case 1: packet_walk<DIAG, 1>(p, lane, s_e, s_h, s_mh, dslot, t_start, valid, eye, dir, inv, hit); break;
        case 2: packet_walk<DIAG, 2>(p, lane, s_e, s_h, s_mh, dslot, t_start, valid, eye, dir, inv, hit); break;
        case 3: packet_walk<DIAG, 3>(p, lane, s_e, s_h, s_mh, dslot, t_start, valid, eye, dir, inv, hit); break;
        case 4: packet_walk<DIAG, 4>(p, lane, s_e, s_h, s_mh, dslot, t_start, valid, eye, dir, inv, hit); break;
        case 5: packet_walk<DIAG, 5>(p, lane, s_e, s_h, s_mh, dslot, t_start, valid, eye, dir, inv, hit); break;
        case 6: packet_walk<DIAG, 6>(p, lane, s_e, s_h, s_mh, dslot, t_start, valid, eye, dir, inv, hit); break;
        case 7: packet_walk<DIAG, 7>(p, lane, s_e, s_h, s_mh, dslot, t_start, valid, eye, dir, inv, hit); break;
        default: packet_walk<DIAG, 8>(p, lane, s_e, s_h, s_mh, dslot, t_start, valid, eye, dir, inv, hit); break;
    }
#else
    packet_walk<DIAG, 8>(p, lane, s_e, s_h, s_mh, dslot, t_start, valid, eye, dir, inv, hit);
#endif
    if (!valid) return;
    const uint32_t o32 = lr * p.width + x;
    uint32_t packed = MISS_PACKED;
    float nzv = 0.0f;
    if (hit.id != NO_TRI) packed = shade_hit(p, hit.id, hit.u, hit.v, nzv);
    p.packed[(size_t)lr * p.pitch_u32 + x] = packed;
    p.tri_id[o32] = hit.id;
    p.t[o32] = hit.t;
    if (p.nz) p.nz[o32] = nzv;
}


// Tile order. BM_PK_SCHED 0 (default): one tile per wave in screen order (grid = tiles / 4 blocks; the
// hardware dispatcher balances). 1 (A/B, measured slower: filled view 302 -> 355 us, C4 284 -> 356): a
// persistent grid (the blocks the device keeps resident) whose block b owns the tiles b, b + B, ...
// (B = blocks) and hands them to its four waves by an LDS ticket; with p.sched == 2 and a cost table
// (the render target's previous trace: 10-ns ticks per 8x8 tile, rewritten as tiles complete) the share
// goes out longest first (LPT, the quad kernel's cost-ordered schedule). The driver loop costs the
// kernel 9 SGPRs and 39 spills, and the tiles it starts first run slower on cold caches.
#ifndef BM_PK_SCHED
#define BM_PK_SCHED 0
#endif
template <int SH, bool DIAG = false>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(BM_PACKET_WAVES))) void k_trace_packet(
    const TraceParams p) {
    static_assert(SH == SH_NONE, "packets: primary rays");
    __shared__ uint4 s_e[WAVES][PK_DEPTH];  // (child ref, lanes lo, lanes hi, parent << 2 | slot) or (lo.xyz, ref)
#if !BM_PK_POP_SLOAD
    __shared__ uint4 s_h[WAVES][PK_DEPTH];  // (hi.xyz, lanes lo)
    __shared__ uint32_t s_mh[WAVES][PK_DEPTH];  // lanes hi
    uint4* const sh = s_h[0];
    uint32_t* const smh = s_mh[0];
#else
    uint4* const sh = nullptr;
    uint32_t* const smh = nullptr;
#endif
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t tiles_x = (p.width + 7) / 8, tiles_y = (p.local_rows + 7) / 8;
    const uint32_t ntiles = tiles_x * tiles_y;
#if BM_PK_SCHED == 0
    const uint32_t tile = blockIdx.x * WAVES + (uint32_t)w;
    if (tile >= ntiles) return;
    packet_tile<DIAG>(p, tile, tiles_x, lane, s_e[w], sh ? sh + w * PK_DEPTH : nullptr, smh ? smh + w * PK_DEPTH : nullptr,
                      DIAG ? p.diag + 4 * (size_t)tile : nullptr);
#else
    __shared__ uint32_t s_ticket;
    __shared__ uint32_t s_order[LPT_MAX];
    const uint32_t B = gridDim.x;
    const uint32_t share = ntiles > blockIdx.x ? (ntiles - blockIdx.x + B - 1) / B : 0u;
    const bool lpt = p.sched == 2 && p.tile_cost != nullptr && share <= LPT_MAX;
    if (lpt) {  // the share by descending cost: bitonic in LDS, key = cost << 7 | (127 - k)
        for (uint32_t k = tid; k < LPT_MAX; k += BLOCK) {
            const uint32_t cst = k < share ? min(p.tile_cost[blockIdx.x + k * B], (1u << 24) - 2u) + 1u : 0u;
            s_order[k] = (cst << 7) | (LPT_MAX - 1u - k);
        }
        __syncthreads();
        for (uint32_t size = 2; size <= LPT_MAX; size <<= 1)
            for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
                for (uint32_t k = tid; k < LPT_MAX; k += BLOCK) {
                    const uint32_t o = k ^ stride;
                    if (o > k) {
                        const uint32_t a = s_order[k], b = s_order[o];
                        const bool desc = (k & size) == 0;
                        if (desc ? a < b : a > b) {
                            s_order[k] = b;
                            s_order[o] = a;
                        }
                    }
                }
                __syncthreads();
            }
        for (uint32_t k = tid; k < LPT_MAX; k += BLOCK) s_order[k] = LPT_MAX - 1u - (s_order[k] & (LPT_MAX - 1u));
    }
    if (tid == 0) s_ticket = WAVES;
    __syncthreads();
    for (uint32_t k = (uint32_t)w; k < share;) {
        uint32_t knext = 0;
        if (lane == 0) knext = atomicAdd(&s_ticket, 1u);
        knext = __builtin_amdgcn_readfirstlane(knext);
        const uint32_t tile = blockIdx.x + (lpt ? s_order[k] : k) * B;
        const uint64_t t0 = lpt ? __builtin_amdgcn_s_memrealtime() : 0;
        packet_tile<DIAG>(p, tile, tiles_x, lane, s_e[w], sh ? sh + w * PK_DEPTH : nullptr,
                          smh ? smh + w * PK_DEPTH : nullptr, DIAG ? p.diag + 4 * (size_t)tile : nullptr);
        if (p.tile_cost && lane == 0) p.tile_cost[tile] = (uint32_t)(__builtin_amdgcn_s_memrealtime() - t0);
        k = knext;
    }
#endif
}

// Persistent launch on min(p.persistent_blocks, the kernel's resident blocks); *grid gets the size.
template <typename K>
void launch_persistent(K kernel, const TraceParams& p, hipStream_t s, uint32_t* grid) {
    const uint32_t g = std::min(p.persistent_blocks, resident_blocks(kernel, BLOCK));
    if (grid) *grid = g;
    kernel<<<g, BLOCK, 0, s>>>(p);
}

}  // namespace
}  // namespace bm
