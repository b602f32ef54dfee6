// bm_trace_ab.hip — trace variants measured slower than the product kernels and kept for A/B
// measurements (tools/); compiled only into A/B builds (-DBM_TRACE_AB=1, e.g.
// tools/build_ab.py <out.so> BM_TRACE_AB=1), never into the in-tree library:
//   k_trace_tiles        one 16x16 tile per workgroup (round 1's first kernel; scratch / no overflow)
//   k_trace_persistent   single-lane persistent variants: LDS stack 16/8/12 without the priority
//                        boost, LDS 8 with it, dynamic tile tickets from one global atomic
//   k_trace_pair         two lanes per ray (8x4 pixels per wave): +5-16 % against quads
//   k_trace_quad_fetch   ray quads with in-wave ray refill: slower than block-dynamic tiles
//   k_trace_quad<.., 8>  BVH8 records, two children per lane: 12-16 % slower than BVH4
// Each gives the oracle's frames and counters exactly like the product kernels (same traversal
// order), which the A/B build's variant tests check.
#if BM_TRACE_AB
#include "bm_trace_dev.h"

namespace bm {
namespace {

// One 16x16 pixel tile per workgroup (each wave an 8x8 quadrant).
template <bool COUNT, int LDS_N, int OVF, int SH = SH_NONE, int W = 2>
__global__ __launch_bounds__(BLOCK) void k_trace_tiles(const TraceParams p) {
    __shared__ uint32_t s_ref[LDS_N][BLOCK];
    __shared__ float s_t[LDS_N][BLOCK];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const uint32_t x = blockIdx.x * 16 + (w & 1) * 8 + (lane & 7);
    const uint32_t lr = blockIdx.y * 16 + (w >> 1) * 8 + (lane >> 3);
    const uint32_t gy = global_row(p, lr);
    if (x >= p.width || lr >= p.local_rows || gy >= p.height) return;
    Stack<LDS_N, OVF> st;
    st.s_ref = s_ref;
    st.s_t = s_t;
    st.tid = tid;
    const uint32_t slot = (blockIdx.y * gridDim.x + blockIdx.x) * BLOCK + tid;
    st.g_ref = p.ovf_ref + slot;
    st.g_t = p.ovf_t + slot;
    st.stride = p.ovf_stride;
    unsigned long long cn = 0, ct = 0, ch = 0, csh[3] = {0, 0, 0};
    const bool hit = trace_pixel<COUNT, decltype(st), 0, SH, W>(p, st, x, lr, gy, cn, ct, ch, csh);
    if (SH == SH_QUEUE) enqueue_hit(p, hit, lr * p.width + x);
    flush_counters<COUNT>(p, cn, ct, ch, csh);
}

// ---- ray pairs: two lanes per ray over the BVH4 (TRACE_PAIR) ------------------------------------
// A wave traces an 8x4 pixel tile: lane 2r+h works for ray r and holds children 2h and 2h+1 of a
// record — adjacent dwords of every SoA plane, so a plane is one 8-B load and the two children's
// slab distances are packed f32 operations. Per ray and visit this spends half the lanes of a quad
// on the same slab work, and the per-ray bookkeeping (ranks, hit count, pushes, next child) is
// replicated over two lanes instead of four; at a leaf each lane tests every other triangle. The
// children's order keys, ranks, stack positions and the traversal are quad_visit's (order_key), so
// frames and COUNT counters are the oracle's step for step.
constexpr int PRAYS = BLOCK / 2;  // rays per workgroup
constexpr int PAIR_LDS = 16;      // LDS stack entries per ray (8 B each: 16 KiB per workgroup)

template <typename PS>
__device__ __forceinline__ uint32_t pair_visit(const TraceParams& p, uint32_t node, uint32_t h, const vec3f o,
                                               const vec3f inv, float tmax, bool key_t, const PS& st, int& sp) {
    const uint2* nd = reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(p.nodes) + ((node << 7) | (h << 3)));
    const uint2 lxp = nd[0], lyp = nd[2], lzp = nd[4], hxp = nd[6], hyp = nd[8], hzp = nd[10], rp = nd[12];
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
    const uint32_t ka = ha ? order_key(tna, 2u * h) : ~0u, kb = hb ? order_key(tnb, 2u * h + 1u) : ~0u;
    const uint32_t pa = dpp_u<QP_X1>(ka), pb = dpp_u<QP_X1>(kb);  // the partner lane's two children
    const uint32_t ra = (uint32_t)(kb < ka) + (uint32_t)(pa < ka) + (uint32_t)(pb < ka);
    const uint32_t rb = (uint32_t)(ka < kb) + (uint32_t)(pa < kb) + (uint32_t)(pb < kb);
    // hit count: a missing child's key ~0u ranks after every hit, so its rank is the hit count
    const uint32_t m = min(ha ? 4u : ra, hb ? 4u : rb);
    const uint32_t nh = min(m, dpp_u<QP_X1>(m));
    if (ha && ra > 0) st.put(sp + (int)(nh - 1u - ra), rp.x, key_t ? tna : 0.0f);
    if (hb && rb > 0) st.put(sp + (int)(nh - 1u - rb), rp.y, key_t ? tnb : 0.0f);
    sp += max((int)nh - 1, 0);
    uint32_t nx = (ha && ra == 0) ? rp.x : ((hb && rb == 0) ? rp.y : EMPTY_REF);
    nx = min(nx, dpp_u<QP_X1>(nx));
    return nx;
}

// Closest hit of one ray over the pair: quad_closest's loop with two lanes per ray.
template <bool COUNT, uint32_t PRIO, typename PS>
__device__ __forceinline__ void pair_closest(const TraceParams& p, const PS& st, uint32_t h, const vec3f eye,
                                             const vec3f dir, const vec3f inv, float& tbest, uint32_t& ibest,
                                             float& bu, float& bv, unsigned long long& cn, unsigned long long& ct) {
    int sp = 0;
    uint32_t next = p.num_tris ? 0u : EMPTY_REF;
    uint32_t iter = 0;
    for (;;) {
        prio_boost<PRIO>(p, iter);
        if (next != EMPTY_REF && (next & LEAF_BIT)) {
            const uint32_t first = next & FIRST_MASK, cnt = ((next >> 27) & 15u) + 1u;
            for (uint32_t k0 = 0; k0 < cnt; k0 += 2) {
                const uint32_t k = first + k0 + h;
                float t = __builtin_inff(), u = 0.f, v = 0.f;
                uint32_t id = NO_TRI;
                if (k0 + h < cnt) {
                    const float4 a = p.tris[3 * k + 0], b = p.tris[3 * k + 1], cc = p.tris[3 * k + 2];
                    float tt, uu, vv;
                    if (tri_test(a, b, cc, eye, dir, tt, uu, vv) && tt > 0.0f && tt != 3.40282347e+38f) {
                        t = tt;
                        id = f2u(a.w);
                        u = uu;
                        v = vv;
                    }
                }
                quad_min_step<QP_X1>(t, id, u, v);
                if (t < tbest || (t == tbest && id < ibest)) {
                    tbest = t;
                    ibest = id;
                    bu = u;
                    bv = v;
                }
            }
            if (COUNT && h == 0) ct += cnt;
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
        if (COUNT && h == 0) ++cn;
        next = pair_visit(p, next, h, eye, inv, tbest, true, st, sp);
        if (next != EMPTY_REF && !(next & LEAF_BIT)) {
            if (COUNT && h == 0) ++cn;
            next = pair_visit(p, next, h, eye, inv, tbest, true, st, sp);
        }
    }
}

// Persistent pair kernel: 8x4 pixel tiles handed to the block's waves from an LDS ticket (the
// block's share in screen order, XCD-aware runs as in k_trace_quad; frames do not depend on it).
template <bool COUNT, int LDS_N, uint32_t PRIO>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(COUNT ? 1 : BM_QUAD_WAVES))) void k_trace_pair(const TraceParams p) {
    __shared__ uint2 s_stk[LDS_N][PRAYS];
    __shared__ uint32_t s_ticket;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const uint32_t h = (uint32_t)lane & 1u, r = (uint32_t)lane >> 1;
    QStack<LDS_N, PRAYS> st;
    st.s = s_stk;
    st.ray = w * 32 + (int)r;
    const uint32_t slot = blockIdx.x * PRAYS + st.ray;
    st.g_ref = p.ovf_ref;
    st.g_t = p.ovf_t;
    st.slot = slot;
    st.stride = p.ovf_stride;
    const uint32_t tiles_x = (p.width + 7) / 8, tiles_y = (p.local_rows + 3) / 4;
    const uint32_t ntiles = tiles_x * tiles_y;
    const vec3f eye = v3(p.eye[0], p.eye[1], p.eye[2]);
    unsigned long long cn = 0, ct = 0, ch = 0, csh[3] = {0, 0, 0};
    const bool xcd_map = (gridDim.x & 7u) == 0;
    const uint32_t xcd = blockIdx.x & 7u, xj = blockIdx.x >> 3, xblocks = gridDim.x >> 3;
    auto tile_of = [&](uint32_t k) -> uint32_t {
        if (!xcd_map) return blockIdx.x + k * gridDim.x;
        const uint32_t l = xj + k * xblocks;  // this XCD's k-th local tile; runs of 4 tiles (32 px) per XCD
        return 4u * (xcd + 8u * (l >> 2)) + (l & 3u);
    };
    if (tid == 0) s_ticket = WAVES;
    __syncthreads();
    for (uint32_t i = tile_of((uint32_t)w); i < ntiles;) {
        uint32_t knext = 0;
        if (lane == 0) knext = atomicAdd(&s_ticket, 1u);
        knext = __builtin_amdgcn_readfirstlane(knext);
        const uint32_t x = (i % tiles_x) * 8 + (r & 7u);
        const uint32_t lr = (i / tiles_x) * 4 + (r >> 3);
        const uint32_t gy = lr < p.local_rows ? global_row(p, lr) : p.height;
        i = tile_of(knext);
        if (x >= p.width || gy >= p.height) continue;  // whole pairs only
        __builtin_amdgcn_s_setprio(0);
        const vec3f dir = primary_dir(p, x, gy);
        float tbest = __builtin_inff(), bu = 0.f, bv = 0.f;
        uint32_t ibest = NO_TRI;
        const vec3f inv = v3(1.f / dir.x, 1.f / dir.y, 1.f / dir.z);
        pair_closest<COUNT, PRIO>(p, st, h, eye, dir, inv, tbest, ibest, bu, bv, cn, ct);
        const size_t o = (size_t)lr * p.width + x;
        uint32_t packed = MISS_PACKED;
        float nzv = 0.0f;
        if (ibest != NO_TRI) {
            packed = shade_hit(p, ibest, bu, bv, nzv);
            if (COUNT && h == 0) ++ch;
        }
        if (h == 0) {
            p.packed[(size_t)lr * p.pitch_u32 + x] = packed;
            p.tri_id[o] = ibest;
        } else {
            p.t[o] = tbest;
            if (p.nz) p.nz[o] = nzv;
        }
    }
    flush_counters<COUNT>(p, cn, ct, ch, csh);
}

// Ray quads with in-wave ray refill: the wave's rays (its static 4x4 tiles, 16 rays each, in order)
// are handed to idle quads as the quads finish, so a quad never waits for the slowest ray of its
// tile (the persistent "while-while with ray fetch" scheme of Aila & Laine, HPG 2009, at quad
// granularity; the hand-out is a wave ballot + popcount, no atomics). Idle quads are refilled once
// at least refill_min of the 16 are idle (the setup of a ray is ~150 instructions of the whole
// wave). Every ray's traversal is the quad kernel's, step for step: frames and counters are those
// of trace_pixel / orc_bvh_trace.
template <bool COUNT, int LDS_N>
__global__ __launch_bounds__(BLOCK) BM_TRACE_OCCUPANCY void k_trace_quad_fetch(const TraceParams p) {
    __shared__ uint2 s_stk[LDS_N][QRAYS];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int c = lane & 3, q = lane >> 2;
    QStack<LDS_N> st;
    st.s = s_stk;
    st.ray = w * 16 + q;
    const uint32_t slot = blockIdx.x * QRAYS + st.ray;
    st.g_ref = p.ovf_ref;
    st.g_t = p.ovf_t;
    st.slot = slot;
    st.stride = p.ovf_stride;
    const uint32_t tiles_x = (p.width + 3) / 4, tiles_y = (p.local_rows + 3) / 4;
    const uint32_t ntiles = tiles_x * tiles_y;
    const uint32_t nwaves = gridDim.x * WAVES;
    const uint32_t wg = __builtin_amdgcn_readfirstlane(blockIdx.x * WAVES + w);
    const uint32_t R = wg < ntiles ? 16u * ((ntiles - wg + nwaves - 1) / nwaves) : 0u;  // this wave's rays
    const uint32_t refill_min = p.refill_min ? min(p.refill_min, 16u) : 8u;
    const vec3f eye = v3(p.eye[0], p.eye[1], p.eye[2]);
    const unsigned long long below = (1ull << (4 * q)) - 1ull;  // lanes of the quads before this one
    uint32_t r_next = 0;
    bool active = false;
    uint32_t x = 0, lr = 0, ibest = NO_TRI, next = EMPTY_REF;
    vec3f dir = v3(0.f, 0.f, 0.f), inv = dir;
    float tbest = 0.f, bu = 0.f, bv = 0.f;
    int sp = 0;
    unsigned long long cn = 0, ct = 0, ch = 0;
    __builtin_amdgcn_s_setprio(0);
    for (;;) {
        if (r_next < R) {
            const unsigned long long idle = ballot(!active && c == 0);  // bit 4q per idle quad
            const uint32_t nidle = (uint32_t)__popcll(idle);
            if (nidle >= refill_min) {
                if (!active) {
                    const uint32_t r = r_next + (uint32_t)__popcll(idle & below);
                    if (r < R) {
                        const uint32_t tile = wg + (r >> 4) * nwaves, j = r & 15u;
                        x = (tile % tiles_x) * 4 + (j & 3u);
                        lr = (tile / tiles_x) * 4 + (j >> 2);
                        const uint32_t gy = lr < p.local_rows ? global_row(p, lr) : p.height;
                        if (x < p.width && gy < p.height) {
                            dir = primary_dir(p, x, gy);
                            inv = v3(1.f / dir.x, 1.f / dir.y, 1.f / dir.z);
                            tbest = __builtin_inff();
                            ibest = NO_TRI;
                            bu = bv = 0.f;
                            sp = 0;
                            next = p.num_tris ? 0u : EMPTY_REF;
                            active = true;
                        }
                    }
                }
                r_next += nidle;
                // the wave's last rays hold its critical path: raise its issue priority
                if (r_next >= R) __builtin_amdgcn_s_setprio(1);
            }
        } else if (ballot(active) == 0) {
            break;
        }
        if (!active) continue;
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
            if (!found) {
                // ray done: shade and write its four planes (one per lane of the quad)
                const size_t o = (size_t)lr * p.width + x;
                uint32_t packed = MISS_PACKED;
                float nzv = 0.0f;
                if (ibest != NO_TRI) {
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
                if (c == 0) p.packed[(size_t)lr * p.pitch_u32 + x] = packed;
                else if (c == 1) p.tri_id[o] = ibest;
                else if (c == 2) p.t[o] = tbest;
                else if (p.nz) p.nz[o] = nzv;
                active = false;
                continue;
            }
        }
        if (next & LEAF_BIT) {
            const uint32_t first = next & FIRST_MASK, cnt = ((next >> 27) & 15u) + 1u;
            for (uint32_t k0 = 0; k0 < cnt; k0 += 4) {
                const uint32_t k = first + k0 + c;
                float t = __builtin_inff(), u = 0.f, v = 0.f;
                uint32_t id = NO_TRI;
                if (k0 + c < cnt) {
                    const float4 a = p.tris[3 * k + 0], b = p.tris[3 * k + 1], cc = p.tris[3 * k + 2];
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
            continue;
        }
        if (COUNT && c == 0) ++cn;
        next = quad_visit(p, next, c, eye, inv, tbest, true, st, sp);
    }
    const unsigned long long zero[3] = {0, 0, 0};
    flush_counters<COUNT>(p, cn, ct, ch, zero);
}

template <bool COUNT, int SH, int W>
hipError_t launch_variant_ab(const TraceParams& p, int variant, hipStream_t s, uint32_t* grid) {
    const dim3 tiles((p.width + 15) / 16, (p.local_rows + 15) / 16);
    switch (variant) {
        case TRACE_TILES_SCRATCH16: k_trace_tiles<COUNT, 16, OVF_SCRATCH, SH, W><<<tiles, BLOCK, 0, s>>>(p); break;
        case TRACE_TILES_NOOVF16: k_trace_tiles<COUNT, 16, OVF_NONE, SH, W><<<tiles, BLOCK, 0, s>>>(p); break;
        case TRACE_PERSIST_GLOBAL16:
            launch_persistent(k_trace_persistent<COUNT, 16, OVF_GLOBAL, 0, SH, W>, p, s, grid);
            break;
        case TRACE_PERSIST_GLOBAL8: launch_persistent(k_trace_persistent<COUNT, 8, OVF_GLOBAL, 0, SH, W>, p, s, grid); break;
        case TRACE_PERSIST_GLOBAL12:
            launch_persistent(k_trace_persistent<COUNT, 12, OVF_GLOBAL, 0, SH, W>, p, s, grid);
            break;
        case TRACE_PERSIST_PRIO8: launch_persistent(k_trace_persistent<COUNT, 8, OVF_GLOBAL, 1, SH, W>, p, s, grid); break;
        case TRACE_PERSIST_DYN12:
            launch_persistent(k_trace_persistent<COUNT, 12, OVF_GLOBAL, 1, SH, W, true>, p, s, grid);
            break;
        case TRACE_PERSIST_DYN16:
            launch_persistent(k_trace_persistent<COUNT, 16, OVF_GLOBAL, 1, SH, W, true>, p, s, grid);
            break;
        case TRACE_PAIR:
            if constexpr (W == 4 && SH == SH_NONE) {
                launch_persistent(k_trace_pair<COUNT, PAIR_LDS, 1>, p, s, grid);
                break;
            }
            [[fallthrough]];
        case TRACE_QUAD_FETCH:
            if constexpr (W == 4 && SH == SH_NONE) {
                launch_persistent(k_trace_quad_fetch<COUNT, QUAD_LDS>, p, s, grid);
                break;
            }
            // shadow rays or BVH2: what the product's TRACE_QUAD runs for them (bm_trace.hip)
            if constexpr (W == 4 && SH != SH_QUEUE)
                launch_persistent(k_trace_quad<COUNT, QUAD_LDS, 1, SH>, p, s, grid);
            else
                launch_persistent(k_trace_persistent<COUNT, 12, OVF_GLOBAL, 1, SH, W>, p, s, grid);
            break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <bool COUNT, int SH>
hipError_t launch_ab(const TraceParams& p, hipStream_t s, uint32_t* grid) {
    if (p.bvh_width == 8) {  // BVH8: the quad kernel only (primary or fused shadow rays)
        if constexpr (SH == SH_QUEUE) {
            return hipErrorInvalidValue;
        } else {
            if (COUNT && p.diag) launch_persistent(k_trace_quad<true, QUAD_LDS, 1, SH, true, 8>, p, s, grid);
            else launch_persistent(k_trace_quad<COUNT, QUAD_LDS, 1, SH, false, 8>, p, s, grid);
            return hipGetLastError();
        }
    }
    return p.bvh_width == 4 ? launch_variant_ab<COUNT, SH, 4>(p, p.variant, s, grid)
                            : launch_variant_ab<COUNT, SH, 2>(p, p.variant, s, grid);
}

}  // namespace

hipError_t launch_trace_ab(const TraceParams& p, bool count, int sh, hipStream_t s, uint32_t* grid) {
    switch (sh) {
        case SH_NONE: return count ? launch_ab<true, SH_NONE>(p, s, grid) : launch_ab<false, SH_NONE>(p, s, grid);
        case SH_FUSED: return count ? launch_ab<true, SH_FUSED>(p, s, grid) : launch_ab<false, SH_FUSED>(p, s, grid);
        default: return count ? launch_ab<true, SH_QUEUE>(p, s, grid) : launch_ab<false, SH_QUEUE>(p, s, grid);
    }
}

}  // namespace bm
#endif  // BM_TRACE_AB
