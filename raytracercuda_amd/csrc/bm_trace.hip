// bm_trace.hip — per-pixel primary-ray trace for gfx950 (replaces bmMarchKernel,
// Raytracer/BuildTree.cu:367-499; Trace.cu and Trace2.cu carry no live semantics).
//
// The product kernels (device code in bm_trace_dev.h):
//   k_trace_quad    ray quads (four lanes per ray over the BVH4, 4x4 pixels per wave), persistent
//                   grid, block-dynamic LDS tile tickets, XCD-aware runs, cost-ordered schedule;
//                   primary rays or primary + fused shadow rays
//   k_cull + k_trace_rays  frames in flight over sparse views: lane-per-ray root cull with ballot
//                   compaction, then quads over the survivors
//   k_trace_persistent<.., 12, OVF_GLOBAL, 1>  one lane per pixel (8x8 tiles per wave): BVH2 scenes
//                   and the shadow-queue study; k_shadow_persistent drains that queue
//   k_reshade, k_clear, k_pin_ops  multi-GPU reshading, render-target clear, the glm-pin self-test
// The ray direction is rebuilt on the device from the camera's column/row tables with the
// reference's exact arithmetic (Camera.cpp:51-66), so no 12-byte-per-pixel ray table is read.
// Traversal stacks live in LDS, with a global overflow area indexed by the thread's slot in the
// persistent grid (no scratch).
#include "bm_trace_dev.h"

namespace bm {
namespace {

// Shadow pass: persistent waves over the compacted queue of hit pixels, 64 entries per wave step
// (SURVEY §8(d) C5). The primary t is read back from the t plane; the ray direction is rebuilt
// exactly as in trace_pixel.
template <bool COUNT, int LDS_N, uint32_t PRIO, int W>
__global__ __launch_bounds__(BLOCK) void k_shadow_persistent(const TraceParams p) {
    __shared__ uint32_t s_ref[LDS_N][BLOCK];
    __shared__ float s_t[LDS_N][BLOCK];
    const int tid = threadIdx.x;
    Stack<LDS_N, OVF_GLOBAL> st;
    st.s_ref = s_ref;
    st.s_t = s_t;
    st.tid = tid;
    const uint32_t slot = blockIdx.x * BLOCK + tid;
    st.g_ref = p.ovf_ref + slot;
    st.g_t = p.ovf_t + slot;
    st.stride = p.ovf_stride;
    const uint32_t count = *p.queue_count;
    const vec3f eye = v3(p.eye[0], p.eye[1], p.eye[2]);
    unsigned long long cn = 0, ct = 0, co = 0;
    for (uint32_t q = slot; q - (tid & 63) < count; q += gridDim.x * BLOCK) {  // wave-uniform bound
        if (q >= count) continue;
        const uint32_t pix = p.queue[q];
        const uint32_t lr = pix / p.width, x = pix - lr * p.width;
        const vec3f dir = primary_dir(p, x, global_row(p, lr));
        vec3f o, d;
        shadow_segment(p, eye, dir, p.t[pix], o, d);
        __builtin_amdgcn_s_setprio(0);
        const bool occ = shadow_ray<COUNT, decltype(st), PRIO, W>(p, st, o, d, cn, ct);
        p.shadow[pix] = occ ? 1 : 0;
        if (COUNT) co += occ;
    }
    if (COUNT) {
        atomicAdd(&p.shadow_counters[0], cn);
        atomicAdd(&p.shadow_counters[1], ct);
        atomicAdd(&p.shadow_counters[2], co);
    }
}

// Self-test of the scalar primitives (bm_debug_primitives): one record per thread in the layout of
// oracle/beam_oracle.c orc_pin_ops — orient_mul, 1/dir, tri_test (the trace's Möller-Trumbore with
// its exact-safe early reject, on e1 = v1 - v0, e2 = v2 - v0 as the build computes them) and
// shade_normals — the device code the trace kernels run, checked against the reference's glm.
__global__ __launch_bounds__(256) void k_pin_ops(uint32_t n, const float* __restrict__ in, float* __restrict__ out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float* a = in + 36 * (size_t)i;
    float* o = out + 12 * (size_t)i;
    const vec3f d = orient_mul(a + 6, v3(a[3], a[4], a[5]));
    o[0] = d.x, o[1] = d.y, o[2] = d.z;
    o[3] = 1.f / d.x, o[4] = 1.f / d.y, o[5] = 1.f / d.z;
    const vec3f v0 = v3(a[15], a[16], a[17]);
    const vec3f e1 = sub(v3(a[18], a[19], a[20]), v0), e2 = sub(v3(a[21], a[22], a[23]), v0);
    float t, u, v;
    const bool in_tri = tri_test(make_float4(v0.x, v0.y, v0.z, 0.f), make_float4(e1.x, e1.y, e1.z, 0.f),
                                 make_float4(e2.x, e2.y, e2.z, 0.f), v3(a[0], a[1], a[2]), d, t, u, v);
    o[6] = in_tri ? t : 3.40282347e+38f;
    o[7] = in_tri ? u : 0.f;
    o[8] = in_tri ? v : 0.f;
    float z;
    o[9] = u2f(shade_normals(a + 24, a[33], a[34], z));
    o[10] = z;
    o[11] = 0.f;
}

// Multi-GPU exchange by triangle id (bm_options.gather_planes == 0): only the id plane travels, and
// the root rebuilds each hit pixel's t, |n.z| and packed colour by re-running Möller-Trumbore on
// that triangle for that pixel's ray — the same operations on the same operands as the trace that
// chose it (tri_orig holds the bit-identical (v0, e1, e2) records the trace's copies came from),
// so every plane equals a single-device trace bit for bit. Misses: the miss colour, +inf, 0.
__global__ __launch_bounds__(256) void k_reshade(const TraceParams p, const float4* __restrict__ tri_orig) {
    const uint32_t x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
    if (x >= p.width || y >= p.height) return;
    const size_t o = (size_t)y * p.width + x;
    const uint32_t id = p.tri_id[o];
    uint32_t packed = MISS_PACKED;
    float tout = __builtin_inff(), nzv = 0.0f;
    if (id != NO_TRI) {
        const vec3f dir = primary_dir(p, x, y);
        const vec3f eye = v3(p.eye[0], p.eye[1], p.eye[2]);
        float t = 0.f, u = 0.f, v = 0.f;
        (void)tri_test(tri_orig[3 * (size_t)id], tri_orig[3 * (size_t)id + 1], tri_orig[3 * (size_t)id + 2], eye, dir,
                       t, u, v);
        // bmFaceInterpolate<vec3> + normalize + pack (CudaComon.cuh:253-266, BuildTree.cu:489-491)
        const float* n = p.nrm + 9 * (size_t)id;
        const float ww = 1.f - (u + v);
        const vec3f nn = v3((n[0] * ww + n[3] * u) + n[6] * v, (n[1] * ww + n[4] * u) + n[7] * v,
                            (n[2] * ww + n[5] * u) + n[8] * v);
        const float il = 1.f / sqrtf(dot(nn, nn));
        const float z = nn.z * il;
        const float rr = fabsf(z * 255.f);
        packed = ((rr == rr) ? (uint32_t)rr : 0u) << 16;
        nzv = fabsf(z);
        tout = t;
    }
    p.packed[(size_t)y * p.pitch_u32 + x] = packed;
    p.t[o] = tout;
    if (p.nz) p.nz[o] = nzv;
}

__global__ __launch_bounds__(256) void k_clear(uint32_t* buf, uint32_t pitch_u32, uint32_t width, uint32_t height,
                                               uint32_t value) {
    const uint32_t x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
    if (x < width && y < height) buf[(size_t)y * pitch_u32 + x] = value;
}

template <bool COUNT, int SH, int W>
hipError_t launch_variant(const TraceParams& p, int variant, hipStream_t s, uint32_t* grid) {
    switch (variant) {
        case TRACE_PERSIST_DIAG12:
            if (!COUNT || SH) return hipErrorInvalidValue;
            launch_persistent(k_trace_persistent<true, 12, OVF_GLOBAL, 1, SH_NONE, W, false, true>, p, s, grid);
            break;
        case TRACE_PERSIST_PRIO12: launch_persistent(k_trace_persistent<COUNT, 12, OVF_GLOBAL, 1, SH, W>, p, s, grid); break;
        case TRACE_COMPACT:
            if constexpr (W == 4 && SH != SH_QUEUE) {
                if (p.rayq) {  // the host sized the ray queue (trace_compact_layout)
                    k_cull<COUNT, SH><<<p.rayq_regions, BLOCK, 0, s>>>(p);
                    if (COUNT && p.diag) launch_persistent(k_trace_rays<true, QUAD_LDS, 1, SH, true>, p, s, grid);
                    else if (p.prio_after == 0) launch_persistent(k_trace_rays<COUNT, QUAD_LDS, 0, SH>, p, s, grid);
                    else launch_persistent(k_trace_rays<COUNT, QUAD_LDS, 1, SH>, p, s, grid);
                    break;
                }
            }
            [[fallthrough]];
        case TRACE_PACKET:
            // wave packets: BVH4 primary rays, non-counting (a packet's visit order is not the oracle's)
            if constexpr (W == 4 && SH == SH_NONE && !COUNT) {
                const uint32_t tiles = ((p.width + 7) / 8) * ((p.local_rows + 7) / 8);
                if (BM_PK_SCHED == 0) {
                    if (grid) *grid = 0;
                    if (p.diag) k_trace_packet<SH_NONE, true><<<(tiles + WAVES - 1) / WAVES, BLOCK, 0, s>>>(p);
                    else k_trace_packet<SH_NONE><<<(tiles + WAVES - 1) / WAVES, BLOCK, 0, s>>>(p);
                } else if (p.diag) {
                    launch_persistent(k_trace_packet<SH_NONE, true>, p, s, grid);
                } else {
                    launch_persistent(k_trace_packet<SH_NONE>, p, s, grid);
                }
                break;
            }
            [[fallthrough]];
        case TRACE_QUAD:
            // ray quads need the BVH4 layout; BVH2 scenes and the shadow queue take the single-lane kernel
            if constexpr (W == 4 && SH != SH_QUEUE)
                if (COUNT && p.diag) launch_persistent(k_trace_quad<true, QUAD_LDS, 1, SH, true>, p, s, grid);
                else launch_persistent(k_trace_quad<COUNT, QUAD_LDS, 1, SH>, p, s, grid);
            else
                launch_persistent(k_trace_persistent<COUNT, 12, OVF_GLOBAL, 1, SH, W>, p, s, grid);
            break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <bool COUNT, int SH>
hipError_t launch_width(const TraceParams& p, hipStream_t s, uint32_t* grid) {
    if (p.bvh_width == 8 || !trace_variant_product(p.variant)) {  // A/B builds only (bm_trace_ab.hip)
#if BM_TRACE_AB
        return launch_trace_ab(p, COUNT, SH, s, grid);
#else
        return hipErrorInvalidValue;
#endif
    }
    return p.bvh_width == 4 ? launch_variant<COUNT, SH, 4>(p, p.variant, s, grid)
                            : launch_variant<COUNT, SH, 2>(p, p.variant, s, grid);
}

}  // namespace

bool trace_variant_persistent(int variant) { return variant >= TRACE_PERSIST_GLOBAL16 && variant != TRACE_PACKET; }

bool trace_variant_product(int variant) {
    return variant == TRACE_PERSIST_DIAG12 || variant == TRACE_PERSIST_PRIO12 || variant == TRACE_QUAD ||
           variant == TRACE_COMPACT || variant == TRACE_PACKET;
}

bool trace_variant_built(int variant) {
#if BM_TRACE_AB
    return variant >= 0 && variant < TRACE_NUM_VARIANTS;
#else
    return trace_variant_product(variant);
#endif
}

uint32_t quad_tiles(uint32_t width, uint32_t local_rows) {
    return ((width + QTW - 1) / QTW) * ((local_rows + QTH - 1) / QTH);
}

bool trace_compact_layout(uint32_t width, uint32_t local_rows, uint32_t min_tpr, uint32_t* regions,
                          uint32_t* tiles_per_region) {
    if (width == 0 || local_rows == 0 || width > 0xFFFFu || local_rows > 0xFFFFu) return false;
    const uint64_t ntiles = (uint64_t)((width + CULL_TILE - 1) / CULL_TILE) * ((local_rows + CULL_TILE - 1) / CULL_TILE);
    uint64_t tpr = min_tpr >= 4 ? (min_tpr + 3) / 4 * 4 : 32;  // tiles per region (a multiple of the 4 waves; 32: C2 in flight +1.7 %, C3 +3.4 % over 16)
    while ((ntiles + tpr - 1) / tpr > CULL_MAX_REGIONS) tpr += 4;
    *tiles_per_region = (uint32_t)tpr;
    *regions = (uint32_t)((ntiles + tpr - 1) / tpr);
    return true;
}

uint32_t trace_variant_lds(int variant) {
    switch (variant) {
        case TRACE_PERSIST_GLOBAL8: return 8;
        case TRACE_PERSIST_GLOBAL12:
        case TRACE_PERSIST_PRIO12: return 12;
        case TRACE_PERSIST_PRIO8: return 8;
        case TRACE_PERSIST_DYN12:
        case TRACE_PERSIST_DIAG12:
        case TRACE_QUAD:
        case TRACE_QUAD_FETCH:
        case TRACE_PAIR:
        case TRACE_COMPACT: return 12;  // sizes the overflow area: the quad kernel's fallback keeps 12 in LDS
        default: return 16;
    }
}

// Upper bound of the persistent grid (sizes the overflow area): 8 blocks of 4 waves per CU, the
// most a CU holds. Each launch uses min(this, what that kernel keeps resident: resident_blocks).
uint32_t trace_persistent_blocks(int variant, int device) {
    (void)variant;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return 0;
    return 8u * (uint32_t)prop.multiProcessorCount;
}

hipError_t launch_trace(const TraceParams& p, bool count, hipStream_t s, uint32_t* grid) {
    if (grid) *grid = 0;
    if (p.width == 0 || p.local_rows == 0) return hipSuccess;
    if (p.shadow && p.shadow_queue)
        return count ? launch_width<true, SH_QUEUE>(p, s, grid) : launch_width<false, SH_QUEUE>(p, s, grid);
    if (p.shadow) return count ? launch_width<true, SH_FUSED>(p, s, grid) : launch_width<false, SH_FUSED>(p, s, grid);
    return count ? launch_width<true, SH_NONE>(p, s, grid) : launch_width<false, SH_NONE>(p, s, grid);
}

template <int W>
void launch_shadow_w(const TraceParams& p, bool count, hipStream_t s) {
    switch (trace_variant_lds(p.variant)) {
        case 8:
            if (count) launch_persistent(k_shadow_persistent<true, 8, 1, W>, p, s, nullptr);
            else launch_persistent(k_shadow_persistent<false, 8, 1, W>, p, s, nullptr);
            break;
        case 16:
            if (count) launch_persistent(k_shadow_persistent<true, 16, 1, W>, p, s, nullptr);
            else launch_persistent(k_shadow_persistent<false, 16, 1, W>, p, s, nullptr);
            break;
        default:
            if (count) launch_persistent(k_shadow_persistent<true, 12, 1, W>, p, s, nullptr);
            else launch_persistent(k_shadow_persistent<false, 12, 1, W>, p, s, nullptr);
            break;
    }
}

hipError_t launch_shadow(const TraceParams& p, bool count, hipStream_t s) {
    if (p.width == 0 || p.local_rows == 0 || !p.shadow || !p.shadow_queue) return hipSuccess;
    if (p.bvh_width == 4) launch_shadow_w<4>(p, count, s);
    else launch_shadow_w<2>(p, count, s);
    return hipGetLastError();
}

hipError_t launch_pin_ops(uint32_t n, const float* in, float* out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    k_pin_ops<<<(n + 255) / 256, 256, 0, s>>>(n, in, out);
    return hipGetLastError();
}

hipError_t launch_reshade(const TraceParams& p, const float4* tri_orig, hipStream_t s) {
    if (p.width == 0 || p.height == 0) return hipSuccess;
    k_reshade<<<dim3((p.width + 255) / 256, p.height), 256, 0, s>>>(p, tri_orig);
    return hipGetLastError();
}

hipError_t launch_clear(uint32_t* buf, uint32_t pitch_u32, uint32_t width, uint32_t height, uint32_t value,
                        hipStream_t s) {
    if (width == 0 || height == 0) return hipSuccess;
    k_clear<<<dim3((width + 255) / 256, height), 256, 0, s>>>(buf, pitch_u32, width, height, value);
    return hipGetLastError();
}

}  // namespace bm

