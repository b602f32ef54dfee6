// bm_api.cpp — the C ABI (include/beam_c.h) over HIP: contexts, meshes, scenes, cameras and
// offscreen render targets. Host-side counterpart of the reference's Scene/SceneTree/Mesh/
// Camera/RenderTarget/DeviceBuffer classes (Raytracer/*.cpp), minus GL interop.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/beam_c.h"
#include "bm_internal.h"

#define BM_VERSION_STRING "beam-mi355x 0.1 (gfx950, LBVH + wave64 trace)"

struct bm_context {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    uint32_t leaf_size = 4;
    bool auto_packet = true;  // dense coherent views: wave packets (trace_impl)
    int trace_variant = bm::TRACE_QUAD;  // ray quads, block-dynamic tile order (BVH2 and the shadow queue: single-lane)
    uint32_t persistent_blocks = 0;
    uint32_t scramble = 0;
    uint32_t prio_after = 24, prio_level = 2;
    uint32_t refill_min = 8;
    // quad tiles: 2 = block-dynamic, longest first by the last trace of the render target (frames one
    // at a time: the heavy tiles must not start last); 1 = block-dynamic in screen order (targets on
    // their own streams: overlapping frames fill each other's tails, and screen order measured
    // faster there, 72.7 vs 76.3 us per bunny frame); -1 = that choice per target, else forced
    int sched = -1;
    uint32_t cull_tpr = 0;  // compacted trace: tiles per culling workgroup (0: 32)
    // frames in flight on sparse views: cull + compacted quads (TRACE_COMPACT) instead of plain quads
    // when the scene's box covers under half the frame (trace_impl); BM_TRACE_AUTO=0 turns it off
    bool auto_compact = true;
    bool shadow_queue = false;  // BM_OPT_SHADOW_QUEUE
    bool reference_kd = false;    // BM_OPT_REFERENCE_KD
    bool reference_hash = false;  // BM_OPT_REFERENCE_HASH
    uint32_t bvh_width = 4;     // BM_OPT_BVH2 -> 2
    void* ovf = nullptr;  // traversal-stack overflow area of the persistent trace grid
    size_t ovf_cap = 0;
    unsigned long long* tile_ctr = nullptr;  // ticket counter of the dynamic trace variants
    unsigned long long tile_base = 0;        // its value at the next launch
    // render targets with their own stream (bm_rt_set_stream): traces into them run there, ordered
    // after the context stream's work by `ready` (recorded when `epoch` moved on since the target's
    // last trace), and the context stream waits for their last trace before it rebuilds anything
    std::vector<bm_rt*> rt_streams;
    std::vector<bm_rt*> rts;  // every live render target (detached by bm_context_destroy)
    hipEvent_t ready = nullptr;
    uint64_t epoch = 1;
    uint32_t* post = nullptr;   // pinned coherent host words of readback (64 x u32)
    uint32_t* post_dev = nullptr;
    uint32_t post_seq = 0;
    std::string last_error;
    // multi-GPU (bm_options.devices / comm_*): this context is the root; peers[g-1] is a plain
    // single-device context for device g, holding the replicas of every object made here
    std::vector<bm_context*> peers;
    std::vector<int> devices;   // devices[g] of the band layout (root first)
    uint32_t band_h = 16;
    uint32_t gather = 0;        // resolved transport: BM_GATHER_PEER or BM_GATHER_RCCL
    uint32_t planes = 0;        // BM_PLANE_* mask gathered
    const bm::Rccl* rccl = nullptr;
    std::vector<void*> nccl;    // one process, RCCL transport: ncclComm_t per device
    void* comm = nullptr;       // several processes: ncclComm_t of this rank (or the loopback's)
    bool rccl_loopback = false; // one process, RCCL over a repeated device list: self send/recv
    int comm_rank = 0, comm_size = 1;
    bm::Tuning tune;            // bm_context_set_param (BM_PARAM_*); the fields above follow it (apply_params)
    bool multi() const { return !peers.empty() || comm_size > 1; }
    uint32_t bands_n() const { return comm_size > 1 ? (uint32_t)comm_size : (uint32_t)devices.size(); }
};

namespace {

int32_t fail(bm_context* ctx, int32_t code, const std::string& msg) {
    if (ctx) ctx->last_error = msg;
    return code;
}

int32_t hip_fail(bm_context* ctx, hipError_t e, const char* what) {
    std::string m = std::string(what) + ": " + hipGetErrorName(e) + " (" + hipGetErrorString(e) + ")";
    return fail(ctx, e == hipErrorOutOfMemory ? BM_ERROR_GPU_ALLOC_FAIL : BM_ERROR_DEVICE, m);
}

#define BM_HIP(ctx, expr)                                       \
    do {                                                        \
        hipError_t e__ = (expr);                                \
        if (e__ != hipSuccess) return hip_fail(ctx, e__, #expr); \
    } while (0)

// Grow-only device buffer (the reference's DeviceBuffer, DeviceBuffer.cpp:7-58, without the
// per-call cudaMalloc).
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t reserve(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        hipError_t e = hipMalloc(&p, bytes ? bytes : 16);
        if (e == hipSuccess) cap = bytes;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <class T>
    T* as() const {
        return reinterpret_cast<T*>(p);
    }
};

}  // namespace

struct bm_mesh {
    bm_context* ctx = nullptr;
    std::vector<bm_mesh*> rep;  // replicas on the context's peer devices
    uint32_t num_vertices = 0;
    uint32_t num_indices = 0;
    uint32_t max_index = 0;  // host-side bound check before any kernel reads through the indices
    DevBuf slot[BM_VERTEX_DATA_COUNT];
    uint32_t slot_comp[BM_VERTEX_DATA_COUNT] = {};
    DevBuf idx;
};

struct bm_scene {
    bm_context* ctx = nullptr;
    std::vector<bm_scene*> rep;  // replicas on the context's peer devices
    std::vector<bm_mesh*> meshes;
    bool built = false;
    uint32_t n = 0, nrec = 0, leaf_size = 4, width = 4;
    std::vector<std::pair<bm_mesh*, uint32_t>> built_with;  // meshes + triangle counts of the last build
    // reference mode (bm_kd.hip)
    bool kd = false;
    uint32_t kd_pairs = 0, kd_leaves = 0;
    // hashed-grid mode (Hash.cu): sorted (bucket, triangle) pairs in kd_keys/kd_vals(2), bucket ranges
    bool hash = false;
    DevBuf hash_bstart, hash_bend;
    bool kd_sorted_in_scratch = false;
    bool kd_top_rank = false;  // the last reference-mode build sorted its pairs with the ranked top digit
    DevBuf kd_counts, kd_offsets, kd_sums, kd_total, kd_keys, kd_vals, kd_keys2, kd_vals2, kd_smeta,
        kd_leaf_of, kd_leaf_key, kd_leaf_start, kd_leaf_count, kd_lch, kd_rch, kd_first, kd_last, kd_pleaf, kd_pint,
        kd_nodes, kd_leafrec, kd_ftris, kd_node_key, kd_cnodes,  // march records (launch_kd_records, launch_kd_leaves)
        kd_ubox,   // union of the leaf cells (launch_kd_records): the march's exact miss cull
        kd_cache,  // the count pass's first leaves per triangle (KdBuild::cache)
        kd_queue, kd_fill;  // split descent: queued subtrees (+ count word), emit cursors
    DevBuf mesh_table, tri_orig, nrm, aabb, cen, bounds, keys, vals, keys2, vals2, lch, rch, first, last,
        parent_leaf, parent_int, ibox, pre, suf, table, records, records2, tris;  // records2: BVH8 builds' BVH2 records
    bm::MeshDesc* staging = nullptr;  // pinned host copy of the mesh table
    size_t staging_cap = 0;
    bool replicas_clean = false;       // bounds' gather replicas left zero by the last LBVH build/refit (bm_build.hip)
    uint32_t* hbounds = nullptr;       // pinned: the last build's scene box (ordered images, 6 words)
    hipEvent_t hbounds_ev = nullptr;   // ... valid once this has completed; word 8: the build's sort skew word
    hipEvent_t staging_done = nullptr, ev0 = nullptr, ev1 = nullptr;
    uint32_t sort_path = 0;            // BM_SORT_* of the last build (MSD until its skew word is read)
    bool orig_valid = false;           // tri_orig holds the last build's original-order records (reshade)
    // tri_orig was rebuilt lazily by a multi-device trace on a render target's stream (the scene was built
    // before the context had peers): every later reshade, on whatever stream, waits for orig_ev
    bool orig_lazy = false;
    hipEvent_t orig_ev = nullptr;
    // reference mode: the leaf count reaches the host after the build (k_post into this pinned area, word 0;
    // sequence in POST_SEQ_WORD), read by kd_leaves_ready when a trace or kdStats needs it
    uint32_t* kd_post = nullptr;
    uint32_t* kd_post_dev = nullptr;
    uint32_t kd_post_seq = 0;
    bool kd_leaves_pending = false;
    uint32_t kd_leaf_cap = 0;          // leaf-side buffers' capacity of the last build (min(pairs, leaf limit))
    bool kd_cnodes_valid = false;      // the last build wrote the child-box records (BM_PARAM_KD_MARCH 3)
    uint32_t scan_epoch = 0;           // launch_exclusive_scan's call epoch on kd_sums (no zero fill per call)
    uint32_t num_meshes = 0;           // mesh-table entries of the last build
};

struct bm_camera {
    bm_context* ctx = nullptr;
    std::vector<bm_camera*> rep;  // replicas on the context's peer devices
    uint32_t width = 0, height = 0;
    float left = 0.f, top = 0.f, dx = 0.f, dy = 0.f;  // setInitialRays' screen window
    float zoom = 1.f, z2 = 1.f;
    DevBuf rx, ry;
    DevBuf counters;
};

struct bm_rt {
    bm_context* ctx = nullptr;
    uint32_t width = 0, height = 0, pitch = 0;
    bool external = false, locked = false;
    DevBuf storage;
    uint32_t* packed = nullptr;
    uint32_t* tri = nullptr;
    float* t = nullptr;
    float* nz = nullptr;
    DevBuf shadow;  // u8 plane (width x height), allocated by the first shadow trace
    DevBuf queue;   // shadow-pass queue: count word, then up to width x height pixel indices
    DevBuf rayq;    // compacted trace: region counts, then the regions' ray entries
    DevBuf tile_cost;  // cost-ordered schedule (sched 2): last trace's time per quad-kernel tile
    hipStream_t stream = nullptr;  // bm_rt_set_stream; null: the context stream
    hipEvent_t done = nullptr;     // recorded after each trace on `stream`
    uint64_t epoch = 0;            // context epoch this target's stream last synchronised with
    DevBuf ovf;                    // traversal-stack overflow area of traces on `stream`
    int32_t last_kind = -1;        // BM_TRACE_KIND_* of the last trace into this target
    // multi-GPU traces into this (root) target: per band source g, a compact band buffer on device
    // g's context with its own stream; RCCL staging on the root; start/done events
    std::vector<bm_rt*> band;
    std::vector<hipStream_t> band_stream;  // owned (null for a band buffer on this target's stream)
    std::vector<hipEvent_t> band_done;     // recorded on band_stream[g] after its gather step
    hipEvent_t mg_start = nullptr;         // recorded on this target's stream as a multi trace begins
    hipEvent_t mg_t[3] = {};               // timing: trace start, band 0 traced, exchange done (bm_rt_last_timing)
    bool mg_timed = false;                 // mg_t holds a recorded frame
    DevBuf stage;                          // RCCL: the other sources' band planes, received on the root
};

namespace {

// The stream a render target's traces, clears and readbacks run on.
hipStream_t rt_stream(const bm_rt* rt) { return rt->stream ? rt->stream : rt->ctx->stream; }

// Context-stream work that traces read (builds, ray tables) is about to change: wait (on the
// device) for the last trace of every render target with its own stream, and open a new epoch.
hipError_t ctx_drain(bm_context* ctx) {
    for (bm_rt* r : ctx->rt_streams) {
        hipError_t e = hipStreamWaitEvent(ctx->stream, r->done, 0);
        if (e != hipSuccess) return e;
    }
    ++ctx->epoch;
    return hipSuccess;
}

// Host wait for the context stream and every render-target stream.
hipError_t ctx_sync_all(bm_context* ctx) {
    hipError_t e = hipStreamSynchronize(ctx->stream);
    for (bm_rt* r : ctx->rt_streams)
        if (e == hipSuccess) e = hipStreamSynchronize(r->stream);
    return e;
}

// Grow-only reallocation of buffers that traces read (records, triangles, normals, ray tables):
// hipFree gives no ordering guarantee against work still queued on other streams, so before the
// first buffer of an update actually grows, wait on the host for the context stream and every
// render-target stream (growth is rare: a larger scene or frame than any before).
struct GrowGuard {
    bm_context* ctx;
    bool synced = false;
    hipError_t reserve(DevBuf& b, size_t bytes) {
        if (bytes > b.cap && !synced) {
            hipError_t e = ctx_sync_all(ctx);
            if (e != hipSuccess) return e;
            synced = true;
        }
        return b.reserve(bytes);
    }
};

// Before a trace on a render target's own stream: order it after the context stream's work.
hipError_t rt_acquire(bm_rt* rt) {
    bm_context* ctx = rt->ctx;
    if (!rt->stream || rt->epoch == ctx->epoch) return hipSuccess;
    hipError_t e = hipEventRecord(ctx->ready, ctx->stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(rt->stream, ctx->ready, 0);
    if (e == hipSuccess) rt->epoch = ctx->epoch;
    return e;
}

}  // namespace

// Multi-GPU state of a (root) render target: its band buffers on every device, their streams and
// events, the RCCL staging area. Recreated by the next multi-device trace.
static void mg_release(bm_rt* rt) {
    for (size_t g = 0; g < rt->band.size(); ++g) {
        const int dev = rt->band[g]->ctx ? rt->band[g]->ctx->device : -1;
        bm_rt_destroy(rt->band[g]);  // waits for its stream
        if (dev >= 0) (void)hipSetDevice(dev);
        if (rt->band_stream[g]) (void)hipStreamDestroy(rt->band_stream[g]);
        if (rt->band_done[g]) (void)hipEventDestroy(rt->band_done[g]);
    }
    rt->band.clear();
    rt->band_stream.clear();
    rt->band_done.clear();
    if (rt->ctx) (void)hipSetDevice(rt->ctx->device);
    if (rt->mg_start) (void)hipEventDestroy(rt->mg_start);
    rt->mg_start = nullptr;
    for (hipEvent_t& e : rt->mg_t) {
        if (e) (void)hipEventDestroy(e);
        e = nullptr;
    }
    rt->mg_timed = false;
    rt->stage.release();
}

// Release a render target's device resources (its work is finished) and unlink it from its context.
static void detach_rt(bm_rt* rt) {
    if (rt->done) (void)hipEventDestroy(rt->done);
    rt->done = nullptr;
    rt->ovf.release();
    if (!rt->external) rt->storage.release();
    rt->packed = nullptr;
    rt->tri = nullptr;
    rt->t = nullptr;
    rt->nz = nullptr;
    rt->shadow.release();
    rt->queue.release();
    rt->rayq.release();
    rt->tile_cost.release();
    rt->stream = nullptr;
    rt->ctx = nullptr;
}

// Options of one trace call (the public entry points below fill these in).
struct TraceReq {
    uint32_t band_h = 16, band_step = 1, band_first = 0;
    bool exact = true;  // the render target must be exactly the camera's size
    bool count = false;
    unsigned long long* counters = nullptr;         // [3] primary
    unsigned long long* shadow_counters = nullptr;  // [3] shadow pass
    const float* light = nullptr;                   // non-null: add the shadow pass
    int variant_override = -1;
    unsigned long long* diag = nullptr;
    uint32_t* grid_out = nullptr;  // persistent grid of the primary launch
};

// A replica's call failed on a peer device: report it on the root context.
static int32_t peer_fail(bm_context* root, const bm_context* peer, int32_t rc) {
    if (root != peer) root->last_error = "device " + std::to_string(peer->device) + ": " + peer->last_error;
    return rc;
}

extern "C" {

// "+ab": an A/B build carrying the measured-slower trace variants and BVH8 (bm_trace_ab.hip)
const char* bm_version(void) { return BM_TRACE_AB ? BM_VERSION_STRING "+ab" : BM_VERSION_STRING; }

// The trace schedule fields of a context from its tuning parameters (defaults where unset).
static void apply_params(bm_context* ctx) {
    const bm::Tuning& t = ctx->tune;
    const int64_t v = t.get(BM_PARAM_TRACE_VARIANT, -1);
    ctx->trace_variant = v >= 0 ? (int)v : bm::TRACE_QUAD;
    ctx->scramble = (uint32_t)t.get(BM_PARAM_TRACE_SCRAMBLE, 0);
    ctx->prio_after = (uint32_t)t.get(BM_PARAM_TRACE_PRIO_AFTER, 24);
    ctx->prio_level = (uint32_t)t.get(BM_PARAM_TRACE_PRIO_LEVEL, 2);
    ctx->refill_min = (uint32_t)t.get(BM_PARAM_TRACE_REFILL_MIN, 8);
    ctx->sched = (int)t.get(BM_PARAM_TRACE_SCHED, -1);
    ctx->cull_tpr = (uint32_t)t.get(BM_PARAM_CULL_TILES, 0);
    // an explicit variant stays as set: no switch to the compacted trace on sparse views
    ctx->auto_compact = t.get(BM_PARAM_TRACE_AUTO_COMPACT, v >= 0 ? 0 : 1) != 0;
    ctx->auto_packet = t.get(BM_PARAM_TRACE_AUTO_PACKET, v >= 0 ? 0 : 1) != 0;
    ctx->persistent_blocks = bm::trace_persistent_blocks(ctx->trace_variant, ctx->device);
    const int64_t grid = t.get(BM_PARAM_TRACE_GRID, 0);
    if (grid > 0) ctx->persistent_blocks = std::min<uint32_t>(ctx->persistent_blocks, (uint32_t)grid);
}

static int32_t context_create_single(const bm_options& o, bm_context** out) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return BM_ERROR_DEVICE;
    if (o.device < 0 || o.device >= count) return BM_ERROR_INVALID_PARAMETER;
    if (o.leaf_size > 16) return BM_ERROR_INVALID_PARAMETER;
    if (hipSetDevice(o.device) != hipSuccess) return BM_ERROR_DEVICE;
    bm_context* ctx = new (std::nothrow) bm_context();
    if (!ctx) return BM_ERROR_GPU_ALLOC_FAIL;
    ctx->device = o.device;
    ctx->leaf_size = o.leaf_size ? o.leaf_size : 4;
    ctx->shadow_queue = (o.flags & BM_OPT_SHADOW_QUEUE) != 0;
    ctx->bvh_width = (o.flags & BM_OPT_BVH2) ? 2u : (o.flags & BM_OPT_BVH8) ? 8u : 4u;
#if !BM_TRACE_AB
    if (o.flags & BM_OPT_BVH8) {  // measured slower than BVH4: A/B builds only
        delete ctx;
        return BM_ERROR_INVALID_PARAMETER;
    }
#endif
    if ((o.flags & BM_OPT_BVH2) && (o.flags & BM_OPT_BVH8)) {
        delete ctx;
        return BM_ERROR_INVALID_PARAMETER;
    }
    ctx->reference_kd = (o.flags & BM_OPT_REFERENCE_KD) != 0;
    ctx->reference_hash = (o.flags & BM_OPT_REFERENCE_HASH) != 0;
    if (ctx->reference_kd && ctx->reference_hash) {
        delete ctx;
        return BM_ERROR_INVALID_PARAMETER;
    }
    apply_params(ctx);
    if (o.stream || (o.flags & BM_OPT_NULL_STREAM)) {
        ctx->stream = reinterpret_cast<hipStream_t>(o.stream);
    } else {
        if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
            delete ctx;
            return BM_ERROR_DEVICE;
        }
        ctx->own_stream = true;
    }
    ctx->devices.assign(1, ctx->device);
    *out = ctx;
    return BM_ERROR_ALL_FINE;
}

int32_t bm_context_create(const bm_options* opts, bm_context** out) {
    if (!out) return BM_ERROR_INVALID_PARAMETER;
    *out = nullptr;
    bm_options o{};
    if (opts) o = *opts;
    const bool procs = o.comm_size > 1;
    if (o.num_devices > BM_MAX_DEVICES || o.comm_size < 0 || o.comm_size > (int32_t)bm::MAX_BAND_SOURCES ||
        (procs && (o.comm_rank < 0 || o.comm_rank >= o.comm_size || o.num_devices > 1)) || o.gather > BM_GATHER_RCCL ||
        (o.gather_planes & ~(uint32_t)(BM_PLANE_PACKED | BM_PLANE_TRI_ID | BM_PLANE_T | BM_PLANE_NZ | BM_PLANE_SHADOW)))
        return BM_ERROR_INVALID_PARAMETER;
    if (o.num_devices >= 1) o.device = o.devices[0];
    const uint32_t n = procs ? 1u : std::max<uint32_t>(o.num_devices, 1u);
    if ((n > 1 || procs) && (o.flags & (BM_OPT_REFERENCE_KD | BM_OPT_REFERENCE_HASH)))
        return BM_ERROR_INVALID_PARAMETER;  // reference modes trace whole frames on one device
    bm_options root = o;
    root.num_devices = 0;
    int32_t rc = context_create_single(root, out);
    if (rc) return rc;
    bm_context* ctx = *out;
    ctx->band_h = o.band_height ? o.band_height : 16u;
    ctx->planes = o.gather_planes;  // 0: triangle ids (+ shadows) travel, the root reshades
    if (n == 1 && !procs) return BM_ERROR_ALL_FINE;
    *out = nullptr;
    if (procs) {  // one device per process: one RCCL communicator over the ranks
        rc = bm_context_start_comm(ctx, o.comm_rank, o.comm_size, o.comm_id);
        if (rc) {
            bm_context_destroy(ctx);
            return rc;
        }
        *out = ctx;
        return BM_ERROR_ALL_FINE;
    }
    // one process, n devices: a plain context per extra device (its own stream)
    bool distinct = true;
    for (uint32_t g = 1; g < n; ++g) {
        bm_options po = o;
        po.num_devices = 0;
        po.device = o.devices[g];
        po.stream = nullptr;
        po.flags &= ~BM_OPT_NULL_STREAM;
        bm_context* p = nullptr;
        rc = context_create_single(po, &p);
        if (rc) {
            bm_context_destroy(ctx);
            return rc;
        }
        ctx->peers.push_back(p);
        ctx->devices.push_back(o.devices[g]);
        for (uint32_t k = 0; k < g; ++k) distinct = distinct && o.devices[k] != o.devices[g];
    }
    // peer access: every other device writes the root's planes (BM_GATHER_PEER)
    bool peer_ok = true;
    for (uint32_t g = 1; g < n; ++g) {
        if (ctx->devices[g] == ctx->device) continue;
        int can = 0;
        if (hipDeviceCanAccessPeer(&can, ctx->devices[g], ctx->device) != hipSuccess || !can) {
            peer_ok = false;
            continue;
        }
        (void)hipSetDevice(ctx->devices[g]);
        const hipError_t e = hipDeviceEnablePeerAccess(ctx->device, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) peer_ok = false;
        (void)hipGetLastError();  // clear a sticky "already enabled"
    }
    (void)hipSetDevice(ctx->device);
    uint32_t gather = o.gather;
    if (gather == BM_GATHER_AUTO) gather = peer_ok || !distinct ? BM_GATHER_PEER : BM_GATHER_RCCL;
    if (gather == BM_GATHER_PEER && !peer_ok) {
        bm_context_destroy(ctx);
        return BM_ERROR_INVALID_PARAMETER;  // PEER needs peer access
    }
    ctx->gather = gather;
    if (gather == BM_GATHER_RCCL) {
        const char* why = "";
        ctx->rccl = bm::rccl_load(&why);
        if (!ctx->rccl) {
            bm_context_destroy(ctx);
            return BM_ERROR_DEVICE;
        }
        if (distinct) {  // one rank per device (ncclCommInitAll)
            ctx->nccl.assign(n, nullptr);
            if (bm::rccl_init_all(ctx->rccl, ctx->nccl.data(), (int)n, ctx->devices.data()) != 0) {
                bm_context_destroy(ctx);
                return BM_ERROR_DEVICE;
            }
        } else {
            // A repeated device (RCCL refuses two ranks on one GPU): one single-rank communicator
            // on the root, made like a multi-process one (unique id + ncclCommInitRank), and every
            // band source's planes travel as grouped send/recv to itself into the root's staging
            // area, then the same multi-source scatter — the RCCL gather path rehearsed on one GPU.
            uint8_t id[BM_COMM_ID_BYTES];
            ctx->rccl_loopback = true;
            if (bm::rccl_unique_id(ctx->rccl, id) != 0 || bm::rccl_init_rank(ctx->rccl, &ctx->comm, 1, id, 0) != 0) {
                bm_context_destroy(ctx);
                return BM_ERROR_DEVICE;
            }
        }
        (void)hipSetDevice(ctx->device);
    }
    *out = ctx;
    return BM_ERROR_ALL_FINE;
}

int32_t bm_context_start_comm(bm_context* ctx, int32_t rank, int32_t size, const uint8_t* comm_id) {
    if (!ctx) return BM_ERROR_INVALID_PARAMETER;
    if (!comm_id || size < 2 || size > (int32_t)bm::MAX_BAND_SOURCES || rank < 0 || rank >= size)
        return fail(ctx, BM_ERROR_INVALID_PARAMETER, "start_comm: rank/size out of range or no unique id");
    if (ctx->multi() || !ctx->rts.empty() || ctx->reference_kd || ctx->reference_hash)
        return fail(ctx, BM_ERROR_INVALID_PARAMETER,
                    "start_comm: needs a single-device context without render targets (not a reference mode)");
    const char* why = "";
    const bm::Rccl* r = bm::rccl_load(&why);
    if (!r) return fail(ctx, BM_ERROR_DEVICE, std::string("start_comm: RCCL unavailable: ") + why);
    BM_HIP(ctx, hipSetDevice(ctx->device));
    void* comm = nullptr;
    const int e = bm::rccl_init_rank(r, &comm, size, comm_id, rank);  // collective: every rank enters it
    if (e != 0) return fail(ctx, BM_ERROR_DEVICE, std::string("ncclCommInitRank: ") + bm::rccl_error_string(r, e));
    ctx->rccl = r;
    ctx->comm = comm;
    ctx->gather = BM_GATHER_RCCL;
    ctx->comm_rank = rank;
    ctx->comm_size = size;
    return BM_ERROR_ALL_FINE;
}

int32_t bm_context_set_param(bm_context* ctx, uint32_t key, int64_t value) {
    if (!ctx) return BM_ERROR_INVALID_PARAMETER;
    if (key >= BM_PARAM_COUNT || value < -1) return fail(ctx, BM_ERROR_INVALID_PARAMETER, "set_param: unknown key or value");
    if (key == BM_PARAM_TRACE_VARIANT && value >= 0 && !bm::trace_variant_built((int)value))
        return fail(ctx, BM_ERROR_INVALID_PARAMETER, "set_param: trace variant not compiled into this library");
    if (key == BM_PARAM_TRACE_SCHED && value > 2) return fail(ctx, BM_ERROR_INVALID_PARAMETER, "set_param: sched 0..2");
    if (key == BM_PARAM_KD_TB && value >= 0 && value != 64 && value != 256)
        return fail(ctx, BM_ERROR_INVALID_PARAMETER, "set_param: KD_TB is 64 or 256");
    if (key == BM_PARAM_KD_MARCH && value > 3) return fail(ctx, BM_ERROR_INVALID_PARAMETER, "set_param: KD_MARCH 0..3");
    if (key == BM_PARAM_TRACE_PRIO_LEVEL && value > 3) return fail(ctx, BM_ERROR_INVALID_PARAMETER, "set_param: prio 0..3");
    // k_front (one-launch gather + keys + top-digit pass) was removed in round 5
    if (key == BM_PARAM_FRONT_MAX_N && value > 0)
        return fail(ctx, BM_ERROR_INVALID_PARAMETER, "set_param: FRONT_MAX_N: k_front was removed (always 0)");
    // a top-digit-first sort's device-side LSD fallback covers at most RADIX tiles: 2^22 keys is the
    // largest scene it is correct for (bm_build.hip msd_sort clamps to it as well)
    if (key == BM_PARAM_MSD_MAX_N && value > (int64_t)bm::MSD_MAX_N_CAP)
        return fail(ctx, BM_ERROR_INVALID_PARAMETER, "set_param: MSD_MAX_N is at most 2^22");
    for (bm_context* p : ctx->peers) {
        const int32_t rc = bm_context_set_param(p, key, value);
        if (rc) return peer_fail(ctx, p, rc);
    }
    BM_HIP(ctx, hipSetDevice(ctx->device));
    ctx->tune.v[key] = value;
    apply_params(ctx);
    return BM_ERROR_ALL_FINE;
}

int64_t bm_context_get_param(const bm_context* ctx, uint32_t key) {
    if (!ctx || key >= BM_PARAM_COUNT) return INT64_MIN;
    return ctx->tune.v[key];
}

uint32_t bm_context_num_devices(const bm_context* ctx) { return ctx ? ctx->bands_n() : 0; }

int32_t bm_comm_available(void) { return bm::rccl_load(nullptr) ? BM_ERROR_ALL_FINE : BM_ERROR_DEVICE; }

uint32_t bm_context_gather(const bm_context* ctx) {
    if (!ctx || !ctx->multi()) return 0;
    return ctx->rccl_loopback ? BM_GATHER_RCCL_LOOPBACK : ctx->gather;
}

int32_t bm_comm_unique_id(uint8_t* id) {
    if (!id) return BM_ERROR_INVALID_PARAMETER;
    const bm::Rccl* r = bm::rccl_load(nullptr);
    if (!r) return BM_ERROR_DEVICE;
    return bm::rccl_unique_id(r, id) == 0 ? BM_ERROR_ALL_FINE : BM_ERROR_DEVICE;
}

void bm_context_destroy(bm_context* ctx) {
    if (!ctx) return;
    (void)bm_sync(ctx);
    // render targets still alive (a caller error: handles go before their context) are detached:
    // their band buffers on the peers go first, then their own device memory; a later
    // bm_rt_destroy only frees the handle
    for (bm_rt* rt : ctx->rts) mg_release(rt);
    for (void* c : ctx->nccl)
        if (c) bm::rccl_destroy(ctx->rccl, c);
    if (ctx->comm) bm::rccl_destroy(ctx->rccl, ctx->comm);
    for (bm_context* p : ctx->peers) bm_context_destroy(p);
    ctx->peers.clear();
    (void)hipSetDevice(ctx->device);
    for (bm_rt* rt : ctx->rts) detach_rt(rt);
    if (ctx->own_stream && ctx->stream) (void)hipStreamDestroy(ctx->stream);
    if (ctx->ovf) (void)hipFree(ctx->ovf);
    if (ctx->tile_ctr) (void)hipFree(ctx->tile_ctr);
    if (ctx->ready) (void)hipEventDestroy(ctx->ready);
    if (ctx->post) (void)hipHostFree(ctx->post);
    delete ctx;
}

int32_t bm_sync(bm_context* ctx) {
    if (!ctx) return BM_ERROR_INVALID_PARAMETER;
    for (bm_context* p : ctx->peers) {
        BM_HIP(ctx, hipSetDevice(p->device));
        BM_HIP(ctx, ctx_sync_all(p));
    }
    BM_HIP(ctx, hipSetDevice(ctx->device));
    BM_HIP(ctx, ctx_sync_all(ctx));
    return BM_ERROR_ALL_FINE;
}

const char* bm_last_error_string(const bm_context* ctx) { return ctx ? ctx->last_error.c_str() : "null context"; }

void* bm_context_stream(const bm_context* ctx) { return ctx ? reinterpret_cast<void*>(ctx->stream) : nullptr; }

// ---- mesh (Mesh.cpp:30-54) -------------------------------------------------------------------
int32_t bm_mesh_create(bm_context* ctx, bm_mesh** out) {
    if (!ctx || !out) return BM_ERROR_INVALID_PARAMETER;
    bm_mesh* m = new (std::nothrow) bm_mesh();
    if (!m) return BM_ERROR_GPU_ALLOC_FAIL;
    m->ctx = ctx;
    for (bm_context* p : ctx->peers) {
        bm_mesh* r = nullptr;
        const int32_t rc = bm_mesh_create(p, &r);
        if (rc) {
            bm_mesh_destroy(m);
            return peer_fail(ctx, p, rc);
        }
        m->rep.push_back(r);
    }
    *out = m;
    return BM_ERROR_ALL_FINE;
}

int32_t bm_mesh_set_vertex_data(bm_mesh* m, const float* data, uint32_t num_vertices, uint32_t num_components,
                                uint32_t slot) {
    if (!m) return BM_ERROR_INVALID_PARAMETER;
    bm_context* ctx = m->ctx;
    if (!data || num_vertices == 0 || slot >= BM_VERTEX_DATA_COUNT || num_components == 0 || num_components > 4 ||
        (m->num_vertices != 0 && m->num_vertices != num_vertices) ||
        (slot == BM_VERTEX_DATA_POSITION && num_components != 3))
        return fail(ctx, BM_ERROR_INVALID_PARAMETER, "setVertexData: invalid parameter (Mesh.cpp:32-37)");
    BM_HIP(ctx, hipSetDevice(ctx->device));
    const size_t bytes = sizeof(float) * (size_t)num_components * num_vertices;
    GrowGuard grow{ctx};  // a build still queued may read the old slot
    BM_HIP(ctx, grow.reserve(m->slot[slot], bytes));
    // synchronous copy, as the reference's DeviceBuffer::copyFrom(wait=true)
    BM_HIP(ctx, hipMemcpyAsync(m->slot[slot].p, data, bytes, hipMemcpyHostToDevice, ctx->stream));
    BM_HIP(ctx, hipStreamSynchronize(ctx->stream));
    m->slot_comp[slot] = num_components;
    m->num_vertices = num_vertices;  // the reference leaves m_numVertices at 0 (Mesh.cpp); we record it
    for (bm_mesh* r : m->rep) {
        const int32_t rc = bm_mesh_set_vertex_data(r, data, num_vertices, num_components, slot);
        if (rc) return peer_fail(ctx, r->ctx, rc);
    }
    return BM_ERROR_ALL_FINE;
}

int32_t bm_mesh_set_indices(bm_mesh* m, const uint32_t* indices, uint32_t num_indices) {
    if (!m) return BM_ERROR_INVALID_PARAMETER;
    bm_context* ctx = m->ctx;
    if (!indices || (num_indices % 3) != 0)
        return fail(ctx, BM_ERROR_INVALID_PARAMETER, "setIndices: null or not a multiple of 3 (Mesh.cpp:48)");
    BM_HIP(ctx, hipSetDevice(ctx->device));
    uint32_t mx = 0;
    for (uint32_t i = 0; i < num_indices; ++i) mx = std::max(mx, indices[i]);
    GrowGuard grow{ctx};
    BM_HIP(ctx, grow.reserve(m->idx, sizeof(uint32_t) * (size_t)num_indices));
    if (num_indices) {
        BM_HIP(ctx, hipMemcpyAsync(m->idx.p, indices, sizeof(uint32_t) * (size_t)num_indices,
                                   hipMemcpyHostToDevice, ctx->stream));
        BM_HIP(ctx, hipStreamSynchronize(ctx->stream));
    }
    m->num_indices = num_indices;
    m->max_index = mx;
    for (bm_mesh* r : m->rep) {
        const int32_t rc = bm_mesh_set_indices(r, indices, num_indices);
        if (rc) return peer_fail(ctx, r->ctx, rc);
    }
    return BM_ERROR_ALL_FINE;
}

void bm_mesh_destroy(bm_mesh* m) {
    if (!m) return;
    for (bm_mesh* r : m->rep) bm_mesh_destroy(r);
    (void)hipSetDevice(m->ctx->device);
    (void)hipStreamSynchronize(m->ctx->stream);
    for (auto& s : m->slot) s.release();
    m->idx.release();
    delete m;
}

// ---- scene (Scene.cpp, SceneTree.cpp) --------------------------------------------------------
int32_t bm_scene_create(bm_context* ctx, bm_scene** out) {
    if (!ctx || !out) return BM_ERROR_INVALID_PARAMETER;
    BM_HIP(ctx, hipSetDevice(ctx->device));
    bm_scene* s = new (std::nothrow) bm_scene();
    if (!s) return BM_ERROR_GPU_ALLOC_FAIL;
    s->ctx = ctx;
    s->leaf_size = ctx->leaf_size;
    if (hipEventCreate(&s->staging_done) != hipSuccess || hipEventCreate(&s->ev0) != hipSuccess ||
        hipEventCreate(&s->ev1) != hipSuccess ||
        hipEventCreateWithFlags(&s->orig_ev, hipEventDisableTiming) != hipSuccess) {
        delete s;
        return fail(ctx, BM_ERROR_DEVICE, "hipEventCreate failed");
    }
    for (bm_context* p : ctx->peers) {
        bm_scene* r = nullptr;
        const int32_t rc = bm_scene_create(p, &r);
        if (rc) {
            bm_scene_destroy(s);
            return peer_fail(ctx, p, rc);
        }
        s->rep.push_back(r);
    }
    *out = s;
    return BM_ERROR_ALL_FINE;
}

int32_t bm_scene_add_mesh(bm_scene* s, bm_mesh* m) {
    if (!s || !m || m->ctx != s->ctx || m->rep.size() != s->rep.size()) return BM_ERROR_INVALID_PARAMETER;
    for (size_t i = 0; i < s->rep.size(); ++i) {
        const int32_t rc = bm_scene_add_mesh(s->rep[i], m->rep[i]);
        if (rc) return peer_fail(s->ctx, s->rep[i]->ctx, rc);
    }
    s->meshes.push_back(m);
    s->built = false;
    return BM_ERROR_ALL_FINE;
}

int32_t bm_scene_remove_mesh(bm_scene* s, bm_mesh* m) {
    if (!s || !m) return BM_ERROR_INVALID_PARAMETER;
    auto it = std::find(s->meshes.begin(), s->meshes.end(), m);
    if (it == s->meshes.end()) return fail(s->ctx, BM_ERROR_INVALID_PARAMETER, "removeMesh: mesh not in scene");
    for (size_t i = 0; i < s->rep.size(); ++i) (void)bm_scene_remove_mesh(s->rep[i], m->rep[i]);
    s->meshes.erase(it);  // the reference forgets to mark its mesh table dirty (Scene.cpp:43-56)
    s->built = false;
    return BM_ERROR_ALL_FINE;
}

// A few device words to the host in the middle of a build (the counts that size the next buffers),
// without a stream synchronisation: k_post writes them into pinned coherent host memory and releases a
// sequence number there, on which this thread spins (checking the stream every few thousand polls, so
// a failed kernel ends the wait with its error). A synchronisation's wake-up and a pageable copy cost
// ~40 us per readback on the kd build; BM_PARAM_READBACK_SYNC 1 restores them for an A/B.
static int32_t post_wait(bm_context* ctx, hipStream_t st, const uint32_t* flag, uint32_t seq);
static int32_t readback(bm_context* ctx, hipStream_t st, const uint32_t* a, uint32_t na, const uint32_t* b,
                        uint32_t nb, uint32_t* out) {
    if (ctx->tune.get(BM_PARAM_READBACK_SYNC, 0) != 0) {
        if (na) BM_HIP(ctx, hipMemcpyAsync(out, a, 4 * (size_t)na, hipMemcpyDeviceToHost, st));
        if (nb) BM_HIP(ctx, hipMemcpyAsync(out + na, b, 4 * (size_t)nb, hipMemcpyDeviceToHost, st));
        BM_HIP(ctx, hipStreamSynchronize(st));
        return BM_ERROR_ALL_FINE;
    }
    if (!ctx->post) {
        void* h = nullptr;
        BM_HIP(ctx, hipHostMalloc(&h, 4 * (bm::POST_SEQ_WORD + 1), hipHostMallocCoherent | hipHostMallocMapped));
        std::memset(h, 0, 4 * (bm::POST_SEQ_WORD + 1));
        void* d = nullptr;
        const hipError_t e = hipHostGetDevicePointer(&d, h, 0);
        if (e != hipSuccess) {
            (void)hipHostFree(h);
            return hip_fail(ctx, e, "readback: hipHostGetDevicePointer");
        }
        ctx->post = static_cast<uint32_t*>(h);
        ctx->post_dev = static_cast<uint32_t*>(d);
    }
    if (++ctx->post_seq == 0) ctx->post_seq = 1;
    const uint32_t seq = ctx->post_seq;
    BM_HIP(ctx, bm::launch_post(a, na, b, nb, ctx->post_dev, seq, st));
    const int32_t r = post_wait(ctx, st, ctx->post + bm::POST_SEQ_WORD, seq);
    if (r != BM_ERROR_ALL_FINE) return r;
    std::memcpy(out, ctx->post, 4 * (size_t)(na + nb));
    return BM_ERROR_ALL_FINE;
}

// Spin until k_post released `seq` into *flag (pinned host memory), checking the stream every few thousand
// polls so that a failed kernel ends the wait with its error.
static int32_t post_wait(bm_context* ctx, hipStream_t st, const uint32_t* flag, uint32_t seq) {
    // spin for the short waits (the counts usually land within tens of microseconds); past ~50 us of
    // polling yield the core between polls, so a long wait (a large scene's count pass) does not burn
    // a host core that other ranks' or frames' threads share
    const auto t0 = std::chrono::steady_clock::now();
    bool yield = false;
    for (uint32_t i = 1; __atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq; ++i) {
        if ((i & 4095) == 0) {
            const hipError_t q = hipStreamQuery(st);
            if (q != hipErrorNotReady && __atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) {
                if (q != hipSuccess) return hip_fail(ctx, q, "readback: stream");
                return fail(ctx, BM_ERROR_DEVICE, "readback: the stream drained without posting the words");
            }
        }
        if (!yield && (i & 255) == 0)
            yield = std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(50);
        if (yield) {
            std::this_thread::yield();
        } else {
#if defined(__x86_64__) || defined(__i386__)
            __builtin_ia32_pause();
#endif
        }
    }
    return BM_ERROR_ALL_FINE;
}

// Scratch of launch_exclusive_scan: grown like any buffer, zero-filled when (re)allocated; each call gets
// the next epoch (20 bits, never 0), so its status words from earlier calls read as not ready.
static int32_t scan_scratch(bm_context* ctx, bm_scene* s, GrowGuard& grow, uint32_t n, uint32_t* epoch) {
    const size_t cap = s->kd_sums.cap;
    BM_HIP(ctx, grow.reserve(s->kd_sums, 4 * (size_t)bm::scan_sums_words(n)));
    // The epoch is the scene's own (its status words hold only its epochs). When it wraps, a word written
    // 2^20 - 1 calls ago could carry the new epoch (a tile the scene used before it shrank and regrew):
    // zero-fill then, as on a reallocation.
    s->scan_epoch = (s->scan_epoch + 1) & ((1u << 20) - 1u);
    const bool wrapped = s->scan_epoch == 0;
    if (wrapped) s->scan_epoch = 1;
    if (s->kd_sums.cap != cap || wrapped) BM_HIP(ctx, hipMemsetAsync(s->kd_sums.p, 0, s->kd_sums.cap, ctx->stream));
    *epoch = s->scan_epoch;
    return BM_ERROR_ALL_FINE;
}

// Reference mode (bm_kd.hip): the reference's kd-tree. Two host reads of a count (pairs, leaves)
// size the next buffers; each is a spin on pinned host memory (readback), not a stream sync.
static constexpr float KD_WORLD_MIN = -30.f, KD_WORLD_MAX = 30.f;  // SceneTree.cpp:44-45

static int32_t kd_build(bm_context* ctx, bm_scene* s, const bm::BuildBuffers& b, GrowGuard& grow) {
    hipStream_t st = ctx->stream;
    const uint32_t n = b.n;
    const int leaf_depth = bm::kd_leaf_depth(KD_WORLD_MIN, KD_WORLD_MAX);
    if (leaf_depth > 31) return fail(ctx, BM_ERROR_INVALID_PARAMETER, "reference mode: kd leaves deeper than 31");
    const size_t nn = n ? n : 1;
    BM_HIP(ctx, bm::launch_gather(b, st));
    BM_HIP(ctx, grow.reserve(s->kd_counts, 4 * nn));
    BM_HIP(ctx, grow.reserve(s->kd_offsets, 4 * nn));
    BM_HIP(ctx, grow.reserve(s->kd_total, 16));
    BM_HIP(ctx, grow.reserve(s->kd_cache, 4 * (size_t)bm::KD_LEAF_CACHE * nn));
    bm::KdBuild kb{b.meshes, b.num_meshes, n, KD_WORLD_MIN, KD_WORLD_MAX, leaf_depth,
                   s->kd_counts.as<uint32_t>(), s->kd_offsets.as<uint32_t>(), nullptr, nullptr,
                   s->kd_cache.as<uint32_t>()};
    kb.tune = &ctx->tune;
    kb.split = bm::kd_split_depth(leaf_depth, ctx->tune);
    if (kb.split) {  // queue: 4 items per triangle (+ 1 count word), walked in place beyond that
        kb.queue_cap = (uint32_t)std::min<size_t>(4 * nn + 1024, 1u << 28);
        // test hooks (read per build): small queues force the walk-on paths (tests/test_gpu_reference_mode.py)
        const int64_t qc = ctx->tune.get(BM_PARAM_KD_QUEUE_CAP, 0), lq = ctx->tune.get(BM_PARAM_KD_LQ_CAP, 0);
        if (qc > 0) kb.queue_cap = (uint32_t)std::min<int64_t>(qc, kb.queue_cap);
        if (lq > 0) kb.lq_cap = (uint32_t)std::min<int64_t>(lq, 1u << 20);
        BM_HIP(ctx, grow.reserve(s->kd_queue, 8 * (size_t)kb.queue_cap));
        BM_HIP(ctx, grow.reserve(s->kd_fill, 4 * nn));
        kb.queue = reinterpret_cast<uint2*>(s->kd_queue.p);
        kb.qcount = b.bounds;  // words 0 (count) and 1 (overflow flag), zeroed by launch_gather above
        kb.qcount_zeroed = true;
        // word 2: top-bit count, then the top-bit map (zeroed with them): the sort's ranked top digit
        if (leaf_depth == 31 && ctx->tune.get(BM_PARAM_KD_TOP_RANK, 1) != 0) {
            kb.topcount = b.bounds + 2;
            kb.topmap = b.bounds + 3;
        }
        kb.fill = s->kd_fill.as<uint32_t>();
    }
    BM_HIP(ctx, bm::launch_kd_count(kb, st));
    uint32_t ep = 0;
    if (const int32_t r = scan_scratch(ctx, s, grow, n, &ep)) return r;
    BM_HIP(ctx, bm::launch_exclusive_scan(kb.counts, kb.offsets, n, s->kd_sums.as<uint32_t>(),
                                          s->kd_total.as<uint32_t>(), st, s->kd_total.as<unsigned long long>() + 1, ep));
    // kd_total words (u64 pairs in [2..3]), then qcount, overflow flag, top-bit count
    uint32_t rb[7] = {0, 0, 0, 0, 0, 1, ~0u};
    const bool q = kb.split && kb.qcount;
    {
        const int32_t r = readback(ctx, st, s->kd_total.as<uint32_t>(), 4, q ? kb.qcount : nullptr,
                                   q ? (kb.topmap ? 3u : 2u) : 0u, rb);
        if (r != BM_ERROR_ALL_FINE) return r;
    }
    const uint64_t tot[2] = {0, (uint64_t)rb[2] | ((uint64_t)rb[3] << 32)};
    const uint32_t qinfo[3] = {rb[4], rb[5], rb[6]};
    // The emit pass may skip the walk from the root only if the count pass's queue holds every
    // (triangle, node at depth split) item and no leaf lies at depth <= split (k_kd_top never emits
    // a leaf itself). Halving is uniform per level, so every node at depth d has the extents of the
    // world box halved along the axes d % 3 has cycled through, and the stop rule (min extent <
    // 0.03 or depth 37, BuildTree.cu:200) fires at one depth for all nodes: kd_leaf_depth.
    // Leaves therefore lie exactly at leaf_depth, and kd_split_depth keeps split below it.
    kb.reuse_queue = kb.split && kb.split < leaf_depth && qinfo[1] == 0;
    // the ranked top digit needs every leaf below a queued node (the map holds their top bits) and at most
    // 1,024 values present (ranks in one 10-bit digit); otherwise the four plain passes
    const bool top_rank = kb.topmap && kb.reuse_queue && qinfo[2] <= 1024u;
    if (tot[1] > bm::MAX_PAIRS)
        return fail(ctx, BM_ERROR_GPU_ALLOC_FAIL, "reference mode: more than 2^31 (leaf, face) pairs");
    const uint32_t m = (uint32_t)tot[1];
    const size_t mm = m ? m : 1;
    for (DevBuf* d : {&s->kd_keys, &s->kd_vals, &s->kd_keys2, &s->kd_vals2, &s->kd_leaf_of})
        BM_HIP(ctx, grow.reserve(*d, 4 * mm));
    BM_HIP(ctx, grow.reserve(s->kd_smeta, 4 * bm::sort_meta_words(m, leaf_depth)));
    kb.keys = s->kd_keys.as<uint32_t>();
    kb.vals = s->kd_vals.as<uint32_t>();
    bool smeta_zeroed = false;  // the emit pass zero-fills the sort's metadata on the side (no fill launch)
    kb.zero_ptr = s->kd_smeta.as<uint32_t>();
    kb.zero_words = (uint32_t)bm::sort_meta_words(m, leaf_depth);
    kb.zeroed = &smeta_zeroed;
    BM_HIP(ctx, bm::launch_kd_emit(kb, st));
    bool scratch = false;
    BM_HIP(ctx, bm::launch_sort_pairs(kb.keys, kb.vals, s->kd_keys2.as<uint32_t>(), s->kd_vals2.as<uint32_t>(), m,
                                      leaf_depth, s->kd_smeta.as<uint32_t>(), st, &scratch, smeta_zeroed,
                                      top_rank ? kb.topmap : nullptr));
    s->kd_top_rank = top_rank;
    const uint32_t* skeys = scratch ? s->kd_keys2.as<uint32_t>() : kb.keys;
    BM_HIP(ctx, grow.reserve(s->kd_ubox, 32));
    if (const int32_t r = scan_scratch(ctx, s, grow, std::max(m, n), &ep)) return r;
    // leaf index of each pair's run: the scan of the run starts, taken from the sorted keys directly
    BM_HIP(ctx, bm::launch_exclusive_scan(nullptr, s->kd_leaf_of.as<uint32_t>(), m, s->kd_sums.as<uint32_t>(),
                                          s->kd_total.as<uint32_t>() + 1, st, nullptr, ep, skeys));
    // The leaf count stays on the device (kd_total word 1): the leaf-side buffers are sized by the pair
    // count (an upper bound), the kernels read the count themselves, and the host learns it after the
    // build (k_post into the scene's pinned words, read by kd_leaves_ready) — no mid-build readback.
    const uint32_t* nl_dev = s->kd_total.as<uint32_t>() + 1;
    // capacity: the pair count bounds the leaves, and a tree of more than KD_MAX_LEAVES is refused anyway
    // (BM_PARAM_KD_MAX_LEAVES lowers that limit: test hook); a device count above the capacity leaves the
    // leaf-side kernels idle and kd_leaves_ready reports it (no garbage records in between)
    const uint32_t leaf_limit = (uint32_t)std::min<int64_t>(ctx->tune.get(BM_PARAM_KD_MAX_LEAVES, bm::KD_MAX_LEAVES),
                                                            bm::KD_MAX_LEAVES);
    const uint32_t nlc = std::min(m, leaf_limit);
    s->kd_leaf_cap = nlc;
    const size_t nln = nlc ? nlc : 1, nli = nlc > 1 ? nlc - 1 : 1;
    for (DevBuf* d : {&s->kd_leaf_key, &s->kd_leaf_start, &s->kd_leaf_count, &s->kd_pleaf})
        BM_HIP(ctx, grow.reserve(*d, 4 * nln));
    for (DevBuf* d : {&s->kd_lch, &s->kd_rch, &s->kd_first, &s->kd_last, &s->kd_pint}) BM_HIP(ctx, grow.reserve(*d, 4 * nli));
    BM_HIP(ctx, grow.reserve(s->kd_ftris, 48 * mm));
    BM_HIP(ctx, bm::launch_kd_leaves(skeys, m, nullptr, s->kd_leaf_of.as<uint32_t>(),
                                     s->kd_leaf_key.as<uint32_t>(), s->kd_leaf_start.as<uint32_t>(),
                                     nullptr, nlc, st, nl_dev, s->kd_ubox.as<uint32_t>(),  // counts: k_kd_records
                                     scratch ? s->kd_vals2.as<const uint32_t>() : kb.vals, b.tri_orig,
                                     s->kd_ftris.as<float4>()));
    BM_HIP(ctx, bm::launch_radix_tree(s->kd_leaf_key.as<uint32_t>(), nlc, s->kd_lch.as<uint32_t>(),
                                      s->kd_rch.as<uint32_t>(), s->kd_first.as<uint32_t>(), s->kd_last.as<uint32_t>(),
                                      s->kd_pleaf.as<uint32_t>(), s->kd_pint.as<uint32_t>(), st, nl_dev));
    BM_HIP(ctx, grow.reserve(s->kd_nodes, 32 * nli));
    BM_HIP(ctx, grow.reserve(s->kd_leafrec, 32 * nln));
    BM_HIP(ctx, grow.reserve(s->kd_node_key, 4 * nli));
    const bool child_steps = ctx->tune.get(BM_PARAM_KD_MARCH, 3) == 3;  // only that march reads cnodes
    if (child_steps) BM_HIP(ctx, grow.reserve(s->kd_cnodes, 64 * nli));
    s->kd_cnodes_valid = child_steps;
    bm::KdMarch km{s->kd_leaf_key.as<const uint32_t>(), s->kd_leaf_start.as<const uint32_t>(),
                   s->kd_leaf_count.as<const uint32_t>(), nullptr, s->kd_lch.as<const uint32_t>(),
                   s->kd_rch.as<const uint32_t>(), s->kd_first.as<const uint32_t>(), s->kd_last.as<const uint32_t>(),
                   nlc, leaf_depth, KD_WORLD_MIN, KD_WORLD_MAX, nullptr, nullptr, nullptr, nullptr};
    km.num_leaves_dev = nl_dev;
    km.no_grid = ctx->tune.get(BM_PARAM_KD_GRID, 1) == 0;  // the parameter governs the records too
    if (!s->kd_post) {
        void* h = nullptr;
        BM_HIP(ctx, hipHostMalloc(&h, 4 * (bm::POST_SEQ_WORD + 1), hipHostMallocCoherent | hipHostMallocMapped));
        std::memset(h, 0, 4 * (bm::POST_SEQ_WORD + 1));
        void* d = nullptr;
        const hipError_t e = hipHostGetDevicePointer(&d, h, 0);
        if (e != hipSuccess) {
            (void)hipHostFree(h);
            return hip_fail(ctx, e, "kd build: hipHostGetDevicePointer");
        }
        s->kd_post = static_cast<uint32_t*>(h);
        s->kd_post_dev = static_cast<uint32_t*>(d);
    }
    if (++s->kd_post_seq == 0) s->kd_post_seq = 1;
    // the records kernel also posts the leaf count for kd_leaves_ready (no k_post launch after it)
    BM_HIP(ctx, bm::launch_kd_records(km, m, s->kd_nodes.as<uint4>(), s->kd_leafrec.as<uint4>(),
                                      s->kd_node_key.as<uint32_t>(), st, child_steps ? s->kd_cnodes.as<uint4>() : nullptr,
                                      s->kd_ubox.as<uint32_t>(), s->kd_post_dev, s->kd_post_seq));
    s->kd_leaves_pending = true;
    const uint32_t nl = 0;  // until kd_leaves_ready
    s->kd_pairs = m;
    s->kd_leaves = nl;
    s->kd_sorted_in_scratch = scratch;
    return BM_ERROR_ALL_FINE;
}

// The last reference-mode build's leaf count on the host: waits (once per build) for its k_post.
static int32_t kd_leaves_ready(bm_scene* s) {
    if (!s->kd_leaves_pending) return BM_ERROR_ALL_FINE;
    bm_context* ctx = s->ctx;
    const int32_t r = post_wait(ctx, ctx->stream, s->kd_post + bm::POST_SEQ_WORD, s->kd_post_seq);
    if (r != BM_ERROR_ALL_FINE) return r;
    s->kd_leaves = s->kd_post[0];
    s->kd_leaves_pending = false;
    if (s->kd_leaves > s->kd_leaf_cap) {  // the leaf-side kernels wrote nothing (capacity guard)
        s->built = false;
        return fail(ctx, BM_ERROR_GPU_ALLOC_FAIL, "reference mode: more kd leaves (" + std::to_string(s->kd_leaves) +
                                                      ") than the build accepts (" + std::to_string(s->kd_leaf_cap) + ")");
    }
    return BM_ERROR_ALL_FINE;
}

// Hashed-grid mode (BM_OPT_REFERENCE_HASH): the reference's alternative accelerator (Hash.cu:132-178)
// as (bucket, triangle) pairs sorted by bucket; see bm_kd.hip.
static int32_t hash_build(bm_context* ctx, bm_scene* s, const bm::BuildBuffers& b, GrowGuard& grow) {
    hipStream_t st = ctx->stream;
    const uint32_t n = b.n;
    const size_t nn = n ? n : 1;
    BM_HIP(ctx, bm::launch_gather(b, st));
    BM_HIP(ctx, grow.reserve(s->kd_counts, 4 * nn));
    BM_HIP(ctx, grow.reserve(s->kd_offsets, 4 * nn));
    // kd_total words: [0] u32 scan total, [1] too-large flag, [2..3] u64 pair count
    BM_HIP(ctx, grow.reserve(s->kd_total, 16));
    BM_HIP(ctx, hipMemsetAsync(s->kd_total.p, 0, 16, st));
    bm::HashBuild hb{b.meshes, b.num_meshes, n, s->kd_counts.as<uint32_t>(), s->kd_offsets.as<uint32_t>(),
                     nullptr, nullptr, s->kd_total.as<uint32_t>() + 1};
    BM_HIP(ctx, bm::launch_hash_count(hb, st));
    uint32_t ep = 0;
    if (const int32_t r = scan_scratch(ctx, s, grow, n, &ep)) return r;
    BM_HIP(ctx, bm::launch_exclusive_scan(hb.counts, hb.offsets, n, s->kd_sums.as<uint32_t>(),
                                          s->kd_total.as<uint32_t>(), st, s->kd_total.as<unsigned long long>() + 1, ep));
    uint32_t tot[4] = {0, 0, 0, 0};
    {
        const int32_t r = readback(ctx, st, s->kd_total.as<uint32_t>(), 4, nullptr, 0, tot);
        if (r != BM_ERROR_ALL_FINE) return r;
    }
    if (tot[1]) return fail(ctx, BM_ERROR_INVALID_PARAMETER, "hashed grid: a triangle spans more than 2^20 cells");
    const uint64_t pairs = (uint64_t)tot[2] | ((uint64_t)tot[3] << 32);
    if (pairs > bm::MAX_PAIRS) return fail(ctx, BM_ERROR_GPU_ALLOC_FAIL, "hashed grid: more than 2^31 (cell, face) pairs");
    const uint32_t m = (uint32_t)pairs;
    const size_t mm = m ? m : 1;
    for (DevBuf* d : {&s->kd_keys, &s->kd_vals, &s->kd_keys2, &s->kd_vals2}) BM_HIP(ctx, grow.reserve(*d, 4 * mm));
    BM_HIP(ctx, grow.reserve(s->kd_smeta, 4 * bm::sort_meta_words(m, 16)));
    hb.keys = s->kd_keys.as<uint32_t>();
    hb.vals = s->kd_vals.as<uint32_t>();
    BM_HIP(ctx, bm::launch_hash_emit(hb, st));
    bool scratch = false;
    BM_HIP(ctx, bm::launch_sort_pairs(hb.keys, hb.vals, s->kd_keys2.as<uint32_t>(), s->kd_vals2.as<uint32_t>(), m, 16,
                                      s->kd_smeta.as<uint32_t>(), st, &scratch));
    BM_HIP(ctx, grow.reserve(s->hash_bstart, 4 * (size_t)bm::HG_NUM_BUCKETS));
    BM_HIP(ctx, grow.reserve(s->hash_bend, 4 * (size_t)bm::HG_NUM_BUCKETS));
    BM_HIP(ctx, bm::launch_hash_ranges(scratch ? s->kd_keys2.as<uint32_t>() : hb.keys, m,
                                       s->hash_bstart.as<uint32_t>(), s->hash_bend.as<uint32_t>(), st));
    s->kd_pairs = m;
    s->kd_sorted_in_scratch = scratch;
    return BM_ERROR_ALL_FINE;
}

static int32_t scene_build_impl(bm_scene* s, bm_build_stats* stats, bool refit) {
    if (!s) return BM_ERROR_INVALID_PARAMETER;
    bm_context* ctx = s->ctx;
    if (refit) {
        bool same = s->built && s->built_with.size() == s->meshes.size();
        for (size_t i = 0; same && i < s->meshes.size(); ++i)
            same = s->built_with[i].first == s->meshes[i] && s->built_with[i].second == s->meshes[i]->num_indices / 3;
        if (!same)
            return fail(ctx, BM_ERROR_INVALID_PARAMETER,
                        "refit needs the meshes and triangle counts of the last build (call updateGPUScene)");
    }
    BM_HIP(ctx, hipSetDevice(ctx->device));
    BM_HIP(ctx, ctx_drain(ctx));  // traces on render-target streams may still read the old build
    uint64_t n64 = 0;
    std::vector<bm::MeshDesc> table;
    for (bm_mesh* m : s->meshes) {
        if (!m->slot[BM_VERTEX_DATA_POSITION].p || m->slot_comp[BM_VERTEX_DATA_POSITION] != 3)
            return fail(ctx, BM_ERROR_NO_VERTICES, "mesh without a 3-component position slot");
        if (m->num_indices && !m->idx.p) return fail(ctx, BM_ERROR_INVALID_PARAMETER, "mesh indices missing");
        if (!m->slot[BM_VERTEX_DATA_NORMAL].p || m->slot_comp[BM_VERTEX_DATA_NORMAL] != 3)
            return fail(ctx, BM_ERROR_INVALID_FORMAT,
                        "mesh without 3-component normals (the reference dereferences NULL, BuildTree.cu:489)");
        if (m->num_indices && m->max_index >= m->num_vertices)
            return fail(ctx, BM_ERROR_INVALID_PARAMETER, "index out of range of the mesh's vertices");
        bm::MeshDesc d;
        d.pos = m->slot[BM_VERTEX_DATA_POSITION].as<const float>();
        d.nrm = m->slot[BM_VERTEX_DATA_NORMAL].as<const float>();
        d.idx = m->idx.as<const uint32_t>();
        d.tri_offset = (uint32_t)n64;
        d.num_tris = m->num_indices / 3;
        n64 += d.num_tris;
        table.push_back(d);
    }
    if (n64 >= bm::MAX_TRIS) return fail(ctx, BM_ERROR_INVALID_PARAMETER, "more than 2^27 triangles");
    const uint32_t n = (uint32_t)n64;
    const uint32_t nrec = bm::num_records(n);
    const size_t ni = n > 1 ? n - 1 : 1;
    const size_t nn = n ? n : 1;
    // previous mesh-table upload must be done before the pinned staging buffer is rewritten
    BM_HIP(ctx, hipEventSynchronize(s->staging_done));
    if (table.size() > s->staging_cap) {
        if (s->staging) (void)hipHostFree(s->staging);
        s->staging = nullptr;
        s->staging_cap = 0;
        BM_HIP(ctx, hipHostMalloc((void**)&s->staging, sizeof(bm::MeshDesc) * table.size(), hipHostMallocDefault));
        s->staging_cap = table.size();
    }
    GrowGuard grow{ctx};
    BM_HIP(ctx, grow.reserve(s->mesh_table, sizeof(bm::MeshDesc) * std::max<size_t>(table.size(), 1)));
    BM_HIP(ctx, grow.reserve(s->tri_orig, 48 * nn));
    BM_HIP(ctx, grow.reserve(s->nrm, 36 * nn));
    BM_HIP(ctx, grow.reserve(s->aabb, 24 * nn));
    BM_HIP(ctx, grow.reserve(s->cen, 12 * nn));
    const size_t bounds_cap = s->bounds.cap;
    BM_HIP(ctx, grow.reserve(s->bounds, 4 * bm::build_meta_words(n)));
    if (s->bounds.cap != bounds_cap) s->replicas_clean = false;  // a fresh allocation holds anything
    BM_HIP(ctx, grow.reserve(s->keys, 4 * nn));
    BM_HIP(ctx, grow.reserve(s->vals, 4 * nn));
    BM_HIP(ctx, grow.reserve(s->keys2, 4 * nn));
    BM_HIP(ctx, grow.reserve(s->vals2, 4 * nn));
    BM_HIP(ctx, grow.reserve(s->lch, 4 * ni));
    BM_HIP(ctx, grow.reserve(s->rch, 4 * ni));
    BM_HIP(ctx, grow.reserve(s->first, 4 * ni));
    BM_HIP(ctx, grow.reserve(s->last, 4 * ni));
    BM_HIP(ctx, grow.reserve(s->parent_leaf, 4 * nn));
    BM_HIP(ctx, grow.reserve(s->parent_int, 4 * ni));
    BM_HIP(ctx, grow.reserve(s->pre, 24 * nn));
    BM_HIP(ctx, grow.reserve(s->suf, 24 * nn));
    BM_HIP(ctx, grow.reserve(s->table, 4 * bm::chunk_table_floats(n)));
    BM_HIP(ctx, grow.reserve(s->ibox, 24 * ni));
    const uint32_t width = refit ? s->width : ctx->bvh_width;
    BM_HIP(ctx, grow.reserve(s->records, (width == 8 ? 256 : width == 4 ? 128 : 64) * (size_t)nrec));
    if (width == 8) BM_HIP(ctx, grow.reserve(s->records2, 64 * (size_t)nrec));
    BM_HIP(ctx, grow.reserve(s->tris, 48 * nn));
    if (!table.empty()) {
        std::memcpy(s->staging, table.data(), sizeof(bm::MeshDesc) * table.size());
        BM_HIP(ctx, hipMemcpyAsync(s->mesh_table.p, s->staging, sizeof(bm::MeshDesc) * table.size(),
                                   hipMemcpyHostToDevice, ctx->stream));
    }
    BM_HIP(ctx, hipEventRecord(s->staging_done, ctx->stream));
    bm::BuildBuffers b;
    b.n = n;
    b.num_meshes = (uint32_t)table.size();
    b.leaf_size = s->leaf_size;
    b.width = width;
    b.records2 = width == 8 ? s->records2.as<uint32_t>() : nullptr;
    b.meshes = s->mesh_table.as<const bm::MeshDesc>();
    b.tri_orig = s->tri_orig.as<float4>();
    b.nrm = s->nrm.as<float>();
    b.aabb = s->aabb.as<float>();
    b.cen = s->cen.as<float>();
    b.bounds = s->bounds.as<uint32_t>();
    b.keys = s->keys.as<uint32_t>();
    b.vals = s->vals.as<uint32_t>();
    b.keys2 = s->keys2.as<uint32_t>();
    b.vals2 = s->vals2.as<uint32_t>();
    b.lch = s->lch.as<uint32_t>();
    b.rch = s->rch.as<uint32_t>();
    b.first = s->first.as<uint32_t>();
    b.last = s->last.as<uint32_t>();
    b.parent_leaf = s->parent_leaf.as<uint32_t>();
    b.parent_int = s->parent_int.as<uint32_t>();
    b.pre = s->pre.as<float>();
    b.suf = s->suf.as<float>();
    b.table = s->table.as<float>();
    b.ibox = s->ibox.as<float>();
    b.records = s->records.as<uint32_t>();
    b.tris = s->tris.as<float4>();
    b.replicas_clean = s->replicas_clean && !ctx->reference_kd && !ctx->reference_hash;
    b.tune = &ctx->tune;
    bool front = false;  // k_front (gather + keys + top-digit pass in one launch) was removed in round 5
    // a multi-device root rebuilds t, |n.z| and colours from the original-order records (reshade)
    b.orig_records = ctx->multi() && ctx->tune.get(BM_PARAM_ORIG_LAZY, 0) == 0;
    bool orig = true;  // reference modes' gathers write them
    b.orig_written = &orig;
    s->replicas_clean = false;  // until this build's kernels are enqueued (a failed launch leaves them unknown)
    BM_HIP(ctx, hipEventRecord(s->ev0, ctx->stream));
    if (ctx->reference_kd || ctx->reference_hash) {
        if (refit) return fail(ctx, BM_ERROR_INVALID_PARAMETER, "refit: not available in reference mode");
        const int32_t e = ctx->reference_kd ? kd_build(ctx, s, b, grow) : hash_build(ctx, s, b, grow);
        if (e) return e;
    } else {
        BM_HIP(ctx, refit ? bm::launch_refit(b, ctx->stream) : bm::launch_build(b, ctx->stream));
        s->replicas_clean = n > 0;  // its last replica reader clears them (n == 0: nothing gathered, memset path)
        // build_ms covers the build's kernels; the scene-bounds readback for the host below is not part of it
        BM_HIP(ctx, hipEventRecord(s->ev1, ctx->stream));
        if (!s->hbounds) {
            BM_HIP(ctx, hipHostMalloc((void**)&s->hbounds, 64, hipHostMallocDefault));
            std::memset(s->hbounds, 0, 64);
            BM_HIP(ctx, hipEventCreateWithFlags(&s->hbounds_ev, hipEventDisableTiming));
        }
        BM_HIP(ctx, hipMemcpyAsync(s->hbounds, b.bounds, 6 * sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->stream));
        s->sort_path = refit ? 0u : bm::msd_sort(n, ctx->tune) ? BM_SORT_MSD : BM_SORT_LSD;
        if (s->sort_path == BM_SORT_MSD)  // the device may have switched that sort to the LSD passes
            BM_HIP(ctx, hipMemcpyAsync(s->hbounds + 8, b.bounds + bm::build_sort_skew_word(), sizeof(uint32_t),
                                       hipMemcpyDeviceToHost, ctx->stream));
        BM_HIP(ctx, hipEventRecord(s->hbounds_ev, ctx->stream));
    }
    s->kd = ctx->reference_kd;
    s->hash = ctx->reference_hash;
    if (ctx->reference_kd || ctx->reference_hash) BM_HIP(ctx, hipEventRecord(s->ev1, ctx->stream));
    if (!refit) {
        s->built_with.clear();
        for (bm_mesh* m : s->meshes) s->built_with.emplace_back(m, m->num_indices / 3);
    }
    s->n = n;
    s->nrec = nrec;
    s->width = width;
    s->built = true;
    s->orig_valid = orig;
    s->orig_lazy = false;  // the build wrote (or invalidated) tri_orig on the context stream
    s->num_meshes = (uint32_t)table.size();
    if (ctx->reference_hash) s->sort_path = 0;
    if (ctx->reference_kd) s->sort_path = !n ? 0u : s->kd_top_rank ? BM_SORT_KD_RANKED : BM_SORT_LSD;  // the pair sort
    if (stats) {
        BM_HIP(ctx, hipEventSynchronize(s->ev1));
        if (s->sort_path == BM_SORT_MSD) {
            BM_HIP(ctx, hipEventSynchronize(s->hbounds_ev));
            if (s->hbounds[8]) s->sort_path = BM_SORT_MSD_SKEW;
        }
        stats->sort_path = s->sort_path;
        stats->fused_front = front ? 1u : 0u;
        float ms = 0.f;
        BM_HIP(ctx, hipEventElapsedTime(&ms, s->ev0, s->ev1));
        stats->num_meshes = (uint32_t)table.size();
        stats->num_tris = n;
        stats->num_records = nrec;
        stats->leaf_size = s->leaf_size;
        stats->bvh_width = s->width;
        stats->build_ms = ms;
    }
    return BM_ERROR_ALL_FINE;
}

// Replicas first (each on its own device and stream, all concurrent), then the root: build_ms is the
// root device's time.
static int32_t scene_build_all(bm_scene* s, bm_build_stats* stats, bool refit) {
    if (!s) return BM_ERROR_INVALID_PARAMETER;
    for (bm_scene* r : s->rep) {
        const int32_t rc = scene_build_impl(r, nullptr, refit);
        if (rc) return peer_fail(s->ctx, r->ctx, rc);
    }
    return scene_build_impl(s, stats, refit);
}

int32_t bm_scene_build(bm_scene* s, bm_build_stats* stats) { return scene_build_all(s, stats, false); }

#ifdef BM_BUILD_DIAG
// Diagnostic builds only (tools/build_diag.py): reset (out == NULL) or read the build kernels' span
// words of the current device (64 x u64; not part of the C ABI).
extern "C" int32_t bm_debug_build_diag(uint64_t* out) {
    auto* o = reinterpret_cast<unsigned long long*>(out);
    return bm::build_diag(o) == hipSuccess && bm::kd_build_diag(o) == hipSuccess ? BM_ERROR_ALL_FINE : BM_ERROR_DEVICE;
}
#endif

int32_t bm_scene_refit(bm_scene* s, bm_build_stats* stats) { return scene_build_all(s, stats, true); }

int32_t bm_scene_kd_stats(bm_scene* s, uint64_t out[4]) {
    if (!s || !out) return BM_ERROR_INVALID_PARAMETER;
    bm_context* ctx = s->ctx;
    if (!s->built || !s->kd) return fail(ctx, BM_ERROR_NOT_BUILT, "no reference-mode build");
    BM_HIP(ctx, hipSetDevice(ctx->device));
    if (const int32_t r = kd_leaves_ready(s)) return r;
    std::vector<uint32_t> cnt(s->kd_leaves);
    if (s->kd_leaves)
        BM_HIP(ctx, hipMemcpyAsync(cnt.data(), s->kd_leaf_count.p, 4 * (size_t)s->kd_leaves, hipMemcpyDeviceToHost,
                                   ctx->stream));
    BM_HIP(ctx, hipStreamSynchronize(ctx->stream));
    uint64_t stored = 0, dropped = 0, mx = 0;
    for (uint32_t c : cnt) {
        stored += std::min<uint32_t>(c, 256);
        dropped += c > 256 ? c - 256 : 0;
        mx = std::max<uint64_t>(mx, c);
    }
    out[0] = s->kd_leaves;
    out[1] = stored;
    out[2] = dropped;
    out[3] = mx;
    return BM_ERROR_ALL_FINE;
}

int32_t bm_scene_grid_stats(bm_scene* s, uint64_t out[4]) {
    if (!s || !out) return BM_ERROR_INVALID_PARAMETER;
    bm_context* ctx = s->ctx;
    if (!s->built || !s->hash) return fail(ctx, BM_ERROR_NOT_BUILT, "no hashed-grid build");
    BM_HIP(ctx, hipSetDevice(ctx->device));
    std::vector<uint32_t> b0(bm::HG_NUM_BUCKETS), b1(bm::HG_NUM_BUCKETS);
    BM_HIP(ctx, hipMemcpyAsync(b0.data(), s->hash_bstart.p, 4 * b0.size(), hipMemcpyDeviceToHost, ctx->stream));
    BM_HIP(ctx, hipMemcpyAsync(b1.data(), s->hash_bend.p, 4 * b1.size(), hipMemcpyDeviceToHost, ctx->stream));
    BM_HIP(ctx, hipStreamSynchronize(ctx->stream));
    uint64_t nonempty = 0, mx = 0, dropped = 0;
    for (size_t i = 0; i < b0.size(); ++i) {
        const uint64_t c = b1[i] - b0[i];
        nonempty += c != 0;
        mx = std::max(mx, c);
        dropped += c > 256 ? c - 256 : 0;
    }
    out[0] = s->kd_pairs;
    out[1] = nonempty;
    out[2] = mx;
    out[3] = dropped;
    return BM_ERROR_ALL_FINE;
}

int32_t bm_scene_grid_export(bm_scene* s, uint32_t* bucket_start, uint32_t* bucket_end, uint32_t* faces) {
    if (!s) return BM_ERROR_INVALID_PARAMETER;
    bm_context* ctx = s->ctx;
    if (!s->built || !s->hash) return fail(ctx, BM_ERROR_NOT_BUILT, "no hashed-grid build");
    BM_HIP(ctx, hipSetDevice(ctx->device));
    const size_t nb = 4 * (size_t)bm::HG_NUM_BUCKETS;
    if (bucket_start) BM_HIP(ctx, hipMemcpyAsync(bucket_start, s->hash_bstart.p, nb, hipMemcpyDeviceToHost, ctx->stream));
    if (bucket_end) BM_HIP(ctx, hipMemcpyAsync(bucket_end, s->hash_bend.p, nb, hipMemcpyDeviceToHost, ctx->stream));
    if (faces && s->kd_pairs)
        BM_HIP(ctx, hipMemcpyAsync(faces, (s->kd_sorted_in_scratch ? s->kd_vals2 : s->kd_vals).p, 4 * (size_t)s->kd_pairs,
                                   hipMemcpyDeviceToHost, ctx->stream));
    BM_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return BM_ERROR_ALL_FINE;
}

int32_t bm_scene_export(bm_scene* s, uint32_t* records, uint32_t* tris, uint32_t* keys, uint32_t* perm) {
    if (!s) return BM_ERROR_INVALID_PARAMETER;
    bm_context* ctx = s->ctx;
    if (!s->built) return fail(ctx, BM_ERROR_NOT_BUILT, "scene not built");
    if (s->kd || s->hash) return fail(ctx, BM_ERROR_INVALID_PARAMETER, "export: not available in reference mode");
    BM_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    if (records)
        BM_HIP(ctx, hipMemcpyAsync(records, s->records.p, (s->width == 8 ? 256 : s->width == 4 ? 128 : 64) * (size_t)s->nrec,
                                   hipMemcpyDeviceToHost, st));
    if (s->n) {
        if (tris) BM_HIP(ctx, hipMemcpyAsync(tris, s->tris.p, 48 * (size_t)s->n, hipMemcpyDeviceToHost, st));
        if (keys) BM_HIP(ctx, hipMemcpyAsync(keys, s->keys.p, 4 * (size_t)s->n, hipMemcpyDeviceToHost, st));
        if (perm) BM_HIP(ctx, hipMemcpyAsync(perm, s->vals.p, 4 * (size_t)s->n, hipMemcpyDeviceToHost, st));
    }
    BM_HIP(ctx, hipStreamSynchronize(st));
    return BM_ERROR_ALL_FINE;
}

void bm_scene_destroy(bm_scene* s) {
    if (!s) return;
    for (bm_scene* r : s->rep) bm_scene_destroy(r);
    (void)hipSetDevice(s->ctx->device);
    (void)ctx_sync_all(s->ctx);
    for (DevBuf* b : {&s->mesh_table, &s->tri_orig, &s->nrm, &s->aabb, &s->cen, &s->bounds, &s->keys, &s->vals, &s->keys2,
                      &s->vals2, &s->lch, &s->rch, &s->first, &s->last, &s->parent_leaf, &s->parent_int,
                      &s->ibox, &s->pre, &s->suf, &s->table, &s->records, &s->records2, &s->tris, &s->kd_counts, &s->kd_offsets,
                      &s->kd_sums, &s->kd_total, &s->kd_keys, &s->kd_vals, &s->kd_keys2, &s->kd_vals2, &s->kd_smeta,
                      &s->kd_leaf_of, &s->kd_leaf_key, &s->kd_leaf_start, &s->kd_leaf_count,
                      &s->kd_lch, &s->kd_rch, &s->kd_first, &s->kd_last, &s->kd_pleaf, &s->kd_pint, &s->kd_nodes, &s->kd_cnodes,
                      &s->kd_leafrec, &s->kd_ftris, &s->kd_node_key, &s->kd_ubox, &s->kd_cache,
                      &s->kd_queue, &s->kd_fill, &s->hash_bstart, &s->hash_bend})
        b->release();
    if (s->staging) (void)hipHostFree(s->staging);
    if (s->hbounds) (void)hipHostFree(s->hbounds);
    if (s->kd_post) (void)hipHostFree(s->kd_post);
    if (s->hbounds_ev) (void)hipEventDestroy(s->hbounds_ev);
    if (s->staging_done) (void)hipEventDestroy(s->staging_done);
    if (s->ev0) (void)hipEventDestroy(s->ev0);
    if (s->ev1) (void)hipEventDestroy(s->ev1);
    if (s->orig_ev) (void)hipEventDestroy(s->orig_ev);
    delete s;
}

// ---- camera (Camera.cpp) ---------------------------------------------------------------------
int32_t bm_camera_create(bm_context* ctx, bm_camera** out) {
    if (!ctx || !out) return BM_ERROR_INVALID_PARAMETER;
    bm_camera* c = new (std::nothrow) bm_camera();
    if (!c) return BM_ERROR_GPU_ALLOC_FAIL;
    c->ctx = ctx;
    for (bm_context* p : ctx->peers) {
        bm_camera* r = nullptr;
        const int32_t rc = bm_camera_create(p, &r);
        if (rc) {
            bm_camera_destroy(c);
            return peer_fail(ctx, p, rc);
        }
        c->rep.push_back(r);
    }
    *out = c;
    return BM_ERROR_ALL_FINE;
}

// Camera::setInitialRays (Camera.cpp:43-72). The ray at pixel (x,y) is a function of the x-th
// term of the column recurrence and the y-th term of the row recurrence only, so the camera keeps
// those two tables (W + H floats) and the trace kernel rebuilds each direction with the same
// arithmetic; the per-pixel validation of the reference is kept here.
static int32_t camera_rays_impl(bm_camera* c, uint32_t width, uint32_t height, float left, float right, float top,
                                float bottom, float zoom, bool validate) {
    bm_context* ctx = c->ctx;
    if (width == 0 || height == 0) return fail(ctx, BM_ERROR_INVALID_PARAMETER, "setInitialRays: zero size");
    const float dx = (right - left) / (float)width;
    const float dy = (bottom - top) / (float)height;
    const float z2 = zoom * zoom;
    std::vector<float> rx(width), ry(height);
    float v = top + dy * .5f;
    for (uint32_t y = 0; y < height; y++, v += dy) ry[y] = v;
    v = left + dx * .5f;
    for (uint32_t x = 0; x < width; x++, v += dx) rx[x] = v;
    for (uint32_t y = 0; validate && y < height; ++y) {
        const float ryy = ry[y] * ry[y];
        for (uint32_t x = 0; x < width; ++x) {
            const float d = 1.f / std::sqrt(z2 + rx[x] * rx[x] + ryy);
            if (std::isnan(d) || d <= 0.f)
                return fail(ctx, BM_ERROR_INVALID_PARAMETER, "setInitialRays: NaN or non-positive ray (Camera.cpp:62)");
        }
    }
    BM_HIP(ctx, hipSetDevice(ctx->device));
    BM_HIP(ctx, ctx_drain(ctx));
    GrowGuard grow{ctx};
    BM_HIP(ctx, grow.reserve(c->rx, 4 * (size_t)width));
    BM_HIP(ctx, grow.reserve(c->ry, 4 * (size_t)height));
    BM_HIP(ctx, hipMemcpyAsync(c->rx.p, rx.data(), 4 * (size_t)width, hipMemcpyHostToDevice, ctx->stream));
    BM_HIP(ctx, hipMemcpyAsync(c->ry.p, ry.data(), 4 * (size_t)height, hipMemcpyHostToDevice, ctx->stream));
    BM_HIP(ctx, hipStreamSynchronize(ctx->stream));
    c->width = width;
    c->height = height;
    c->zoom = zoom;
    c->z2 = z2;
    c->left = left;
    c->top = top;
    c->dx = dx;
    c->dy = dy;
    return BM_ERROR_ALL_FINE;
}

int32_t bm_camera_set_initial_rays(bm_camera* c, uint32_t width, uint32_t height, float left, float right, float top,
                                   float bottom, float zoom) {
    if (!c) return BM_ERROR_INVALID_PARAMETER;
    int32_t rc = camera_rays_impl(c, width, height, left, right, top, bottom, zoom, true);
    for (size_t i = 0; rc == BM_ERROR_ALL_FINE && i < c->rep.size(); ++i) {  // same tables, validated once
        rc = camera_rays_impl(c->rep[i], width, height, left, right, top, bottom, zoom, false);
        if (rc) return peer_fail(c->ctx, c->rep[i]->ctx, rc);
    }
    return rc;
}

// Upper bound of the fraction of the frame whose rays can reach the scene's box: the box's eight
// corners projected through the camera (orient^-1, then the pinhole x/z, y/z of setInitialRays'
// window), their bounding rectangle clipped to the frame. 1 when unknown (build still running), when
// the eye is inside the box or a corner is not in front of the camera.
static double scene_coverage(const bm_camera* c, const bm_scene* s, const float* eye3, const float* m) {
    if (!s->hbounds || hipEventQuery(s->hbounds_ev) != hipSuccess || s->n == 0) return 1.0;
    double lo[3], hi[3];
    for (int a = 0; a < 3; ++a) {
        lo[a] = bm::bounds_lo(s->hbounds[a]);
        hi[a] = bm::bounds_hi(s->hbounds[3 + a]);
        if (!(lo[a] <= hi[a])) return 1.0;
    }
    bool inside = true;
    for (int a = 0; a < 3; ++a) inside = inside && eye3[a] >= lo[a] && eye3[a] <= hi[a];
    if (inside) return 1.0;
    // dir = M r with M column-major (m[3*col + row]); r = M^-1 dir
    const double a00 = m[0], a10 = m[1], a20 = m[2], a01 = m[3], a11 = m[4], a21 = m[5], a02 = m[6], a12 = m[7],
                 a22 = m[8];
    const double det = a00 * (a11 * a22 - a12 * a21) - a01 * (a10 * a22 - a12 * a20) + a02 * (a10 * a21 - a11 * a20);
    if (!(std::fabs(det) > 1e-12)) return 1.0;
    const double inv[9] = {(a11 * a22 - a12 * a21) / det, (a02 * a21 - a01 * a22) / det, (a01 * a12 - a02 * a11) / det,
                           (a12 * a20 - a10 * a22) / det, (a00 * a22 - a02 * a20) / det, (a02 * a10 - a00 * a12) / det,
                           (a10 * a21 - a11 * a20) / det, (a01 * a20 - a00 * a21) / det, (a00 * a11 - a01 * a10) / det};
    double x0 = 1e300, x1 = -1e300, y0 = 1e300, y1 = -1e300;
    for (int k = 0; k < 8; ++k) {
        const double v[3] = {((k & 1) ? hi[0] : lo[0]) - eye3[0], ((k & 2) ? hi[1] : lo[1]) - eye3[1],
                             ((k & 4) ? hi[2] : lo[2]) - eye3[2]};
        double r[3];
        for (int i = 0; i < 3; ++i) r[i] = inv[3 * i] * v[0] + inv[3 * i + 1] * v[1] + inv[3 * i + 2] * v[2];
        if (!(r[2] > 1e-9)) return 1.0;
        const double sx = r[0] / r[2] * c->zoom, sy = r[1] / r[2] * c->zoom;  // ray (rx, ry, zoom) direction
        const double px = (sx - c->left) / c->dx - 0.5, py = (sy - c->top) / c->dy - 0.5;
        x0 = std::min(x0, px), x1 = std::max(x1, px), y0 = std::min(y0, py), y1 = std::max(y1, py);
    }
    const double W = c->width, H = c->height;
    const double w = std::max(0.0, std::min(W, x1 + 2.0) - std::max(0.0, x0 - 2.0));
    const double h = std::max(0.0, std::min(H, y1 + 2.0) - std::max(0.0, y0 - 2.0));
    return w * h / (W * H);
}

static int32_t trace_impl(bm_camera* c, const float* eye3, const float* orient3x3, bm_scene* s, bm_rt* rt,
                          const TraceReq& rq) {
    if (!c) return BM_ERROR_INVALID_PARAMETER;
    bm_context* ctx = c->ctx;
    if (!eye3 || !orient3x3 || !s || c->width == 0 || c->height == 0 || !c->rx.p)
        return fail(ctx, BM_ERROR_INVALID_PARAMETER, "traceScene: invalid parameter (Camera.cpp:88-92)");
    if (!rt) return fail(ctx, BM_ERROR_NO_RENDER_TARGET, "traceScene: no render target");
    if (rq.band_h == 0 || rq.band_step == 0 || rq.band_first >= rq.band_step)
        return fail(ctx, BM_ERROR_INVALID_PARAMETER, "trace: invalid band partition");
    const uint32_t bands = (c->height + rq.band_h - 1) / rq.band_h;
    const uint32_t my_bands = bands > rq.band_first ? (bands - rq.band_first + rq.band_step - 1) / rq.band_step : 0;
    const uint32_t rows = my_bands * rq.band_h;
    // the reference requires equal sizes (Scene.cpp:90-94); a band target needs room for its rows
    if (rt->width != c->width || (rq.exact ? rt->height != c->height : rt->height < std::min(rows, c->height)))
        return fail(ctx, BM_ERROR_RT_CAM_MISMATCH, "render target and camera sizes differ (Scene.cpp:90-94)");
    if (!s->built) return fail(ctx, BM_ERROR_NOT_BUILT, "scene has no current build (call updateGPUScene)");
    if (rq.light && !(std::isfinite(rq.light[0]) && std::isfinite(rq.light[1]) && std::isfinite(rq.light[2])))
        return fail(ctx, BM_ERROR_INVALID_PARAMETER, "shadow trace: light position must be finite");
    BM_HIP(ctx, hipSetDevice(ctx->device));
    const hipStream_t st = rt_stream(rt);
    BM_HIP(ctx, rt_acquire(rt));
    if (s->hash || s->kd) {  // reference modes: the reference's own accelerators and marches
        if (!rq.exact || rq.band_step != 1 || rq.light || (s->hash && (rq.count || rq.diag)))
            return fail(ctx, BM_ERROR_INVALID_PARAMETER, "reference mode: full-frame traceScene only");
        bm::TraceParams p{};
        p.tris = s->tri_orig.as<const float4>();  // original order: the reference's face ids
        p.nrm = s->nrm.as<const float>();
        p.rx = c->rx.as<const float>();
        p.ry = c->ry.as<const float>();
        p.z2 = c->z2;
        p.zoom = c->zoom;
        std::memcpy(p.eye, eye3, sizeof(p.eye));
        std::memcpy(p.orient, orient3x3, sizeof(p.orient));
        p.width = c->width;
        p.height = c->height;
        p.pitch_u32 = rt->pitch / 4;
        p.packed = rt->packed;
        p.tri_id = rt->tri;
        p.t = rt->t;
        p.nz = rt->nz;
        p.counters = rq.counters;
        p.diag = rq.diag;
        if (rq.grid_out) *rq.grid_out = ((c->width + 7) / 8) * ((c->height + 7) / 8);  // one wave per 8x8 tile
        const uint32_t* faces = (s->kd_sorted_in_scratch ? s->kd_vals2 : s->kd_vals).as<const uint32_t>();
        rt->last_kind = s->hash ? BM_TRACE_KIND_HASH_MARCH : BM_TRACE_KIND_KD_MARCH;
        if (s->hash) {  // Hash.cu:235-302
            BM_HIP(ctx, bm::launch_hash_march(p, s->hash_bstart.as<const uint32_t>(),
                                              s->hash_bend.as<const uint32_t>(), faces, st));
        } else {  // BuildTree.cu:367-499
            if (const int32_t r = kd_leaves_ready(s)) return r;
            bm::KdMarch k{s->kd_leaf_key.as<const uint32_t>(), s->kd_leaf_start.as<const uint32_t>(),
                          s->kd_leaf_count.as<const uint32_t>(), faces,
                          s->kd_lch.as<const uint32_t>(), s->kd_rch.as<const uint32_t>(),
                          s->kd_first.as<const uint32_t>(), s->kd_last.as<const uint32_t>(), s->kd_leaves,
                          bm::kd_leaf_depth(KD_WORLD_MIN, KD_WORLD_MAX), KD_WORLD_MIN, KD_WORLD_MAX,
                          s->kd_nodes.as<const uint4>(), s->kd_leafrec.as<const uint4>(),
                          s->kd_node_key.as<const uint32_t>(),
                          s->kd_ftris.as<const float4>(), s->kd_ubox.as<const uint32_t>()};
            k.march_variant = (int)ctx->tune.get(BM_PARAM_KD_MARCH, 3);
            // child-box records exist only when the build ran with march 3 (the same frames either way)
            if (k.march_variant == 3 && !s->kd_cnodes_valid) k.march_variant = 2;
            k.cnodes = s->kd_cnodes_valid ? s->kd_cnodes.as<const uint4>() : nullptr;
            BM_HIP(ctx, bm::launch_kd_march(p, k, rq.count, st));
        }
        if (rt->stream) BM_HIP(ctx, hipEventRecord(rt->done, st));
        return BM_ERROR_ALL_FINE;
    }
    bm::TraceParams p{};
    p.nodes = s->records.as<const uint4>();
    p.tris = s->tris.as<const float4>();
    p.nrm = s->nrm.as<const float>();
    p.rx = c->rx.as<const float>();
    p.ry = c->ry.as<const float>();
    p.z2 = c->z2;
    p.zoom = c->zoom;
    std::memcpy(p.eye, eye3, sizeof(p.eye));
    std::memcpy(p.orient, orient3x3, sizeof(p.orient));
    p.width = c->width;
    p.height = c->height;
    p.band_h = rq.band_h;
    p.band_step = rq.band_step;
    p.band_first = rq.band_first;
    p.local_rows = std::min(rows, rt->height);
    p.pitch_u32 = rt->pitch / 4;
    p.num_tris = s->n;
    p.packed = rt->packed;
    p.tri_id = rt->tri;
    p.t = rt->t;
    p.nz = rt->nz;
    p.counters = rq.counters;
    p.variant = rq.variant_override >= 0 ? rq.variant_override : ctx->trace_variant;
    p.bvh_width = s->width;
    if (rq.variant_override < 0 && p.variant == bm::TRACE_QUAD && s->width == 4 && !rq.diag &&
        (ctx->auto_compact || ctx->auto_packet)) {
        const double cov = scene_coverage(c, s, eye3, orient3x3);
        // dense coherent views: wave packets (k_trace_packet) when the scene box covers >= 1M of this
        // target's pixels (0.5M with frames in flight: a target on its own stream, whose packets' longest
        // waves overlap the other frames) at >= 4 of them per triangle — enough 8x8 packets to fill the
        // machine, each sharing its node records over most of its 64 rays (measured, DESIGN §12: the
        // filled view and C4 -40 % / -13 % one frame at a time, -53 % / -25 % in flight; C2 at 0.55M
        // covered pixels -8 % in flight, +7 % one frame at a time; C3 at 2 pixels per triangle stays faster
        // as quads)
        const double covered = cov * (double)c->width * (double)p.local_rows;
        const double min_covered = rt->stream ? 0.5e6 : 1.0e6;
        if (ctx->auto_packet && !rq.count && !rq.light && covered >= min_covered && covered >= 4.0 * (double)s->n)
            p.variant = bm::TRACE_PACKET;
        // frames in flight over a sparse view: most rays miss the scene, so the lane-per-ray root cull and
        // compacted quads (TRACE_COMPACT) cost less per frame than quads for every ray (measured in flight:
        // bunny 1080p +21 %, armadillo proxy +18 %; filled view -9 %, one frame at a time no gain)
        else if (ctx->auto_compact && rt->stream && cov < 0.5)
            p.variant = bm::TRACE_COMPACT;
    }

    p.diag = rq.diag;
    p.scramble = ctx->scramble;
    p.prio_after = ctx->prio_after;
    p.prio_level = ctx->prio_level;
    p.refill_min = ctx->refill_min;
    p.sched = ctx->sched >= 0 ? (uint32_t)ctx->sched : rt->stream ? 1u : 2u;
    const bool packet = p.variant == bm::TRACE_PACKET && !rq.count && !rq.light && s->width == 4;
    if (packet) p.persistent_blocks = ctx->persistent_blocks;  // the packet kernel's persistent grid (no overflow area)
    if (p.sched == 2 && (p.variant == bm::TRACE_QUAD || packet)) {  // (quad tiles outnumber 8x8 packet tiles)
        const size_t ntiles = bm::quad_tiles(p.width, p.local_rows);
        if (rt->tile_cost.cap < 4 * ntiles) {
            BM_HIP(ctx, hipStreamSynchronize(st));
            BM_HIP(ctx, rt->tile_cost.reserve(4 * ntiles));
            BM_HIP(ctx, hipMemsetAsync(rt->tile_cost.p, 0, 4 * ntiles, st));
        }
        p.tile_cost = rt->tile_cost.as<uint32_t>();
    }
    const bool shadow = rq.light != nullptr;
    if (shadow && p.variant == bm::TRACE_PERSIST_DIAG12)
        return fail(ctx, BM_ERROR_INVALID_PARAMETER, "shadow trace: not available with the diagnostic variant");
    // wave packets run only for non-counting BVH4 primary traces; otherwise that variant takes the quad
    // (or BVH2 single-lane) kernel, whose overflow area is sized here
    if (bm::trace_variant_persistent(p.variant) || shadow || (p.variant == bm::TRACE_PACKET && !packet)) {
        const uint32_t blocks = ctx->persistent_blocks ? ctx->persistent_blocks : 1024;
        const size_t slots = (size_t)blocks * 256;
        const size_t bytes =
            slots * ((p.bvh_width == 8 ? bm::MAX_STACK8 : bm::MAX_STACK) - bm::trace_variant_lds(p.variant)) * 8;
        void* ovf;
        size_t ovf_cap;
        if (rt->stream) {  // concurrent with other streams' traces: the target's own area
            if (bytes > rt->ovf.cap) BM_HIP(ctx, hipStreamSynchronize(st));
            BM_HIP(ctx, rt->ovf.reserve(bytes));
            ovf = rt->ovf.p;
            ovf_cap = rt->ovf.cap;
        } else {
            if (bytes > ctx->ovf_cap) {
                // grow-only, outside any capture: the first trace of a context allocates it
                BM_HIP(ctx, hipStreamSynchronize(st));
                if (ctx->ovf) (void)hipFree(ctx->ovf);
                ctx->ovf = nullptr;
                ctx->ovf_cap = 0;
                BM_HIP(ctx, hipMalloc(&ctx->ovf, bytes));
                ctx->ovf_cap = bytes;
            }
            ovf = ctx->ovf;
            ovf_cap = ctx->ovf_cap;
        }
        p.persistent_blocks = blocks;
        p.ovf_stride = (uint32_t)slots;
        p.ovf_ref = reinterpret_cast<uint32_t*>(ovf);
        p.ovf_t = reinterpret_cast<float*>(reinterpret_cast<char*>(ovf) + ovf_cap / 2);
    }
    if (shadow) {
        const size_t px = (size_t)rt->width * rt->height;
        const size_t qbytes = ctx->shadow_queue ? 4 * (64 + px) : 0;
        if (rt->shadow.cap < px || rt->queue.cap < qbytes) BM_HIP(ctx, hipStreamSynchronize(st));
        BM_HIP(ctx, rt->shadow.reserve(px));
        p.shadow = rt->shadow.as<uint8_t>();
        std::memcpy(p.light, rq.light, sizeof(p.light));
        p.shadow_counters = rq.shadow_counters;
        if (ctx->shadow_queue) {
            BM_HIP(ctx, rt->queue.reserve(qbytes));
            p.shadow_queue = true;
            p.queue_count = rt->queue.as<uint32_t>();
            p.queue = rt->queue.as<uint32_t>() + 64;
            BM_HIP(ctx, hipMemsetAsync(p.queue_count, 0, 4, st));
        }
    }
    uint32_t regions = 0, tpr = 0;
    if (p.variant == bm::TRACE_COMPACT && p.bvh_width == 4 && !(shadow && ctx->shadow_queue) &&
        bm::trace_compact_layout(p.width, p.local_rows, ctx->cull_tpr, &regions, &tpr)) {
        const size_t region = (size_t)tpr * 64;
        const size_t bytes = 4 * (regions + (size_t)regions * region);
        if (rt->rayq.cap < bytes) BM_HIP(ctx, hipStreamSynchronize(st));
        BM_HIP(ctx, rt->rayq.reserve(bytes));
        p.rayq_count = rt->rayq.as<uint32_t>();
        p.rayq = p.rayq_count + regions;
        // near-orthonormal orient (columns unit and pairwise orthogonal within 2^-10): the cull's
        // approximate ray directions stay within 2^-20 relative of the exact ones
        double worst = 0;
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) {
                double d = 0;
                for (int k = 0; k < 3; ++k) d += (double)orient3x3[3 * i + k] * (double)orient3x3[3 * j + k];
                worst = std::max(worst, std::fabs(d - (i == j ? 1.0 : 0.0)));
            }
        p.fast_cull = worst < 0x1p-10 ? 1u : 0u;
        p.rayq_region = (uint32_t)region;
        p.rayq_tpr = tpr;
        p.rayq_regions = regions;
    }
    const bool dyn = p.variant == bm::TRACE_PERSIST_DYN12 || p.variant == bm::TRACE_PERSIST_DYN16;
    if (dyn && rt->stream)
        return fail(ctx, BM_ERROR_INVALID_PARAMETER, "trace: the global-ticket variants need the context stream");
    if (dyn) {
        if (!ctx->tile_ctr) {
            BM_HIP(ctx, hipMalloc(&ctx->tile_ctr, sizeof(unsigned long long)));
            BM_HIP(ctx, hipMemsetAsync(ctx->tile_ctr, 0, sizeof(unsigned long long), st));
            ctx->tile_base = 0;
        }
        p.tile_ctr = ctx->tile_ctr;
        p.tile_base = ctx->tile_base;
    }
    uint32_t grid = 0;
    if (p.bvh_width == 8 && ((shadow && ctx->shadow_queue) ||
                             (p.variant != bm::TRACE_QUAD && p.variant != bm::TRACE_COMPACT)))
        return fail(ctx, BM_ERROR_INVALID_PARAMETER, "BVH8 scenes trace with the quad kernel only");
    rt->last_kind = packet ? BM_TRACE_KIND_PACKETS
                    : (p.variant == bm::TRACE_COMPACT && p.rayq) ? BM_TRACE_KIND_CULL_QUADS
                    : ((p.variant == bm::TRACE_QUAD || p.variant == bm::TRACE_COMPACT || p.variant == bm::TRACE_PACKET) &&
                       p.bvh_width >= 4 &&
                       !(shadow && ctx->shadow_queue))
                        ? BM_TRACE_KIND_QUADS
                        : BM_TRACE_KIND_LANES;
    BM_HIP(ctx, bm::launch_trace(p, rq.count, st, &grid));
    if (rq.grid_out) *rq.grid_out = grid;
    if (dyn) ctx->tile_base += (unsigned long long)((p.width + 7) / 8) * ((p.local_rows + 7) / 8) + 4ull * grid;
    if (shadow) BM_HIP(ctx, bm::launch_shadow(p, rq.count, st));
    if (rt->stream) BM_HIP(ctx, hipEventRecord(rt->done, st));
    return BM_ERROR_ALL_FINE;
}

static TraceReq bands_req(uint32_t band_height, uint32_t band_step, uint32_t band_first) {
    TraceReq rq;
    rq.band_h = band_height;
    rq.band_step = band_step;
    rq.band_first = band_first;
    rq.exact = false;
    return rq;
}

// ---- multi-GPU trace: screen bands over the devices + one gather to the root ------
static constexpr uint32_t ALL_PLANES = BM_PLANE_PACKED | BM_PLANE_TRI_ID | BM_PLANE_T | BM_PLANE_NZ | BM_PLANE_SHADOW;
static_assert(BM_PLANE_PACKED == bm::PLANE_PACKED && BM_PLANE_TRI_ID == bm::PLANE_TRI_ID && BM_PLANE_T == bm::PLANE_T &&
                  BM_PLANE_NZ == bm::PLANE_NZ && BM_PLANE_SHADOW == bm::PLANE_SHADOW,
              "plane bits");

// Bytes of each plane of a band buffer of `px` pixels, in gather order (packed, tri, t, nz, shadow).
static const uint32_t PLANE_BYTES[5] = {4, 4, 4, 4, 1};

static bm::BandPlanes band_planes(const bm_rt* b, uint32_t band_first, uint32_t rows) {
    return bm::BandPlanes{b->packed, b->tri, b->t, b->nz, b->shadow.as<const uint8_t>(), band_first, rows};
}

static void* band_plane_ptr(const bm_rt* b, int p) {
    switch (p) {
        case 0: return b->packed;
        case 1: return b->tri;
        case 2: return b->t;
        case 3: return b->nz;
        default: return b->shadow.p;
    }
}

// Staging area of source k (RCCL receive on the root): planes of rows*width pixels back to back.
static char* stage_plane(bm_rt* rt, uint32_t k, int p, size_t px) {
    size_t off = (size_t)k * px * 17;
    for (int q = 0; q < p; ++q) off += px * PLANE_BYTES[q];
    return rt->stage.as<char>() + off;
}

// First multi-device trace into rt: one compact band buffer per band source this process traces
// (each device of a one-process context, on its own stream; a multi-process rank's own, on rt's
// stream), events, and the root's RCCL staging area.
static int32_t mg_prepare(bm_rt* rt, uint32_t rows) {
    bm_context* ctx = rt->ctx;
    const bool procs = ctx->comm_size > 1;
    const uint32_t nsrc = procs ? 1u : (uint32_t)ctx->devices.size();
    for (uint32_t g = 0; g < nsrc; ++g) {
        bm_context* xg = g ? ctx->peers[g - 1] : ctx;
        BM_HIP(ctx, hipSetDevice(xg->device));
        hipStream_t bs = nullptr;
        if (!procs) BM_HIP(ctx, hipStreamCreateWithFlags(&bs, hipStreamNonBlocking));
        bm_rt* b = nullptr;
        int32_t rc = bm_rt_create_offscreen(xg, rt->width, rows, 0, &b);
        if (rc) {
            if (bs) (void)hipStreamDestroy(bs);
            return peer_fail(ctx, xg, rc);
        }
        xg->rts.pop_back();  // internal: owned by rt, released with it
        hipEvent_t ev = nullptr;
        (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
        rt->band.push_back(b);
        rt->band_stream.push_back(bs);
        rt->band_done.push_back(ev);
        if (!ev) return fail(ctx, BM_ERROR_DEVICE, "hipEventCreate failed");
        rc = bm_rt_set_stream(b, bs ? reinterpret_cast<void*>(bs) : reinterpret_cast<void*>(rt->stream));
        if (rc) return peer_fail(ctx, xg, rc);
    }
    BM_HIP(ctx, hipSetDevice(ctx->device));
    BM_HIP(ctx, hipEventCreateWithFlags(&rt->mg_start, hipEventDisableTiming));
    for (hipEvent_t& e : rt->mg_t) BM_HIP(ctx, hipEventCreate(&e));
    const uint32_t staged = ctx->gather != BM_GATHER_RCCL ? 0u : procs ? (ctx->comm_rank == 0 ? ctx->comm_size - 1 : 0)
                                                                       : nsrc - 1;
    if (staged) BM_HIP(ctx, rt->stage.reserve((size_t)staged * rows * rt->width * 17));
    return BM_ERROR_ALL_FINE;
}

#define BM_NCCL(ctx, expr)                                                                              \
    do {                                                                                                \
        const int e__ = (expr);                                                                         \
        if (e__ != 0)                                                                                   \
            return fail(ctx, BM_ERROR_DEVICE, std::string(#expr) + ": " + bm::rccl_error_string((ctx)->rccl, e__)); \
    } while (0)

static int32_t trace_multi(bm_camera* c, const float* eye3, const float* orient3x3, bm_scene* s, bm_rt* rt,
                           const float* light) {
    bm_context* ctx = c->ctx;
    if (!eye3 || !orient3x3 || !s || c->width == 0 || c->height == 0 || !c->rx.p)
        return fail(ctx, BM_ERROR_INVALID_PARAMETER, "traceScene: invalid parameter (Camera.cpp:88-92)");
    if (!rt) return fail(ctx, BM_ERROR_NO_RENDER_TARGET, "traceScene: no render target");
    if (rt->ctx != ctx || s->ctx != ctx) return fail(ctx, BM_ERROR_INVALID_PARAMETER, "objects of another context");
    if (rt->width != c->width || rt->height != c->height)
        return fail(ctx, BM_ERROR_RT_CAM_MISMATCH, "render target and camera sizes differ (Scene.cpp:90-94)");
    if (!s->built) return fail(ctx, BM_ERROR_NOT_BUILT, "scene has no current build (call updateGPUScene)");
    const bool procs = ctx->comm_size > 1;
    const uint32_t G = ctx->bands_n(), bh = ctx->band_h, W = rt->width, H = rt->height;
    const uint32_t rows = (((H + bh - 1) / bh + G - 1) / G) * bh;  // every source's (padded) band rows
    const size_t px = (size_t)rows * W;
    BM_HIP(ctx, hipSetDevice(ctx->device));
    const hipStream_t st = rt_stream(rt);
    BM_HIP(ctx, rt_acquire(rt));
    if (rt->band.empty()) {
        const int32_t rc = mg_prepare(rt, rows);
        if (rc) return rc;
    }
    // default exchange: the triangle-id plane (+ the u8 shadow plane), 4 (5) B/pixel; the root rebuilds
    // packed, t and |n.z| from the ids (launch_reshade). An explicit gather_planes mask moves those
    // planes as they are.
    const bool by_id = ctx->planes == 0;
    const uint32_t planes = (by_id ? (BM_PLANE_TRI_ID | BM_PLANE_SHADOW) : ctx->planes) &
                            (light ? ALL_PLANES : ALL_PLANES & ~BM_PLANE_SHADOW);
    if (light && (!procs || ctx->comm_rank == 0) && rt->shadow.cap < (size_t)W * H) {
        BM_HIP(ctx, hipStreamSynchronize(st));
        BM_HIP(ctx, rt->shadow.reserve((size_t)W * H));
    }
    const bm::FramePlanes dst{rt->packed, rt->pitch / 4, rt->tri, rt->t, rt->nz, rt->shadow.as<uint8_t>(), W, H};
    BM_HIP(ctx, hipEventRecord(rt->mg_start, st));  // the target's earlier work (reads) precedes the writes
    rt->mg_timed = false;  // set again only once all three events of this frame are recorded
    BM_HIP(ctx, hipEventRecord(rt->mg_t[0], st));
    for (uint32_t g = 0; g < rt->band.size(); ++g) {
        bm_camera* cg = g ? c->rep[g - 1] : c;
        bm_scene* sg = g ? s->rep[g - 1] : s;
        bm_rt* b = rt->band[g];
        bm_context* xg = b->ctx;
        const uint32_t first = procs ? (uint32_t)ctx->comm_rank : g;
        BM_HIP(ctx, hipSetDevice(xg->device));
        const hipStream_t bs = rt_stream(b);
        BM_HIP(ctx, hipStreamWaitEvent(bs, rt->mg_start, 0));
        TraceReq rq = bands_req(bh, G, first);
        rq.light = light;
        const int32_t rc = trace_impl(cg, eye3, orient3x3, sg, b, rq);
        if (rc) return peer_fail(ctx, xg, rc);
        if (g == 0) BM_HIP(ctx, hipEventRecord(rt->mg_t[1], bs));  // band 0's trace done (root device)
        if (ctx->gather == BM_GATHER_PEER) {  // this device writes its rows into the root's planes
            const bm::BandPlanes src = band_planes(b, first, rows);
            BM_HIP(ctx, bm::launch_band_scatter(&src, 1, dst, bh, G, planes, bs));
        }
        BM_HIP(ctx, hipEventRecord(rt->band_done[g], bs));
    }
    BM_HIP(ctx, hipSetDevice(ctx->device));
    if (ctx->gather == BM_GATHER_PEER) {
        for (hipEvent_t e : rt->band_done) BM_HIP(ctx, hipStreamWaitEvent(st, e, 0));
    } else if (!procs && ctx->rccl_loopback) {  // one GPU listed N times: send/recv to self, on st
        for (hipEvent_t e : rt->band_done) BM_HIP(ctx, hipStreamWaitEvent(st, e, 0));
        BM_NCCL(ctx, bm::rccl_group_start(ctx->rccl));
        for (uint32_t g = 1; g < G; ++g)
            for (int p = 0; p < 5; ++p) {
                if (!(planes & (1u << p))) continue;
                BM_NCCL(ctx, bm::rccl_send(ctx->rccl, band_plane_ptr(rt->band[g], p), px * PLANE_BYTES[p], 0,
                                           ctx->comm, st));
                BM_NCCL(ctx, bm::rccl_recv(ctx->rccl, stage_plane(rt, g - 1, p, px), px * PLANE_BYTES[p], 0,
                                           ctx->comm, st));
            }
        BM_NCCL(ctx, bm::rccl_group_end(ctx->rccl));
    } else if (!procs) {  // one process, RCCL: every peer's band planes into the root's staging area
        BM_HIP(ctx, hipStreamWaitEvent(st, rt->band_done[0], 0));
        BM_NCCL(ctx, bm::rccl_group_start(ctx->rccl));
        for (uint32_t g = 1; g < G; ++g)
            for (int p = 0; p < 5; ++p) {
                if (!(planes & (1u << p))) continue;
                BM_NCCL(ctx, bm::rccl_send(ctx->rccl, band_plane_ptr(rt->band[g], p), px * PLANE_BYTES[p], 0,
                                           ctx->nccl[g], rt->band_stream[g]));
                BM_NCCL(ctx, bm::rccl_recv(ctx->rccl, stage_plane(rt, g - 1, p, px), px * PLANE_BYTES[p], (int)g,
                                           ctx->nccl[0], st));
            }
        BM_NCCL(ctx, bm::rccl_group_end(ctx->rccl));
    } else if (ctx->comm_rank != 0) {  // several processes: this rank's band planes to rank 0
        BM_NCCL(ctx, bm::rccl_group_start(ctx->rccl));
        for (int p = 0; p < 5; ++p)
            if (planes & (1u << p))
                BM_NCCL(ctx, bm::rccl_send(ctx->rccl, band_plane_ptr(rt->band[0], p), px * PLANE_BYTES[p], 0,
                                           ctx->comm, st));
        BM_NCCL(ctx, bm::rccl_group_end(ctx->rccl));
    } else {
        BM_NCCL(ctx, bm::rccl_group_start(ctx->rccl));
        for (int r = 1; r < ctx->comm_size; ++r)
            for (int p = 0; p < 5; ++p)
                if (planes & (1u << p))
                    BM_NCCL(ctx, bm::rccl_recv(ctx->rccl, stage_plane(rt, r - 1, p, px), px * PLANE_BYTES[p], r,
                                               ctx->comm, st));
        BM_NCCL(ctx, bm::rccl_group_end(ctx->rccl));
    }
    if (ctx->gather == BM_GATHER_RCCL && (!procs || ctx->comm_rank == 0)) {  // root: one scatter of all sources
        bm::BandPlanes src[bm::MAX_BAND_SOURCES];
        src[0] = band_planes(rt->band[0], 0, rows);
        for (uint32_t k = 1; k < G; ++k)
            src[k] = bm::BandPlanes{reinterpret_cast<const uint32_t*>(stage_plane(rt, k - 1, 0, px)),
                                    reinterpret_cast<const uint32_t*>(stage_plane(rt, k - 1, 1, px)),
                                    reinterpret_cast<const float*>(stage_plane(rt, k - 1, 2, px)),
                                    reinterpret_cast<const float*>(stage_plane(rt, k - 1, 3, px)),
                                    reinterpret_cast<const uint8_t*>(stage_plane(rt, k - 1, 4, px)), k, rows};
        BM_HIP(ctx, bm::launch_band_scatter(src, G, dst, bh, G, planes, st));
    }
    if (by_id && (!procs || ctx->comm_rank == 0)) {
        bm::TraceParams p{};
        p.nrm = s->nrm.as<const float>();
        p.rx = c->rx.as<const float>();
        p.ry = c->ry.as<const float>();
        p.z2 = c->z2;
        p.zoom = c->zoom;
        std::memcpy(p.eye, eye3, sizeof(p.eye));
        std::memcpy(p.orient, orient3x3, sizeof(p.orient));
        p.width = W;
        p.height = H;
        p.pitch_u32 = rt->pitch / 4;
        p.packed = rt->packed;
        p.tri_id = rt->tri;
        p.t = rt->t;
        p.nz = rt->nz;
        if (!s->orig_valid) {  // built before this context had peers: the records it did not need then
            bm::BuildBuffers ob;
            ob.n = s->n;
            ob.num_meshes = s->num_meshes;
            ob.meshes = s->mesh_table.as<const bm::MeshDesc>();
            ob.tri_orig = s->tri_orig.as<float4>();
            ob.bounds = s->bounds.as<uint32_t>();
            BM_HIP(ctx, hipStreamWaitEvent(st, s->ev1, 0));  // the build (and its mesh-table upload) first
            BM_HIP(ctx, bm::launch_orig_records(ob, st));
            // a target on another stream (frames in flight) must not reshade from tri_orig
            // before this launch has written it
            BM_HIP(ctx, hipEventRecord(s->orig_ev, st));
            s->orig_valid = true;
            s->orig_lazy = true;
        } else if (s->orig_lazy) {
            BM_HIP(ctx, hipStreamWaitEvent(st, s->orig_ev, 0));
        }
        BM_HIP(ctx, bm::launch_reshade(p, s->tri_orig.as<const float4>(), st));
    }
    BM_HIP(ctx, hipEventRecord(rt->mg_t[2], st));
    rt->mg_timed = true;
    if (rt->stream) BM_HIP(ctx, hipEventRecord(rt->done, st));
    return BM_ERROR_ALL_FINE;
}

int32_t bm_rt_last_timing(bm_rt* rt, float out_ms[2]) {
    if (!rt || !out_ms || !rt->ctx) return BM_ERROR_INVALID_PARAMETER;
    bm_context* ctx = rt->ctx;
    if (!rt->mg_timed) return fail(ctx, BM_ERROR_NOT_BUILT, "last_timing: no multi-device trace into this target");
    BM_HIP(ctx, hipSetDevice(ctx->device));
    BM_HIP(ctx, hipEventSynchronize(rt->mg_t[2]));
    BM_HIP(ctx, hipEventElapsedTime(&out_ms[0], rt->mg_t[0], rt->mg_t[1]));
    BM_HIP(ctx, hipEventElapsedTime(&out_ms[1], rt->mg_t[1], rt->mg_t[2]));
    return BM_ERROR_ALL_FINE;
}

int32_t bm_camera_trace(bm_camera* c, const float* eye3, const float* orient3x3, bm_scene* s, bm_rt* rt) {
    if (c && c->ctx->multi()) return trace_multi(c, eye3, orient3x3, s, rt, nullptr);
    return trace_impl(c, eye3, orient3x3, s, rt, TraceReq{});
}

int32_t bm_camera_trace_bands(bm_camera* c, const float* eye3, const float* orient3x3, bm_scene* s, bm_rt* rt,
                              uint32_t band_height, uint32_t band_step, uint32_t band_first) {
    return trace_impl(c, eye3, orient3x3, s, rt, bands_req(band_height, band_step, band_first));
}

int32_t bm_camera_trace_shadow(bm_camera* c, const float* eye3, const float* orient3x3, bm_scene* s, bm_rt* rt,
                               const float* light3) {
    if (!light3) return c ? fail(c->ctx, BM_ERROR_INVALID_PARAMETER, "shadow trace: no light") : BM_ERROR_INVALID_PARAMETER;
    if (c->ctx->multi()) return trace_multi(c, eye3, orient3x3, s, rt, light3);
    TraceReq rq;
    rq.light = light3;
    return trace_impl(c, eye3, orient3x3, s, rt, rq);
}

int32_t bm_camera_trace_shadow_bands(bm_camera* c, const float* eye3, const float* orient3x3, bm_scene* s,
                                     bm_rt* rt, uint32_t band_height, uint32_t band_step, uint32_t band_first,
                                     const float* light3) {
    if (!light3) return c ? fail(c->ctx, BM_ERROR_INVALID_PARAMETER, "shadow trace: no light") : BM_ERROR_INVALID_PARAMETER;
    TraceReq rq = bands_req(band_height, band_step, band_first);
    rq.light = light3;
    return trace_impl(c, eye3, orient3x3, s, rt, rq);
}

int32_t bm_camera_trace_counters(bm_camera* c, const float* eye3, const float* orient3x3, bm_scene* s, bm_rt* rt,
                                 uint64_t out[3]) {
    if (!c || !out) return BM_ERROR_INVALID_PARAMETER;
    bm_context* ctx = c->ctx;
    if (!rt) return fail(ctx, BM_ERROR_NO_RENDER_TARGET, "traceScene: no render target");
    const hipStream_t st = rt_stream(rt);
    BM_HIP(ctx, hipSetDevice(ctx->device));
    BM_HIP(ctx, c->counters.reserve(6 * sizeof(unsigned long long)));
    BM_HIP(ctx, hipMemsetAsync(c->counters.p, 0, 6 * sizeof(unsigned long long), st));
    TraceReq rq;
    rq.count = true;
    rq.counters = c->counters.as<unsigned long long>();
    int32_t e = trace_impl(c, eye3, orient3x3, s, rt, rq);
    if (e) return e;
    unsigned long long h[3];
    BM_HIP(ctx, hipMemcpyAsync(h, c->counters.p, sizeof(h), hipMemcpyDeviceToHost, st));
    BM_HIP(ctx, hipStreamSynchronize(st));
    for (int i = 0; i < 3; ++i) out[i] = h[i];
    return BM_ERROR_ALL_FINE;
}

int32_t bm_camera_trace_shadow_counters(bm_camera* c, const float* eye3, const float* orient3x3, bm_scene* s,
                                        bm_rt* rt, const float* light3, uint64_t out[6]) {
    if (!c || !out || !light3) return BM_ERROR_INVALID_PARAMETER;
    bm_context* ctx = c->ctx;
    if (!rt) return fail(ctx, BM_ERROR_NO_RENDER_TARGET, "traceScene: no render target");
    const hipStream_t st = rt_stream(rt);
    BM_HIP(ctx, hipSetDevice(ctx->device));
    BM_HIP(ctx, c->counters.reserve(6 * sizeof(unsigned long long)));
    BM_HIP(ctx, hipMemsetAsync(c->counters.p, 0, 6 * sizeof(unsigned long long), st));
    TraceReq rq;
    rq.count = true;
    rq.counters = c->counters.as<unsigned long long>();
    rq.shadow_counters = rq.counters + 3;
    rq.light = light3;
    int32_t e = trace_impl(c, eye3, orient3x3, s, rt, rq);
    if (e) return e;
    unsigned long long h[6];
    BM_HIP(ctx, hipMemcpyAsync(h, c->counters.p, sizeof(h), hipMemcpyDeviceToHost, st));
    BM_HIP(ctx, hipStreamSynchronize(st));
    for (int i = 0; i < 6; ++i) out[i] = h[i];
    return BM_ERROR_ALL_FINE;
}

int32_t bm_camera_trace_profile(bm_camera* c, const float* eye3, const float* orient3x3, bm_scene* s, bm_rt* rt,
                                uint64_t* per_wave, uint32_t max_waves, uint32_t* num_waves) {
    if (!c || !num_waves) return BM_ERROR_INVALID_PARAMETER;
    bm_context* ctx = c->ctx;
    if (!rt) return fail(ctx, BM_ERROR_NO_RENDER_TARGET, "traceScene: no render target");
    const hipStream_t st = rt_stream(rt);
    // waves of the largest persistent grid; reference mode and wave packets: one wave per 8x8 tile
    const bool packet = ctx->trace_variant == bm::TRACE_PACKET && s && !s->kd && s->width == 4;
    const uint32_t tiles = ((c->width + 7) / 8) * ((c->height + 7) / 8);
    const uint32_t cap = (s && s->kd) || packet ? tiles : ctx->persistent_blocks * 4;
    *num_waves = cap;
    if (!per_wave || max_waves < cap) return fail(ctx, BM_ERROR_INVALID_PARAMETER, "trace_profile: buffer too small");
    BM_HIP(ctx, hipSetDevice(ctx->device));
    DevBuf d;
    BM_HIP(ctx, d.reserve((size_t)cap * 32));
    BM_HIP(ctx, hipMemsetAsync(d.p, 0, (size_t)cap * 32, st));
    BM_HIP(ctx, c->counters.reserve(6 * sizeof(unsigned long long)));
    TraceReq rq;
    // the quad and compacted variants carry their own diagnostic builds; others: DIAG12
    rq.variant_override = (ctx->trace_variant == bm::TRACE_COMPACT || ctx->trace_variant == bm::TRACE_QUAD || packet)
                              ? ctx->trace_variant
                              : bm::TRACE_PERSIST_DIAG12;
    rq.diag = d.as<unsigned long long>();
    rq.count = !packet;  // packets: per-wave step counts instead of the oracle's counters
    rq.counters = c->counters.as<unsigned long long>();
    uint32_t grid = 0;
    rq.grid_out = &grid;
    int32_t e = trace_impl(c, eye3, orient3x3, s, rt, rq);
    if (e) {
        d.release();
        return e;
    }
    *num_waves = s->kd ? grid : packet ? tiles : grid * 4;
    BM_HIP(ctx, hipMemcpyAsync(per_wave, d.p, (size_t)*num_waves * 32, hipMemcpyDeviceToHost, st));
    BM_HIP(ctx, hipStreamSynchronize(st));
    d.release();
    return BM_ERROR_ALL_FINE;
}

void bm_camera_destroy(bm_camera* c) {
    if (!c) return;
    for (bm_camera* r : c->rep) bm_camera_destroy(r);
    (void)hipSetDevice(c->ctx->device);
    (void)ctx_sync_all(c->ctx);
    c->rx.release();
    c->ry.release();
    c->counters.release();
    delete c;
}

// ---- render target (RenderTarget.cpp, offscreen) ---------------------------------------------
int32_t bm_rt_create_offscreen(bm_context* ctx, uint32_t width, uint32_t height, uint32_t pitch, bm_rt** out) {
    if (!ctx || !out || width == 0 || height == 0) return BM_ERROR_INVALID_PARAMETER;
    if (width >= (1u << 30) || (uint64_t)width * height >= (1ull << 32))  // trace kernels index planes in 32 bits
        return fail(ctx, BM_ERROR_INVALID_PARAMETER, "render target of 2^32 pixels or more");
    if (pitch == 0) pitch = width * 4;
    if (pitch < width * 4 || (pitch % 4) != 0)
        return fail(ctx, BM_ERROR_INVALID_PARAMETER, "pitch < width*4 (RenderTarget.cpp:19)");
    BM_HIP(ctx, hipSetDevice(ctx->device));
    bm_rt* rt = new (std::nothrow) bm_rt();
    if (!rt) return BM_ERROR_GPU_ALLOC_FAIL;
    rt->ctx = ctx;
    rt->width = width;
    rt->height = height;
    rt->pitch = pitch;
    const size_t plane = 4 * (size_t)width * height;
    const size_t packed_bytes = ((size_t)pitch * height + 255) & ~(size_t)255;
    hipError_t e = rt->storage.reserve(packed_bytes + 3 * plane);
    if (e != hipSuccess) {
        delete rt;
        return hip_fail(ctx, e, "render target allocation");
    }
    char* base = rt->storage.as<char>();
    rt->packed = reinterpret_cast<uint32_t*>(base);
    rt->tri = reinterpret_cast<uint32_t*>(base + packed_bytes);
    rt->t = reinterpret_cast<float*>(base + packed_bytes + plane);
    rt->nz = reinterpret_cast<float*>(base + packed_bytes + 2 * plane);
    ctx->rts.push_back(rt);
    *out = rt;
    return BM_ERROR_ALL_FINE;
}

int32_t bm_rt_create_external(bm_context* ctx, uint32_t width, uint32_t height, uint32_t pitch, void* packed,
                              void* tri_id, void* t, void* nz, bm_rt** out) {
    if (!ctx || !out || width == 0 || height == 0 || !packed || !tri_id || !t) return BM_ERROR_INVALID_PARAMETER;
    if (width >= (1u << 30) || (uint64_t)width * height >= (1ull << 32)) return BM_ERROR_INVALID_PARAMETER;
    if (pitch == 0) pitch = width * 4;
    if (pitch < width * 4 || (pitch % 4) != 0) return BM_ERROR_INVALID_PARAMETER;
    bm_rt* rt = new (std::nothrow) bm_rt();
    if (!rt) return BM_ERROR_GPU_ALLOC_FAIL;
    rt->ctx = ctx;
    rt->width = width;
    rt->height = height;
    rt->pitch = pitch;
    rt->external = true;
    rt->packed = reinterpret_cast<uint32_t*>(packed);
    rt->tri = reinterpret_cast<uint32_t*>(tri_id);
    rt->t = reinterpret_cast<float*>(t);
    rt->nz = reinterpret_cast<float*>(nz);
    ctx->rts.push_back(rt);
    *out = rt;
    return BM_ERROR_ALL_FINE;
}

uint32_t bm_rt_width(const bm_rt* rt) { return rt ? rt->width : 0; }
uint32_t bm_rt_height(const bm_rt* rt) { return rt ? rt->height : 0; }
uint32_t bm_rt_pitch(const bm_rt* rt) { return rt ? rt->pitch : 0; }
void* bm_rt_buffer(const bm_rt* rt) { return rt ? rt->packed : nullptr; }
void* bm_rt_tri_id(const bm_rt* rt) { return rt ? rt->tri : nullptr; }
void* bm_rt_t(const bm_rt* rt) { return rt ? rt->t : nullptr; }
void* bm_rt_nz(const bm_rt* rt) { return rt ? rt->nz : nullptr; }
void* bm_rt_shadow(const bm_rt* rt) { return rt ? rt->shadow.p : nullptr; }

int32_t bm_rt_read_shadow(bm_rt* rt, uint8_t* out) {
    if (!rt || !out) return BM_ERROR_INVALID_PARAMETER;
    bm_context* ctx = rt->ctx;
    if (!rt->shadow.p) return fail(ctx, BM_ERROR_INVALID_PARAMETER, "no shadow plane: trace with a light first");
    BM_HIP(ctx, hipSetDevice(ctx->device));
    BM_HIP(ctx, hipMemcpyAsync(out, rt->shadow.p, (size_t)rt->width * rt->height, hipMemcpyDeviceToHost, rt_stream(rt)));
    BM_HIP(ctx, hipStreamSynchronize(rt_stream(rt)));
    return BM_ERROR_ALL_FINE;
}

int32_t bm_rt_lock(bm_rt* rt) {
    if (!rt) return BM_ERROR_INVALID_PARAMETER;
    if (rt->locked) return BM_ERROR_UNLOCK_FIRST;
    rt->locked = true;
    return BM_ERROR_ALL_FINE;
}

int32_t bm_rt_unlock(bm_rt* rt) {
    if (!rt) return BM_ERROR_INVALID_PARAMETER;
    if (!rt->locked) return BM_ERROR_LOCK_FIRST;
    rt->locked = false;
    return BM_ERROR_ALL_FINE;
}

int32_t bm_rt_clear(bm_rt* rt, uint32_t value) {
    if (!rt) return BM_ERROR_INVALID_PARAMETER;
    bm_context* ctx = rt->ctx;
    BM_HIP(ctx, hipSetDevice(ctx->device));
    BM_HIP(ctx, bm::launch_clear(rt->packed, rt->pitch / 4, rt->width, rt->height, value, rt_stream(rt)));
    return BM_ERROR_ALL_FINE;
}

int32_t bm_rt_read(bm_rt* rt, uint32_t* packed, uint32_t* tri_id, float* t, float* rgb) {
    if (!rt) return BM_ERROR_INVALID_PARAMETER;
    bm_context* ctx = rt->ctx;
    BM_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t st = rt_stream(rt);
    const size_t plane = 4 * (size_t)rt->width * rt->height;
    if (packed)
        BM_HIP(ctx, hipMemcpy2DAsync(packed, 4 * (size_t)rt->width, rt->packed, rt->pitch, 4 * (size_t)rt->width,
                                     rt->height, hipMemcpyDeviceToHost, st));
    if (tri_id) BM_HIP(ctx, hipMemcpyAsync(tri_id, rt->tri, plane, hipMemcpyDeviceToHost, st));
    if (t) BM_HIP(ctx, hipMemcpyAsync(t, rt->t, plane, hipMemcpyDeviceToHost, st));
    std::vector<float> nz;
    std::vector<uint32_t> tri;
    if (rgb) {
        if (!rt->nz) return fail(ctx, BM_ERROR_INVALID_PARAMETER, "rgb readback needs the nz plane");
        nz.resize((size_t)rt->width * rt->height);
        tri.resize(nz.size());
        BM_HIP(ctx, hipMemcpyAsync(nz.data(), rt->nz, plane, hipMemcpyDeviceToHost, st));
        BM_HIP(ctx, hipMemcpyAsync(tri.data(), rt->tri, plane, hipMemcpyDeviceToHost, st));
    }
    BM_HIP(ctx, hipStreamSynchronize(st));
    if (rgb) {
        for (size_t i = 0; i < nz.size(); ++i) {
            const bool hit = tri[i] != BM_NO_TRIANGLE;
            rgb[3 * i + 0] = hit ? nz[i] : 0.f;
            rgb[3 * i + 1] = hit ? 0.f : 1.f;
            rgb[3 * i + 2] = 0.f;
        }
    }
    return BM_ERROR_ALL_FINE;
}

int32_t bm_rt_set_stream(bm_rt* rt, void* stream) {
    if (!rt) return BM_ERROR_INVALID_PARAMETER;
    bm_context* ctx = rt->ctx;
    hipStream_t ns = reinterpret_cast<hipStream_t>(stream);
    if (ns == ctx->stream) ns = nullptr;
    if (ns == rt->stream) return BM_ERROR_ALL_FINE;
    mg_release(rt);  // multi-device band buffers are remade on the new stream by the next trace
    BM_HIP(ctx, hipSetDevice(ctx->device));
    BM_HIP(ctx, hipStreamSynchronize(rt_stream(rt)));  // the old stream's work on this target is done
    if (!ctx->ready) BM_HIP(ctx, hipEventCreateWithFlags(&ctx->ready, hipEventDisableTiming));
    if (!rt->done) BM_HIP(ctx, hipEventCreateWithFlags(&rt->done, hipEventDisableTiming));
    if (rt->stream && !ns) ctx->rt_streams.erase(std::find(ctx->rt_streams.begin(), ctx->rt_streams.end(), rt));
    if (!rt->stream && ns) ctx->rt_streams.push_back(rt);
    rt->stream = ns;
    rt->epoch = 0;  // the first trace on the new stream waits for the context stream
    if (ns) BM_HIP(ctx, hipEventRecord(rt->done, ns));
    return BM_ERROR_ALL_FINE;
}

void* bm_rt_stream(const bm_rt* rt) { return rt ? reinterpret_cast<void*>(rt_stream(rt)) : nullptr; }

int32_t bm_rt_trace_kind(const bm_rt* rt) { return rt ? rt->last_kind : -1; }

int32_t bm_rt_save_ppm(bm_rt* rt, const char* path) {
    if (!rt || !path) return BM_ERROR_INVALID_PARAMETER;
    std::vector<uint32_t> px((size_t)rt->width * rt->height);
    const int32_t rc = bm_rt_read(rt, px.data(), nullptr, nullptr, nullptr);
    if (rc != BM_ERROR_ALL_FINE) return rc;
    // binary P6, rows top to bottom as stored; packed 0x00RRGGBB -> R, G, B bytes
    std::vector<unsigned char> rgb(3 * px.size());
    for (size_t i = 0; i < px.size(); ++i) {
        rgb[3 * i + 0] = (unsigned char)(px[i] >> 16);
        rgb[3 * i + 1] = (unsigned char)(px[i] >> 8);
        rgb[3 * i + 2] = (unsigned char)px[i];
    }
    FILE* f = std::fopen(path, "wb");
    if (!f) return fail(rt->ctx, BM_ERROR_INVALID_PARAMETER, "save_ppm: cannot open the output file");
    const bool ok = std::fprintf(f, "P6\n%u %u\n255\n", rt->width, rt->height) > 0 &&
                    std::fwrite(rgb.data(), 1, rgb.size(), f) == rgb.size();
    if (std::fclose(f) != 0 || !ok) return fail(rt->ctx, BM_ERROR_INVALID_PARAMETER, "save_ppm: write failed");
    return BM_ERROR_ALL_FINE;
}

int32_t bm_debug_primitives(bm_context* ctx, uint32_t n, const float* in, float* out) {
    if (!ctx || (n && (!in || !out))) return BM_ERROR_INVALID_PARAMETER;
    if (n == 0) return BM_ERROR_ALL_FINE;
    BM_HIP(ctx, hipSetDevice(ctx->device));
    DevBuf din, dout;  // scratch of this call only
    const size_t bin = (size_t)n * 36 * sizeof(float), bout = (size_t)n * 12 * sizeof(float);
    hipError_t e = din.reserve(bin);
    if (e == hipSuccess) e = dout.reserve(bout);
    if (e == hipSuccess) e = hipMemcpyAsync(din.p, in, bin, hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess) e = bm::launch_pin_ops(n, din.as<const float>(), dout.as<float>(), ctx->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(out, dout.p, bout, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    din.release();
    dout.release();
    BM_HIP(ctx, e);
    return BM_ERROR_ALL_FINE;
}

void bm_rt_destroy(bm_rt* rt) {
    if (!rt) return;
    bm_context* ctx = rt->ctx;
    if (ctx) {  // null: detached by bm_context_destroy, nothing left on the device
        mg_release(rt);
        (void)hipSetDevice(ctx->device);
        (void)hipStreamSynchronize(ctx->stream);
        if (rt->stream) {
            (void)hipStreamSynchronize(rt->stream);
            ctx->rt_streams.erase(std::find(ctx->rt_streams.begin(), ctx->rt_streams.end(), rt));
        }
        auto it = std::find(ctx->rts.begin(), ctx->rts.end(), rt);  // band buffers are not listed
        if (it != ctx->rts.end()) ctx->rts.erase(it);
        detach_rt(rt);
    }
    delete rt;
}

}  // extern "C"
