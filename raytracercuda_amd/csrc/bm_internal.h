// bm_internal.h — launch interface between the C-ABI layer (bm_api.cpp) and the kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/beam_c.h"
#include "bm_common.h"

// A/B builds (tools/build_ab.py ... BM_TRACE_AB=1) add the trace variants measured slower than the
// product kernels (bm_trace_ab.hip) and BVH8; the in-tree library is built without them.
#ifndef BM_TRACE_AB
#define BM_TRACE_AB 0
#endif

namespace bm {

// A context's tuning parameters (bm_context_set_param, BM_PARAM_* in beam_c.h): -1 = the library
// default. Launch code reads them from here; nothing is read from the environment.
struct Tuning {
    int64_t v[BM_PARAM_COUNT];
    Tuning() {
        for (int64_t& x : v) x = -1;
    }
    int64_t get(int key, int64_t dflt) const { return v[key] >= 0 ? v[key] : dflt; }
};

// Device buffers of one acceleration-structure build (all owned by the scene, grow-only).
struct BuildBuffers {
    uint32_t n = 0;          // triangles
    uint32_t num_meshes = 0;
    uint32_t leaf_size = 4;
    uint32_t width = 4;           // BVH4 (128-B records), BVH2 (64-B) or BVH8 (256-B, from the BVH2 records)
    const MeshDesc* meshes = nullptr;
    float4* tri_orig = nullptr;   // 3n, original order (written only when need_orig: orig_records, n == 1)
    bool orig_records = false;    // the caller needs tri_orig after the build (a multi-device root's reshade)
    bool* orig_written = nullptr; // out: launch_build / launch_refit wrote tri_orig
    float* nrm = nullptr;         // 9n, original order (corner normals)
    float* aabb = nullptr;        // 6n, original order (written only when need_aabb: n == 1, non-mesh-direct)
    float* cen = nullptr;         // 3n, original order: AABB centres (the Morton keys' input)
    uint32_t* bounds = nullptr;   // build metadata block (build_meta_words(n), zero-filled per build):
                                  // BOUNDS_SLOTS bounds, gather tickets, the radix-sort counters and
                                  // histograms, then per-block partial bounds (bm_build.hip)
    uint32_t* keys = nullptr;     // n  (sorted on return)
    uint32_t* vals = nullptr;     // n  (sorted position -> global id on return)
    uint32_t* keys2 = nullptr;    // n  scratch
    uint32_t* vals2 = nullptr;    // n  scratch
    uint32_t* lch = nullptr;      // n-1
    uint32_t* rch = nullptr;      // n-1
    uint32_t* first = nullptr;    // n-1
    uint32_t* last = nullptr;     // n-1
    uint32_t* parent_leaf = nullptr;  // n
    uint32_t* parent_int = nullptr;   // n-1
    float* ibox = nullptr;            // 6(n-1): boxes of nodes whose range lies in one refit chunk
    float* pre = nullptr;             // 6n: in-chunk prefix unions of sorted leaf boxes
    float* suf = nullptr;             // 6n: in-chunk suffix unions
    float* table = nullptr;           // 6 * chunk_table_floats(n) / 6: sparse table of chunk unions
    uint32_t* records = nullptr;      // (width 8: 64, 4: 32, 2: 16) * max(n-1, 1)
    uint32_t* records2 = nullptr;     // width 8 only: the BVH2 records it is collapsed from (16 * max(n-1, 1))
    float4* tris = nullptr;           // 3n, sorted order
    // the gather's bound replicas in `bounds` are already zero (the previous LBVH build or refit of
    // this buffer cleared them after their last reader): launch_build / launch_refit skip the memset
    bool replicas_clean = false;
    const Tuning* tune = nullptr;  // the context's parameters (BM_PARAM_MSD_*, NRM_DEFER, BUCKET_LDS_CAP)
};

size_t build_meta_words(uint32_t n);
// largest top-digit-first sort: the device-side LSD fallback's last pass runs in RADIX (1,024) bucket
// workgroups of one tile each, i.e. at most 1,024 top-digit tiles (2^22 keys take 512)
constexpr uint32_t MSD_MAX_N_CAP = 1u << 22;
bool msd_sort(uint32_t n, const Tuning& t);  // launch_build sorts the top digit first, then each bucket
uint32_t build_sort_skew_word();             // meta word: nonzero when that sort fell back to LSD passes
size_t chunk_table_floats(uint32_t n);
uint32_t num_records(uint32_t n);
hipError_t launch_build(const BuildBuffers& b, hipStream_t s);
// Refit: new triangle data and boxes over the topology (vals, tree arrays) of the last launch_build
// with the same buffers and triangle count.
hipError_t launch_refit(const BuildBuffers& b, hipStream_t s);

// Triangle records (original order), corner normals and AABBs only (reference modes: no scene bounds);
// zeroes b.bounds words 0 and 1 (the reference-mode split descent keeps its queue count and overflow
// flag there, so the count pass needs no fill launch).
hipError_t launch_gather(const BuildBuffers& b, hipStream_t s);
// The original-order triangle records only (b.meshes, b.num_meshes, b.n, b.tri_orig): for a reshade
// after a build that did not write them (need_orig false at build time).
hipError_t launch_orig_records(const BuildBuffers& b, hipStream_t s);
#ifdef BM_BUILD_DIAG
hipError_t build_diag(unsigned long long* out);     // diagnostic builds: per-wave slots, LBVH build rows (bm_build.hip)
hipError_t kd_build_diag(unsigned long long* out);  // the same, kd build rows (bm_kd.hip)
#endif

// Readback of na words at a and nb at b (na + nb < POST_SEQ_WORD) into pinned coherent host memory
// `host` (device view), then `seq` released into host[POST_SEQ_WORD] (bm_api.cpp readback spins on it).
constexpr uint32_t POST_SEQ_WORD = 63;
hipError_t launch_post(const uint32_t* a, uint32_t na, const uint32_t* b, uint32_t nb, uint32_t* host, uint32_t seq,
                       hipStream_t s);

// Generic stable sort of (key, value) u32 pairs on the low key_bits bits (10-bit one-sweep passes).
// smeta: sort_meta_words(n, key_bits) words of scratch. *in_scratch: the result is in keys2/vals2.
// topmap (31-bit keys only): a 2,048-bit map of the values of bits 20-30 present (at most 1,024 set):
// three passes, the last on the rank of those bits (bm_build.hip build_top_rank) — the same order.
size_t sort_meta_words(uint32_t n, int key_bits);
constexpr uint32_t KD_TOPMAP_WORDS = 64;  // 2,048 bits
hipError_t launch_sort_pairs(uint32_t* keys, uint32_t* vals, uint32_t* keys2, uint32_t* vals2, uint32_t n,
                             int key_bits, uint32_t* smeta, hipStream_t s, bool* in_scratch, bool meta_zeroed = false,
                             const uint32_t* topmap = nullptr);
// Karras radix tree over n sorted keys (equal keys: position tiebreak), as in the BVH build.
hipError_t launch_radix_tree(const uint32_t* keys, uint32_t n, uint32_t* lch, uint32_t* rch, uint32_t* first,
                             uint32_t* last, uint32_t* parent_leaf, uint32_t* parent_int, hipStream_t s,
                             const uint32_t* n_dev = nullptr);

// Trace kernel variants (LDS stack depth / overflow policy / grid shape); the C ABI picks one per
// context (BM_TRACE_VARIANT overrides it for A/B measurements).
enum TraceVariant {
    TRACE_TILES_SCRATCH16 = 0,   // 16x16 tile per workgroup, LDS stack 16, scratch overflow
    TRACE_TILES_NOOVF16 = 1,     // experiment only: no overflow (drops beyond 16 entries)
    TRACE_PERSIST_GLOBAL16 = 2,  // persistent waves over 8x8 tiles, LDS 16, global overflow
    TRACE_PERSIST_GLOBAL8 = 3,
    TRACE_PERSIST_GLOBAL12 = 4,
    TRACE_PERSIST_DIAG12 = 5,    // diagnostic: PRIO12 + per-wave timestamps (bm_camera_trace_profile only)
    TRACE_PERSIST_PRIO12 = 6,    // persistent LDS 12 + s_setprio boost of long-running waves
    TRACE_PERSIST_PRIO8 = 7,     // persistent LDS 8 + the same boost
    TRACE_PERSIST_DYN12 = 8,     // persistent LDS 12 + boost, tiles taken dynamically (atomic ticket)
    TRACE_PERSIST_DYN16 = 9,
    TRACE_QUAD = 10,             // persistent, four lanes per ray over the BVH4 (4x4 pixel tile per wave)
    TRACE_QUAD_FETCH = 11,       // ray quads + in-wave ray refill (idle quads take the wave's next rays)
    TRACE_COMPACT = 12,          // lane-per-ray setup + root cull and ray queue, then quads over the survivors
    TRACE_PAIR = 13,             // persistent, two lanes per ray over the BVH4 (8x4 pixel tile per wave)
    TRACE_PACKET = 14,           // wave packets: one 8x8 tile per wave, wave-uniform stack, scalar record loads
    TRACE_NUM_VARIANTS
};
// Traversal stack bound: a Karras tree over 30-bit keys + 32-bit position tiebreak is < 64 levels
// deep; BVH2 pushes at most one entry per level, BVH4 (half the levels) at most three.
constexpr int MAX_STACK = 96;
constexpr int MAX_STACK8 = 160;  // BVH8: up to 7 pushes per node step

struct TraceParams {
    const uint4* nodes;          // records as 4 x uint4 (BVH2) or 8 x uint4 (BVH4)
    const float4* tris;          // sorted triangle records
    const float* nrm;            // 9 per original triangle
    const float* rx;             // camera column table (W)
    const float* ry;             // camera row table (H)
    float z2, zoom;
    float eye[3];
    float orient[9];             // column-major glm mat3
    uint32_t width, height;      // full frame
    uint32_t band_h, band_step, band_first;
    uint32_t local_rows;         // rows present in the render target
    uint32_t pitch_u32;          // packed-plane row stride (u32 elements)
    uint32_t num_tris;           // 0 -> every pixel misses
    uint32_t* packed;
    uint32_t* tri_id;
    float* t;
    float* nz;
    unsigned long long* counters;  // [3], counting build only
    uint32_t* ovf_ref;             // global stack overflow [MAX_STACK - lds][ovf_stride]
    float* ovf_t;
    uint32_t ovf_stride;           // = persistent_blocks * 256
    uint32_t persistent_blocks;    // upper bound of a persistent grid (each launch: min with residency)
    uint32_t scramble;             // persistent grid: scrambled tile order
    uint32_t prio_after;           // priority-boost variants: traversal steps before s_setprio
    uint32_t prio_level;
    uint32_t refill_min;           // quad-fetch variant: idle quads (of 16) that trigger a refill
    uint32_t sched;                // quad variant: 0 static tile order, 1 block-dynamic (LDS ticket),
                                   // 2 block-dynamic, longest first by the last trace's tile times
    uint32_t* tile_cost;           // sched 2: per quad-kernel tile, 10-ns ticks of its last trace (render target)
    int variant;
    uint32_t bvh_width;            // 2 or 4 (the scene's record layout)
    unsigned long long* tile_ctr;  // dynamic variants: monotonic ticket counter of the context
    unsigned long long tile_base;  // its value when this launch starts (tickets = tiles + waves)
    unsigned long long* diag;      // [4 per wave of the persistent grid], diagnostic build only
    // shadow rays (null shadow: primary rays only). Fused: the primary kernel traces each hit's
    // shadow ray itself. Queue (shadow_queue): the primary kernel zeroes the shadow plane and appends
    // every hit pixel (local index lr*width + x) to queue; k_shadow_persistent drains it.
    uint8_t* shadow;
    bool shadow_queue;
    uint32_t* queue;
    uint32_t* queue_count;
    float light[3];
    unsigned long long* shadow_counters;  // [3], counting build only
    // compacted variant (TRACE_COMPACT): rays that enter the root, region r at rayq + r * rayq_region
    // (x | local row << 16), rayq_count[r] of them; a region = rayq_tpr consecutive 8x8 tiles
    uint32_t* rayq;
    uint32_t* rayq_count;
    uint32_t rayq_region, rayq_tpr, rayq_regions;
    uint32_t fast_cull;  // orient is near-orthonormal: k_cull may use approximate ray setup
};

bool trace_variant_persistent(int variant);
// The product kernels (TRACE_QUAD, TRACE_COMPACT, the single-lane PRIO12 and its DIAG12 build); the
// other variants and BVH8 exist only in A/B builds (-DBM_TRACE_AB=1, bm_trace_ab.hip).
bool trace_variant_product(int variant);
bool trace_variant_built(int variant);  // compiled into this library
#if BM_TRACE_AB
hipError_t launch_trace_ab(const TraceParams& p, bool count, int shadow_mode, hipStream_t s, uint32_t* grid);
#endif
// Pixel tiles of the quad kernel for a frame (one wave each): sizes the cost-ordered schedule's table.
uint32_t quad_tiles(uint32_t width, uint32_t local_rows);
// Ray-queue geometry of TRACE_COMPACT for a frame (false: the frame does not fit its 16-bit pixel
// coordinates; the quad kernel traces it instead).
bool trace_compact_layout(uint32_t width, uint32_t local_rows, uint32_t min_tpr, uint32_t* regions,
                          uint32_t* tiles_per_region);
uint32_t trace_variant_lds(int variant);
uint32_t trace_persistent_blocks(int variant, int device);

// *grid receives the persistent grid launched (0 for the tile kernels): a dynamic variant consumes
// tiles + 4 * grid tickets.
hipError_t launch_trace(const TraceParams& p, bool count, hipStream_t s, uint32_t* grid);
// Shadow pass over the queue the preceding launch_trace (with p.shadow set) filled.
hipError_t launch_shadow(const TraceParams& p, bool count, hipStream_t s);
// ---- reference mode (bm_kd.hip): the reference's kd-tree and march ---------------------------------
struct KdBuild {
    const MeshDesc* meshes;
    uint32_t num_meshes, n;
    float wmin, wmax;
    int leaf_depth;
    uint32_t* counts;   // n: leaves reached per triangle
    uint32_t* offsets;  // n: exclusive scan of counts
    uint32_t* keys;     // leaf path keys of the (key, triangle) pairs
    uint32_t* vals;
    uint32_t* cache;    // KD_LEAF_CACHE x n: the first leaves the count pass reached (slot i of g at i * n + g)
    // split descent (k_kd_top + k_kd_sub): split = 0 or >= leaf_depth walks each triangle in one lane
    int split = 0;
    uint2* queue = nullptr;      // queue_cap (triangle, path) items: the nodes reached at depth `split`
    uint32_t queue_cap = 0;
    uint32_t* qcount = nullptr;  // 2 words: queue length, overflow flag (a subtree walked on, not queued)
    // count pass: the 2,048-bit map of the queued nodes' top 11 path bits (KD_TOPMAP_WORDS words, zeroed)
    // and the number of bits set (one word, zeroed) — the pair sort's ranked top digit (launch_sort_pairs)
    uint32_t* topmap = nullptr;
    uint32_t* topcount = nullptr;
    bool reuse_queue = false;    // emit: the count pass's queue is complete (flag read back 0)
    uint32_t* fill = nullptr;    // n: emit cursors
    uint32_t lq_cap = 0;         // LDS queue items per workgroup (0 or above the kernel's array: the array size)
    bool qcount_zeroed = false;  // qcount/overflow words already zero (launch_gather): the count pass skips its fill
    // emit pass: k_kd_sub also zero-fills these words (the pair sort's metadata: no fill launch before it);
    // *zeroed reports whether it ran
    uint32_t* zero_ptr = nullptr;
    uint32_t zero_words = 0;
    bool* zeroed = nullptr;
    const Tuning* tune = nullptr;  // BM_PARAM_KD_GRID / KD_PAIR / KD_TB
};
// Depth at which the reference-mode build hands subtrees to other lanes (BM_PARAM_KD_SPLIT overrides; 0 = off)
int kd_split_depth(int leaf_depth, const Tuning& t);
#ifndef BM_KD_LEAF_CACHE
#define BM_KD_LEAF_CACHE 8
#endif
constexpr uint32_t KD_LEAF_CACHE = BM_KD_LEAF_CACHE;  // a triangle reaching at most this many leaves is not descended twice
struct KdMarch {
    const uint32_t *leaf_key, *leaf_start, *leaf_count, *faces, *lch, *rch, *first, *last;
    uint32_t num_leaves;
    int leaf_depth;
    float wmin, wmax;
    const uint4* nodes;   // march records (launch_kd_records): 2 x uint4 per internal node (num_leaves - 1)
    const uint4* leaves;  // 2 x uint4 per leaf
    const uint32_t* node_key;  // key of each internal node's first leaf
    const float4* ftris;  // 3 per sorted (leaf, face) pair: the face's triangle record (launch_kd_leaves)
    const uint32_t* ubox = nullptr;  // union of the leaf cells, 6 bound-slot images (launch_kd_records); null: no cull
    int march_variant = 3;  // 3: child-box steps (cnodes); 2: wave-cooperative leaves; 1 / 0: lane-per-ray leaves
    const uint32_t* num_leaves_dev = nullptr;  // build: the leaf count on the device (num_leaves bounds the grid)
    const uint4* cnodes = nullptr;  // child-box records: 4 x uint4 per internal node (launch_kd_records); null: none
    bool no_grid = false;  // BM_PARAM_KD_GRID 0: node boxes by the halving recurrence, never the closed form
};
// Build the march's node and leaf records from the Karras arrays of a reference-mode build.
// cnodes (optional): the child-box records the product march steps with (4 x uint4 per internal node).
// ubox (optional): the union of the leaf cells' boxes into ubox[6] as bound-slot images (bkey_lo of
// the minima, bkey of the maxima; ubox zero-filled by launch_kd_leaves first).
// The leaves' pair counts too (into k.leaf_count, from k.leaf_start and the pair count m). post_host
// (optional): launch_post's readback of *k.num_leaves_dev with sequence post_seq, done by the kernel itself.
hipError_t launch_kd_records(const KdMarch& k, uint32_t m, uint4* nodes, uint4* leaves, uint32_t* node_key,
                             hipStream_t s, uint4* cnodes = nullptr, uint32_t* ubox = nullptr,
                             uint32_t* post_host = nullptr, uint32_t post_seq = 0);
int kd_leaf_depth(float wmin, float wmax);
uint32_t scan_sums_words(uint32_t n);
// Exclusive scan of n u32 in one launch (decoupled look-back). sums: scan_sums_words(n) words of
// scratch, zero-filled once when allocated, then reused with a new epoch (1..2^20-1, != the last call's)
// per call; in/out 16-byte aligned. *grand_total = the u32 total and, with total64, *total64 = the exact
// 64-bit total (the pair-count guard of the reference-mode builds). run_keys (in unused): the scan of
// the run-start flags of n sorted keys (1 where key i differs from key i - 1), computed on the fly.
hipError_t launch_exclusive_scan(const uint32_t* in, uint32_t* out, uint32_t n, uint32_t* sums,
                                 uint32_t* grand_total, hipStream_t s, unsigned long long* total64, uint32_t epoch,
                                 const uint32_t* run_keys = nullptr);
hipError_t launch_kd_count(const KdBuild& k, hipStream_t s);
constexpr uint64_t MAX_PAIRS = 0x7FFFFFFFull;  // (key, triangle) pairs a reference-mode build accepts
hipError_t launch_kd_emit(const KdBuild& k, hipStream_t s);
// leaf_count null: no count pass here (launch_kd_records computes the counts); flags null: run starts
// from the keys; ubox: zero-filled (the union words of launch_kd_records); ftris: the march's face
// records gathered in pair order too (faces[i]'s tri_orig record)
hipError_t launch_kd_leaves(const uint32_t* keys, uint32_t m, const uint32_t* flags, const uint32_t* leaf_of,
                            uint32_t* leaf_key, uint32_t* leaf_start, uint32_t* leaf_count, uint32_t nl,
                            hipStream_t s, const uint32_t* nl_dev = nullptr, uint32_t* ubox = nullptr,
                            const uint32_t* faces = nullptr, const float4* tri_orig = nullptr, float4* ftris = nullptr);
// Leaf-side kernels given the device leaf count (nl_dev) treat their host `nl` as the buffers' capacity:
// a device count above it (a build past BM_PARAM_KD_MAX_LEAVES) makes them write nothing, and the host
// reports the error when it reads the count (kd_leaves_ready).
constexpr uint32_t KD_MAX_LEAVES = 1u << 25;  // k_kd_records packs child indices below 2^25 with the split depth
// count: node records visited, face tests, hits into p.counters; p.diag: per-wave timeline (8x8 waves)
hipError_t launch_kd_march(const TraceParams& p, const KdMarch& k, bool count, hipStream_t s);

// ---- reference mode, hashed grid (bm_kd.hip): the reference's alternative accelerator (Hash.cu) ----
constexpr uint32_t HG_NUM_BUCKETS = 65536;     // MAX_HASH_ELEMENTS, BuildTree.cuh:21
constexpr uint32_t HG_MAX_CELLS = 1u << 20;    // cells per triangle AABB a build accepts
struct HashBuild {
    const MeshDesc* meshes;
    uint32_t num_meshes, n;
    uint32_t* counts;     // n: accepted cells per triangle
    uint32_t* offsets;    // n: exclusive scan of counts
    uint32_t* keys;       // bucket of each (cell, triangle) pair
    uint32_t* vals;       // its triangle id
    uint32_t* too_large;  // set when some triangle's AABB spans more than HG_MAX_CELLS cells
};
hipError_t launch_hash_count(const HashBuild& h, hipStream_t s);
hipError_t launch_hash_emit(const HashBuild& h, hipStream_t s);
hipError_t launch_hash_ranges(const uint32_t* keys, uint32_t m, uint32_t* bstart, uint32_t* bend, hipStream_t s);
hipError_t launch_hash_march(const TraceParams& p, const uint32_t* bstart, const uint32_t* bend,
                             const uint32_t* faces, hipStream_t s);
hipError_t launch_clear(uint32_t* buf, uint32_t pitch_u32, uint32_t width, uint32_t height, uint32_t value,
                        hipStream_t s);

// ---- multi-GPU exchange (bm_gather.hip) -------------------------------------------------------------
constexpr uint32_t PLANE_PACKED = 1, PLANE_TRI_ID = 2, PLANE_T = 4, PLANE_NZ = 8, PLANE_SHADOW = 16;
constexpr uint32_t MAX_BAND_SOURCES = 8;
struct BandPlanes {  // one device's band buffer: compact rows, row stride = frame width
    const uint32_t* packed;
    const uint32_t* tri;
    const float* t;
    const float* nz;        // may be null
    const uint8_t* shadow;  // may be null
    uint32_t band_first;    // the device's index: it holds bands b with b % band_step == band_first
    uint32_t rows;          // compact rows present
};
struct FramePlanes {  // the root render target
    uint32_t* packed;
    uint32_t pitch_u32;
    uint32_t* tri;
    float* t;
    float* nz;
    uint8_t* shadow;
    uint32_t width, height;
};
// Copy band rows of nsrc sources into their frame rows (the planes in `planes`). The launch runs on
// `s`'s device; source and destination may be on other devices when peer access is enabled.
hipError_t launch_band_scatter(const BandPlanes* src, uint32_t nsrc, const FramePlanes& dst, uint32_t band_h,
                               uint32_t band_step, uint32_t planes, hipStream_t s);

// Multi-GPU exchange by triangle id: rebuild packed, t and |n.z| of a full frame (p.width x p.height,
// p.tri_id filled) on the root from the ids, the camera tables and the scene's original-order
// triangle records (bm_trace.hip).
hipError_t launch_reshade(const TraceParams& p, const float4* tri_orig, hipStream_t s);
// Self-test of the trace's scalar primitives on n records (bm_debug_primitives; layouts: orc_pin_ops).
hipError_t launch_pin_ops(uint32_t n, const float* in, float* out, hipStream_t s);

// ---- RCCL, loaded on first use (bm_rccl.cpp): librccl.so.1, the same library torch uses ---------------
struct Rccl;
// nullptr (and *why set) when librccl.so.1 or one of its entry points cannot be loaded.
const Rccl* rccl_load(const char** why);
int rccl_unique_id(const Rccl* r, uint8_t* id128);
int rccl_init_rank(const Rccl* r, void** comm, int size, const uint8_t* id128, int rank);
int rccl_init_all(const Rccl* r, void** comms, int n, const int* devices);
void rccl_destroy(const Rccl* r, void* comm);
int rccl_group_start(const Rccl* r);
int rccl_group_end(const Rccl* r);
// bytes as ncclUint8 (0 = ncclSuccess)
int rccl_send(const Rccl* r, const void* buf, size_t bytes, int peer, void* comm, hipStream_t s);
int rccl_recv(const Rccl* r, void* buf, size_t bytes, int peer, void* comm, hipStream_t s);
const char* rccl_error_string(const Rccl* r, int code);

}  // namespace bm
