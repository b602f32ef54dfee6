/*
 * beam_c.h — C ABI of the MI355X-native Beam primary-ray path (libbeam_hip.so).
 *
 * Drop-in boundary for the reference's hot path. The reference splits its host API
 * (Raytracer/Beam.h:32-72, C++ classes) from its device entry points (extern "C" declarations at
 * Raytracer/SceneTree.cpp:11-35 and Raytracer/Camera.cpp:16-19), and those pass glm types by value
 * and by reference, so they are not a real C ABI. Everything here is POD: opaque handles, plain
 * pointers, sizes and int32 error codes. include/beam/Beam.h rebuilds the reference's C++
 * interface classes on top of it; INTEGRATION.md shows the ctypes / C++ bindings.
 *
 * Threading and streams: one host thread per context. Every device operation is enqueued on the
 * context's HIP stream (its own, or one supplied in bm_options) and returns without waiting,
 * like the reference's launches on the legacy default stream; bm_sync() waits. Mesh uploads copy
 * from the caller's host memory before returning (the reference's synchronous cudaMemcpy,
 * DeviceBuffer.cpp:44-58). Handles must be destroyed before their context.
 *
 * Errors: the reference's u32 codes (Raytracer/Beam.h:8-16) plus BM_ERROR_DEVICE for any HIP
 * failure (the reference calls exit(1) from CUDA_CALL, CudaComon.cuh:59-68) and
 * BM_ERROR_NOT_BUILT for tracing a scene that has no current build.
 * bm_last_error_string() describes the last failure on a context.
 */
#ifndef BEAM_C_H
#define BEAM_C_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BM_ERROR_ALL_FINE 0
#define BM_ERROR_NO_VERTICES 1
#define BM_ERROR_INVALID_PARAMETER 2
#define BM_ERROR_GPU_ALLOC_FAIL 3
#define BM_ERROR_INVALID_FORMAT 4
#define BM_ERROR_RT_CAM_MISMATCH 5
#define BM_ERROR_UNLOCK_FIRST 6
#define BM_ERROR_LOCK_FIRST 7
#define BM_ERROR_NO_RENDER_TARGET 8
#define BM_ERROR_DEVICE 9
#define BM_ERROR_NOT_BUILT 10

/* Vertex data slots (Raytracer/Beam.h:19-29). */
#define BM_VERTEX_DATA_POSITION 0
#define BM_VERTEX_DATA_NORMAL 1
#define BM_VERTEX_DATA_UV1 2
#define BM_VERTEX_DATA_UV2 3
#define BM_VERTEX_DATA_TANGENT 4
#define BM_VERTEX_DATA_BITANGENT 5
#define BM_VERTEX_DATA_EXTRA1 6
#define BM_VERTEX_DATA_EXTRA2 7
#define BM_VERTEX_DATA_EXTRA3 8
#define BM_VERTEX_DATA_EXTRA4 9
#define BM_VERTEX_DATA_COUNT 10

/* Framebuffer values (Raytracer/BuildTree.cu:486-496; pixel format 0x00RRGGBB, GLinterop.h). */
#define BM_MISS_PACKED 0x0000FF00u
#define BM_NO_TRIANGLE 0xFFFFFFFFu

typedef struct bm_context bm_context;
typedef struct bm_mesh bm_mesh;
typedef struct bm_scene bm_scene;
typedef struct bm_camera bm_camera;
typedef struct bm_rt bm_rt;

#define BM_MAX_DEVICES 8
#define BM_COMM_ID_BYTES 128

typedef struct bm_options {
    int32_t device;      /* HIP device ordinal (the reference picks the last one, Program.cpp:122-124) */
    void* stream;        /* hipStream_t to enqueue on, or NULL for a stream owned by the context */
    uint32_t leaf_size;  /* BVH leaf collapse size, 1..16 (0 = default 4) */
    uint32_t flags;      /* BM_OPT_* bits */
    /* ---- multi-GPU; all zero = one device. The reference has no device control
     * beyond cudaSetDevice(count-1) in its demo (TestProgram/Program.cpp:121-124). ---------------- */
    /* One process, several devices: devices[0..num_devices) (1..8; 0 = `device` alone). Every mesh,
     * scene and camera created on the context is replicated on each device (the build is
     * deterministic, so the replicas are bit-identical); a trace deals the frame's screen bands
     * (band_height rows, band b -> device b % n) to the devices and gathers them into the render
     * target, which lives on devices[0] (the root; `stream` applies to it). A device may be listed
     * more than once (several band streams sharing one GPU: a one-GPU rehearsal of the n-way path). */
    uint32_t num_devices;
    int32_t devices[BM_MAX_DEVICES];
    uint32_t band_height;    /* rows per screen band, 0 = 16 */
    uint32_t gather;         /* BM_GATHER_* transport of the band buffers to the root */
    uint32_t gather_planes;  /* 0: the triangle-id plane (+ shadow bytes) travels and the root rebuilds
                                t, |n.z| and the packed colour from it (4 B/pixel, every plane exact);
                                else a BM_PLANE_* mask of planes moved as traced */
    /* Several processes, one device each (e.g. launched by torchrun): rank comm_rank of comm_size
     * (0 or 1: no communicator), joined by the RCCL unique id rank 0 made with bm_comm_unique_id and
     * handed to the other ranks by the caller. A trace then covers this rank's bands and gathers
     * every rank's bands into rank 0's render target over RCCL (the render targets of other ranks
     * are left unwritten); builds are replicated per rank as above. */
    int32_t comm_rank;
    int32_t comm_size;
    uint8_t comm_id[BM_COMM_ID_BYTES];
} bm_options;

/* Gather transports (bm_options.gather). */
#define BM_GATHER_AUTO 0u  /* PEER for one process, RCCL between processes */
#define BM_GATHER_PEER 1u  /* each device writes its bands into the root's planes over xGMI (peer
                              access; a kernel on the source device, no staging copy) */
#define BM_GATHER_RCCL 2u  /* one RCCL communicator over the devices (ncclCommInitAll): grouped
                              ncclSend/ncclRecv into root staging buffers, then one scatter kernel
                              on the root. A device list that repeats a device (RCCL refuses two
                              ranks on one GPU) gets one single-rank communicator instead (unique id
                              + ncclCommInitRank) and every band travels as a send/recv to itself:
                              the same staging and scatter, rehearsed on one GPU */
/* bm_context_gather's answer for that single-rank rehearsal (never an option value). */
#define BM_GATHER_RCCL_LOOPBACK 3u
/* Planes a multi-device trace gathers (bm_options.gather_planes). */
#define BM_PLANE_PACKED 1u  /* the reference's framebuffer, 0x00RRGGBB */
#define BM_PLANE_TRI_ID 2u
#define BM_PLANE_T 4u
#define BM_PLANE_NZ 8u      /* |n.z| of the shading normal (rgb readback) */
#define BM_PLANE_SHADOW 16u /* u8 shadow plane of shadow traces */

/* Enqueue on the legacy default (null) stream, e.g. torch's default stream, whose handle is 0. */
#define BM_OPT_NULL_STREAM 1u
/* Shadow rays as a separate wavefront pass over a device queue of the hit pixels (compacted with
 * wave64 ballots) instead of fused into the primary kernel; same results, a compaction study. */
#define BM_OPT_SHADOW_QUEUE 2u
/* Build BVH2 (binary, 64-B records) instead of the default BVH4 (128-B records, every other level
 * of the binary tree collapsed). Same frames; fewer, wider node steps with BVH4. */
#define BM_OPT_BVH2 4u
/* Build BVH8 (256-B records, three binary levels per node, collapsed from the BVH2 records) and
 * trace it with ray quads (two children per lane): a third fewer node steps, but each step costs
 * more than it saves — measured 12-16 % slower than the default BVH4. Compiled into
 * A/B builds only (bm_version() ending in "+ab", tools/build_ab.py); the product library rejects the
 * flag with BM_ERROR_INVALID_PARAMETER. Primary and fused shadow rays with the default trace (no
 * shadow queue, no trace variants); excludes BM_OPT_BVH2. */
#define BM_OPT_BVH8 32u
/* Reference mode: scenes build the reference's own sparse kd-tree (world box [-30,30]³, SAT
 * insertion, 31 levels, 256-face leaves; BuildTree.cu:154-362) and traces march it with the
 * first-hit-leaf early-out (BuildTree.cu:367-499), so every pixel equals the reference framebuffer,
 * including the pixels where that early-out returns a farther triangle than the closest hit.
 * Full-frame bm_camera_trace only (no bands, shadows, refit or export; bm_camera_trace_counters
 * returns node records visited, face tests and hits; bm_camera_trace_profile a wave per 8x8 tile).
 * One device only. */
#define BM_OPT_REFERENCE_KD 8u
/* Hashed-grid mode: the reference's alternative accelerator (Raytracer/Hash.cu, compiled there only
 * with TREE_TYPE==HASH): 0.03 cells hashed into 65,536 buckets by Fletcher-16, every
 * SAT-accepted cell of a triangle's AABB (the insert loop's row reset fixed), 256 faces per bucket;
 * the march steps cell by cell from the eye (at most 400) and returns the closest hit of the first
 * bucket with any hit, collisions included. Full-frame bm_camera_trace only; excludes
 * BM_OPT_REFERENCE_KD. A comparison study, not a renderer: see DESIGN.md §7. */
#define BM_OPT_REFERENCE_HASH 16u

/* bm_build_stats.sort_path: how the build sorted its Morton keys. */
#define BM_SORT_LSD 1u      /* three 10-bit LSD one-sweep passes */
#define BM_SORT_MSD 2u      /* the top digit first, then every bucket in one workgroup's LDS */
#define BM_SORT_MSD_SKEW 3u /* the top-digit histogram showed a bucket too large for LDS: the same
                               build sorted with the LSD passes instead (decided on the device) */
/* reference mode (BM_OPT_REFERENCE_KD) reports its (leaf, face) pair sort: BM_SORT_LSD (four 10-bit
 * passes over the 31-bit leaf paths) or BM_SORT_KD_RANKED (three: the last on the rank of the paths'
 * top 11 bits among those present, when at most 1,024 are) — the same order either way */
#define BM_SORT_KD_RANKED 4u
typedef struct bm_build_stats {
    uint32_t num_meshes;
    uint32_t num_tris;
    uint32_t num_records;  /* node record slots (bvh_width 2: 64 B each, 4: 128 B each) */
    uint32_t leaf_size;
    float build_ms;        /* device time gather+bounds+Morton+sort+emit+refit+pack (hipEvents) */
    uint32_t bvh_width;    /* 4 (default), 2 (BM_OPT_BVH2) or 8 (BM_OPT_BVH8, A/B builds only) */
    uint32_t sort_path;    /* the sort this build ran: BM_SORT_* (0 for refits and the hashed grid) */
    uint32_t fused_front;  /* always 0 (round 5: k_front removed; kept for ABI stability) */
} bm_build_stats;

/* ---- context ------------------------------------------------------------------------------ */
int32_t bm_context_create(const bm_options* opts, bm_context** out);
void bm_context_destroy(bm_context* ctx);
int32_t bm_sync(bm_context* ctx);
const char* bm_last_error_string(const bm_context* ctx);
void* bm_context_stream(const bm_context* ctx);       /* the hipStream_t work is enqueued on */
const char* bm_version(void);
/* Devices a context spans (1 for single-device contexts; comm_size for multi-process ones). */
uint32_t bm_context_num_devices(const bm_context* ctx);
/* Multi-process gather: rank 0 makes the RCCL unique id (BM_COMM_ID_BYTES bytes) that every rank
 * passes in bm_options.comm_id. BM_ERROR_DEVICE when RCCL (librccl.so.1) cannot be loaded. */
int32_t bm_comm_unique_id(uint8_t* id);
/* BM_ERROR_ALL_FINE when RCCL (librccl.so.1) resolves in this process, else BM_ERROR_DEVICE: the
 * check every rank makes before any rank enters the collective communicator start. */
int32_t bm_comm_available(void);
/* The transport a multi-device context resolved (BM_GATHER_PEER, BM_GATHER_RCCL or
 * BM_GATHER_RCCL_LOOPBACK); 0 for single-device contexts. */
uint32_t bm_context_gather(const bm_context* ctx);

/* Split start of a multi-process context: create a plain single-device context on every rank
 * first (bm_options without comm_*; band_height and gather_planes are kept for later), let the
 * ranks agree that every one of them has one, then join the RCCL communicator here (the
 * collective ncclCommInitRank). A rank whose device setup fails therefore never leaves the others
 * blocked inside the collective. Needs a context with no devices list, no peers and no render
 * targets yet; size >= 2. Meshes, scenes and cameras made afterwards are this rank's replicas. */
int32_t bm_context_start_comm(bm_context* ctx, int32_t rank, int32_t size, const uint8_t* comm_id);

/* ---- tuning parameters ----------------------------------------------------------------------
 * Measurement and test hooks of the kernels' schedules (the reference's configuration is
 * compile-time only, Types.h:8-13 and BuildTree.cuh:11-21; this library reads nothing from the
 * environment). Per context, set before the work they affect; -1 restores the library default.
 * The defaults are the measured-best settings. BM_ERROR_INVALID_PARAMETER for an
 * unknown key or a value the key does not accept. */
#define BM_PARAM_TRACE_VARIANT 0      /* trace kernel variant (bm_internal.h TraceVariant; A/B builds add more) */
#define BM_PARAM_TRACE_SCHED 1        /* quad tile order: 0 static, 1 screen-order dynamic, 2 cost-ordered */
#define BM_PARAM_TRACE_SCRAMBLE 2     /* lane-per-ray variants: scrambled static tile order */
#define BM_PARAM_TRACE_PRIO_AFTER 3   /* steps before a long-running wave raises its priority */
#define BM_PARAM_TRACE_PRIO_LEVEL 4   /* that priority (0-3) */
#define BM_PARAM_TRACE_REFILL_MIN 5   /* quad-fetch variant: idle quads that trigger a refill */
#define BM_PARAM_CULL_TILES 6         /* compacted trace: 8x8 tiles per culling workgroup region */
#define BM_PARAM_TRACE_AUTO_COMPACT 7 /* 0: never switch sparse in-flight views to cull + compacted quads */
#define BM_PARAM_TRACE_GRID 8         /* cap of the persistent trace grid (workgroups) */
#define BM_PARAM_READBACK_SYNC 9      /* 1: mid-build count readbacks by copy + stream sync (A/B) */
#define BM_PARAM_KD_QUEUE_CAP 10      /* reference-mode build: subtree queue items (small: walk-on paths) */
#define BM_PARAM_KD_LQ_CAP 11         /* reference-mode build: LDS queue items per workgroup */
#define BM_PARAM_KD_SPLIT 12          /* reference-mode build: hand-off depth (0: one lane walks all) */
#define BM_PARAM_KD_GRID 13           /* 0: node boxes by the halving recurrence, never the closed form */
#define BM_PARAM_KD_PAIR 14           /* 0: one lane per walk instead of a lane pair */
#define BM_PARAM_KD_TB 15             /* lanes per workgroup of the reference-mode descent (64 or 256) */
#define BM_PARAM_KD_MARCH 16          /* reference-mode march: 3 wave-cooperative leaves, child-box node steps (default), 2 the same with one box per step, 1/0 lane leaves in 64/256-lane groups */
#define BM_PARAM_MSD_MAX_N 17         /* largest scene sorted top digit first (above: three LSD passes) */
#define BM_PARAM_NRM_DEFER 18         /* 0: corner normals gathered by the gather, not the top-digit pass */
#define BM_PARAM_BUCKET_LDS_CAP 19    /* keys a bucket may hold to sort in LDS (0: every bucket via global) */
#define BM_PARAM_MSD_WIDE_N 20        /* above this many triangles the bucket sort runs 1,024-lane workgroups */
#define BM_PARAM_FRONT_MAX_N 21       /* retired (k_front removed in round 5): only 0 / -1 accepted */
#define BM_PARAM_ORIG_LAZY 22         /* test hook: 1 = builds never write the original-order records, so a
                                         multi-device trace rebuilds them lazily (the path a scene built before
                                         bm_context_start_comm takes) */
#define BM_PARAM_KD_MAX_LEAVES 23     /* reference mode: kd leaves a build accepts (default and cap 2^25; a test
                                         hook below): more leave the tree unbuilt and the first trace or kdStats
                                         reports BM_ERROR_GPU_ALLOC_FAIL */
#define BM_PARAM_TRACE_AUTO_PACKET 24 /* 0: never switch dense coherent views to wave packets (BM_PARAM_TRACE_VARIANT 14) */
#define BM_PARAM_KD_TOP_RANK 25 /* 0: reference-mode pair sort in four plain passes (no ranked top digit; A/B) */
#define BM_PARAM_COUNT 26
int32_t bm_context_set_param(bm_context* ctx, uint32_t key, int64_t value);
/* The value set for key, -1 while the library default is in effect; INT64_MIN for an unknown key. */
int64_t bm_context_get_param(const bm_context* ctx, uint32_t key);

/* ---- mesh: IMesh (Beam.h:47-54, Mesh.cpp:30-54) ------------------------------------------ */
int32_t bm_mesh_create(bm_context* ctx, bm_mesh** out);
/* numComponents <= 4; position must have 3; all slots share one vertex count (Mesh.cpp:32-37). */
int32_t bm_mesh_set_vertex_data(bm_mesh* m, const float* data, uint32_t num_vertices,
                                uint32_t num_components, uint32_t slot);
/* num_indices % 3 == 0 (Mesh.cpp:48). */
int32_t bm_mesh_set_indices(bm_mesh* m, const uint32_t* indices, uint32_t num_indices);
void bm_mesh_destroy(bm_mesh* m);

/* ---- scene: IScene (Beam.h:56-63, Scene.cpp, SceneTree.cpp) ------------------------------ */
int32_t bm_scene_create(bm_context* ctx, bm_scene** out);
/* The scene references (does not own) its meshes; keep them alive while it uses them. */
int32_t bm_scene_add_mesh(bm_scene* s, bm_mesh* m);
int32_t bm_scene_remove_mesh(bm_scene* s, bm_mesh* m);
/* updateGPUScene (SceneTree.cpp:70-91): rebuild the acceleration structure from the current
 * meshes; global triangle id = sum of earlier meshes' triangle counts + local face index.
 * stats may be NULL; when given, the call waits for the build to finish to fill build_ms. */
int32_t bm_scene_build(bm_scene* s, bm_build_stats* stats);
/* Refit-only update for animated meshes: the meshes and triangle counts of the
 * last bm_scene_build, new vertex positions/normals (bm_mesh_set_vertex_data). Keeps the sorted
 * order, radix tree, leaf collapse and node set; recomputes triangle records, boxes and node
 * records (skips Morton codes, sort and emit). Frames are exact as after a rebuild; traversal cost
 * grows as the geometry drifts from the topology. BM_ERROR_INVALID_PARAMETER when the mesh set or
 * a triangle count changed. stats as bm_scene_build (build_ms = the refit's device time). */
int32_t bm_scene_refit(bm_scene* s, bm_build_stats* stats);
/* Reference-mode scenes: out[0] leaves holding faces, out[1] face references stored, out[2] faces
 * dropped by the 256 cap, out[3] largest leaf (before the cap). Synchronous. */
int32_t bm_scene_kd_stats(bm_scene* s, uint64_t out[4]);
/* Hashed-grid scenes: out[0] (cell, face) pairs, out[1] non-empty buckets, out[2] largest bucket,
 * out[3] faces beyond the 256 cap. Synchronous. (Hash.cu:82-89, BuildTree.cuh:21) */
int32_t bm_scene_grid_stats(bm_scene* s, uint64_t out[4]);
/* Hashed-grid scenes: bucket b holds faces[bucket_start[b] .. bucket_end[b]) (65,536 buckets; faces
 * = global triangle ids, out[0] of bm_scene_grid_stats entries). Any pointer may be NULL. */
int32_t bm_scene_grid_export(bm_scene* s, uint32_t* bucket_start, uint32_t* bucket_end, uint32_t* faces);
void bm_scene_destroy(bm_scene* s);

/* ---- camera: ICamera (Beam.h:65-72, Camera.cpp) ----------------------------------------- */
int32_t bm_camera_create(bm_context* ctx, bm_camera** out);
/* setInitialRays (Camera.cpp:43-72): same sequential ray recurrence and validation. */
int32_t bm_camera_set_initial_rays(bm_camera* c, uint32_t width, uint32_t height, float left,
                                   float right, float top, float bottom, float zoom);
/* traceScene (Camera.cpp:85-97 -> SceneTree::march -> bmMarch): one primary ray per pixel,
 * eye[3], orient_colmajor[9] (glm mat3 memory layout). The render target's size must equal the
 * camera's (Scene.cpp:81-97, BM_ERROR_RT_CAM_MISMATCH). On a multi-device context (bm_options
 * devices / comm_*) the frame's bands are traced on every device and gathered into the target;
 * bm_camera_trace_shadow likewise. The band, counter and profile entry points below run on the
 * root device alone. */
int32_t bm_camera_trace(bm_camera* c, const float* eye3, const float* orient3x3, bm_scene* s,
                        bm_rt* rt);
/* Screen-band partition for multi-GPU: trace only global rows in bands b*band_height..+band_height
 * with b % band_step == band_first, writing them compacted into rt (local row r holds global row
 * ((r/band_height)*band_step + band_first)*band_height + r%band_height). rt width must equal the
 * camera width and its height must be >= the compacted row count. band_step=1, band_first=0 is
 * bm_camera_trace. */
int32_t bm_camera_trace_bands(bm_camera* c, const float* eye3, const float* orient3x3, bm_scene* s,
                              bm_rt* rt, uint32_t band_height, uint32_t band_step,
                              uint32_t band_first);
/* Primary trace plus one shadow ray per hit toward a point light (the reference
 * has no shadow rays, so the semantics are this build's): origin = eye + dir * (t * 0.9999f),
 * direction = light3 - origin (unnormalised); the pixel's shadow-plane byte is 1 when any triangle's
 * Möller-Trumbore t_s has 0 < t_s < 1 (any hit), else 0 (also on a primary miss). The primary
 * planes are written exactly as bm_camera_trace writes them; read the shadow plane with
 * bm_rt_read_shadow / bm_rt_shadow. Hit pixels are compacted into a queue on the device (wave64
 * ballots) and the shadow rays run as a second persistent pass over it. */
int32_t bm_camera_trace_shadow(bm_camera* c, const float* eye3, const float* orient3x3, bm_scene* s,
                               bm_rt* rt, const float* light3);
/* bm_camera_trace_bands + the shadow pass over the band's rows. */
int32_t bm_camera_trace_shadow_bands(bm_camera* c, const float* eye3, const float* orient3x3,
                                     bm_scene* s, bm_rt* rt, uint32_t band_height,
                                     uint32_t band_step, uint32_t band_first, const float* light3);
void bm_camera_destroy(bm_camera* c);

/* ---- render target: IRenderTarget (Beam.h:32-45) — offscreen device planes --------------- */
/* Replaces registerGLTBO (RenderTarget.cpp:17-28): device planes owned by the library.
 * pitch (bytes per row of the packed plane) >= width*4, 0 = width*4. */
int32_t bm_rt_create_offscreen(bm_context* ctx, uint32_t width, uint32_t height, uint32_t pitch,
                               bm_rt** out);
/* Wrap caller-owned device memory (e.g. torch tensors): packed (pitch*height bytes), tri_id and t
 * (width*height each) are required, nz (width*height floats, |n.z| of the shading normal) may be
 * NULL. */
int32_t bm_rt_create_external(bm_context* ctx, uint32_t width, uint32_t height, uint32_t pitch,
                              void* packed, void* tri_id, void* t, void* nz, bm_rt** out);
uint32_t bm_rt_width(const bm_rt* rt);
uint32_t bm_rt_height(const bm_rt* rt);
uint32_t bm_rt_pitch(const bm_rt* rt);
/* Device pointers of the planes (IRenderTarget::buffer() is the packed plane). */
void* bm_rt_buffer(const bm_rt* rt);
void* bm_rt_tri_id(const bm_rt* rt);
void* bm_rt_t(const bm_rt* rt);
void* bm_rt_nz(const bm_rt* rt);
/* u8 shadow plane (width*height, row stride width); NULL until the first shadow trace. */
void* bm_rt_shadow(const bm_rt* rt);
/* lock/unlock keep the reference's ordering contract (RenderTarget.cpp:53-83): trace requires a
 * locked target in the C++ layer; in the C ABI the target is passed explicitly. */
int32_t bm_rt_lock(bm_rt* rt);
int32_t bm_rt_unlock(bm_rt* rt);
/* ICamera::clear / bmClear (RTClear.cu:19-48): fill the packed plane (pitch honoured). */
int32_t bm_rt_clear(bm_rt* rt, uint32_t value);
/* Synchronous readback of any subset of planes (NULL = skip). packed is width*height u32 (pitch
 * removed); rgb is width*height*3 floats: (|n.z|,0,0) on a hit, (0,1,0) on a miss. */
int32_t bm_rt_read(bm_rt* rt, uint32_t* packed, uint32_t* tri_id, float* t, float* rgb);
/* Synchronous readback of the shadow plane (width*height bytes). */
int32_t bm_rt_read_shadow(bm_rt* rt, uint8_t* out);
/* Frames in flight. A render target may carry its own HIP stream (NULL or the context stream:
 * the default). Traces into it, and its clear/readback calls, are enqueued there instead of on the
 * context stream, so traces into different targets can run concurrently (the next frame's
 * workgroups fill the CUs the previous frame's tail leaves idle). The library orders them with
 * events: a trace waits for the context stream's work (builds, ray tables) enqueued before it, and
 * a build or setInitialRays waits for the last trace of every such target. bm_sync waits for all
 * of them. Each such target owns its traversal-stack overflow area. The caller keeps the stream
 * alive while the target uses it. Not available with the global-ticket diagnostic variants. */
int32_t bm_rt_set_stream(bm_rt* rt, void* stream);
/* The stream a render target's work runs on (its own, or the context's). */
void* bm_rt_stream(const bm_rt* rt);
/* Which kernels the last trace into this target ran (measurement: names the dominant kernel). A
 * target on its own stream over a sparse view (the scene's box under half the frame) takes the
 * root cull + compacted ray quads; otherwise ray quads (BVH4) or one lane per ray. -1: no trace. */
#define BM_TRACE_KIND_QUADS 0       /* k_trace_quad */
#define BM_TRACE_KIND_CULL_QUADS 1  /* k_cull + k_trace_rays */
#define BM_TRACE_KIND_LANES 2       /* k_trace_persistent / k_trace_tiles (BVH2, shadow queue, variants) */
#define BM_TRACE_KIND_KD_MARCH 3    /* reference mode: k_kd_march_coop */
#define BM_TRACE_KIND_HASH_MARCH 4  /* hashed-grid mode: k_hash_march */
#define BM_TRACE_KIND_PACKETS 5     /* k_trace_packet (BM_PARAM_TRACE_VARIANT 14: wave packets) */
int32_t bm_rt_trace_kind(const bm_rt* rt);
/* Multi-device contexts: the device-time split of the last frame traced into this (root) target,
 * from HIP events on the streams it ran on: out_ms[0] = this process's band trace (its first band
 * source), out_ms[1] = the exchange after it (RCCL send/recv or peer writes, band scatter and
 * reshade; on rank 0 it includes waiting for the slowest rank's bands). Synchronous: waits for
 * that frame. BM_ERROR_NOT_BUILT before the first multi-device trace into rt. */
int32_t bm_rt_last_timing(bm_rt* rt, float out_ms[2]);
/* Host dump of the packed plane as a binary PPM (P6, 8-bit R,G,B from 0x00RRGGBB, rows top to
 * bottom): the frame-loop step after trace that the reference hands to GL (SURVEY 8(f)2,
 * Program.cpp:314-341). Synchronous; BM_ERROR_INVALID_PARAMETER if the file cannot be written. */
int32_t bm_rt_save_ppm(bm_rt* rt, const char* path);
void bm_rt_destroy(bm_rt* rt);

/* ---- self-test --------------------------------------------------------------------------------
 * The trace kernels' scalar primitives on n host records, run on the context's device (synchronous):
 * orient*ray, 1/dir, Möller-Trumbore (bmTriIntersect, CudaComon.cuh:117-155, with the trace's
 * exact-safe early reject), interpolate + normalize + pack (CudaComon.cuh:253-266, BuildTree.cu:
 * 489-491). in: 36 floats per record (orig[3] ray[3] orient[9, column-major] v0[3] v1[3] v2[3]
 * n0[3] n1[3] n2[3] su sv pad); out: 12 floats (dir[3] 1/dir[3] t u v — t = FLT_MAX and u = v = 0 on
 * a reject — packed colour bits, normalised n.z, pad). tests/test_gpu_glm_pin.py compares them bit
 * for bit with the reference's glm 0.9.9.0 (tests/golden/glm_pin.npz). */
int32_t bm_debug_primitives(bm_context* ctx, uint32_t n, const float* in, float* out);

/* ---- OBJ ingest: TestProgram's Model::load (TestProgram/Model.cpp:26-126) without Assimp ------ */
/* Host-side parse (no device work): one mesh per material run (a `usemtl` after faces, or `o`/`g`,
 * starts a new mesh), file face order, polygons as fans (0,j,j+1), corners with equal (v,vt,vn)
 * index triples shared in first-use order, normals vn[ni] and UV1 vt[ti] when every corner has
 * them; for meshes with both, the tangent space Model.cpp:34 asks Assimp for (aiProcess_CalcTangentSpace,
 * restated in bm_obj.cpp: per-corner face tangents projected into the normal's plane, smoothed over
 * corners at the same position within 45 degrees) into slots BM_VERTEX_DATA_TANGENT/BITANGENT, corners
 * with different tangents not sharing a vertex. Floats parsed with strtof. BM_ERROR_INVALID_PARAMETER if the file cannot be opened,
 * BM_ERROR_INVALID_FORMAT on a malformed face. */
#define BM_OBJ_UNSHARED 1u /* one vertex per corner instead of sharing equal index triples */
typedef struct bm_model bm_model;
typedef struct bm_model_info {
    uint32_t num_meshes;
    uint64_t num_faces;
    uint64_t num_vertices;
    float bmin[3], bmax[3]; /* over the referenced positions (Model.cpp:69-79, 119-122) */
} bm_model_info;
int32_t bm_model_load(const char* path, uint32_t flags, bm_model** out);
int32_t bm_model_info_get(const bm_model* m, bm_model_info* info);
/* Host arrays of mesh i (valid until bm_model_destroy); nrm/uv are NULL when absent. */
int32_t bm_model_mesh(const bm_model* m, uint32_t i, const float** pos, const float** nrm, const float** uv,
                      const uint32_t** idx, uint32_t* num_vertices, uint32_t* num_indices,
                      const char** material);
/* Model::load's upload (Model.cpp:49-114): create one bm_mesh per mesh on ctx (once) and, when
 * scene is non-NULL, add each to it num_adds times. The meshes belong to the model: remove them
 * from scenes (or destroy the scenes) before bm_model_destroy. */
int32_t bm_model_upload(bm_model* m, bm_context* ctx, bm_scene* scene, uint32_t num_adds);
/* Tangents and bitangents of mesh i (3 floats per vertex), NULL when the mesh has no normals or no UVs. */
int32_t bm_model_mesh_tangents(const bm_model* m, uint32_t i, const float** tangent, const float** bitangent);
bm_mesh* bm_model_gpu_mesh(const bm_model* m, uint32_t i);
void bm_model_destroy(bm_model* m);

/* ---- measurement ------------------------------------------------------------------------- */
/* Re-trace the camera view with the counting build of the trace kernel and return the totals
 * over all pixels: out[0] BVH node records fetched, out[1] triangle tests, out[2] hits. Output
 * planes are written exactly as bm_camera_trace writes them. Synchronous. */
int32_t bm_camera_trace_counters(bm_camera* c, const float* eye3, const float* orient3x3,
                                 bm_scene* s, bm_rt* rt, uint64_t out[3]);
/* Counting build of bm_camera_trace_shadow: out[0..2] as above for the primary rays, out[3] node
 * records and out[4] triangle tests of the shadow rays, out[5] shadowed pixels. Synchronous. */
int32_t bm_camera_trace_shadow_counters(bm_camera* c, const float* eye3, const float* orient3x3,
                                        bm_scene* s, bm_rt* rt, const float* light3, uint64_t out[6]);
/* Diagnostic trace (same outputs) recording, per wave64 of the persistent launch, four u64: start
 * and end s_memrealtime (100 MHz), (XCC id << 32 | HW_ID), and the sum over the wave's 8x8 tiles of
 * each tile's longest per-lane work (node records + triangle tests). per_wave holds 4*max_waves
 * u64; *num_waves receives the waves launched, or the capacity needed when max_waves is too small
 * (then BM_ERROR_INVALID_PARAMETER). Synchronous; never used for timing. */
int32_t bm_camera_trace_profile(bm_camera* c, const float* eye3, const float* orient3x3, bm_scene* s,
                                bm_rt* rt, uint64_t* per_wave, uint32_t max_waves,
                                uint32_t* num_waves);
/* Export the built BVH for structural parity tests (synchronous; any pointer may be NULL):
 * records[num_records*16] u32, tris[num_tris*12] u32 (sorted order), keys[num_tris] sorted
 * Morton keys, perm[num_tris] sorted position -> global triangle id. */
int32_t bm_scene_export(bm_scene* s, uint32_t* records, uint32_t* tris, uint32_t* keys,
                        uint32_t* perm);

#ifdef __cplusplus
}
#endif
#endif /* BEAM_C_H */
