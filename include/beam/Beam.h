// Beam.h — the reference's C++ host API (Raytracer/Beam.h:32-72), rebuilt header-only over the
// C ABI of libbeam_hip.so (include/beam_c.h). A program written against the reference's
// IScene / IMesh / ICamera / IRenderTarget compiles against this header with two changes:
//   * IRenderTarget::registerGLTBO (GL interop) is replaced by IRenderTarget::createOffscreen;
//   * the device is chosen with Beam::setDevice(n) (default: the BM_DEVICE env var, else 0)
//     instead of cudaSetDevice (TestProgram/Program.cpp:122-124);
//   * Beam::setDevices({d0, d1, ...}) (or env BM_DEVICES="0,1,2,3") renders every frame on several
//     GPUs: scenes are replicated, screen bands dealt round-robin, the frame gathered on d0.
// Error codes, vertex slots, the "current render target" set by lock() (RenderTarget.cpp:53-88)
// and the asynchronous launch behaviour are the reference's. Beam::sync() waits for the device.
#pragma once

#include <cstdint>
#include <cstdlib>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../beam_c.h"

namespace Beam {

using i32 = int32_t;
using i64 = int64_t;
using u32 = uint32_t;
using u64 = uint64_t;
template <typename T>
using sptr = std::shared_ptr<T>;
template <typename T>
using wptr = std::weak_ptr<T>;
template <typename T>
using Array = std::vector<T>;

constexpr u32 ERROR_ALL_FINE = BM_ERROR_ALL_FINE;
constexpr u32 ERROR_NO_VERTICES = BM_ERROR_NO_VERTICES;
constexpr u32 ERROR_INVALID_PARAMETER = BM_ERROR_INVALID_PARAMETER;
constexpr u32 ERROR_GPU_ALLOC_FAIL = BM_ERROR_GPU_ALLOC_FAIL;
constexpr u32 ERROR_INVALID_FORMAT = BM_ERROR_INVALID_FORMAT;
constexpr u32 ERROR_RT_CAM_MISMATCH = BM_ERROR_RT_CAM_MISMATCH;
constexpr u32 ERROR_UNLOCK_FIRST = BM_ERROR_UNLOCK_FIRST;
constexpr u32 ERROR_LOCK_FIRST = BM_ERROR_LOCK_FIRST;
constexpr u32 ERROR_NO_RENDER_TARGET = BM_ERROR_NO_RENDER_TARGET;
constexpr u32 ERROR_DEVICE = BM_ERROR_DEVICE;
constexpr u32 ERROR_NOT_BUILT = BM_ERROR_NOT_BUILT;

constexpr u32 VERTEX_DATA_POSITION = 0;
constexpr u32 VERTEX_DATA_NORMAL = 1;
constexpr u32 VERTEX_DATA_UV1 = 2;
constexpr u32 VERTEX_DATA_UV2 = 3;
constexpr u32 VERTEX_DATA_TANGENT = 4;
constexpr u32 VERTEX_DATA_BITANGENT = 5;
constexpr u32 VERTEX_DATA_EXTRA1 = 6;
constexpr u32 VERTEX_DATA_EXTRA2 = 7;
constexpr u32 VERTEX_DATA_EXTRA3 = 8;
constexpr u32 VERTEX_DATA_EXTRA4 = 9;
constexpr u32 VERTEX_DATA_COUNT = 10;

namespace detail {
inline uint32_t& flags_slot() {  // BM_OPT_* for the context created on first use
    static uint32_t f = (std::getenv("BM_REFERENCE_KD") && std::atoi(std::getenv("BM_REFERENCE_KD"))) ? BM_OPT_REFERENCE_KD
                                                                                                   : 0u;
    return f;
}
struct MultiDevice {  // bm_options multi-GPU fields for the context created on first use
    std::vector<int> devices;
    u32 band_height = 0, gather = BM_GATHER_AUTO;
};
inline MultiDevice& multi_slot() {
    static MultiDevice m = [] {
        MultiDevice d;
        if (const char* e = std::getenv("BM_DEVICES")) {  // "0,1,2,3"
            for (const char* p = e; *p;) {
                char* end = nullptr;
                const long v = std::strtol(p, &end, 10);
                if (end == p) break;
                d.devices.push_back((int)v);
                p = *end == ',' ? end + 1 : end;
            }
        }
        return d;
    }();
    return m;
}
struct Context {
    bm_context* h = nullptr;
    explicit Context(int device) {
        bm_options o{};
        o.device = device;
        o.flags = flags_slot();
        const MultiDevice& m = multi_slot();
        if (m.devices.size() > BM_MAX_DEVICES) throw std::runtime_error("Beam: at most 8 devices");
        o.num_devices = (uint32_t)m.devices.size();
        for (size_t i = 0; i < m.devices.size(); ++i) o.devices[i] = m.devices[i];
        o.band_height = m.band_height;
        o.gather = m.gather;
        if (bm_context_create(&o, &h) != BM_ERROR_ALL_FINE) throw std::runtime_error("Beam: no usable HIP device");
    }
    ~Context() { bm_context_destroy(h); }
};
inline int& device_slot() {
    static int d = std::getenv("BM_DEVICE") ? std::atoi(std::getenv("BM_DEVICE")) : 0;
    return d;
}
inline sptr<Context>& context_slot() {
    static sptr<Context> c;
    return c;
}
inline bm_context* ctx() {
    auto& c = context_slot();
    if (!c) c = std::make_shared<Context>(device_slot());
    return c->h;
}
}  // namespace detail

// Select the device before the first Beam object is created.
inline void setDevice(int device) { detail::device_slot() = device; }
// Render on several devices (1..8; repeats allowed: a one-GPU rehearsal): objects replicated on
// each, screen bands of bandHeight rows (0 = 16) dealt round-robin, the frame gathered on
// devices[0] by `gather` (BM_GATHER_AUTO / _PEER / _RCCL). Before the first Beam object.
inline void setDevices(const std::vector<int>& devices, u32 bandHeight = 0, u32 gather = BM_GATHER_AUTO) {
    detail::multi_slot() = detail::MultiDevice{devices, bandHeight, gather};
}
inline u32 numDevices() { return bm_context_num_devices(detail::ctx()); }
// Reference mode (BM_OPT_REFERENCE_KD; env BM_REFERENCE_KD=1): scenes build the reference's kd-tree
// and traceScene returns its first-hit-leaf answer, pixel for pixel. Before the first Beam object.
inline void setReferenceMode(bool on) {
    if (on) detail::flags_slot() = (detail::flags_slot() | BM_OPT_REFERENCE_KD) & ~BM_OPT_REFERENCE_HASH;
    else detail::flags_slot() &= ~BM_OPT_REFERENCE_KD;
}
// Hashed-grid mode (BM_OPT_REFERENCE_HASH): the reference's alternative accelerator (Hash.cu, built
// there with TREE_TYPE==HASH, SceneHash.cpp) — a comparison study. Before the first Beam object.
inline void setHashGridMode(bool on) {
    if (on) detail::flags_slot() = (detail::flags_slot() | BM_OPT_REFERENCE_HASH) & ~BM_OPT_REFERENCE_KD;
    else detail::flags_slot() &= ~BM_OPT_REFERENCE_HASH;
}
inline u32 sync() { return (u32)bm_sync(detail::ctx()); }
inline std::string lastError() { return bm_last_error_string(detail::ctx()); }

class IRenderTarget {
   public:
    // Offscreen device render target: planes packed (0x00RRGGBB, pitch honoured), triangle id, t.
    static sptr<IRenderTarget> createOffscreen(u32 width, u32 height, u32 pitch = 0) {
        bm_rt* h = nullptr;
        if (bm_rt_create_offscreen(detail::ctx(), width, height, pitch, &h) != BM_ERROR_ALL_FINE) return nullptr;
        return sptr<IRenderTarget>(new IRenderTarget(h));
    }
    // GL interop is not part of this build (offscreen framebuffers only).
    static sptr<IRenderTarget> registerGLTBO(u32, u32, u32, u32) { return nullptr; }
    ~IRenderTarget() {
        if (current() == this) current() = nullptr;
        bm_rt_destroy(h_);
    }
    void* buffer() const { return bm_rt_buffer(h_); }
    template <class T>
    T* buffer() const {
        return reinterpret_cast<T*>(buffer());
    }
    u32 pitch() const { return bm_rt_pitch(h_); }
    u32 width() const { return bm_rt_width(h_); }
    u32 height() const { return bm_rt_height(h_); }
    u32 lock() {
        const u32 e = (u32)bm_rt_lock(h_);
        if (e == ERROR_ALL_FINE) current() = this;
        return e;
    }
    u32 unlock() {
        const u32 e = (u32)bm_rt_unlock(h_);
        if (e == ERROR_ALL_FINE && current() == this) current() = nullptr;
        return e;
    }
    // Host readback (synchronous); any pointer may be null.
    u32 read(u32* packed, u32* triId = nullptr, float* t = nullptr, float* rgb = nullptr) {
        return (u32)bm_rt_read(h_, packed, triId, t, rgb);
    }
    u32 readShadow(unsigned char* out) { return (u32)bm_rt_read_shadow(h_, out); }
    u32 savePPM(const char* path) { return (u32)bm_rt_save_ppm(h_, path); }
    // frames in flight: this target's traces/readbacks on its own HIP stream (nullptr: the context's)
    u32 setStream(void* stream) { return (u32)bm_rt_set_stream(h_, stream); }
    static IRenderTarget*& current() {  // RenderTarget::m_RT (RenderTarget.cpp:85-93)
        static IRenderTarget* rt = nullptr;
        return rt;
    }
    bm_rt* handle() const { return h_; }

   private:
    explicit IRenderTarget(bm_rt* h) : h_(h) {}
    bm_rt* h_;
};

class IScene;

class IMesh {
   public:
    static sptr<IMesh> create() {
        bm_mesh* h = nullptr;
        if (bm_mesh_create(detail::ctx(), &h) != BM_ERROR_ALL_FINE) return nullptr;
        return sptr<IMesh>(new IMesh(h));
    }
    ~IMesh() { bm_mesh_destroy(h_); }
    u32 setVertexData(const float* vertices, u32 numVertices, u32 numComponents, u32 slotId, bool asyncCopy = false) {
        (void)asyncCopy;
        return (u32)bm_mesh_set_vertex_data(h_, vertices, numVertices, numComponents, slotId);
    }
    u32 setIndices(const u32* indices, u32 numIndices, bool asyncCopy = false) {
        (void)asyncCopy;
        return (u32)bm_mesh_set_indices(h_, indices, numIndices);
    }
    wptr<IScene> scene() const { return {}; }
    bm_mesh* handle() const { return h_; }

   private:
    explicit IMesh(bm_mesh* h) : h_(h) {}
    bm_mesh* h_;
};

class IScene {
   public:
    static sptr<IScene> create() {
        bm_scene* h = nullptr;
        if (bm_scene_create(detail::ctx(), &h) != BM_ERROR_ALL_FINE) return nullptr;
        return sptr<IScene>(new IScene(h));
    }
    ~IScene() { bm_scene_destroy(h_); }
    void addMesh(const sptr<IMesh>& mesh) {
        if (bm_scene_add_mesh(h_, mesh->handle()) == BM_ERROR_ALL_FINE) meshes_.push_back(mesh);
    }
    void removeMesh(const IMesh& mesh) {
        bm_scene_remove_mesh(h_, mesh.handle());
        for (auto it = meshes_.begin(); it != meshes_.end(); ++it)
            if (it->get() == &mesh) {
                meshes_.erase(it);
                break;
            }
    }
    // Rebuilds the BVH (asynchronous, like the reference's launches).
    void updateGPUScene() { bm_scene_build(h_, nullptr); }
    u32 updateGPUScene(bm_build_stats* stats) { return (u32)bm_scene_build(h_, stats); }
    // Extension: refit-only update after vertex data changed (same meshes and triangle counts).
    u32 refitGPUScene(bm_build_stats* stats = nullptr) { return (u32)bm_scene_refit(h_, stats); }
    bm_scene* handle() const { return h_; }

   private:
    explicit IScene(bm_scene* h) : h_(h) {}
    bm_scene* h_;
    Array<sptr<IMesh>> meshes_;
};

class ICamera {
   public:
    static sptr<ICamera> create() {
        bm_camera* h = nullptr;
        if (bm_camera_create(detail::ctx(), &h) != BM_ERROR_ALL_FINE) return nullptr;
        return sptr<ICamera>(new ICamera(h));
    }
    ~ICamera() { bm_camera_destroy(h_); }
    u32 setInitialRays(u32 width, u32 height, float left = -1, float right = 1, float top = 1, float bottom = -1,
                       float zoom = 1) {
        return (u32)bm_camera_set_initial_rays(h_, width, height, left, right, top, bottom, zoom);
    }
    u32 clear(u32 value) {
        IRenderTarget* rt = IRenderTarget::current();
        if (!rt) return ERROR_NO_RENDER_TARGET;
        return (u32)bm_rt_clear(rt->handle(), value);
    }
    u32 traceScene(const float* eye3, const float* orient3x3, sptr<IScene>& scene) {
        IRenderTarget* rt = IRenderTarget::current();
        if (!rt) return ERROR_NO_RENDER_TARGET;
        if (!scene) return ERROR_INVALID_PARAMETER;
        return (u32)bm_camera_trace(h_, eye3, orient3x3, scene->handle(), rt->handle());
    }
    // Extension (no reference counterpart): traceScene plus one any-hit shadow ray per hit toward
    // a point light; the current render target's shadow plane (readShadow) gets 1 = shadowed.
    u32 traceSceneShadow(const float* eye3, const float* orient3x3, sptr<IScene>& scene, const float* light3) {
        IRenderTarget* rt = IRenderTarget::current();
        if (!rt) return ERROR_NO_RENDER_TARGET;
        if (!scene) return ERROR_INVALID_PARAMETER;
        return (u32)bm_camera_trace_shadow(h_, eye3, orient3x3, scene->handle(), rt->handle(), light3);
    }

   private:
    explicit ICamera(bm_camera* h) : h_(h) {}
    bm_camera* h_;
};

}  // namespace Beam
