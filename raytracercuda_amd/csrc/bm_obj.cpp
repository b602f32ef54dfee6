// bm_obj.cpp — native OBJ ingest: the TestProgram's Model::load (TestProgram/Model.cpp:26-126)
// without Assimp. The reference reads files through Assimp (ReadFile with Triangulate,
// JoinIdenticalVertices, SortByPType, CalcTangentSpace) and hands every aiMesh to an IMesh:
// indices (:59-81), positions slot 0 (:84), normals slot 1 when present (:86-90), UV sets into
// slots 2.. (:91-105). This reader keeps what the hot path sees from that:
//   * one mesh per material run: a `usemtl` that follows faces starts a new mesh, as does `o`/`g`;
//     meshes and faces keep file order;
//   * polygons become triangle fans (0, j, j+1);
//   * corners with the same (v, vt, vn) index triple share one vertex, numbered in order of first
//     use (BM_OBJ_UNSHARED: one vertex per corner). Positions/normals are the file's floats, parsed
//     with strtof, so every triangle has exactly the file's coordinates whichever way corners are
//     shared, and intersection results cannot depend on it;
//   * normals are vn[ni] (the OBJ rule; a mesh gets a normal slot only when every corner has one),
//     texture coordinates vt[ti].xy into UV1 when every corner has one.
// Assimp itself is absent from the reference (a Windows DLL, no source), so this boundary is
// "parity unpinned" (SURVEY §8(c)); tests pin it against oracle/beam_oracle.c's reader, which
// produced the golden meshes, and against the golden frames.
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <new>
#include <string>
#include <tuple>
#include <vector>

#include "../../include/beam_c.h"

namespace {

struct ObjMesh {
    std::string material;
    std::vector<float> pos, nrm, uv;
    std::vector<uint32_t> idx;
    bool has_nrm = true, has_uv = true;
};

struct Corner {
    long v, t, n;  // 0-based, -1 = absent
};

const char* skip_ws(const char* p, const char* e) {
    while (p < e && (*p == ' ' || *p == '\t' || *p == '\r')) ++p;
    return p;
}

// Resolve an OBJ index (1-based, negative = relative to the current count); -1 when invalid.
long resolve(long i, size_t count) {
    if (i > 0) return (size_t)i <= count ? i - 1 : -1;
    if (i < 0) return (long)count + i >= 0 ? (long)count + i : -1;
    return -1;
}

}  // namespace

struct bm_model {
    std::vector<ObjMesh> meshes;
    std::vector<bm_mesh*> gpu;
    bm_model_info info{};
    std::string error;
};

extern "C" {

int32_t bm_model_load(const char* path, uint32_t flags, bm_model** out) {
    if (!path || !out) return BM_ERROR_INVALID_PARAMETER;
    *out = nullptr;
    FILE* f = std::fopen(path, "rb");
    if (!f) return BM_ERROR_INVALID_PARAMETER;
    std::vector<char> buf;
    char chunk[1 << 16];
    size_t got;
    while ((got = std::fread(chunk, 1, sizeof(chunk), f)) > 0) buf.insert(buf.end(), chunk, chunk + got);
    std::fclose(f);
    buf.push_back('\n');

    bm_model* m = new (std::nothrow) bm_model();
    if (!m) return BM_ERROR_GPU_ALLOC_FAIL;
    std::vector<float> v, vn, vt;
    std::vector<ObjMesh>& meshes = m->meshes;
    meshes.emplace_back();
    std::map<std::tuple<long, long, long>, uint32_t> shared;  // corner triple -> vertex of the current mesh
    const bool unshared = (flags & BM_OBJ_UNSHARED) != 0;
    std::vector<Corner> poly;
    auto begin_mesh = [&](std::string material) {  // by value: emplace_back may move the source
        if (!meshes.back().idx.empty()) {
            meshes.emplace_back();
            shared.clear();
        }
        meshes.back().material = material;
    };
    const char* p = buf.data();
    const char* end = buf.data() + buf.size();
    while (p < end) {
        const char* eol = static_cast<const char*>(std::memchr(p, '\n', (size_t)(end - p)));
        if (!eol) eol = end;
        const char* q = skip_ws(p, eol);
        if (q < eol && *q != '#') {
            const char* kw = q;
            while (q < eol && *q != ' ' && *q != '\t' && *q != '\r') ++q;
            const std::string key(kw, (size_t)(q - kw));
            if (key == "v" || key == "vn" || key == "vt") {
                std::vector<float>& dst = key == "v" ? v : key == "vn" ? vn : vt;
                const int want = key == "vt" ? 2 : 3;
                std::string line(q, (size_t)(eol - q));
                const char* s = line.c_str();
                for (int c = 0; c < want; ++c) {
                    char* e2 = nullptr;
                    float x = std::strtof(s, &e2);
                    if (e2 == s) x = 0.0f;  // vt with one coordinate: v defaults to 0
                    dst.push_back(x);
                    s = e2;
                }
            } else if (key == "f") {
                poly.clear();
                std::string line(q, (size_t)(eol - q));
                const char* s = line.c_str();
                bool ok = true;
                while (true) {
                    while (*s == ' ' || *s == '\t' || *s == '\r') ++s;
                    if (!*s) break;
                    Corner c{-1, -1, -1};
                    char* e2 = nullptr;
                    long a = std::strtol(s, &e2, 10);
                    if (e2 == s) {
                        ok = false;
                        break;
                    }
                    c.v = resolve(a, v.size() / 3);
                    s = e2;
                    if (*s == '/') {
                        ++s;
                        if (*s != '/') {
                            long b = std::strtol(s, &e2, 10);
                            if (e2 != s) c.t = resolve(b, vt.size() / 2);
                            s = e2;
                        }
                        if (*s == '/') {
                            ++s;
                            long n = std::strtol(s, &e2, 10);
                            if (e2 != s) c.n = resolve(n, vn.size() / 3);
                            s = e2;
                        }
                    }
                    if (c.v < 0) {
                        ok = false;
                        break;
                    }
                    poly.push_back(c);
                    while (*s && *s != ' ' && *s != '\t' && *s != '\r') ++s;
                }
                if (!ok) {
                    m->error = "bad face: " + line;
                    delete m;
                    return BM_ERROR_INVALID_FORMAT;
                }
                ObjMesh& mesh = meshes.back();
                auto vertex = [&](const Corner& c) -> uint32_t {
                    const auto key3 = std::make_tuple(c.v, c.t, c.n);
                    if (!unshared) {
                        auto it = shared.find(key3);
                        if (it != shared.end()) return it->second;
                    }
                    const uint32_t id = (uint32_t)(mesh.pos.size() / 3);
                    for (int k = 0; k < 3; ++k) mesh.pos.push_back(v[3 * (size_t)c.v + k]);
                    if (c.n >= 0)
                        for (int k = 0; k < 3; ++k) mesh.nrm.push_back(vn[3 * (size_t)c.n + k]);
                    else {
                        mesh.has_nrm = false;
                        for (int k = 0; k < 3; ++k) mesh.nrm.push_back(0.0f);
                    }
                    if (c.t >= 0) {
                        mesh.uv.push_back(vt[2 * (size_t)c.t]);
                        mesh.uv.push_back(vt[2 * (size_t)c.t + 1]);
                    } else {
                        mesh.has_uv = false;
                        mesh.uv.push_back(0.0f);
                        mesh.uv.push_back(0.0f);
                    }
                    if (!unshared) shared.emplace(key3, id);
                    return id;
                };
                for (size_t j = 1; j + 1 < poly.size(); ++j) {  // fan (0, j, j+1); points/lines dropped
                    mesh.idx.push_back(vertex(poly[0]));
                    mesh.idx.push_back(vertex(poly[j]));
                    mesh.idx.push_back(vertex(poly[j + 1]));
                }
            } else if (key == "usemtl") {
                const char* s = skip_ws(q, eol);
                const char* e2 = eol;
                while (e2 > s && (e2[-1] == ' ' || e2[-1] == '\t' || e2[-1] == '\r')) --e2;
                begin_mesh(std::string(s, (size_t)(e2 - s)));
            } else if (key == "o" || key == "g") {
                begin_mesh(meshes.back().material);
            }  // s, mtllib and anything else: not on the path
        }
        p = eol + 1;
    }
    if (meshes.back().idx.empty() && meshes.size() > 1) meshes.pop_back();
    if (meshes.size() == 1 && meshes[0].idx.empty()) meshes.clear();
    bm_model_info& in = m->info;
    in.num_meshes = (uint32_t)meshes.size();
    for (int c = 0; c < 3; ++c) {
        in.bmin[c] = INFINITY;
        in.bmax[c] = -INFINITY;
    }
    for (ObjMesh& mesh : meshes) {
        if (!mesh.has_nrm) mesh.nrm.clear();
        if (!mesh.has_uv) mesh.uv.clear();
        in.num_faces += mesh.idx.size() / 3;
        in.num_vertices += mesh.pos.size() / 3;
        for (uint32_t i : mesh.idx)
            for (int c = 0; c < 3; ++c) {
                const float x = mesh.pos[3 * (size_t)i + c];
                in.bmin[c] = std::fmin(in.bmin[c], x);
                in.bmax[c] = std::fmax(in.bmax[c], x);
            }
    }
    *out = m;
    return BM_ERROR_ALL_FINE;
}

int32_t bm_model_info_get(const bm_model* m, bm_model_info* info) {
    if (!m || !info) return BM_ERROR_INVALID_PARAMETER;
    *info = m->info;
    return BM_ERROR_ALL_FINE;
}

int32_t bm_model_mesh(const bm_model* m, uint32_t i, const float** pos, const float** nrm, const float** uv,
                      const uint32_t** idx, uint32_t* num_vertices, uint32_t* num_indices, const char** material) {
    if (!m || i >= m->meshes.size()) return BM_ERROR_INVALID_PARAMETER;
    const ObjMesh& mesh = m->meshes[i];
    if (pos) *pos = mesh.pos.data();
    if (nrm) *nrm = mesh.nrm.empty() ? nullptr : mesh.nrm.data();
    if (uv) *uv = mesh.uv.empty() ? nullptr : mesh.uv.data();
    if (idx) *idx = mesh.idx.data();
    if (num_vertices) *num_vertices = (uint32_t)(mesh.pos.size() / 3);
    if (num_indices) *num_indices = (uint32_t)mesh.idx.size();
    if (material) *material = mesh.material.c_str();
    return BM_ERROR_ALL_FINE;
}

// Model::load's upload loop (Model.cpp:49-114): one IMesh per mesh, added num_adds times.
int32_t bm_model_upload(bm_model* m, bm_context* ctx, bm_scene* scene, uint32_t num_adds) {
    if (!m || !ctx) return BM_ERROR_INVALID_PARAMETER;
    if (m->gpu.empty()) {
        for (const ObjMesh& mesh : m->meshes) {
            bm_mesh* g = nullptr;
            int32_t e = bm_mesh_create(ctx, &g);
            if (e) return e;
            m->gpu.push_back(g);
            const uint32_t nv = (uint32_t)(mesh.pos.size() / 3);
            if ((e = bm_mesh_set_indices(g, mesh.idx.data(), (uint32_t)mesh.idx.size()))) return e;
            if ((e = bm_mesh_set_vertex_data(g, mesh.pos.data(), nv, 3, BM_VERTEX_DATA_POSITION))) return e;
            if (!mesh.nrm.empty() && (e = bm_mesh_set_vertex_data(g, mesh.nrm.data(), nv, 3, BM_VERTEX_DATA_NORMAL)))
                return e;
            if (!mesh.uv.empty() && (e = bm_mesh_set_vertex_data(g, mesh.uv.data(), nv, 2, BM_VERTEX_DATA_UV1)))
                return e;
        }
    }
    if (scene)
        for (bm_mesh* g : m->gpu)
            for (uint32_t k = 0; k < num_adds; ++k) {
                int32_t e = bm_scene_add_mesh(scene, g);
                if (e) return e;
            }
    return BM_ERROR_ALL_FINE;
}

bm_mesh* bm_model_gpu_mesh(const bm_model* m, uint32_t i) {
    return (m && i < m->gpu.size()) ? m->gpu[i] : nullptr;
}

void bm_model_destroy(bm_model* m) {
    if (!m) return;
    for (bm_mesh* g : m->gpu) bm_mesh_destroy(g);
    delete m;
}

}  // extern "C"
