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
//     texture coordinates vt[ti].xy into UV1 when every corner has one;
//   * tangents and bitangents (slots 4 and 5, Model.cpp:107-113) for meshes with normals and UVs, by
//     Assimp's CalcTangentSpace step as restated in tangent_space() below; corners that would share a
//     vertex but got different tangents get vertices of their own, as JoinIdenticalVertices (which
//     Assimp runs after that step) compares every attribute.
// Assimp itself is absent from the reference (a Windows DLL, no source), so this boundary is
// "parity unpinned" (SURVEY §8(c)); tests pin it against oracle/beam_oracle.c's reader, which
// produced the golden meshes, and against the golden frames.
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <array>
#include <map>
#include <new>
#include <string>
#include <tuple>
#include <vector>

#include "../../include/beam_c.h"

namespace {

struct Corner {
    long v, t, n;  // 0-based, -1 = absent
};

struct ObjMesh {
    std::string material;
    std::vector<float> pos, nrm, uv, tan, bit;
    std::vector<uint32_t> idx;
    std::vector<Corner> cor;  // 3 per triangle, file order (vertices are made from them at the end)
    bool has_nrm = true, has_uv = true;
};

struct V3 {
    float x, y, z;
};
inline V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 operator*(V3 a, float f) { return {a.x * f, a.y * f, a.z * f}; }
inline float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline V3 cross(V3 a, V3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
// aiVector3t::operator/= (a zero length leaves the vector), Normalize (/= Length) and NormalizeSafe
inline V3 div_len(V3 a, float len) {
    if (len == 0.0f) return a;
    const float inv = 1.0f / len;
    return {a.x * inv, a.y * inv, a.z * inv};
}
inline V3 normalize(V3 a) { return div_len(a, std::sqrt(dot(a, a))); }
inline V3 normalize_safe(V3 a) {
    const float len = std::sqrt(dot(a, a));
    return len > 0.0f ? div_len(a, len) : a;
}
inline bool special(V3 a) { return !std::isfinite(a.x) || !std::isfinite(a.y) || !std::isfinite(a.z); }

// Tangent space of one mesh's corners (position P[i], normal N[i], uv U[i] of corner i, 3 per
// triangle): Assimp's CalcTangentsProcess (code/PostProcessing/CalcTangentsProcess.cpp, the step
// Model.cpp:34 requests), restated from its published algorithm — Assimp is absent here, so this is
// "parity unpinned" like the rest of the OBJ boundary. Assimp runs it on the importer's unshared
// corners, before JoinIdenticalVertices.
//  1. Per triangle (p0, p1, p2): v = p1 - p0, w = p2 - p0, (sx, sy) = uv1 - uv0, (tx, ty) = uv2 - uv0,
//     dir = (tx sy - ty sx) < 0 ? -1 : 1; when sx ty == sy tx the UVs give no direction and
//     (sx, sy, tx, ty) = (0, 1, 1, 0); tangent = (w sy - v ty) dir, bitangent = (w sx - v tx) dir. Each
//     corner projects both into its normal's plane (t - n (t.n)) and NormalizeSafe's them; when exactly
//     one came out with a NaN/inf component it is rebuilt from the other (n x b, or t x n), normalized.
//  2. Smoothing, corners in order: an unvisited corner a finds the corners within posEps of its
//     position (Assimp's SpatialSort: entries ordered by distance along the plane normal (0.8523,
//     0.0812, 0.5165) normalized — ties here by index — squared distance < posEps^2; posEps = 1e-4 x
//     the mesh's bounding-box diagonal) and takes the unvisited ones with normal.n_a >= 0.9999,
//     tangent.t_a >= cos(45 deg) and bitangent.b_a >= cos(45 deg); a itself, unmarked until then, is
//     found again and counted twice, as in Assimp. The group's tangents and bitangents are summed (a
//     first, then in found order), normalized, and written to every member.
void tangent_space(const std::vector<V3>& P, const std::vector<V3>& N, const std::vector<float>& U,
                   std::vector<V3>& T, std::vector<V3>& B) {
    const size_t nc = P.size();
    T.assign(nc, V3{0, 0, 0});
    B.assign(nc, V3{0, 0, 0});
    for (size_t f = 0; f + 2 < nc; f += 3) {
        const size_t p0 = f, p1 = f + 1, p2 = f + 2;
        const V3 v = P[p1] - P[p0], w = P[p2] - P[p0];
        float sx = U[2 * p1] - U[2 * p0], sy = U[2 * p1 + 1] - U[2 * p0 + 1];
        float tx = U[2 * p2] - U[2 * p0], ty = U[2 * p2 + 1] - U[2 * p0 + 1];
        const float dir = (tx * sy - ty * sx) < 0.0f ? -1.0f : 1.0f;
        if (sx * ty == sy * tx) {
            sx = 0.0f;
            sy = 1.0f;
            tx = 1.0f;
            ty = 0.0f;
        }
        const V3 tg{(w.x * sy - v.x * ty) * dir, (w.y * sy - v.y * ty) * dir, (w.z * sy - v.z * ty) * dir};
        const V3 bt{(w.x * sx - v.x * tx) * dir, (w.y * sx - v.y * tx) * dir, (w.z * sx - v.z * tx) * dir};
        for (size_t p = f; p < f + 3; ++p) {
            V3 lt = normalize_safe(tg - N[p] * dot(tg, N[p]));
            V3 lb = normalize_safe(bt - N[p] * dot(bt, N[p]));
            const bool it = special(lt), ib = special(lb);
            if (it != ib) {
                if (it) lt = normalize_safe(cross(N[p], lb));
                else lb = normalize_safe(cross(lt, N[p]));
            }
            T[p] = lt;
            B[p] = lb;
        }
    }
    // position epsilon and the spatial sort
    V3 mn{INFINITY, INFINITY, INFINITY}, mx{-INFINITY, -INFINITY, -INFINITY};
    for (const V3& p : P) {
        mn = {std::fmin(mn.x, p.x), std::fmin(mn.y, p.y), std::fmin(mn.z, p.z)};
        mx = {std::fmax(mx.x, p.x), std::fmax(mx.y, p.y), std::fmax(mx.z, p.z)};
    }
    const V3 ext = mx - mn;
    const float eps = std::sqrt(dot(ext, ext)) * 1e-4f, eps2 = eps * eps;
    const V3 pn = normalize(V3{0.8523f, 0.0812f, 0.5165f});
    std::vector<float> dist(nc);
    std::vector<uint32_t> order(nc);
    for (size_t i = 0; i < nc; ++i) {
        dist[i] = dot(P[i], pn);
        if (std::isnan(dist[i])) dist[i] = INFINITY;  // a NaN position: last, and never within reach
        order[i] = (uint32_t)i;
    }
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return dist[a] < dist[b]; });
    std::vector<float> sorted(nc);
    for (size_t i = 0; i < nc; ++i) sorted[i] = dist[order[i]];
    const float ang_eps = 0.9999f, limit = std::cos(45.0f * 0.0174532925f);
    std::vector<char> done(nc, 0);
    std::vector<uint32_t> group;
    for (size_t a = 0; a < nc; ++a) {
        if (done[a]) continue;
        const V3 pa = P[a], na = N[a], ta = T[a], ba = B[a];
        group.assign(1, (uint32_t)a);
        const float d = dist[a];
        size_t k = (size_t)(std::lower_bound(sorted.begin(), sorted.end(), d - eps) - sorted.begin());
        for (; k < nc && sorted[k] < d + eps; ++k) {
            const uint32_t j = order[k];
            const V3 dp = P[j] - pa;
            if (!(dot(dp, dp) < eps2) || done[j]) continue;
            if (dot(N[j], na) < ang_eps || dot(T[j], ta) < limit || dot(B[j], ba) < limit) continue;
            group.push_back(j);
            done[j] = 1;
        }
        V3 st{0, 0, 0}, sb{0, 0, 0};
        for (uint32_t j : group) {
            st = st + T[j];
            sb = sb + B[j];
        }
        st = normalize(st);
        sb = normalize(sb);
        for (uint32_t j : group) {
            T[j] = st;
            B[j] = sb;
        }
    }
}

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
    const bool unshared = (flags & BM_OBJ_UNSHARED) != 0;
    std::vector<Corner> poly;
    auto begin_mesh = [&](std::string material) {  // by value: emplace_back may move the source
        if (!meshes.back().cor.empty()) meshes.emplace_back();
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
                for (size_t j = 1; j + 1 < poly.size(); ++j) {  // fan (0, j, j+1); points/lines dropped
                    mesh.cor.push_back(poly[0]);
                    mesh.cor.push_back(poly[j]);
                    mesh.cor.push_back(poly[j + 1]);
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
    if (meshes.back().cor.empty() && meshes.size() > 1) meshes.pop_back();
    if (meshes.size() == 1 && meshes[0].cor.empty()) meshes.clear();
    // vertices: corners with equal (v, vt, vn) triples — and, with a tangent space, equal tangent and
    // bitangent bits — share one, numbered in order of first use (BM_OBJ_UNSHARED: one per corner)
    for (ObjMesh& mesh : meshes) {
        const size_t nc = mesh.cor.size();
        for (const Corner& c : mesh.cor) {
            mesh.has_nrm = mesh.has_nrm && c.n >= 0;
            mesh.has_uv = mesh.has_uv && c.t >= 0;
        }
        std::vector<V3> T, B;
        const bool ts = mesh.has_nrm && mesh.has_uv && nc > 0;
        if (ts) {
            std::vector<V3> P(nc), N(nc);
            std::vector<float> Uc(2 * nc);
            for (size_t i = 0; i < nc; ++i) {
                const Corner& c = mesh.cor[i];
                P[i] = {v[3 * (size_t)c.v], v[3 * (size_t)c.v + 1], v[3 * (size_t)c.v + 2]};
                N[i] = {vn[3 * (size_t)c.n], vn[3 * (size_t)c.n + 1], vn[3 * (size_t)c.n + 2]};
                Uc[2 * i] = vt[2 * (size_t)c.t];
                Uc[2 * i + 1] = vt[2 * (size_t)c.t + 1];
            }
            tangent_space(P, N, Uc, T, B);
        }
        auto bits = [](float x) {
            uint32_t u;
            std::memcpy(&u, &x, 4);
            return u;
        };
        std::map<std::array<uint32_t, 9>, uint32_t> shared;
        mesh.idx.reserve(nc);
        for (size_t i = 0; i < nc; ++i) {
            const Corner& c = mesh.cor[i];
            std::array<uint32_t, 9> key{(uint32_t)c.v, (uint32_t)c.t, (uint32_t)c.n, 0, 0, 0, 0, 0, 0};
            if (ts) {
                key[3] = bits(T[i].x), key[4] = bits(T[i].y), key[5] = bits(T[i].z);
                key[6] = bits(B[i].x), key[7] = bits(B[i].y), key[8] = bits(B[i].z);
            }
            if (!unshared) {
                auto it = shared.find(key);
                if (it != shared.end()) {
                    mesh.idx.push_back(it->second);
                    continue;
                }
            }
            const uint32_t id = (uint32_t)(mesh.pos.size() / 3);
            for (int k = 0; k < 3; ++k) mesh.pos.push_back(v[3 * (size_t)c.v + k]);
            for (int k = 0; k < 3; ++k) mesh.nrm.push_back(c.n >= 0 ? vn[3 * (size_t)c.n + k] : 0.0f);
            mesh.uv.push_back(c.t >= 0 ? vt[2 * (size_t)c.t] : 0.0f);
            mesh.uv.push_back(c.t >= 0 ? vt[2 * (size_t)c.t + 1] : 0.0f);
            if (ts) {
                mesh.tan.insert(mesh.tan.end(), {T[i].x, T[i].y, T[i].z});
                mesh.bit.insert(mesh.bit.end(), {B[i].x, B[i].y, B[i].z});
            }
            if (!unshared) shared.emplace(key, id);
            mesh.idx.push_back(id);
        }
        mesh.cor.clear();
        mesh.cor.shrink_to_fit();
    }
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
            if (!mesh.tan.empty() &&
                ((e = bm_mesh_set_vertex_data(g, mesh.tan.data(), nv, 3, BM_VERTEX_DATA_TANGENT)) ||
                 (e = bm_mesh_set_vertex_data(g, mesh.bit.data(), nv, 3, BM_VERTEX_DATA_BITANGENT))))
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

int32_t bm_model_mesh_tangents(const bm_model* m, uint32_t i, const float** tangent, const float** bitangent) {
    if (!m || i >= m->meshes.size()) return BM_ERROR_INVALID_PARAMETER;
    const ObjMesh& mesh = m->meshes[i];
    if (tangent) *tangent = mesh.tan.empty() ? nullptr : mesh.tan.data();
    if (bitangent) *bitangent = mesh.bit.empty() ? nullptr : mesh.bit.data();
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
