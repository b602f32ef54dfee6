// glm_pin.cpp — TEST INFRASTRUCTURE ONLY (oracle/, never linked into the product).
//
// Computes the hot path's scalar primitives with the reference's own vendored math library,
// glm 0.9.9.0 (/root/reference/3rdParty/glm-0.9.9.0, header-only, compiled here unmodified), in the
// formulation of the reference's code, so that the oracle's C restatement of them (orc_pin_ops in
// beam_oracle.c) is pinned bit for bit against glm rather than against a reading of glm:
//   dir = orient * ray                 BuildTree.cu:377-378 (glm mat3 * vec3)
//   invDir = (1/dir.x, 1/dir.y, 1/dir.z)  BuildTree.cu:379
//   bmTriIntersect                     CudaComon.cuh:117-155 (glm cross, dot, vec3 -)
//   bmFaceInterpolate<vec3> + normalize + pack   CudaComon.cuh:253-266, BuildTree.cu:489-491
// Built by oracle/Makefile (target glm_pin, output oracle/_ref/glm_pin) only where /root/reference
// exists; oracle/make_glm_pin.py runs it and commits inputs + outputs as tests/golden/glm_pin.npz.
//
//   glm_pin IN.f32 OUT.f32     (record layouts: beam_oracle.c, orc_pin_ops)
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include <glm/glm.hpp>

namespace {

// Möller-Trumbore in the reference's formulation, glm types and functions throughout.
float tri(const glm::vec3& orig, const glm::vec3& dir, const glm::vec3& v0, const glm::vec3& v1,
          const glm::vec3& v2, float& u, float& v) {
    const glm::vec3 e1 = v1 - v0;
    const glm::vec3 e2 = v2 - v0;
    const glm::vec3 p = glm::cross(dir, e2);
    const float det = glm::dot(e1, p);
    const float inv = 1.f / det;
    const glm::vec3 tv = orig - v0;
    u = glm::dot(tv, p) * inv;
    if (u < 0 || u > 1) return FLT_MAX;
    const glm::vec3 q = glm::cross(tv, e1);
    v = glm::dot(dir, q) * inv;
    if (v < 0 || v + u > 1) return FLT_MAX;
    return glm::dot(e2, q) * inv;
}

glm::vec3 v3(const float* a) { return glm::vec3(a[0], a[1], a[2]); }

}  // namespace

int main(int argc, char** argv) {
    if (argc != 3) {
        std::fprintf(stderr, "usage: glm_pin IN.f32 OUT.f32\n");
        return 2;
    }
    std::FILE* f = std::fopen(argv[1], "rb");
    if (!f) return 1;
    std::vector<float> in;
    float buf[36];
    while (std::fread(buf, sizeof(float), 36, f) == 36) in.insert(in.end(), buf, buf + 36);
    std::fclose(f);
    const size_t n = in.size() / 36;
    std::vector<float> out(n * 12, 0.f);
    for (size_t i = 0; i < n; ++i) {
        const float* a = &in[i * 36];
        float* o = &out[i * 12];
        glm::mat3 m;
        for (int c = 0; c < 3; ++c)
            for (int r = 0; r < 3; ++r) m[c][r] = a[6 + c * 3 + r];
        const glm::vec3 dir = m * v3(a + 3);
        const glm::vec3 inv(1.f / dir.x, 1.f / dir.y, 1.f / dir.z);
        for (int c = 0; c < 3; ++c) {
            o[c] = dir[c];
            o[3 + c] = inv[c];
        }
        float u = 0.f, v = 0.f;
        const float t = tri(v3(a), dir, v3(a + 15), v3(a + 18), v3(a + 21), u, v);
        o[6] = t;
        o[7] = t == FLT_MAX ? 0.f : u;
        o[8] = t == FLT_MAX ? 0.f : v;
        const float su = a[33], sv = a[34];
        const float w = 1 - (su + sv);
        const glm::vec3 nn = v3(a + 24) * w + v3(a + 27) * su + v3(a + 30) * sv;
        const glm::vec3 nz = glm::normalize(nn);
        const float r = std::abs(nz.z * 255);
        const uint32_t packed = (r == r ? (uint32_t)r : 0u) << 16;  // NaN: 0, the oracle's convention
        std::memcpy(&o[9], &packed, 4);
        o[10] = nz.z;
    }
    f = std::fopen(argv[2], "wb");
    if (!f) return 1;
    std::fwrite(out.data(), sizeof(float), out.size(), f);
    std::fclose(f);
    return 0;
}
