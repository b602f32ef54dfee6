// bm_kd.hip — reference mode: the reference's own acceleration structure and march on gfx950,
// for frames identical to the reference's on every pixel (the first-hit-leaf early-out included).
//
// The reference (BuildTree.cu:154-256) inserts each triangle into a sparse kd-tree over the fixed
// world box: spatial-median splits cycling x, y, z; a child is descended into when Akenine-Möller's
// triangle/box test (BoxTriangle.cuh:134-222) passes; a node becomes a leaf when its smallest edge
// is below 0.03 or at depth 37 — for the world box [-30,30]³ every leaf sits at depth 31 — and a
// leaf keeps its first 256 faces (BuildTree.cu:36-61). The march (BuildTree.cu:367-499) walks the
// tree near-first by split plane, tests every face of the first leaf that has a hit and stops there.
//
// Built here without pointers or atomics deciding anything:
//   k_kd_descend<count>  one thread per triangle repeats the reference's descent (same boxes, same
//                        SAT arithmetic) and counts the leaves it reaches (the first KD_LEAF_CACHE
//                        kept, so the emit pass copies them instead of descending again);
//   exclusive scan       per-triangle output offsets (triangle id order);
//   k_kd_descend<emit>   writes (leaf path key, triangle id) pairs — a leaf is named by its 31 split
//                        decisions, so the key is the node;
//   stable sort          by key: within a leaf the faces come out in triangle-id order, the order the
//                        reference's serial (CPU) insertion gives, which decides exact-t ties and the
//                        256-face cap;
//   leaves               runs of equal keys (flags + scan);
//   radix tree           Karras over the distinct leaf keys: its internal nodes are exactly the
//                        reference's nodes with two children (depth = common prefix length); the
//                        reference's single-child nodes between them are replayed by the march (box
//                        test of every level), and nodes without leaves below cannot produce a hit.
// Bit-identical to oracle/beam_oracle.c orc_kd_build + orc_kd_march.
#include <cmath>
#include <cstdlib>
#include <vector>

#include "bm_internal.h"

namespace bm {
namespace {

#include "bm_bdiag.h"

constexpr int BLOCK = 256;
constexpr float KD_MIN_LEAF = .03f;  // MIN_LEAF_SIZE, BuildTree.cuh:18
constexpr int KD_MAX_DEPTH = 38;     // BUILD_TREE_MAX_DEPTH, BuildTree.cuh:15
constexpr uint32_t KD_LEAF_CAP = 256;  // MAX_FACES_PER_BOX, BuildTree.cuh:17
constexpr float FLT_MAXF = 3.40282347e+38f;

__device__ __forceinline__ float rmin(float a, float b) { return a < b ? a : b; }
__device__ __forceinline__ float rmax(float a, float b) { return a > b ? a : b; }

// planeBoxOverlap (BoxTriangle.cuh:57-79)
__device__ __forceinline__ bool plane_box(const float* nrm, const float* vert, const float* maxbox) {
    float vmin[3], vmax[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        const float v = vert[q];
        if (nrm[q] > 0.0f) {
            vmin[q] = -maxbox[q] - v;
            vmax[q] = maxbox[q] - v;
        } else {
            vmin[q] = maxbox[q] - v;
            vmax[q] = -maxbox[q] - v;
        }
    }
    // (dot(vmin) > 0 -> false; dot(vmax) >= 0 -> true; else false), as one expression
    return !((nrm[0] * vmin[0] + nrm[1] * vmin[1]) + nrm[2] * vmin[2] > 0.0f) &&
           (nrm[0] * vmax[0] + nrm[1] * vmax[1]) + nrm[2] * vmax[2] >= 0.0f;
}

__device__ __forceinline__ bool axis_sep(float pa, float pb, float rad) {
    float mn, mx;
    if (pa < pb) {
        mn = pa;
        mx = pb;
    } else {
        mn = pb;
        mx = pa;
    }
    return (mn > rad || mx < -rad);
}

// triBoxOverlap (BoxTriangle.cuh:134-222): the nine cross-axis tests (AXISTEST_* order), the AABB
// test (FINDMINMAX) and the plane test, operation for operation.
__device__ bool tri_box_branchy(const float* bc, const float* hs, const float* tv) {
    float v0[3], v1[3], v2[3], e0[3], e1[3], e2[3], nrm[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        v0[c] = tv[c] - bc[c];
        v1[c] = tv[3 + c] - bc[c];
        v2[c] = tv[6 + c] - bc[c];
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        e0[c] = v1[c] - v0[c];
        e1[c] = v2[c] - v1[c];
        e2[c] = v0[c] - v2[c];
    }
    float fx, fy, fz, a, b, pa, pb, rad;
    fx = fabsf(e0[0]); fy = fabsf(e0[1]); fz = fabsf(e0[2]);
    a = e0[2]; b = e0[1];
    pa = a * v0[1] - b * v0[2]; pb = a * v2[1] - b * v2[2];
    rad = fz * hs[1] + fy * hs[2];
    if (axis_sep(pa, pb, rad)) return false;
    a = e0[2]; b = e0[0];
    pa = -a * v0[0] + b * v0[2]; pb = -a * v2[0] + b * v2[2];
    rad = fz * hs[0] + fx * hs[2];
    if (axis_sep(pa, pb, rad)) return false;
    a = e0[1]; b = e0[0];
    pa = a * v1[0] - b * v1[1]; pb = a * v2[0] - b * v2[1];
    rad = fy * hs[0] + fx * hs[1];
    if (axis_sep(pb, pa, rad)) return false;

    fx = fabsf(e1[0]); fy = fabsf(e1[1]); fz = fabsf(e1[2]);
    a = e1[2]; b = e1[1];
    pa = a * v0[1] - b * v0[2]; pb = a * v2[1] - b * v2[2];
    rad = fz * hs[1] + fy * hs[2];
    if (axis_sep(pa, pb, rad)) return false;
    a = e1[2]; b = e1[0];
    pa = -a * v0[0] + b * v0[2]; pb = -a * v2[0] + b * v2[2];
    rad = fz * hs[0] + fx * hs[2];
    if (axis_sep(pa, pb, rad)) return false;
    a = e1[1]; b = e1[0];
    pa = a * v0[0] - b * v0[1]; pb = a * v1[0] - b * v1[1];
    rad = fy * hs[0] + fx * hs[1];
    if (axis_sep(pa, pb, rad)) return false;

    fx = fabsf(e2[0]); fy = fabsf(e2[1]); fz = fabsf(e2[2]);
    a = e2[2]; b = e2[1];
    pa = a * v0[1] - b * v0[2]; pb = a * v1[1] - b * v1[2];
    rad = fz * hs[1] + fy * hs[2];
    if (axis_sep(pa, pb, rad)) return false;
    a = e2[2]; b = e2[0];
    pa = -a * v0[0] + b * v0[2]; pb = -a * v1[0] + b * v1[2];
    rad = fz * hs[0] + fx * hs[2];
    if (axis_sep(pa, pb, rad)) return false;
    a = e2[1]; b = e2[0];
    pa = a * v1[0] - b * v1[1]; pb = a * v2[0] - b * v2[1];
    rad = fy * hs[0] + fx * hs[1];
    if (axis_sep(pb, pa, rad)) return false;

#pragma unroll
    for (int c = 0; c < 3; ++c) {
        float mn = v0[c], mx = v0[c];
        if (v1[c] < mn) mn = v1[c];
        if (v1[c] > mx) mx = v1[c];
        if (v2[c] < mn) mn = v2[c];
        if (v2[c] > mx) mx = v2[c];
        if (mn > hs[c] || mx < -hs[c]) return false;
    }
    nrm[0] = e0[1] * e1[2] - e0[2] * e1[1];
    nrm[1] = e0[2] * e1[0] - e0[0] * e1[2];
    nrm[2] = e0[0] * e1[1] - e0[1] * e1[0];
    return plane_box(nrm, v0, hs);
}

// The same tests without the early returns: every test's arithmetic is the one above (same operands,
// same order, no contraction), and the reference's function has no side effects, so "false at the
// first separating test, else the plane test" equals "no test separates, and the plane test passes".
// Straight-line code: a wave whose lanes separate at different tests no longer runs the union of
// the return paths with their exec-mask saves (the descent walks ran at ~5k cycles per level with
// the branches; -DBM_KD_SAT_FLAT=0 restores them for an A/B).
#ifndef BM_KD_SAT_FLAT
#define BM_KD_SAT_FLAT 1
#endif
// The test groups of tri_box_flat, each with the operations above (same operands, same order).
struct SatFrame {
    float v0[3], v1[3], v2[3], e0[3], e1[3], e2[3];
};
__device__ __forceinline__ void sat_frame(const float* bc, const float* tv, SatFrame& f) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        f.v0[c] = tv[c] - bc[c];
        f.v1[c] = tv[3 + c] - bc[c];
        f.v2[c] = tv[6 + c] - bc[c];
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        f.e0[c] = f.v1[c] - f.v0[c];
        f.e1[c] = f.v2[c] - f.v1[c];
        f.e2[c] = f.v0[c] - f.v2[c];
    }
}
// edge e0's three cross-axis tests (AXISTEST_X01, _Y02, _Z12)
__device__ __forceinline__ bool sat_sep_e0(const SatFrame& f, const float* hs) {
    const float* v0 = f.v0; const float* v1 = f.v1; const float* v2 = f.v2; const float* e0 = f.e0;
    bool sep = false;
    float fx, fy, fz, a, b, pa, pb, rad;
    fx = fabsf(e0[0]); fy = fabsf(e0[1]); fz = fabsf(e0[2]);
    a = e0[2]; b = e0[1];
    pa = a * v0[1] - b * v0[2]; pb = a * v2[1] - b * v2[2];
    rad = fz * hs[1] + fy * hs[2];
    sep |= axis_sep(pa, pb, rad);
    a = e0[2]; b = e0[0];
    pa = -a * v0[0] + b * v0[2]; pb = -a * v2[0] + b * v2[2];
    rad = fz * hs[0] + fx * hs[2];
    sep |= axis_sep(pa, pb, rad);
    a = e0[1]; b = e0[0];
    pa = a * v1[0] - b * v1[1]; pb = a * v2[0] - b * v2[1];
    rad = fy * hs[0] + fx * hs[1];
    sep |= axis_sep(pb, pa, rad);
    return sep;
}
// edge e1's (AXISTEST_X01, _Y02, _Z0)
__device__ __forceinline__ bool sat_sep_e1(const SatFrame& f, const float* hs) {
    const float* v0 = f.v0; const float* v1 = f.v1; const float* v2 = f.v2; const float* e1 = f.e1;
    bool sep = false;
    float fx, fy, fz, a, b, pa, pb, rad;
    fx = fabsf(e1[0]); fy = fabsf(e1[1]); fz = fabsf(e1[2]);
    a = e1[2]; b = e1[1];
    pa = a * v0[1] - b * v0[2]; pb = a * v2[1] - b * v2[2];
    rad = fz * hs[1] + fy * hs[2];
    sep |= axis_sep(pa, pb, rad);
    a = e1[2]; b = e1[0];
    pa = -a * v0[0] + b * v0[2]; pb = -a * v2[0] + b * v2[2];
    rad = fz * hs[0] + fx * hs[2];
    sep |= axis_sep(pa, pb, rad);
    a = e1[1]; b = e1[0];
    pa = a * v0[0] - b * v0[1]; pb = a * v1[0] - b * v1[1];
    rad = fy * hs[0] + fx * hs[1];
    sep |= axis_sep(pa, pb, rad);
    return sep;
}
// edge e2's (AXISTEST_X2, _Y1, _Z12)
__device__ __forceinline__ bool sat_sep_e2(const SatFrame& f, const float* hs) {
    const float* v0 = f.v0; const float* v1 = f.v1; const float* v2 = f.v2; const float* e2 = f.e2;
    bool sep = false;
    float fx, fy, fz, a, b, pa, pb, rad;
    fx = fabsf(e2[0]); fy = fabsf(e2[1]); fz = fabsf(e2[2]);
    a = e2[2]; b = e2[1];
    pa = a * v0[1] - b * v0[2]; pb = a * v1[1] - b * v1[2];
    rad = fz * hs[1] + fy * hs[2];
    sep |= axis_sep(pa, pb, rad);
    a = e2[2]; b = e2[0];
    pa = -a * v0[0] + b * v0[2]; pb = -a * v1[0] + b * v1[2];
    rad = fz * hs[0] + fx * hs[2];
    sep |= axis_sep(pa, pb, rad);
    a = e2[1]; b = e2[0];
    pa = a * v1[0] - b * v1[1]; pb = a * v2[0] - b * v2[1];
    rad = fy * hs[0] + fx * hs[1];
    sep |= axis_sep(pb, pa, rad);
    return sep;
}
// the AABB test (FINDMINMAX per axis)
__device__ __forceinline__ bool sat_sep_box(const SatFrame& f, const float* hs) {
    bool sep = false;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        float mn = f.v0[c], mx = f.v0[c];
        if (f.v1[c] < mn) mn = f.v1[c];
        if (f.v1[c] > mx) mx = f.v1[c];
        if (f.v2[c] < mn) mn = f.v2[c];
        if (f.v2[c] > mx) mx = f.v2[c];
        sep |= (mn > hs[c] || mx < -hs[c]);
    }
    return sep;
}
__device__ __forceinline__ bool sat_plane(const SatFrame& f, const float* hs) {
    float nrm[3];
    nrm[0] = f.e0[1] * f.e1[2] - f.e0[2] * f.e1[1];
    nrm[1] = f.e0[2] * f.e1[0] - f.e0[0] * f.e1[2];
    nrm[2] = f.e0[0] * f.e1[1] - f.e0[1] * f.e1[0];
    return plane_box(nrm, f.v0, hs);
}
__device__ __forceinline__ bool tri_box_flat(const float* bc, const float* hs, const float* tv) {
    SatFrame f;
    sat_frame(bc, tv, f);
    const bool sep = sat_sep_e0(f, hs) | sat_sep_e1(f, hs) | sat_sep_e2(f, hs) | sat_sep_box(f, hs);
    return !sep && sat_plane(f, hs);
}
// tri_box_flat's tests split over two lanes (round 6): half 0 the cross-axis tests of edges e0 and e1,
// half 1 those of e2, the AABB test and the plane test. Every test is the one above, and the function
// is "no test separates and the plane test passes", so (half 0's result) && (half 1's) is its result.
__device__ __forceinline__ bool tri_box_half(const float* bc, const float* hs, const float* tv, bool half) {
    SatFrame f;
    sat_frame(bc, tv, f);
    if (!half) return !(sat_sep_e0(f, hs) | sat_sep_e1(f, hs));
    return !(sat_sep_e2(f, hs) | sat_sep_box(f, hs)) && sat_plane(f, hs);
}

// tri_box_flat for a triangle whose coordinates are all below 2^60 in magnitude (kd_finite; the walks' boxes
// lie in the world box): every intermediate is then finite — |v| < 2^61, |e| < 2^62, each product below
// 2^124 — and for finite operands "a < b ? a : b" and fminf differ at most in the sign of a zero, which no
// comparison sees, so the min/max forms below give tri_box_flat's answer with fewer instructions (round 6).
__device__ __forceinline__ bool axis_sep_finite(float pa, float pb, float rad) {
    return fminf(pa, pb) > rad || fmaxf(pa, pb) < -rad;
}
__device__ __forceinline__ bool tri_box_finite(const float* bc, const float* hs, const float* tv) {
    SatFrame f;
    sat_frame(bc, tv, f);
    const float* v0 = f.v0; const float* v1 = f.v1; const float* v2 = f.v2;
    bool sep = false;
#pragma unroll
    for (int q = 0; q < 3; ++q) {  // edges e0, e1, e2: AXISTEST_X, _Y, _Z with tri_box_flat's vertex pairs
        const float* e = q == 0 ? f.e0 : q == 1 ? f.e1 : f.e2;
        const float* xa = q == 2 ? v0 : v0;
        const float* xb = q == 2 ? v1 : v2;
        const float fx = fabsf(e[0]), fy = fabsf(e[1]), fz = fabsf(e[2]);
        float a = e[2], b = e[1];
        sep |= axis_sep_finite(a * xa[1] - b * xa[2], a * xb[1] - b * xb[2], fz * hs[1] + fy * hs[2]);
        b = e[0];
        sep |= axis_sep_finite(-a * xa[0] + b * xa[2], -a * xb[0] + b * xb[2], fz * hs[0] + fx * hs[2]);
        a = e[1];
        const float* za = q == 1 ? v0 : v1;
        const float* zb = q == 1 ? v1 : v2;
        sep |= axis_sep_finite(a * za[0] - b * za[1], a * zb[0] - b * zb[1], fy * hs[0] + fx * hs[1]);
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float mn = fminf(fminf(v0[c], v1[c]), v2[c]), mx = fmaxf(fmaxf(v0[c], v1[c]), v2[c]);
        sep |= (mn > hs[c] || mx < -hs[c]);
    }
    return !sep && sat_plane(f, hs);
}
// the triangle qualifies for tri_box_finite (NaN fails the compares)
__device__ __forceinline__ bool kd_finite(const float* tv) {
    bool ok = true;
#pragma unroll
    for (int i = 0; i < 9; ++i) ok = ok && fabsf(tv[i]) < 0x1p60f;
    return ok;
}

__device__ __forceinline__ bool tri_box(const float* bc, const float* hs, const float* tv) {
    return BM_KD_SAT_FLAT ? tri_box_flat(bc, hs, tv) : tri_box_branchy(bc, hs, tv);
}

// Exact shortcuts to triBoxOverlap, an A/B experiment (-DBM_KD_SAT_SHORTCUT=1; measured slower,
// DESIGN.md §8): the result equals tri_box for every input.
//  * false when the test's own AABB step separates: tri_box computes v_i = tv_i - bc first and returns
//    false at a cross-axis test or at this step, so the step's verdict (same operations) decides;
//  * true when every |v_i[c]| <= hs[c] (1 - 2^-20): then no test can separate. A cross-axis test
//    compares p = a v[j] - b v[k] with rad = |a| hs[j] + |b| hs[k] (a, b: one edge's components): in
//    float |p| <= (|a||v[j]| + |b||v[k]|)(1 + u)^2 and rad >= (|a| hs[j] + |b| hs[k])(1 - u)^2 (u = 2^-24,
//    nonnegative terms), so the 16u margin keeps |p| <= rad; the AABB step passes outright; and the plane
//    test's dot products sum terms n[q] * (+-hs[q] - v0[q]) whose factors' signs are exact (hs - |v0| >
//    0 stays nonzero under rounding), all <= 0 for vmin and >= 0 for vmax, so it returns true. The bound
//    is relative: edge components must be 0 or at least 2^-100 (no subnormal products against a
//    normal rad), and hs >= 2^-60.
#ifndef BM_KD_SAT_SHORTCUT
#define BM_KD_SAT_SHORTCUT 0
#endif
__device__ __forceinline__ bool normal_or_zero(float e) { return e == 0.0f || fabsf(e) >= 0x1p-100f; }
#ifndef BM_KD_SAT_FINITE
#define BM_KD_SAT_FINITE 1
#endif
__device__ __forceinline__ bool tri_box_fast(const float* bc, const float* hs, const float* tv, bool fin = false) {
    if (BM_KD_SAT_FINITE && fin) return tri_box_finite(bc, hs, tv);
    if (!BM_KD_SAT_SHORTCUT) return tri_box(bc, hs, tv);
    bool sep = false, inside = true;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float a = tv[c] - bc[c], b = tv[3 + c] - bc[c], d = tv[6 + c] - bc[c];
        float mn = a, mx = a;  // FINDMINMAX order (tri_box)
        if (b < mn) mn = b;
        if (b > mx) mx = b;
        if (d < mn) mn = d;
        if (d > mx) mx = d;
        sep = sep || mn > hs[c] || mx < -hs[c];
        const float lim = hs[c] * (1.0f - 0x1p-20f);
        inside = inside && hs[c] >= 0x1p-60f && fabsf(a) <= lim && fabsf(b) <= lim && fabsf(d) <= lim &&
                 normal_or_zero(b - a) && normal_or_zero(d - b) && normal_or_zero(a - d);
    }
    if (sep) return false;
    if (inside) return true;
    return tri_box(bc, hs, tv);
}

// Box of the node reached by following `path` (bit k = right at depth k, MSB first over `depth`
// bits of a leaf_depth-bit key) from the world box, with the reference's halving arithmetic.
__device__ __forceinline__ void path_box(uint32_t key, int depth, int leaf_depth, float wmin, float wmax, float* mn,
                                         float* mx) {
    for (int c = 0; c < 3; ++c) {
        mn[c] = wmin;
        mx[c] = wmax;
    }
    for (int k = 0; k < depth; ++k) {
        const int a = k % 3;
        const float s = .5f * (mn[a] + mx[a]);
        if ((key >> (leaf_depth - 1 - k)) & 1u) mn[a] = s;
        else mx[a] = s;
    }
}

// path_box in closed form: along each axis the node's interval is the idx-th of 2^j equal cells of the
// world interval (idx = the path's bits on that axis). Used only when kd_grid_exact() showed on the host
// that the halving recurrence is exact for this world box (it is for [-30, 30]: every bound is a
// multiple of 60 / 2^11), so the boxes are the recurrence's bit for bit — without its 31 dependent steps.
// Bits 0, 3, ..., 30 of x packed into bits 0..10 (the Morton decode's mask-and-shift steps).
__device__ __forceinline__ uint32_t compact3_11(uint32_t x) {
    x &= 0x49249249u;
    x = (x | (x >> 2)) & 0x430C30C3u;
    x = (x | (x >> 4)) & 0x0700F00Fu;
    x = (x | (x >> 8)) & 0x070000FFu;
    x = (x | (x >> 16)) & 0x7FFu;
    return x;
}
// The cell indices by mask-and-shift instead of a per-level loop (round 6: ~35 instead of ~165 VALU
// instructions per box, and the walks rebuild a box at every pop). With level k's bit at position 32 - k
// of a 33-bit frame, the x levels (k % 3 == 0) sit at positions = 2 mod 3, y at 1, z at 0, so each axis's
// compaction yields its index left-aligned in 11 bits: f = idx << (11 - n) for its n levels. Then
// (float)f * (wext 2^-11) is the same real number as (float)idx * (wext 2^-n) — both factors exact, no
// underflow — so it rounds to the same float as the recurrence's cell bound.
__device__ __forceinline__ void path_box_grid(uint32_t path, int depth, float wmin, float wext, float* mn, float* mx) {
    const unsigned long long frame = (unsigned long long)path << (33 - depth);
    const uint32_t fx = compact3_11((uint32_t)(frame >> 2)), fy = compact3_11((uint32_t)(frame >> 1)),
                   fz = compact3_11((uint32_t)frame);
    const float c11 = ldexpf(wext, -11);
    const float cx = ldexpf(wext, -((depth + 2) / 3)), cy = ldexpf(wext, -((depth + 1) / 3)),
                cz = ldexpf(wext, -(depth / 3));
    mn[0] = wmin + (float)fx * c11;
    mn[1] = wmin + (float)fy * c11;
    mn[2] = wmin + (float)fz * c11;
    mx[0] = mn[0] + cx;
    mx[1] = mn[1] + cy;
    mx[2] = mn[2] + cz;
}

// path_box with the level loop unrolled (axis k % 3 known per level): the box stays in registers.
__device__ __forceinline__ void path_box_unrolled(uint32_t key, int depth, int leaf_depth, float wmin, float wmax,
                                                  float* mn, float* mx) {
    float lo[3] = {wmin, wmin, wmin}, hi[3] = {wmax, wmax, wmax};
#pragma unroll
    for (int k = 0; k < 32; ++k) {
        if (k < depth) {
            const int c = k % 3;
            const float s = .5f * (lo[c] + hi[c]);
            if ((key >> (leaf_depth - 1 - k)) & 1u) lo[c] = s;
            else hi[c] = s;
        }
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        mn[c] = lo[c];
        mx[c] = hi[c];
    }
}

struct DescendEntry {
    uint32_t path;
    int depth;
};

// bmInsertTriangleInTree (BuildTree.cu:154-256) for one triangle: LIFO descent, left pushed before
// right as in the reference; the leaves reached are counted (EMIT=false) or written (EMIT=true).
// The current node's box is carried down incrementally (one halving per level, the reference's own
// arithmetic: the same operations path_box replays from the root) and the descent continues into
// the right child when both pass, with the left one stacked — the reference's pop order. Only a
// stacked node's box is rebuilt from its path (path_box), once per branch instead of once per level.
template <bool EMIT>
__global__ __launch_bounds__(BLOCK) void k_kd_descend(const MeshDesc* __restrict__ meshes, uint32_t nm, uint32_t n,
                                                      float wmin, float wmax, int leaf_depth,
                                                      uint32_t* __restrict__ counts,
                                                      const uint32_t* __restrict__ offsets,
                                                      uint32_t* __restrict__ keys, uint32_t* __restrict__ vals,
                                                      uint32_t* __restrict__ cache) {
    const uint32_t g = blockIdx.x * BLOCK + threadIdx.x;
    if (g >= n) return;
    if (EMIT) {  // the count pass kept the leaves of this triangle: copy them
        const uint32_t cnt = counts[g];
        if (cnt <= KD_LEAF_CACHE) {
            const uint32_t o = offsets[g];
            for (uint32_t i = 0; i < cnt; ++i) {
                keys[o + i] = cache[(size_t)i * n + g];
                vals[o + i] = g;
            }
            return;
        }
    }
    uint32_t a0 = 0, b0 = nm;
    while (b0 - a0 > 1) {
        const uint32_t mid = (a0 + b0) >> 1;
        if (meshes[mid].tri_offset <= g) a0 = mid;
        else b0 = mid;
    }
    const MeshDesc md = meshes[a0];
    const uint32_t f = g - md.tri_offset;
    float tv[9];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const uint32_t vi = md.idx[3 * f + k];
#pragma unroll
        for (int c = 0; c < 3; ++c) tv[3 * k + c] = md.pos[3 * vi + c];
    }
    DescendEntry st[KD_MAX_DEPTH + 2];
    int top = -1;
    uint32_t path = 0, found = 0, out = EMIT ? offsets[g] : 0u;
    int depth = 0, ax = 0;
    float mn[3] = {wmin, wmin, wmin}, mx[3] = {wmax, wmax, wmax};
    for (;;) {
        const float dmin = rmin(mx[0] - mn[0], rmin(mx[1] - mn[1], mx[2] - mn[2]));
        bool next = false;
        if (dmin < KD_MIN_LEAF || depth == KD_MAX_DEPTH - 1) {
            if (EMIT) {
                keys[out] = path;
                vals[out] = g;
                ++out;
            } else if (found < KD_LEAF_CACHE) {
                cache[(size_t)found * n + g] = path;
            }
            ++found;
        } else {
            const float s = .5f * ((ax == 0 ? mn[0] : ax == 1 ? mn[1] : mn[2]) + (ax == 0 ? mx[0] : ax == 1 ? mx[1] : mx[2]));
            float bc[3], hs[3];
#pragma unroll
            for (int c = 0; c < 3; ++c) {  // left child: [mn, mx with mx[ax] = s]
                const float hi = c == ax ? s : mx[c];
                bc[c] = (hi + mn[c]) * .5f;
                hs[c] = (hi - mn[c]) * .5f;
            }
            const bool b1 = tri_box(bc, hs, tv);
#pragma unroll
            for (int c = 0; c < 3; ++c) {  // right child: [mn with mn[ax] = s, mx]
                const float lo = c == ax ? s : mn[c];
                bc[c] = (mx[c] + lo) * .5f;
                hs[c] = (mx[c] - lo) * .5f;
            }
            const bool b2 = tri_box(bc, hs, tv);
            if (b1 && b2) st[++top] = DescendEntry{path << 1, depth + 1};
            if (b1 || b2) {
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    if (c != ax) continue;
                    if (b2) mn[c] = s;
                    else mx[c] = s;
                }
                path = (path << 1) | (b2 ? 1u : 0u);
                ++depth;
                ax = ax == 2 ? 0 : ax + 1;
                next = true;
            }
        }
        if (next) continue;
        if (top < 0) break;
        const DescendEntry e = st[top--];
        path = e.path;
        depth = e.depth;
        ax = depth % 3;
        path_box(path << (leaf_depth - depth), depth, leaf_depth, wmin, wmax, mn, mx);
    }
    if (!EMIT) counts[g] = found;
}

// ---- split descent: the same walk cut at depth `split` so a large triangle's subtrees spread over lanes
// k_kd_descend's cost is the wave's largest triangle (the bunny's base: ≈80 leaves in one lane).
// Phase A (k_kd_top) walks every triangle from the root and queues each node it reaches at depth
// `split` as a (triangle, path) item; phase B (k_kd_sub) walks one queued node per lane to its leaves.
// A leaf is then counted, cached and emitted through per-triangle atomics instead of a lane-local
// counter: a triangle's pairs land in its own output segment in another order, which the stable sort
// by leaf key makes irrelevant (a triangle reaches a leaf once), so the sorted pairs are the same.

__device__ __forceinline__ void load_tri(const MeshDesc* __restrict__ meshes, uint32_t nm, uint32_t g, float* tv) {
    uint32_t a0 = 0, b0 = nm;
    while (b0 - a0 > 1) {
        const uint32_t mid = (a0 + b0) >> 1;
        if (meshes[mid].tri_offset <= g) a0 = mid;
        else b0 = mid;
    }
    const MeshDesc md = meshes[a0];
    const uint32_t f = g - md.tri_offset;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const uint32_t vi = md.idx[3 * f + k];
#pragma unroll
        for (int c = 0; c < 3; ++c) tv[3 * k + c] = md.pos[3 * vi + c];
    }
}

struct KdSplitArgs {
    uint32_t n;
    float wmin, wmax;
    int leaf_depth, split;
    uint32_t* counts;         // count: leaves per triangle (zeroed; atomics)
    const uint32_t* offsets;  // emit: segment start per triangle
    uint32_t* fill;           // emit: pairs written per triangle (zeroed; atomics)
    uint32_t *keys, *vals, *cache;
    uint2* queue;             // (triangle, path) of the nodes at depth `split`
    uint32_t cap;
    uint32_t* qcount;
    int grid_exact;           // path_box_grid == path_box for this world box (kd_grid_exact)
    uint32_t lcap;            // LDS queue items per workgroup (<= KD_LQ_CAP)
    uint32_t* oflow;          // set when a node at depth `split` was walked on instead of queued
    uint32_t* zero_ptr;       // emit pass: words k_kd_sub zero-fills on the side (the pair sort's metadata)
    uint32_t zero_words;
    uint32_t* topmap;         // count pass: map of the queued nodes' top 11 path bits (KdBuild::topmap)
    uint32_t* topcount;       // and the number of its bits set
    uint32_t copy_first;      // emit pass: k_kd_sub's workgroups from this index do k_kd_copy's work (0: none)
};

// GRID (a.grid_exact, decided at launch): the closed form; else the halving recurrence, unrolled
template <bool GRID>
__device__ __forceinline__ void walk_box(const KdSplitArgs& a, uint32_t path, int depth, float* mn, float* mx) {
    if (GRID) path_box_grid(path, depth, a.wmin, a.wmax - a.wmin, mn, mx);
    else path_box_unrolled(path << (a.leaf_depth - depth), depth, a.leaf_depth, a.wmin, a.wmax, mn, mx);
}

__device__ __forceinline__ bool enqueue(uint2* lq, uint32_t* lqn, uint32_t lcap, uint32_t g, uint32_t path) {
    const uint32_t slot = atomicAdd(lqn, 1u);  // the counter may pass lcap: readers clamp it
    if (slot >= lcap) return false;
    lq[slot] = make_uint2(g, path);
    return true;
}

// The walk of k_kd_descend from node (path, depth) of triangle g. With `lq` (phase A) a node reached at
// depth a.split is handed to the block's LDS queue when it has room (else walked on here).
template <bool EMIT>
__device__ __forceinline__ void kd_leaf_write(const KdSplitArgs& a, uint32_t g, uint32_t base, uint32_t ticket,
                                              uint32_t path) {
    if (EMIT) {
        a.keys[base + ticket] = path;
        a.vals[base + ticket] = g;
    } else if (ticket < KD_LEAF_CACHE) {
        a.cache[(size_t)ticket * a.n + g] = path;
    }
}

// The stack lives in LDS (KD_WALK_STACK entries per walk, interleaved: entry i of walk w at st[i * (TB / W)
// + w], the walk's lanes writing the same words), one word per entry: the path with a sentinel bit above it
// (depth = its position).
constexpr int KD_WALK_STACK = 32;
// PAIR: two lanes per walk — the lead lane tests the left child, its partner (lane ^ 1) the right one,
// and each takes the other's answer by a lane swap; both keep the same walk state (so they branch
// together) and only the lead lane writes. Twice the waves, half the SAT work per lane and level.
template <bool PAIR>
__device__ __forceinline__ int pair_swap(int v) {
    return PAIR ? __shfl_xor(v, 1) : v;
}
// Lanes per walk with PAIR (round 6): 2 as above, or 4 — lanes 2c and 2c + 1 of a walk's four test child c
// (c = 0 left, 1 right), each running half of the triangle/box tests (tri_box_half); the halves' answers
// combine by a lane swap inside the pair, the children's by a swap between the pairs. The node visits, tests
// and leaves are the two-lane walk's (GPU tests green with it), but the halves are different code, so a wave
// runs both one after the other: measured slower (bunny kd build 0.32 -> 0.36 ms, merged 1.28 -> 1.88 ms),
// an A/B define only.
#ifndef BM_KD_WALK_LANES
#define BM_KD_WALK_LANES 2
#endif
constexpr uint32_t KD_PW = BM_KD_WALK_LANES;
static_assert(KD_PW == 2 || KD_PW == 4, "lanes per walk: 2 or 4");
template <bool PAIR>
constexpr uint32_t kd_w() { return PAIR ? KD_PW : 1u; }
template <bool PAIR>
__device__ __forceinline__ bool kd_lead() { return !PAIR || (threadIdx.x & (KD_PW - 1u)) == 0u; }
// the walk's lead lane's value on every lane of the walk
template <bool PAIR>
__device__ __forceinline__ int kd_from_lead(int v) {
    if (!PAIR) return v;
    if (KD_PW == 4) return __builtin_amdgcn_mov_dpp(v, 0x00, 0xF, 0xF, false);  // quad_perm [0,0,0,0]
    const int o = __shfl_xor(v, 1);
    return (threadIdx.x & 1u) ? o : v;
}
// Both children's tests of a node (split plane s on axis ax) on the walk's lanes.
template <bool PAIR>
__device__ __forceinline__ void kd_child_tests(const float* mn, const float* mx, int ax, float s, const float* tv,
                                               bool fin, bool& b1, bool& b2) {
    float bc[3], hs[3];
    if (PAIR) {  // left child [mn, mx with mx[ax] = s], right [mn with mn[ax] = s, mx]
        const uint32_t r = threadIdx.x & (KD_PW - 1u);
        const bool right = KD_PW == 4 ? (r >> 1) != 0u : r != 0u;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float lo = (c == ax && right) ? s : mn[c];
            const float up = (c == ax && !right) ? s : mx[c];
            bc[c] = (up + lo) * .5f;
            hs[c] = (up - lo) * .5f;
        }
        int mine, other;
        if (KD_PW == 4) {
            mine = tri_box_half(bc, hs, tv, (r & 1u) != 0u) ? 1 : 0;
            mine &= __builtin_amdgcn_mov_dpp(mine, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]: the other half
            other = __builtin_amdgcn_mov_dpp(mine, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]: the other child
        } else {
            mine = tri_box_fast(bc, hs, tv, fin) ? 1 : 0;
            other = pair_swap<PAIR>(mine);
        }
        b1 = (right ? other : mine) != 0;
        b2 = (right ? mine : other) != 0;
    } else {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float up = c == ax ? s : mx[c];
            bc[c] = (up + mn[c]) * .5f;
            hs[c] = (up - mn[c]) * .5f;
        }
        b1 = tri_box_fast(bc, hs, tv, fin);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float lo = c == ax ? s : mn[c];
            bc[c] = (mx[c] + lo) * .5f;
            hs[c] = (mx[c] - lo) * .5f;
        }
        b2 = tri_box_fast(bc, hs, tv, fin);
    }
}

template <bool EMIT, bool PAIR, int TB, bool GRID>
__device__ __forceinline__ void kd_walk(const KdSplitArgs& a, uint32_t g, const float* tv, uint32_t path, int depth,
                                        uint2* lq, uint32_t* lqn, uint32_t lcap, uint32_t* st) {
    const bool lead = kd_lead<PAIR>();
    const bool fin = kd_finite(tv);
    constexpr uint32_t SW = TB / kd_w<PAIR>();  // stack stride: one column per walk (its lanes write the same words)
    float mn[3], mx[3];
    walk_box<GRID>(a, path, depth, mn, mx);
    int ax = depth % 3;
    int top = -1;
    const uint32_t base = EMIT ? a.offsets[g] : 0u;
    uint32_t ticket = 0, pend_path = 0;
    bool pend = false;
    for (;;) {
        const float dmin = rmin(mx[0] - mn[0], rmin(mx[1] - mn[1], mx[2] - mn[2]));
        const bool leaf = dmin < KD_MIN_LEAF || depth == KD_MAX_DEPTH - 1;
        bool queued = false;
        if (!leaf && lq && depth == a.split) {
            int q = 0;
            if (lead) {
                q = (int)enqueue(lq, lqn, lcap, g, path);
                if (!q) *a.oflow = 1u;  // the queue then misses this subtree: the emit pass walks again
            }
            queued = kd_from_lead<PAIR>(q) != 0;
        }
        bool next = false;
        if (leaf) {
            // the ticket's write waits for the next leaf (or the end): the returning atomic's latency
            // then overlaps the walk instead of stalling it once per leaf
            if (lead) {
                if (pend) kd_leaf_write<EMIT>(a, g, base, ticket, pend_path);
                ticket = atomicAdd((EMIT ? a.fill : a.counts) + g, 1u);
                pend_path = path;
                pend = true;
            }
        } else if (!queued) {
            const float s = .5f * ((ax == 0 ? mn[0] : ax == 1 ? mn[1] : mn[2]) + (ax == 0 ? mx[0] : ax == 1 ? mx[1] : mx[2]));
            bool b1, b2;
            kd_child_tests<PAIR>(mn, mx, ax, s, tv, fin, b1, b2);
            if (b1 && b2) st[(++top) * SW] = (path << 1) | (1u << (depth + 1));
            if (b1 || b2) {
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    if (c != ax) continue;
                    if (b2) mn[c] = s;
                    else mx[c] = s;
                }
                path = (path << 1) | (b2 ? 1u : 0u);
                ++depth;
                ax = ax == 2 ? 0 : ax + 1;
                next = true;
            }
        }
        if (next) continue;
        if (top < 0) break;
        const uint32_t e = st[(top--) * SW];
        depth = 31 - __builtin_clz(e);
        path = e ^ (1u << depth);
        ax = depth % 3;
        walk_box<GRID>(a, path, depth, mn, mx);
    }
    if (pend) kd_leaf_write<EMIT>(a, g, base, ticket, pend_path);
}

// ---- wave-shared work in the descent (round 5) ------------------------------------------------------
// A straddling triangle's walk (both children hit at many levels) set k_kd_top's span: ~100 node visits on
// one lane pair while most pairs of its wave had finished. In a one-wave workgroup the walks now
// share work: a pair that finds both children hit hands the second one to a pair that has nothing left to
// walk (the wave's donation list in LDS — a step donates at most one entry per idle pair, so it never holds
// more entries than the wave has walks), else pushes it on its own stack as kd_walk does. An idle pair takes a donated (triangle
// slot, node) entry and walks it with that triangle's vertices from LDS. The nodes visited, tests made and
// leaves reached are kd_walk's; only which lanes make them changes (a triangle's leaves reach its output
// segment in another order, which the stable sort by leaf key makes irrelevant, as in the split descent).
#ifndef BM_KD_SHARE
#define BM_KD_SHARE 1
#endif
constexpr int KD_SHARE = 64;  // walks per one-wave workgroup (32 lane pairs, or 64 single lanes)
struct KdShare {
    float tv[KD_SHARE][9];
    uint32_t g[KD_SHARE];
    uint2 don[KD_SHARE];  // donated entries: (slot, path | sentinel bit at depth)
};

template <bool EMIT, bool PAIR, bool GRID>
__device__ __forceinline__ void kd_walk_shared(const KdSplitArgs& a, bool have, uint32_t path0, int depth0, uint2* lq,
                                               uint32_t* lqn, uint32_t lcap, uint32_t* st, KdShare& S) {
    constexpr uint32_t W = kd_w<PAIR>();
    constexpr uint32_t SW = 64 / W;  // stack stride: one column per walk (its lanes write the same words)
    const uint32_t lane = threadIdx.x & 63;
    const bool lead = kd_lead<PAIR>();
    const uint32_t lead_lane = lane & ~(W - 1u);
    bool walking = have;
    uint32_t wslot = threadIdx.x / W, g = have ? S.g[wslot] : 0u, path = path0;
    int depth = depth0;
    float tv[9];
#pragma unroll
    for (int q = 0; q < 9; ++q) tv[q] = S.tv[wslot][q];
    bool fin = kd_finite(tv);
    float mn[3], mx[3];
    walk_box<GRID>(a, path, depth, mn, mx);
    int ax = depth % 3;
    int top = -1;
    uint32_t base = (EMIT && walking) ? a.offsets[g] : 0u;
    uint32_t ticket = 0, pend_path = 0;
    bool pend = false;
    uint32_t ndon = 0;  // wave-uniform: entries in S.don
    for (;;) {
        if (ndon) {  // idle pairs take donated entries, the most recent first
            const unsigned long long idle = ballot(lead && !walking);
            const uint32_t r = (uint32_t)__popcll(idle & ((1ull << lane) - 1ull));
            const int takes = (lead && !walking && r < ndon) ? 1 : 0;
            const int take = __shfl(takes, (int)lead_lane);
            const uint32_t ri = (uint32_t)__shfl((int)r, (int)lead_lane);
            const uint32_t nidle = (uint32_t)__popcll(idle);
            if (take) {
                const uint2 e = S.don[ndon - 1 - ri];
                wslot = e.x;
                g = S.g[wslot];
#pragma unroll
                for (int q = 0; q < 9; ++q) tv[q] = S.tv[wslot][q];
                fin = kd_finite(tv);
                depth = 31 - __builtin_clz(e.y);
                path = e.y ^ (1u << depth);
                ax = depth % 3;
                walk_box<GRID>(a, path, depth, mn, mx);
                base = EMIT ? a.offsets[g] : 0u;
                top = -1;
                walking = true;
            }
            ndon -= nidle < ndon ? nidle : ndon;
        }
        if (!ballot(walking)) break;  // nothing walking: every donation was taken (ndon == 0)
        bool want_push = false;
        uint32_t push_e = 0;
        if (walking) {  // one node of kd_walk's loop
            const float dmin = rmin(mx[0] - mn[0], rmin(mx[1] - mn[1], mx[2] - mn[2]));
            const bool leaf = dmin < KD_MIN_LEAF || depth == KD_MAX_DEPTH - 1;
            bool queued = false;
            if (!leaf && lq && depth == a.split) {
                int q = 0;
                if (lead) {
                    q = (int)enqueue(lq, lqn, lcap, g, path);
                    if (!q) *a.oflow = 1u;
                }
                queued = kd_from_lead<PAIR>(q) != 0;
            }
            bool next = false;
            if (leaf) {
                if (lead) {
                    if (pend) kd_leaf_write<EMIT>(a, g, base, ticket, pend_path);
                    ticket = atomicAdd((EMIT ? a.fill : a.counts) + g, 1u);
                    pend_path = path;
                    pend = true;
                }
            } else if (!queued) {
                const float sp = .5f * ((ax == 0 ? mn[0] : ax == 1 ? mn[1] : mn[2]) + (ax == 0 ? mx[0] : ax == 1 ? mx[1] : mx[2]));
                bool b1, b2;
                kd_child_tests<PAIR>(mn, mx, ax, sp, tv, fin, b1, b2);
                if (b1 && b2) {
                    want_push = true;
                    push_e = (path << 1) | (1u << (depth + 1));
                }
                if (b1 || b2) {
#pragma unroll
                    for (int c = 0; c < 3; ++c) {
                        if (c != ax) continue;
                        if (b2) mn[c] = sp;
                        else mx[c] = sp;
                    }
                    path = (path << 1) | (b2 ? 1u : 0u);
                    ++depth;
                    ax = ax == 2 ? 0 : ax + 1;
                    next = true;
                }
            }
            if (!next) {
                if (top >= 0) {
                    const uint32_t e = st[(top--) * SW];
                    depth = 31 - __builtin_clz(e);
                    path = e ^ (1u << depth);
                    ax = depth % 3;
                    walk_box<GRID>(a, path, depth, mn, mx);
                } else {  // this walk is done: its last leaf out, then the pair is idle
                    if (pend) kd_leaf_write<EMIT>(a, g, base, ticket, pend_path);
                    pend = false;
                    walking = false;
                }
            }
        }
        // the second children: to pairs left idle by this step (beyond the entries already listed), else
        // on the pair's own stack
        const unsigned long long idle2 = ballot(lead && !walking);
        const unsigned long long pushers = ballot(lead && want_push);
        const uint32_t ni = (uint32_t)__popcll(idle2), np = (uint32_t)__popcll(pushers);
        const uint32_t avail = ni > ndon ? ni - ndon : 0u;
        const uint32_t p = (uint32_t)__popcll(pushers & ((1ull << lead_lane) - 1ull));
        const bool donate = want_push && p < avail;
        if (donate && lead) S.don[ndon + p] = make_uint2(wslot, push_e);
        if (want_push && !donate) st[(++top) * SW] = push_e;
        ndon += np < avail ? np : avail;
        __builtin_amdgcn_wave_barrier();  // the donations are in LDS before the next step reads them
    }
}

constexpr uint32_t KD_TOP_BITS = 11;  // the pair sort's ranked top digit: path bits of depths 0-10
constexpr uint32_t KD_LQ_CAP = 4 * BLOCK;  // LDS queue items per workgroup of BLOCK lanes (4 per lane)
constexpr int KD_SPLIT_ABOVE_LEAF = 6;     // default split depth = leaf depth - 6 (cells 4x the leaf's per axis)

// Phase A. The LDS queue keeps the global queue's atomics to one per workgroup; a node that finds the LDS
// queue full is walked on by its lane(s), one that finds the global queue full by the flushing lane(s).
// TB lanes per workgroup (64 by default: a one-wave workgroup flushes its queue as soon as its own walks
// end instead of waiting at the barrier for the workgroup's longest walk). Each triangle's leaf counter
// (count pass) or fill counter (emit pass) is zeroed here by its lead lane before any walk of the
// workgroup can reach a leaf (the flush walks only this workgroup's triangles, after the barrier).
template <bool EMIT, bool PAIR, int TB, bool GRID>
__global__ __launch_bounds__(TB) void k_kd_top(const MeshDesc* __restrict__ meshes, uint32_t nm, KdSplitArgs a) {
    BDIAG(9);
    constexpr uint32_t W = kd_w<PAIR>(), LQ = 4 * TB;
    __shared__ uint2 lq[LQ];
    __shared__ uint32_t stk[KD_WALK_STACK * (TB / W)];
    __shared__ uint32_t lqn, gbase;
    __shared__ KdShare S;  // one-wave workgroups (TB 64): round 0's walks share work (kd_walk_shared)
    __shared__ uint32_t s_top[KD_TOPMAP_WORDS];  // count pass: top 11 path bits of this workgroup's queued nodes
    const uint32_t lcap = a.lcap < LQ ? a.lcap : LQ;
    if (threadIdx.x == 0) lqn = 0;
    if (!EMIT && threadIdx.x < KD_TOPMAP_WORDS) s_top[threadIdx.x] = 0u;
    const bool lead = kd_lead<PAIR>();
    const uint32_t g = (blockIdx.x * TB + threadIdx.x) / W;
    if (g < a.n && lead) {
        (EMIT ? a.fill : a.counts)[g] = 0u;
        if (!EMIT && a.fill) a.fill[g] = 0u;  // the emit pass's counters too (its copy then runs beside its walks)
    }
    __syncthreads();
    bool walk = g < a.n;
    if (walk && EMIT) {  // the count pass kept all leaves of this triangle: copy them
        const uint32_t cnt = a.counts[g];
        if (cnt <= KD_LEAF_CACHE) {
            const uint32_t o = a.offsets[g];
            for (uint32_t i = 0; lead && i < cnt; ++i) {
                a.keys[o + i] = a.cache[(size_t)i * a.n + g];
                a.vals[o + i] = g;
            }
            walk = false;
        }
    }
    // One call site of the walk (its code, and the registers it needs, once): round 0 walks this
    // lane's triangle from the root, queueing the nodes at depth `split` in LDS; after the flush of that
    // queue to the global one, the later rounds walk on the items the global queue had no room for.
    uint32_t wg = g, wpath = 0, i = 0, nq = 0;
    int wdepth = 0;
    if constexpr (TB == 64 && BM_KD_SHARE) {  // round 0 with shared work: every lane of the wave takes part
        float tv[9];
        if (walk) load_tri(meshes, nm, g, tv);
        if (lead) {
            S.g[threadIdx.x / W] = g;
#pragma unroll
            for (int q = 0; q < 9; ++q) S.tv[threadIdx.x / W][q] = tv[q];
        }
        __syncthreads();
        BDIAG_MARK(0);
        kd_walk_shared<EMIT, PAIR, GRID>(a, walk, 0u, 0, lq, &lqn, lcap, stk + threadIdx.x / W, S);
        BDIAG_MARK(1);
        walk = false;
    }
    for (bool first = true;; first = false) {
        if (walk) {
            float tv[9];
            load_tri(meshes, nm, wg, tv);
            BDIAG_MARK(first ? 0 : 2);
            kd_walk<EMIT, PAIR, TB, GRID>(a, wg, tv, wpath, wdepth, first ? lq : nullptr, &lqn, lcap,
                                          stk + threadIdx.x / W);
            BDIAG_MARK(first ? 1 : 3);
        }
        if (first) {
            __syncthreads();
            nq = lqn < lcap ? lqn : lcap;
            if (threadIdx.x == 0) gbase = nq ? atomicAdd(a.qcount, nq) : 0u;
            __syncthreads();
            i = threadIdx.x / W;
        }
        walk = false;
        for (; i < nq; i += TB / W) {  // the next queued item: to the global queue, or walked here
            const uint2 it = lq[i];
            const uint32_t j = gbase + i;
            if (j < a.cap) {
                if (lead) {
                    a.queue[j] = it;
                    if (!EMIT && a.topmap) {
                        const uint32_t top = it.y >> (a.split - (int)KD_TOP_BITS);
                        atomicOr(&s_top[top >> 5], 1u << (top & 31u));
                    }
                }
            } else {
                if (lead) *a.oflow = 1u;
                wg = it.x;
                wpath = it.y;
                wdepth = a.split;
                walk = true;
                i += TB / W;
                break;
            }
        }
        if (!walk) break;
    }
    if (!EMIT && a.topmap) {  // the workgroup's map words into the global map; newly set bits counted once
        __syncthreads();
        if (threadIdx.x < KD_TOPMAP_WORDS && s_top[threadIdx.x]) {
            const uint32_t old = atomicOr(&a.topmap[threadIdx.x], s_top[threadIdx.x]);
            const uint32_t fresh = s_top[threadIdx.x] & ~old;
            if (fresh) atomicAdd(a.topcount, (uint32_t)__popc(fresh));
        }
    }
}

// Emit pass when the count pass queued every node at depth `split` (no overflow): triangles with at most
// KD_LEAF_CACHE leaves copy them from the cache; k_kd_sub<true> then re-walks only the queued subtrees of
// the others — no second walk from the root. By default its work runs as extra workgroups of k_kd_sub<true>'s
// launch (BM_KD_FUSE_COPY; the fill counters k_kd_sub<true> bumps are then zeroed by the count pass).
__global__ __launch_bounds__(BLOCK) void k_kd_copy(KdSplitArgs a) {
    BDIAG(12);
    const uint32_t g = blockIdx.x * BLOCK + threadIdx.x;
    if (g >= a.n) return;
    a.fill[g] = 0u;
    const uint32_t cnt = a.counts[g];
    if (cnt > KD_LEAF_CACHE) return;
    const uint32_t o = a.offsets[g];
    for (uint32_t i = 0; i < cnt; ++i) {
        a.keys[o + i] = a.cache[(size_t)i * a.n + g];
        a.vals[o + i] = g;
    }
}

// Phase B: one queued node per lane (pair) — grid-stride over the queue's length, read on the device.
// At least 4 waves per SIMD: the walk sits just above 128 VGPRs without the SLP vectorizer (build.py),
// which would cost a wave per SIMD.
template <bool EMIT, bool PAIR, int TB, bool GRID>
__global__ __launch_bounds__(TB) __attribute__((amdgpu_waves_per_eu(4))) void k_kd_sub(const MeshDesc* __restrict__ meshes, uint32_t nm, KdSplitArgs a) {
    BDIAG(EMIT ? 11 : 10);
    constexpr uint32_t W = kd_w<PAIR>();
    __shared__ uint32_t stk[KD_WALK_STACK * (TB / W)];
    if (EMIT)  // the next kernel's metadata, in place of a fill launch (nothing here reads it)
        for (uint32_t z = blockIdx.x * TB + threadIdx.x; z < a.zero_words; z += gridDim.x * TB) a.zero_ptr[z] = 0u;
    if (EMIT && a.copy_first && blockIdx.x >= a.copy_first) {  // k_kd_copy's work, in the same launch
        const uint32_t g = (blockIdx.x - a.copy_first) * TB + threadIdx.x;
        if (g >= a.n) return;
        const uint32_t cnt = a.counts[g];
        if (cnt > KD_LEAF_CACHE) return;
        const uint32_t o = a.offsets[g];
        for (uint32_t i = 0; i < cnt; ++i) {
            a.keys[o + i] = a.cache[(size_t)i * a.n + g];
            a.vals[o + i] = g;
        }
        return;
    }
    const uint32_t q = *a.qcount < a.cap ? *a.qcount : a.cap;
    const uint32_t stride = (a.copy_first ? a.copy_first : gridDim.x) * (TB / W);
    if constexpr (TB == 64 && BM_KD_SHARE) {  // rounds of one item per pair, the round's walks sharing work
        __shared__ KdShare S;
        const bool lead = kd_lead<PAIR>();
        for (uint32_t i = (blockIdx.x * TB + threadIdx.x) / W;;) {
            uint2 it = make_uint2(0u, 0u);
            bool have = false;
            for (; i < q; i += stride) {
                it = a.queue[i];
                if (EMIT && a.counts[it.x] <= KD_LEAF_CACHE) continue;  // copied from the cache
                have = true;
                i += stride;
                break;
            }
            if (!ballot(have)) break;
            float tv[9];
            if (have) load_tri(meshes, nm, it.x, tv);
            if (lead) {
                S.g[threadIdx.x / W] = it.x;
#pragma unroll
                for (int c = 0; c < 9; ++c) S.tv[threadIdx.x / W][c] = tv[c];
            }
            __syncthreads();
            kd_walk_shared<EMIT, PAIR, GRID>(a, have, it.y, a.split, nullptr, nullptr, 0, stk + threadIdx.x / W, S);
            __syncthreads();
        }
        return;
    }
    for (uint32_t i = (blockIdx.x * TB + threadIdx.x) / W;;) {  // one walk call site, as k_kd_top
        uint2 it = make_uint2(0u, 0u);
        bool walk = false;
        for (; i < q; i += stride) {
            it = a.queue[i];
            if (EMIT && a.counts[it.x] <= KD_LEAF_CACHE) continue;  // copied from the cache (k_kd_copy / k_kd_top)
            walk = true;
            i += stride;
            break;
        }
        if (!walk) break;
        float tv[9];
        load_tri(meshes, nm, it.x, tv);
        kd_walk<EMIT, PAIR, TB, GRID>(a, it.x, tv, it.y, a.split, nullptr, nullptr, 0, stk + threadIdx.x / W);
    }
}

// ---- exclusive scan (u32), one pass: decoupled look-back (Merrill & Garland) ---------------------------
// Round 5: one launch instead of three (block scans, one workgroup over the block sums, add: ~15 us and
// two kernel boundaries per scan on the kd build). A tile of SCAN_BLOCK x 4 values takes a ticket (the
// counter resets itself: its last holder zeroes it), reduces, publishes its aggregate, looks back over its
// predecessors 64 at a time (one wave, one round trip per 64 tiles), publishes its inclusive prefix and
// writes its outputs. Status word per tile (u64): epoch (20 bits) | flag (2) | value (42): a word of
// another call's epoch reads as not ready, so the words need no zero fill between calls (only on
// allocation, bm_api.cpp). Values and the total are exact in 64 bits; the outputs are u32 (the callers
// bound the total: MAX_PAIRS).
constexpr int SCAN_BLOCK = 1024, SCAN_ITEMS = 4, SCAN_TILE = SCAN_BLOCK * SCAN_ITEMS;
constexpr unsigned long long SC_AGG = 1ull << 42, SC_INC = 2ull << 42, SC_VAL = (1ull << 42) - 1;
__device__ __forceinline__ unsigned long long sc_word(uint32_t epoch, unsigned long long flag, unsigned long long v) {
    return ((unsigned long long)epoch << 44) | flag | (v & SC_VAL);
}

__global__ __launch_bounds__(SCAN_BLOCK) void k_scan1(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                       uint32_t n, unsigned long long* __restrict__ status,
                                                       uint32_t* __restrict__ ticket, uint32_t epoch, uint32_t nt,
                                                       uint32_t* __restrict__ total32,
                                                       unsigned long long* __restrict__ total64,
                                                       const uint32_t* __restrict__ run_keys) {
    __shared__ uint32_t s_tile;
    __shared__ unsigned long long s_wsum[SCAN_BLOCK / 64], s_excl;
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
    if (t == 0) {
        const uint32_t k = atomicAdd(ticket, 1u);
        if (k == nt - 1) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // all taken
        s_tile = k;
    }
    __syncthreads();
    const uint32_t tile = s_tile;
    const uint32_t i0 = tile * SCAN_TILE + SCAN_ITEMS * t;
    uint32_t v[SCAN_ITEMS];
    if (run_keys) {  // the values: 1 where a run of equal keys starts (not stored)
        uint32_t k[SCAN_ITEMS];
        if (i0 + SCAN_ITEMS <= n) {
            const uint4 q = *reinterpret_cast<const uint4*>(run_keys + i0);
            k[0] = q.x, k[1] = q.y, k[2] = q.z, k[3] = q.w;
        } else {
#pragma unroll
            for (int j = 0; j < SCAN_ITEMS; ++j) k[j] = i0 + j < n ? run_keys[i0 + j] : 0u;
        }
        const uint32_t prev = (i0 > 0 && i0 - 1 < n) ? run_keys[i0 - 1] : ~k[0];
#pragma unroll
        for (int j = 0; j < SCAN_ITEMS; ++j) v[j] = (i0 + j < n && k[j] != (j ? k[j - 1] : prev)) ? 1u : 0u;
    } else if (i0 + SCAN_ITEMS <= n) {
        const uint4 q = *reinterpret_cast<const uint4*>(in + i0);
        v[0] = q.x;
        v[1] = q.y;
        v[2] = q.z;
        v[3] = q.w;
    } else {
#pragma unroll
        for (int k = 0; k < SCAN_ITEMS; ++k) v[k] = i0 + k < n ? in[i0 + k] : 0u;
    }
    unsigned long long mine = 0;
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; ++k) mine += v[k];
    unsigned long long incl = mine;  // inclusive wave scan of the threads' sums
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long y = __shfl_up(incl, o);
        if (lane >= (uint32_t)o) incl += y;
    }
    if (lane == 63) s_wsum[w] = incl;
    __syncthreads();
    unsigned long long wbase = 0, agg = 0;
#pragma unroll
    for (uint32_t q = 0; q < SCAN_BLOCK / 64; ++q) {
        if (q < w) wbase += s_wsum[q];
        agg += s_wsum[q];
    }
    if (w == 0) {  // publish, look back, publish the inclusive prefix
        if (lane == 0)
            __hip_atomic_store(status + tile, sc_word(epoch, tile == 0 ? SC_INC : SC_AGG, agg), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        unsigned long long excl = 0;
        for (long long j = (long long)tile - 1; j >= 0;) {
            const long long jj = j - (long long)lane;  // lane L reads predecessor j - L
            unsigned long long x = 0;
            if (jj >= 0) x = __hip_atomic_load(status + jj, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const bool mine_ok = jj >= 0 && (uint32_t)(x >> 44) == epoch && (x & (SC_AGG | SC_INC));
            const bool is_inc = mine_ok && (x & SC_INC);
            const unsigned long long incm = ballot(is_inc), okm = ballot(mine_ok || jj < 0);
            // lanes up to the first inclusive one (or all 64) must be ready
            const uint32_t stop = incm ? (uint32_t)__ffsll((long long)incm) - 1 : 63;
            const unsigned long long need = stop == 63 ? ~0ull : ((2ull << stop) - 1);
            if ((okm & need) != need) continue;  // a predecessor not published yet: read again
            unsigned long long add = (lane <= stop && jj >= 0) ? (x & SC_VAL) : 0;
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) add += __shfl_xor(add, o);
            excl += add;
            if (incm) break;
            j -= 64;
        }
        if (lane == 0) {
            if (tile > 0)
                __hip_atomic_store(status + tile, sc_word(epoch, SC_INC, excl + agg), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            s_excl = excl;
            if (tile == nt - 1) {
                *total32 = (uint32_t)(excl + agg);
                if (total64) *total64 = excl + agg;
            }
        }
    }
    __syncthreads();
    uint32_t run = (uint32_t)(s_excl + wbase + incl - mine);
    uint32_t o[SCAN_ITEMS];
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; ++k) {
        o[k] = run;
        run += v[k];
    }
    if (i0 + SCAN_ITEMS <= n) {
        *reinterpret_cast<uint4*>(out + i0) = make_uint4(o[0], o[1], o[2], o[3]);
    } else {
#pragma unroll
        for (int k = 0; k < SCAN_ITEMS; ++k)
            if (i0 + k < n) out[i0 + k] = o[k];
    }
}

// ---- small device -> host readbacks without a stream synchronisation (bm_api.cpp readback) ----------
// Lanes copy the words into pinned, coherent host memory; then, after a system-scope fence, lane 0
// releases the sequence number in word POST_SEQ_WORD, on which the host spins.
__global__ __launch_bounds__(64) void k_post(const uint32_t* __restrict__ a, uint32_t na,
                                             const uint32_t* __restrict__ b, uint32_t nb, uint32_t* host,
                                             uint32_t seq) {
    const uint32_t t = threadIdx.x;
    if (t < na) host[t] = a[t];
    else if (t < na + nb) host[t] = b[t - na];
    __threadfence_system();
    __syncthreads();
    if (t == 0) __hip_atomic_store(host + POST_SEQ_WORD, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---- leaves: runs of equal keys ------------------------------------------------------------------
// nl_dev (when given): the leaf count as the scan left it on the device; nl then only bounds the grid.
__global__ __launch_bounds__(BLOCK) void k_kd_leaf_count(const uint32_t* __restrict__ leaf_start, uint32_t nl,
                                                         uint32_t m, uint32_t* __restrict__ leaf_count,
                                                         const uint32_t* __restrict__ nl_dev) {
    if (nl_dev) nl = *nl_dev <= nl ? *nl_dev : 0u;  // above the capacity: nothing (KD_MAX_LEAVES)
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i < nl) leaf_count[i] = (i + 1 < nl ? leaf_start[i + 1] : m) - leaf_start[i];
}

// flags null: a run starts where the key differs from the previous one (computed here); ubox: zeroed
// (the union words k_kd_records max-reduces into) when given.
__global__ __launch_bounds__(BLOCK) void k_kd_leaves(const uint32_t* __restrict__ keys, uint32_t m,
                                                     const uint32_t* __restrict__ flags,
                                                     const uint32_t* __restrict__ leaf_of,
                                                     uint32_t* __restrict__ leaf_key,
                                                     uint32_t* __restrict__ leaf_start, uint32_t cap,
                                                     uint32_t* __restrict__ ubox, const uint32_t* __restrict__ faces,
                                                     const float4* __restrict__ tri_orig, float4* __restrict__ ftris) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i < 6 && ubox) ubox[i] = 0u;
    if (ftris && i < m) {  // the march's face records (v0|id, e1, e2 of tri_orig) in pair order
        const size_t g = 3 * (size_t)faces[i];
        ftris[3 * (size_t)i + 0] = tri_orig[g + 0];
        ftris[3 * (size_t)i + 1] = tri_orig[g + 1];
        ftris[3 * (size_t)i + 2] = tri_orig[g + 2];
    }
    const bool start = i < m && (flags ? flags[i] != 0u : (i == 0 || keys[i] != keys[i - 1]));
    if (start && leaf_of[i] < cap) {  // leaves beyond the buffers' capacity: not stored
        leaf_key[leaf_of[i]] = keys[i];
        leaf_start[leaf_of[i]] = i;
    }
}

inline uint32_t blocks_for(uint32_t n, uint32_t per) { return (n + per - 1) / per; }

// ---- the march (bmMarchKernel, BuildTree.cu:367-499) ---------------------------------------------
// bmBoxRayIntersect (CudaComon.cuh:158-172), with the reference's _min/_max (second argument on NaN).
__device__ __forceinline__ float kd_box_ray(const float* bmn, const float* bmx, const vec3f o, const vec3f inv) {
    const float t0[3] = {(bmn[0] - o.x) * inv.x, (bmn[1] - o.y) * inv.y, (bmn[2] - o.z) * inv.z};
    const float t1[3] = {(bmx[0] - o.x) * inv.x, (bmx[1] - o.y) * inv.y, (bmx[2] - o.z) * inv.z};
    const float ftmax = rmin(rmax(t0[0], t1[0]), rmin(rmax(t0[1], t1[1]), rmax(t0[2], t1[2])));
    if (ftmax < 0.f) return FLT_MAXF;
    const float ftmin = rmax(rmin(t0[0], t1[0]), rmax(rmin(t0[1], t1[1]), rmin(t0[2], t1[2])));
    const float dist = rmax(0.f, ftmin);
    return (ftmax >= ftmin ? dist : FLT_MAXF);
}

struct KdView {
    const uint4* nodes;     // 2 per internal node (k_kd_records)
    const uint4* leaves;    // 2 per leaf
    const uint32_t* node_key;
    const uint32_t* leaf_key;
    const float4* ftris;    // per (leaf, face) pair, in leaf order: the face's (v0|id, e1, e2) record
    uint32_t num_leaves;
    int leaf_depth;
    float wmin, wmax;
    const uint32_t* ubox;  // union of the leaf cells (k_kd_records), or null
    const uint4* cnodes;   // child-box records (k_kd_records), or null: one-box steps
};

// Union of the leaf cells: a ray whose box test misses it enters no leaf, so the reference's march
// tests no face and ends in a miss. The test is exact: bmBoxRayIntersect is monotone under nesting
// when every 1/dir component is finite (kd_visit), every leaf box lies inside the union, so a miss
// of the union is a miss of every leaf; lanes with an infinite 1/dir component are not culled.
// Reduced by k_kd_records (one block reduction, then six atomics per workgroup).

// Node records of the march: 32 B per node, one visit = one 32-B load. The box is the node's own
// (the reference's box at the node's split depth: the last of its chain of single-child nodes),
// computed here with the reference's halving recurrence:
//   internal node i: (box lo.xyz, lch | split depth << 25) (box hi.xyz, rch)
//   leaf j:          (box lo.xyz, first face)              (box hi.xyz, face count capped at 256)
// (child refs: LEAF_BIT | index < 2^25). node_key[i] = key of node i's first leaf (for lanes that
// replay chains level by level).
// Child-box records (cnodes, 64 B per internal node, the product march's): node i's children's own
// boxes, its split plane and depth —
//   (left box lo.xyz, lch) (left box hi.xyz, rch) (right box lo.xyz, split plane s) (right box hi.xyz, split depth)
// with s = .5f * (hi + lo) of i's own box on axis depth % 3, the value kd_split computes from i's record.
// A march step at node i then tests both children against the ray from one record: a child whose box
// is missed is never visited (the reference's visit of it tests that box and pops on).
// Continue path_box's halving recurrence from a node's box at depth d0 down to depth d1 along `key`:
// a child's box from its parent's (the child's key shares the parent's first d0 bits), bit for bit
// path_box(key, d1) without repeating the parent's levels.
__device__ __forceinline__ void path_box_from(uint32_t key, int d0, int d1, int leaf_depth, float* mn, float* mx) {
    for (int k = d0; k < d1; ++k) {
        const int a = k % 3;
        const float s = .5f * (mn[a] + mx[a]);
        if ((key >> (leaf_depth - 1 - k)) & 1u) mn[a] = s;
        else mx[a] = s;
    }
}

__global__ __launch_bounds__(BLOCK) void k_kd_records(const uint32_t* __restrict__ leaf_key,
                                                      const uint32_t* __restrict__ leaf_start,
                                                      uint32_t* __restrict__ leaf_count, uint32_t m,
                                                      const uint32_t* __restrict__ lch, const uint32_t* __restrict__ rch,
                                                      const uint32_t* __restrict__ first,
                                                      const uint32_t* __restrict__ last, uint32_t nl, int leaf_depth,
                                                      float wmin, float wmax, uint4* __restrict__ nodes,
                                                      uint4* __restrict__ leaves, uint32_t* __restrict__ node_key,
                                                      const uint32_t* __restrict__ nl_dev, uint4* __restrict__ cnodes,
                                                      int grid_exact, uint32_t* __restrict__ ubox,
                                                      uint32_t* __restrict__ post_host, uint32_t post_seq) {
    BDIAG(13);
    if (post_host && blockIdx.x == 0 && threadIdx.x == 0) {  // k_post's readback of the leaf count, folded in:
        post_host[0] = *nl_dev;                               // the count is final before this launch
        __threadfence_system();
        __hip_atomic_store(post_host + POST_SEQ_WORD, post_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (nl_dev) nl = *nl_dev <= nl ? *nl_dev : 0u;
    if (blockIdx.x * BLOCK >= nl) return;  // the whole workgroup past the leaves (the grid is the capacity)
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    float mn[3], mx[3];
    uint32_t v[6] = {0, 0, 0, 0, 0, 0};  // the union of the leaf cells (block max, then atomics)
    if (i < nl) {
        // (grid-exact worlds: the closed form, bit for bit the recurrence without its dependent steps)
        if (grid_exact) path_box_grid(leaf_key[i], leaf_depth, wmin, wmax - wmin, mn, mx);
        else path_box(leaf_key[i], leaf_depth, leaf_depth, wmin, wmax, mn, mx);
        // the leaf's pair count (k_kd_leaf_count's, folded in): up to the next leaf's start, or m
        const uint32_t cnt = (i + 1 < nl ? leaf_start[i + 1] : m) - leaf_start[i];
        leaf_count[i] = cnt;
        leaves[2 * (size_t)i] = make_uint4(__float_as_uint(mn[0]), __float_as_uint(mn[1]), __float_as_uint(mn[2]),
                                           leaf_start[i]);
        leaves[2 * (size_t)i + 1] = make_uint4(__float_as_uint(mx[0]), __float_as_uint(mx[1]),
                                               __float_as_uint(mx[2]), min(cnt, KD_LEAF_CAP));
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            v[c] = bkey_lo(mn[c]);
            v[3 + c] = bkey(mx[c]);
        }
    }
    if (ubox) {  // block max, then six atomics per workgroup (ubox zeroed by k_kd_leaves)
        __shared__ uint32_t red[6][BLOCK / 64];
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            uint32_t x = v[k];
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) x = max(x, (uint32_t)__shfl_xor((int)x, o));
            if (lane == 0) red[k][w] = x;
        }
        __syncthreads();
        if (threadIdx.x < 6) {
            uint32_t x = 0;
            for (int j = 0; j < BLOCK / 64; ++j) x = max(x, red[threadIdx.x][j]);
            atomicMax(&ubox[threadIdx.x], x);
        }
    }
    if (i + 1 < nl) {
        const uint32_t k0 = leaf_key[first[i]], k1 = leaf_key[last[i]];
        const uint32_t split = (uint32_t)__clz((int)((k0 ^ k1) << (32 - leaf_depth)));
        if (grid_exact) path_box_grid(split ? k0 >> (leaf_depth - (int)split) : 0u, (int)split, wmin, wmax - wmin, mn, mx);
        else path_box(k0, (int)split, leaf_depth, wmin, wmax, mn, mx);
        nodes[2 * (size_t)i] = make_uint4(__float_as_uint(mn[0]), __float_as_uint(mn[1]), __float_as_uint(mn[2]),
                                          lch[i] | (split << 25));
        nodes[2 * (size_t)i + 1] = make_uint4(__float_as_uint(mx[0]), __float_as_uint(mx[1]),
                                              __float_as_uint(mx[2]), rch[i]);
        node_key[i] = k0;
        if (cnodes) {
            const int a = (int)(split % 3u);
            const float sp = .5f * (mx[a] + mn[a]);
            // Karras split g: the left child covers [first, g], the right [g + 1, last]
            const uint32_t lc = lch[i], rc = rch[i], g = lc & ~LEAF_BIT;
            const uint32_t kg = leaf_key[g], kg1 = leaf_key[g + 1];
            const int sh = 32 - leaf_depth;
            const int dl = (lc & LEAF_BIT) ? leaf_depth : (int)(uint32_t)__clz((int)((k0 ^ kg) << sh));
            const int dr = (rc & LEAF_BIT) ? leaf_depth : (int)(uint32_t)__clz((int)((kg1 ^ k1) << sh));
            float lmn[3] = {mn[0], mn[1], mn[2]}, lmx[3] = {mx[0], mx[1], mx[2]};
            float rmn[3] = {mn[0], mn[1], mn[2]}, rmx[3] = {mx[0], mx[1], mx[2]};
            path_box_from(k0, (int)split, dl, leaf_depth, lmn, lmx);
            path_box_from(kg1, (int)split, dr, leaf_depth, rmn, rmx);
            uint4* c = cnodes + 4 * (size_t)i;
            c[0] = make_uint4(__float_as_uint(lmn[0]), __float_as_uint(lmn[1]), __float_as_uint(lmn[2]), lc);
            c[1] = make_uint4(__float_as_uint(lmx[0]), __float_as_uint(lmx[1]), __float_as_uint(lmx[2]), rc);
            c[2] = make_uint4(__float_as_uint(rmn[0]), __float_as_uint(rmn[1]), __float_as_uint(rmn[2]),
                              __float_as_uint(sp));
            c[3] = make_uint4(__float_as_uint(rmx[0]), __float_as_uint(rmx[1]), __float_as_uint(rmx[2]), split);
        }
    }
}

// The march (bmMarchKernel, BuildTree.cu:367-499), one lane per pixel, 8x8 pixels per wave.
// Traversal order is the reference's: at a node the far child is pushed and the near child taken
// next (the reference pushes both and pops the near one at once); a Karras node stands for the chain
// of the reference's single-child nodes above its split, each box-tested in turn on the way down.
// The stack lives in LDS (32 entries per lane: at most one push per Karras level, leaf_depth <= 31),
// one u32 per entry: leaf bit | depth << 25 | node index.
constexpr int KD_STACK = 32;
constexpr uint32_t KD_DEPTH_SHIFT = 25, KD_INDEX_MASK = (1u << 25) - 1u;

// bmBoxRayIntersect with hardware min/max: equal to kd_box_ray whenever no slab term is NaN (the
// ternaries differ from v_min/v_max only on NaN operands and in the sign of a zero, which no caller's
// decision sees: every comparison treats -0 == +0 and pp = eye + (+-0) * dir compares alike).
__device__ __forceinline__ float kd_box_ray_fast(const uint4 r0, const uint4 r1, const vec3f o, const vec3f inv) {
    const float tx0 = (__uint_as_float(r0.x) - o.x) * inv.x, tx1 = (__uint_as_float(r1.x) - o.x) * inv.x;
    const float ty0 = (__uint_as_float(r0.y) - o.y) * inv.y, ty1 = (__uint_as_float(r1.y) - o.y) * inv.y;
    const float tz0 = (__uint_as_float(r0.z) - o.z) * inv.z, tz1 = (__uint_as_float(r1.z) - o.z) * inv.z;
    const float ftmax = fminf(fmaxf(tx0, tx1), fminf(fmaxf(ty0, ty1), fmaxf(tz0, tz1)));
    const float ftmin = fmaxf(fminf(tx0, tx1), fmaxf(fminf(ty0, ty1), fminf(tz0, tz1)));
    return (ftmax < 0.f || !(ftmax >= ftmin)) ? FLT_MAXF : fmaxf(0.f, ftmin);
}

// Does the ray's box test miss the union of the leaf cells (exact cull, k_kd_records' union)?
__device__ __forceinline__ bool kd_culled(const KdView& kv, bool exact_chain, const vec3f eye, const vec3f inv) {
    if (!kv.ubox || exact_chain) return false;
    const uint4 lo = make_uint4(__float_as_uint(bounds_lo(kv.ubox[0])), __float_as_uint(bounds_lo(kv.ubox[1])),
                                __float_as_uint(bounds_lo(kv.ubox[2])), 0u);
    const uint4 hi = make_uint4(__float_as_uint(bounds_hi(kv.ubox[3])), __float_as_uint(bounds_hi(kv.ubox[4])),
                                __float_as_uint(bounds_hi(kv.ubox[5])), 0u);
    return kd_box_ray_fast(lo, hi, eye, inv) == FLT_MAXF;
}

// One node visit: the node's record (r0, r1) and the entry distance of its box, FLT_MAXF when the
// ray misses it or any box of its chain of single-child nodes. Chains in one test: the reference
// box-tests each node of a chain in turn and stops at the first miss; chain boxes are nested, and
// bmBoxRayIntersect is monotone under nesting when no slab term can be NaN (every 1/dir component
// finite: (b - o) * inv is then finite or +-inf, and rounding preserves the order of nested
// planes), so the innermost box passes iff every box of the chain does. A lane whose 1/dir has an
// infinite component (a zero or denormal direction component: 0 * inf = NaN terms are possible)
// replays the chain level by level from `dep`, exactly as the reference does.
__device__ __forceinline__ float kd_visit(const KdView& kv, uint32_t ref, int dep, bool exact_chain, const vec3f eye,
                                          const vec3f inv, uint4& r0, uint4& r1) {
    const bool leaf = (ref & LEAF_BIT) != 0;
    const uint32_t idx = ref & ~LEAF_BIT;
    const uint4* rp = (leaf ? kv.leaves : kv.nodes) + 2 * (size_t)idx;
    r0 = rp[0];
    r1 = rp[1];
    if (!exact_chain) return kd_box_ray_fast(r0, r1, eye, inv);
    const uint32_t key = leaf ? kv.leaf_key[idx] : kv.node_key[idx];
    const int target = leaf ? kv.leaf_depth : (int)((r0.w >> KD_DEPTH_SHIFT) & 63u);
    float mn[3], mx[3];
    path_box(key, dep, kv.leaf_depth, kv.wmin, kv.wmax, mn, mx);
    float box = kd_box_ray(mn, mx, eye, inv);
    for (int d2 = dep; box != FLT_MAXF && d2 < target; ++d2) {
        const int a = d2 % 3;
        const float s = .5f * (mx[a] + mn[a]);
        if ((key >> (kv.leaf_depth - 1 - d2)) & 1u) mn[a] = s;
        else mx[a] = s;
        box = kd_box_ray(mn, mx, eye, inv);
    }
    return box;
}

// Internal node split: the near child is taken next, the far child pushed (depth target + 1).
__device__ __forceinline__ void kd_split(const uint4 r0, const uint4 r1, float box, const float* eyea,
                                         const float* dira, uint32_t& nearc, uint32_t& farc, int& target) {
    target = (int)((r0.w >> KD_DEPTH_SHIFT) & 63u);
    const int a = target % 3;
    const float lo = __uint_as_float(a == 0 ? r0.x : a == 1 ? r0.y : r0.z);
    const float hi = __uint_as_float(a == 0 ? r1.x : a == 1 ? r1.y : r1.z);
    const float s = .5f * (hi + lo);
    const float pp = eyea[a] + box * dira[a];
    const uint32_t lc = r0.w & ~(63u << KD_DEPTH_SHIFT), rc = r1.w;
    nearc = pp < s ? lc : rc;
    farc = pp < s ? rc : lc;
}

// TB = 256: 16x16 pixels per workgroup (four 8x8 waves); TB = 64: one 8x8 wave per workgroup, so a
// finished wave frees its LDS stack at once instead of waiting for its slowest neighbour.
// COUNT: node records visited, face tests and hits into p.counters[0..2]; DIAG (TB = 64): per wave
// s_memrealtime at start and end, (XCC id << 32 | HW_ID), the lane-max of visits + face tests.
template <int TB, bool COUNT = false, bool DIAG = false>
__global__ __launch_bounds__(TB) void k_kd_march(const TraceParams p, const KdView kv) {
    __shared__ uint32_t stack[KD_STACK * TB];
    const uint64_t t_start = DIAG ? __builtin_amdgcn_s_memrealtime() : 0;
    uint32_t c_nodes = 0, c_faces = 0;
    constexpr int BLOCK = TB;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const uint32_t x = TB == 256 ? blockIdx.x * 16 + (w & 1) * 8 + (lane & 7) : blockIdx.x * 8 + (lane & 7);
    const uint32_t y = TB == 256 ? blockIdx.y * 16 + (w >> 1) * 8 + (lane >> 3) : blockIdx.y * 8 + (lane >> 3);
    const bool inside = x < p.width && y < p.height;
    if (!DIAG && !inside) return;
    // Camera::setInitialRays for this pixel (Camera.cpp:61-66), dir = orient * ray
    const float rx = p.rx[inside ? x : 0], ry = p.ry[inside ? y : 0];
    const float d = 1.f / sqrtf(p.z2 + rx * rx + ry * ry);
    const vec3f r = v3(rx * d, ry * d, p.zoom * d);
    const float* m = p.orient;
    const vec3f dir = v3((m[0] * r.x + m[3] * r.y) + m[6] * r.z, (m[1] * r.x + m[4] * r.y) + m[7] * r.z,
                         (m[2] * r.x + m[5] * r.y) + m[8] * r.z);
    const vec3f inv = v3(1.f / dir.x, 1.f / dir.y, 1.f / dir.z);
    const vec3f eye = v3(p.eye[0], p.eye[1], p.eye[2]);
    const float eyea[3] = {eye.x, eye.y, eye.z}, dira[3] = {dir.x, dir.y, dir.z};

    float dclosest = FLT_MAXF, tu = 0.f, tvv = 0.f;
    uint32_t fclosest = NO_TRI;
    // Single-child chains in one test. The reference box-tests each node of a chain of single-child
    // nodes in turn and stops at the first miss; only the outcome and the last box's entry distance
    // matter. Chain boxes are nested, and bmBoxRayIntersect is monotone under nesting when no slab
    // term can be NaN (every 1/dir component finite: then (b - o) * inv is finite or +-inf, and
    // rounding preserves the order of nested planes), so the innermost box passes iff every box of
    // the chain does: one test of the node's own box decides. A lane whose 1/dir has an infinite
    // component (a zero or denormal direction component: 0 * inf = NaN terms are possible) replays
    // the chain level by level exactly as the reference does.
    const bool exact_chain = !(fabsf(inv.x) <= FLT_MAXF && fabsf(inv.y) <= FLT_MAXF && fabsf(inv.z) <= FLT_MAXF);
    int top = 0;  // entries in this lane's LDS stack
    // the counting builds march every ray (their counters are the reference algorithm's work)
    bool have = kv.num_leaves > 0 && inside && (COUNT || !kd_culled(kv, exact_chain, eye, inv));
    uint32_t ref = kv.num_leaves == 1 ? LEAF_BIT : 0u;
    int dep = 0;  // depth at which the current node's chain starts
    while (have) {
        const bool leaf = (ref & LEAF_BIT) != 0;
        if (COUNT) ++c_nodes;
        uint4 r0, r1;
        const float box = kd_visit(kv, ref, dep, exact_chain, eye, inv, r0, r1);
        bool next_from_stack = true;
        if (box != FLT_MAXF) {
            if (leaf) {
                const uint32_t cnt = r1.w, start = r0.w;
                if (COUNT) c_faces += cnt;
                const float4* ft = kv.ftris + 3 * (size_t)start;
                // the leaf's face records are contiguous: the next face's loads go out before this
                // face's test (no dependent id load, one face in flight ahead)
                float4 na = make_float4(0.f, 0.f, 0.f, 0.f), nb = na, nc = na;
                if (cnt) {
                    na = ft[0];
                    nb = ft[1];
                    nc = ft[2];
                }
                for (uint32_t k = 0; k < cnt; ++k) {
                    const float4 ta = na, tb = nb, tc = nc;
                    if (k + 1 < cnt) {
                        na = ft[3 * k + 3];
                        nb = ft[3 * k + 4];
                        nc = ft[3 * k + 5];
                    }
                    // bmTriIntersect (CudaComon.cuh:117-155) with the exact-safe early reject
                    float t, u, v;
                    if (tri_test(ta, tb, tc, eye, dir, t, u, v) && t < dclosest) {
                        dclosest = t;
                        fclosest = __float_as_uint(ta.w);
                        tu = u;
                        tvv = v;
                    }
                }
                if (dclosest != FLT_MAXF) break;  // first leaf with a hit ends the march (:427-431)
            } else {
                // split plane of this node (its box is the chain's last): push the far child, take
                // the near one, which the reference pops next
                uint32_t nearc, farc;
                int target;
                kd_split(r0, r1, box, eyea, dira, nearc, farc, target);
                stack[top * BLOCK + tid] = (farc & LEAF_BIT) | ((uint32_t)(target + 1) << KD_DEPTH_SHIFT) |
                                           (farc & KD_INDEX_MASK);
                ++top;
                dep = target + 1;
                ref = nearc;
                next_from_stack = false;
            }
        }
        if (next_from_stack) {
            if (top == 0) break;
            const uint32_t e = stack[--top * BLOCK + tid];
            ref = (e & LEAF_BIT) | (e & KD_INDEX_MASK);
            dep = (int)((e >> KD_DEPTH_SHIFT) & 63u);
        }
    }
    const size_t o = (size_t)y * p.width + x;
    uint32_t packed = MISS_PACKED;
    float nzv = 0.0f, tout = __builtin_inff();
    if (fclosest != NO_TRI) {
        const float* n = p.nrm + 9 * (size_t)fclosest;
        const float ww = 1.f - (tu + tvv);
        const vec3f nn = v3((n[0] * ww + n[3] * tu) + n[6] * tvv, (n[1] * ww + n[4] * tu) + n[7] * tvv,
                            (n[2] * ww + n[5] * tu) + n[8] * tvv);
        const float il = 1.f / sqrtf(dot(nn, nn));
        const float z = nn.z * il;
        const float rr = fabsf(z * 255.f);
        packed = ((rr == rr) ? (uint32_t)rr : 0u) << 16;
        nzv = fabsf(z);
        tout = dclosest;
    }
    if (inside) {
        p.packed[(size_t)y * p.pitch_u32 + x] = packed;
        p.tri_id[o] = fclosest;
        p.t[o] = tout;
        if (p.nz) p.nz[o] = nzv;
    }
    if (COUNT && !DIAG) {  // (a diagnostic trace reports per-wave work; 3 same-address atomics per wave
                           // would serialise its timeline)
        unsigned long long a = c_nodes, b = c_faces, h = fclosest != NO_TRI ? 1u : 0u;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            a += __shfl_xor(a, off);
            b += __shfl_xor(b, off);
            h += __shfl_xor(h, off);
        }
        if (lane == 0) {
            atomicAdd(p.counters + 0, a);
            atomicAdd(p.counters + 1, b);
            atomicAdd(p.counters + 2, h);
        }
    }
    if (DIAG) {
        uint32_t wl = c_nodes + c_faces;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) wl = max(wl, (uint32_t)__shfl_xor((int)wl, off));
        const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
        if (lane == 0) {
            const uint32_t hwid = __builtin_amdgcn_s_getreg((31 << 11) | 4);
            const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);
            const size_t wv = (size_t)blockIdx.y * gridDim.x + blockIdx.x;
            p.diag[4 * wv + 0] = t_start;
            p.diag[4 * wv + 1] = t_end;
            p.diag[4 * wv + 2] = ((uint64_t)xcc << 32) | hwid;
            p.diag[4 * wv + 3] = wl;
        }
    }
}

// The march with wave-cooperative leaves (the default). Per lane the traversal is the one above;
// what changes is who tests a leaf's faces. A lane whose ray enters a leaf records it (below: and may
// walk on) while the others keep traversing; then the wave tests every recorded leaf's faces together:
// the faces are laid end to end (prefix sum of the lanes' counts), each lane takes every 64th face, finds
// its owner lane by a binary search over the prefix sums in LDS and the owner's leaf among its recorded
// ones by shuffles, and tests the face against the owner's ray. Each owner keeps the reference's winner —
// in its first recorded leaf with a hit, the smallest t < FLT_MAX, the earliest face among equal t (the
// sequential `d < dClosest` scan of BuildTree.cu:411-425 from dClosest = FLT_MAX; -0 counts as +0, NaN
// never wins) — through a 64-bit LDS atomic min of (leaf, orderable t, face index), and recomputes that
// face's u, v. A leaf of 256 faces costs four wave steps instead of 256 lane steps.
constexpr uint32_t KD_TRAVERSE = 0, KD_PENDING = 1, KD_DONE = 2;

// The wave body of the cooperative march for the pixel (x, y) of each lane (inside = the lane has a
// pixel): ray setup, traversal, the wave-wide leaf rounds, and the pixel's framebuffer entries.
struct KdCoopLds {
    uint32_t stack[KD_STACK * 64];
    float4 sdir[64];
    uint32_t sincl[64];  // inclusive prefix sums of the lanes' recorded face counts
    unsigned long long sbest[64];
};

// Camera::setInitialRays for pixel (x, y) (Camera.cpp:61-66), dir = orient * ray: the march's exact
// ray setup.
__device__ __forceinline__ vec3f kd_ray_dir(const TraceParams& p, uint32_t x, uint32_t y, bool inside) {
    const float rx = p.rx[inside ? x : 0], ry = p.ry[inside ? y : 0];
    const float d = 1.f / sqrtf(p.z2 + rx * rx + ry * ry);
    const vec3f r = v3(rx * d, ry * d, p.zoom * d);
    const float* m = p.orient;
    return v3((m[0] * r.x + m[3] * r.y) + m[6] * r.z, (m[1] * r.x + m[4] * r.y) + m[7] * r.z,
              (m[2] * r.x + m[5] * r.y) + m[8] * r.z);
}

// Speculative leaves (K > 1, product traces). A lane that enters a leaf records it — up to K per lane, in
// the order the reference's march visits them — and, while another lane of the wave still walks with
// nothing recorded (the wave steps for that lane anyway), walks on past it instead of idling. The wave
// tests the recorded leaves once no walking lane is without one: per lane, the first recorded leaf with
// a hit decides — the leaf the reference's march stops at (:427-431), since the leaves are recorded in
// its visiting order and a leaf without a hit changes nothing — and the walk past it is dropped; a lane
// none of whose leaves hit walks on from where it got. Grazing rays reach their leaves at different
// times, and with one leaf per lane a wave ran a leaf round per lane-leaf, every other lane idle through
// each walk in between (C2's heaviest wave: 702 loop iterations where its longest lane needs 213; the
// oracle model in tools/kd_iters.py). K = 1 is the plain form: counting traces, whose counters are the
// reference's work. A round tests each lane's first recorded leaf only (BM_KD_ROUND_FIRST): testing all
// of them spent face tests on leaves behind the first hit (filled view 1.67 -> 1.59 ms, C5 1.02 ->
// 0.95 ms); with that, K = 4 (C2 0.293 -> 0.272 ms) was where more recorded leaves stopped paying. With the
// rounds' LDS chains gone (ballot owners, DPP prefix) K = 6 is a little better again (C2 0.211 -> 0.207 ms,
// C5 0.637 -> 0.617; K = 8 between).
#ifndef BM_KD_SPEC
#define BM_KD_SPEC 6
#endif
#ifndef BM_KD_CB
#define BM_KD_CB 1  // 0: child-box steps compiled out (A/B builds)
#endif
#ifndef BM_KD_STEPS
#define BM_KD_STEPS 4  // child-box visits per loop iteration for a lane that keeps descending (1/2/3/4/8: C2 0.237/0.217/0.212/0.210/0.220 ms)
#endif
#ifndef BM_KD_DPP_SCAN
#define BM_KD_DPP_SCAN 1  // leaf rounds: the face-count prefix by DPP row shifts and broadcasts (0: shuffles)
#endif
#ifndef BM_KD_OWNER_BALLOT
#define BM_KD_OWNER_BALLOT 1  // leaf rounds: face-slot owners by window ballots (0: binary search per slot)
#endif
#ifndef BM_KD_ROUND_FIRST
#define BM_KD_ROUND_FIRST 1  // a leaf round tests each lane's first recorded leaf only (0: all of them)
#endif
#ifndef BM_KD_XCD
#define BM_KD_XCD 4  // tile columns per XCD run (k_kd_march_coop; 0: screen order)
#endif
constexpr int KD_SPEC = BM_KD_SPEC;
static_assert(KD_SPEC >= 1 && KD_SPEC <= 8, "recorded leaves per lane");

template <bool COUNT, int K, bool CB>
__device__ __forceinline__ void kd_coop_wave(const TraceParams& p, const KdView& kv, KdCoopLds& L, uint32_t x,
                                             uint32_t y, bool inside, uint32_t& c_nodes,
                                             uint32_t& c_faces, bool& hit, uint32_t& iters, uint32_t& rounds,
                                             uint64_t& round_ticks) {
    const int lane = threadIdx.x & 63;
    uint32_t* stack = L.stack;
    const vec3f dir = kd_ray_dir(p, x, y, inside);
    const vec3f inv = v3(1.f / dir.x, 1.f / dir.y, 1.f / dir.z);
    const vec3f eye = v3(p.eye[0], p.eye[1], p.eye[2]);
    const float eyea[3] = {eye.x, eye.y, eye.z}, dira[3] = {dir.x, dir.y, dir.z};
    L.sdir[lane] = make_float4(dir.x, dir.y, dir.z, 0.f);
    // see k_kd_march: one box test per Karras node unless 1/dir has an infinite component
    const bool exact_chain = !(fabsf(inv.x) <= FLT_MAXF && fabsf(inv.y) <= FLT_MAXF && fabsf(inv.z) <= FLT_MAXF);
    float dclosest = FLT_MAXF, tu = 0.f, tvv = 0.f;
    uint32_t fclosest = NO_TRI;
    int top = 0;
    // a ray that misses the union of the leaf cells ends in a miss (kd_culled; not in counting traces,
    // whose counters are the reference algorithm's work — a diagnostic trace culls as the product does)
    uint32_t state = (kv.num_leaves > 0 && inside && ((COUNT && !p.diag) || !kd_culled(kv, exact_chain, eye, inv)))
                         ? KD_TRAVERSE
                         : KD_DONE;
    uint32_t ref = kv.num_leaves == 1 ? LEAF_BIT : 0u;
    int dep = 0;
    // recorded leaves: first face record and the inclusive prefix of their face counts; PENDING = waiting
    // for the round (K recorded, or the walk over); walked = the walk is over
    uint32_t np = 0, pst[K], pin[K];
#pragma unroll
    for (int k = 0; k < K; ++k) pst[k] = pin[k] = 0u;
    bool walked = false;
    // Child-box steps (CB, kv.cnodes): the lane stands at an internal node whose box it hits (entry
    // distance dnext; need_own: recompute it from the node's own record, after a pop) and tests both
    // children from the node's child-box record; children it misses are never visited. Its stack holds
    // plain refs of children whose boxes it hits: a popped leaf is recorded without a load, a popped
    // node visited. Recorded leaves are leaf indices until the round. Lanes with an infinite 1/dir
    // component replay chains (kd_visit) and keep the one-box steps.
    const bool cbl = CB && kv.cnodes != nullptr && kv.num_leaves > 1 && !exact_chain;
    bool need_own = true, need_pop = false;
    float dnext = 0.f;
    auto record = [&](uint32_t a, uint32_t c) {  // (register arrays: indexed by unrolled selects only)
        uint32_t prev = 0;
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (k + 1 == (int)np) prev = pin[k];
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (k == (int)np) {
                pst[k] = a;
                pin[k] = prev + c;
            }
        ++np;
    };
    for (;;) {
        ++iters;
        if (ballot(state == KD_TRAVERSE && np == 0)) {
            if (CB && cbl && state == KD_TRAVERSE) {  // one child-box step
                if (need_pop) {  // pop to the next node to visit, recording the leaves on the way
                    for (;;) {
                        if (np == (uint32_t)K || top == 0) break;
                        const uint32_t e = stack[--top * 64 + lane];
                        if (e & LEAF_BIT) {
                            record(e & ~LEAF_BIT, 0u);
                        } else {
                            ref = e;
                            need_own = true;
                            need_pop = false;
                            break;
                        }
                    }
                }
                // (BM_KD_STEPS) a lane that descends into an internal child visits it in the same
                // iteration: one loop pass (ballot, state checks, pop test) per BM_KD_STEPS levels
#pragma unroll 1
                for (int step = 0; step < BM_KD_STEPS && !need_pop; ++step) {
                    if (COUNT) ++c_nodes;
                    const uint4* cp = kv.cnodes + 4 * (size_t)ref;
                    const uint4 c0 = cp[0], c1 = cp[1], c2 = cp[2], c3 = cp[3];
                    float d = dnext;
                    if (need_own) d = kd_box_ray_fast(kv.nodes[2 * (size_t)ref], kv.nodes[2 * (size_t)ref + 1], eye, inv);
                    need_pop = true;
                    if (d != FLT_MAXF) {  // (only the root can miss here: children are pushed on a hit)
                        // kd_split: near child by the entry point against the split plane
                        const int a = (int)(c3.w % 3u);
                        const bool lnear = eyea[a] + d * dira[a] < __uint_as_float(c2.w);
                        const float dl = kd_box_ray_fast(c0, c1, eye, inv), dr = kd_box_ray_fast(c2, c3, eye, inv);
                        const uint32_t nref = lnear ? c0.w : c1.w, fref = lnear ? c1.w : c0.w;
                        const float dn = lnear ? dl : dr, df = lnear ? dr : dl;
                        if (df != FLT_MAXF) {
                            stack[top * 64 + lane] = fref;
                            ++top;
                        }
                        if (dn != FLT_MAXF) {
                            if (nref & LEAF_BIT) {
                                record(nref & ~LEAF_BIT, 0u);
                            } else {
                                ref = nref;
                                dnext = dn;
                                need_own = false;
                                need_pop = false;
                            }
                        }
                    }
                }
                if (need_pop && top == 0) walked = true;
                if (walked) state = np ? KD_PENDING : KD_DONE;
                else if (np == (uint32_t)K) state = KD_PENDING;
            } else if (state == KD_TRAVERSE) {  // one node visit
                const bool leaf = (ref & LEAF_BIT) != 0;
                if (COUNT) ++c_nodes;
                uint4 r0, r1;
                const float box = kd_visit(kv, ref, dep, exact_chain, eye, inv, r0, r1);
                bool pop = true;
                if (box != FLT_MAXF) {
                    if (leaf) {  // record it, then walk on from the stack
                        record(r0.w, r1.w);
                    } else {
                        uint32_t nearc, farc;
                        int target;
                        kd_split(r0, r1, box, eyea, dira, nearc, farc, target);
                        stack[top * 64 + lane] = (farc & LEAF_BIT) | ((uint32_t)(target + 1) << KD_DEPTH_SHIFT) |
                                                 (farc & KD_INDEX_MASK);
                        ++top;
                        dep = target + 1;
                        ref = nearc;
                        pop = false;
                    }
                }
                if (pop) {
                    if (top == 0) {
                        walked = true;
                        state = np ? KD_PENDING : KD_DONE;
                    } else {
                        const uint32_t e = stack[--top * 64 + lane];
                        ref = (e & LEAF_BIT) | (e & KD_INDEX_MASK);
                        dep = (int)((e >> KD_DEPTH_SHIFT) & 63u);
                    }
                }
                if (np == (uint32_t)K) state = KD_PENDING;
            }
            continue;
        }
        if (!ballot(np != 0)) break;
        // ---- the recorded leaves, tested by the whole wave ------------------------------------------
        ++rounds;
        const uint64_t round_t0 = COUNT ? __builtin_amdgcn_s_memrealtime() : 0;  // (diagnostic traces)
#if BM_KD_ROUND_FIRST
        // each lane's first recorded leaf only: no face is tested past the leaf the reference stops at;
        // a lane whose first leaf has no hit moves its next recorded leaf up for the next round (which
        // runs at once when no lane has to walk)
        uint32_t cstart = 0, ccnt = 0;
        if (np) {
            if (CB && cbl) {  // leaf index -> first face record and face count
                const uint32_t* lw = reinterpret_cast<const uint32_t*>(kv.leaves);
                cstart = lw[8 * (size_t)pst[0] + 3];
                ccnt = lw[8 * (size_t)pst[0] + 7];
            } else {
                cstart = pst[0];
                ccnt = pin[0];
            }
        }
        if (COUNT) c_faces += ccnt;
#if BM_KD_DPP_SCAN
        const uint32_t incl = wave_incl_add(ccnt);
        const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
#else
        uint32_t incl = ccnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t v = __shfl_up(incl, o);
            if (lane >= o) incl += v;
        }
        const uint32_t total = __shfl(incl, 63);
#endif
#if BM_KD_OWNER_BALLOT
        // Owners by window: for the 64 face slots [base, base + 64), each lane with faces whose first
        // slot lies in the window marks that position with its lane id (own[], in sincl's place), a
        // ballot of the marked positions gives each slot the nearest mark at or below it, and a slot
        // before the window's first mark belongs to the previous window's last owner — two LDS round
        // trips and a ballot where the binary search took six dependent reads.
        L.sbest[lane] = ~0ull;
        const uint32_t excl = incl - ccnt;
        uint32_t carry = 0;
        for (uint32_t base = 0; base < total; base += 64) {
            L.sincl[lane] = 64u;
            __builtin_amdgcn_wave_barrier();
            if (ccnt && excl >= base && excl - base < 64u) L.sincl[excl - base] = (uint32_t)lane;
            __builtin_amdgcn_wave_barrier();
            const uint32_t mk = L.sincl[lane];
            const unsigned long long M = ballot(mk != 64u);
            const unsigned long long le = M & (lane == 63 ? ~0ull : ((2ull << lane) - 1ull));
            const uint32_t at = le ? (uint32_t)L.sincl[63 - __builtin_clzll(le)] : carry;
            const uint32_t lo = at;
            carry = (uint32_t)__builtin_amdgcn_readlane((int)at, 63);
            const uint32_t j = base + (uint32_t)lane;
            const uint32_t f = j - (uint32_t)__shfl((int)excl, (int)lo);
            const uint32_t start = (uint32_t)__shfl((int)cstart, (int)lo);
            __builtin_amdgcn_wave_barrier();
#else
        L.sincl[lane] = incl;
        L.sbest[lane] = ~0ull;
        __syncthreads();
        for (uint32_t j = lane; j < ((total + 63) & ~63u); j += 64) {
            // owner: the lowest lane whose inclusive sum exceeds j (lanes with no faces never are); every
            // lane takes part in the shuffle (lanes past the total with the last face's owner)
            const uint32_t jj = min(j, total - 1u);
            uint32_t lo = 0, hi = 63;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (L.sincl[mid] > jj) hi = mid;
                else lo = mid + 1;
            }
            const uint32_t f = jj - (lo ? L.sincl[lo - 1] : 0u);
            const uint32_t start = (uint32_t)__shfl((int)cstart, (int)lo);
#endif
            if (j < total) {
                const float4* ft = kv.ftris + 3 * ((size_t)start + f);
                const float4 od = L.sdir[lo];
                float t, u, v;
                if (tri_test(ft[0], ft[1], ft[2], eye, v3(od.x, od.y, od.z), t, u, v) && t < FLT_MAXF) {
                    // the smallest t, then the earliest face (-0 -> +0: equal t, earliest face)
                    const uint32_t tb = __float_as_uint(t + 0.0f);
                    const uint32_t ot = (tb & 0x80000000u) ? ~tb : (tb | 0x80000000u);
                    atomicMin(&L.sbest[lo], ((unsigned long long)ot << 32) | f);
                }
            }
        }
        __syncthreads();
        if (np) {
            const unsigned long long best = L.sbest[lane];
            if (best != ~0ull) {  // the first leaf with a hit ends the march (:427-431)
                const float4* ft = kv.ftris + 3 * ((size_t)cstart + (uint32_t)best);
                const float4 a = ft[0];
                float t, u, v;
                tri_test(a, ft[1], ft[2], eye, dir, t, u, v);
                dclosest = t;
                fclosest = __float_as_uint(a.w);
                tu = u;
                tvv = v;
                state = KD_DONE;
                np = 0;
            } else {  // the next recorded leaf moves up
#pragma unroll
                for (int k = 0; k + 1 < K; ++k) {
                    pst[k] = pst[k + 1];
                    pin[k] = (CB && cbl) ? 0u : pin[k + 1] - ccnt;
                }
                --np;
                state = np ? (walked ? KD_PENDING : KD_TRAVERSE) : (walked ? KD_DONE : KD_TRAVERSE);
            }
        }
#else
        if (CB && cbl && np) {  // leaf indices -> first face record and face counts (loads issued together)
            const uint32_t* lw = reinterpret_cast<const uint32_t*>(kv.leaves);
            uint32_t acc = 0;
#pragma unroll
            for (int k = 0; k < K; ++k)
                if (k < (int)np) {
                    const uint32_t li = pst[k];
                    pst[k] = lw[8 * (size_t)li + 3];
                    acc += lw[8 * (size_t)li + 7];
                    pin[k] = acc;
                }
        }
        uint32_t cnt = 0;
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (k + 1 == (int)np) cnt = pin[k];
        if (COUNT) c_faces += cnt;
        uint32_t incl = cnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t v = __shfl_up(incl, o);
            if (lane >= o) incl += v;
        }
        const uint32_t total = __shfl(incl, 63);
        L.sincl[lane] = incl;
        L.sbest[lane] = ~0ull;
        __syncthreads();
        for (uint32_t j = lane; j < ((total + 63) & ~63u); j += 64) {
            // owner: the lowest lane whose inclusive sum exceeds j (lanes with no faces never are); every
            // lane takes part in the shuffles below (lanes past the total with the last face's owner)
            const uint32_t jj = min(j, total - 1u);
            uint32_t lo = 0, hi = 63;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (L.sincl[mid] > jj) hi = mid;
                else lo = mid + 1;
            }
            const uint32_t local = jj - (lo ? L.sincl[lo - 1] : 0u);
            // which of the owner's recorded leaves: the first whose inclusive count exceeds `local`
            uint32_t q = 0, base = 0, start = 0, prev = 0;
            bool found = false;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const uint32_t pk = (uint32_t)__shfl((int)pin[k], (int)lo);
                const uint32_t sk = (uint32_t)__shfl((int)pst[k], (int)lo);
                if (!found && local < pk) {
                    found = true;
                    q = (uint32_t)k;
                    base = prev;
                    start = sk;
                }
                prev = pk;
            }
            if (j < total) {
                const uint32_t f = local - base;
                const float4* ft = kv.ftris + 3 * ((size_t)start + f);
                const float4 od = L.sdir[lo];
                float t, u, v;
                if (tri_test(ft[0], ft[1], ft[2], eye, v3(od.x, od.y, od.z), t, u, v) && t < FLT_MAXF) {
                    // the first recorded leaf with a hit, then the smallest t, then the earliest face
                    // (-0 -> +0: equal t, earliest face)
                    const uint32_t tb = __float_as_uint(t + 0.0f);
                    const uint32_t ot = (tb & 0x80000000u) ? ~tb : (tb | 0x80000000u);
                    atomicMin(&L.sbest[lo], ((unsigned long long)q << 40) | ((unsigned long long)ot << 8) | f);
                }
            }
        }
        __syncthreads();
        if (np) {
            const unsigned long long best = L.sbest[lane];
            if (best != ~0ull) {  // the first leaf with a hit ends the march (:427-431)
                const uint32_t q = (uint32_t)(best >> 40), f = (uint32_t)best & 0xFFu;
                uint32_t start = 0;
#pragma unroll
                for (int k = 0; k < K; ++k)
                    if (k == (int)q) start = pst[k];
                const float4* ft = kv.ftris + 3 * ((size_t)start + f);
                const float4 a = ft[0];
                float t, u, v;
                tri_test(a, ft[1], ft[2], eye, dir, t, u, v);
                dclosest = t;
                fclosest = __float_as_uint(a.w);
                tu = u;
                tvv = v;
                state = KD_DONE;
            } else {
                state = walked ? KD_DONE : KD_TRAVERSE;
            }
            np = 0;
        }
#endif
        __syncthreads();  // sincl/sbest are rewritten by the next round
        if (COUNT) round_ticks += __builtin_amdgcn_s_memrealtime() - round_t0;
    }
    const size_t o = (size_t)y * p.width + x;
    uint32_t packed = MISS_PACKED;
    float nzv = 0.0f, tout = __builtin_inff();
    if (fclosest != NO_TRI) {
        const float* n = p.nrm + 9 * (size_t)fclosest;
        const float ww = 1.f - (tu + tvv);
        const vec3f nn = v3((n[0] * ww + n[3] * tu) + n[6] * tvv, (n[1] * ww + n[4] * tu) + n[7] * tvv,
                            (n[2] * ww + n[5] * tu) + n[8] * tvv);
        const float il = 1.f / sqrtf(dot(nn, nn));
        const float z = nn.z * il;
        const float rr = fabsf(z * 255.f);
        packed = ((rr == rr) ? (uint32_t)rr : 0u) << 16;
        nzv = fabsf(z);
        tout = dclosest;
    }
    if (inside) {
        p.packed[(size_t)y * p.pitch_u32 + x] = packed;
        p.tri_id[o] = fclosest;
        p.t[o] = tout;
        if (p.nz) p.nz[o] = nzv;
    }
    hit = fclosest != NO_TRI;
}

template <bool COUNT, bool DIAG>
__global__ __launch_bounds__(64) void k_kd_march_coop(const TraceParams p, const KdView kv) {
    __shared__ KdCoopLds L;
    const uint64_t t_start = DIAG ? __builtin_amdgcn_s_memrealtime() : 0;
    uint32_t c_nodes = 0, c_faces = 0;
    const int lane = threadIdx.x;
    // XCD-aware tile columns: workgroup b runs on XCD b % 8, so with a grid row a multiple of 8 wide,
    // workgroup column c takes tile column G (8 (q / G) + c % 8) + q % G (q = c / 8): runs of G adjacent
    // tile columns share an XCD and its L2 (the kd records their rays walk); measured 1-2 % on C2, C5 and
    // the filled view (G = 4 against screen order, tools/ref_time.py).
    uint32_t bx = blockIdx.x;
    if (BM_KD_XCD > 0 && (gridDim.x & 7u) == 0) {
        constexpr uint32_t G = BM_KD_XCD > 0 ? BM_KD_XCD : 1, SPAN = 8 * G;
        if (bx < gridDim.x / SPAN * SPAN) {
            const uint32_t q = bx >> 3;
            bx = G * (8 * (q / G) + (bx & 7u)) + q % G;
        }
    }
    const uint32_t x = bx * 8 + (lane & 7);
    const uint32_t y = blockIdx.y * 8 + (lane >> 3);
    const bool inside = x < p.width && y < p.height;
    bool hit = false;
    uint32_t iters = 0, rounds = 0;
    uint64_t round_ticks = 0;
    constexpr int K = COUNT && !DIAG ? 1 : KD_SPEC;  // counting traces: the reference's work
    constexpr bool CB = (!COUNT || DIAG) && BM_KD_CB;
    kd_coop_wave<COUNT, K, CB>(p, kv, L, x, y, inside, c_nodes, c_faces, hit, iters, rounds,
                                                                     round_ticks);
    if (COUNT && !DIAG) {  // (a diagnostic trace reports per-wave work; 3 same-address atomics per wave
                           // would serialise its timeline)
        unsigned long long a = c_nodes, b = c_faces, h = hit ? 1u : 0u;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            a += __shfl_xor(a, off);
            b += __shfl_xor(b, off);
            h += __shfl_xor(h, off);
        }
        if (lane == 0) {
            atomicAdd(p.counters + 0, a);
            atomicAdd(p.counters + 1, b);
            atomicAdd(p.counters + 2, h);
        }
    }
    if (DIAG) {
        // bits 0-31: lane-max of node visits + face tests; 32-47: the wave's loop iterations; 48-63: leaf rounds
        uint32_t wl = c_nodes + c_faces;
        const uint32_t nmax = min(iters, 0xFFFFu);
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) wl = max(wl, (uint32_t)__shfl_xor((int)wl, off));
        const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
        if (lane == 0) {
            const size_t wv = (size_t)blockIdx.y * gridDim.x + blockIdx.x;
            p.diag[4 * wv + 0] = t_start;
            p.diag[4 * wv + 1] = t_end;
            p.diag[4 * wv + 2] = round_ticks;  // (the one-box kernel stores its placement here)
            p.diag[4 * wv + 3] = wl | ((uint64_t)nmax << 32) | ((uint64_t)min(rounds, 0xFFFFu) << 48);
        }
    }
}

// ---- hashed uniform grid (Hash.cu, the reference's alternative accelerator) ----------------------
// Cells of 0.03; cell (x, y, z) -> bucket (F16(x) + F16(y) + F16(z)) mod 65536, F16 = Fletcher-16 of
// the four little-endian bytes (bmHash/bmHash3, Hash.cu:15-47). Built here without atomics:
//   k_hash_cells<count>  one thread per triangle visits its AABB's cells (z, y, x loops with the
//                        row indices reset, the fix of Hash.cu:162-164) and counts the cells the
//                        reference's triBoxOverlap accepts;
//   exclusive scan       per-triangle offsets;
//   k_hash_cells<emit>   writes (bucket, triangle) pairs in that order;
//   stable sort          by bucket (16-bit keys): a bucket's faces in triangle-id, then cell order —
//                        the reference's serial insertion order, which decides exact-t ties and its
//                        256-face cap (Hash.cu:82-89);
//   k_hash_ranges        bucket -> [start, end) of the sorted pairs.
// The march (bmMarchKernelSpace, Hash.cu:235-302): from the eye, cell by cell (at most 400), test
// every face of the cell's bucket (first 256) against the ray from the eye; the first bucket with a
// hit ends the march. Bit-identical to oracle/beam_oracle.c orc_hash_build + orc_hash_march.
constexpr uint32_t HG_BUCKETS = 65536;    // MAX_HASH_ELEMENTS, BuildTree.cuh:21
constexpr uint32_t HG_CAP = 256;          // NUM_FACES_PER_CELL, Hash.cu:7
constexpr int HG_ITERS = 400;             // MAX_SEARCH_ITERS, Hash.cu:11
constexpr float HG_CELL = 0.03f;          // CELL_RES
constexpr float HG_INV = 1.f / 0.03f;     // INV_CELL_RES (a float constant)
constexpr float HG_EPS = 0.03f * 0.001f;  // CELL_PINCH_TROUGH_EPSILON

__device__ __forceinline__ uint32_t hg_f16(uint32_t h) {
    uint32_t s1 = 0, s2 = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        s1 = (s1 + ((h >> (8 * b)) & 255u)) % 255u;
        s2 = (s2 + s1) % 255u;
    }
    return (s2 << 8) | s1;
}
__device__ __forceinline__ uint32_t hg_hash3(int32_t x, int32_t y, int32_t z) {
    return (hg_f16((uint32_t)x) + hg_f16((uint32_t)y) + hg_f16((uint32_t)z)) % HG_BUCKETS;
}
// bmMap (Hash.cu:57-60), saturating; NaN -> 0 (as the oracle's hg_map)
__device__ __forceinline__ int32_t hg_map(float f) {
    const float q = floorf(f * HG_INV);
    if (q != q) return 0;
    if (q >= 2147483648.f) return INT32_MAX;
    if (q < -2147483648.f) return INT32_MIN;
    return (int32_t)q;
}

template <bool EMIT>
__global__ __launch_bounds__(BLOCK) void k_hash_cells(const MeshDesc* __restrict__ meshes, uint32_t nm, uint32_t n,
                                                      uint32_t* __restrict__ counts,
                                                      const uint32_t* __restrict__ offsets,
                                                      uint32_t* __restrict__ keys, uint32_t* __restrict__ vals,
                                                      uint32_t* __restrict__ too_large) {
    const uint32_t g = blockIdx.x * BLOCK + threadIdx.x;
    if (g >= n) return;
    uint32_t a0 = 0, b0 = nm;
    while (b0 - a0 > 1) {
        const uint32_t mid = (a0 + b0) >> 1;
        if (meshes[mid].tri_offset <= g) a0 = mid;
        else b0 = mid;
    }
    const MeshDesc md = meshes[a0];
    const uint32_t f = g - md.tri_offset;
    float tv[9];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const uint32_t vi = md.idx[3 * f + k];
#pragma unroll
        for (int c = 0; c < 3; ++c) tv[3 * k + c] = md.pos[3 * vi + c];
    }
    int64_t lo[3], hi[3], span = 1;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        lo[c] = hg_map(rmin(tv[c], rmin(tv[3 + c], tv[6 + c])));
        hi[c] = hg_map(rmax(tv[c], rmax(tv[3 + c], tv[6 + c])));
        span *= hi[c] >= lo[c] ? hi[c] - lo[c] + 1 : 0;
        if (span > HG_MAX_CELLS) {  // the host fails the build (the oracle refuses the same scene)
            if (!EMIT) {
                counts[g] = 0;
                atomicOr(too_large, 1u);
            }
            return;
        }
    }
    uint32_t k = 0, out = EMIT ? offsets[g] : 0u;
    for (int64_t z = lo[2]; z <= hi[2]; ++z)
        for (int64_t y = lo[1]; y <= hi[1]; ++y)
            for (int64_t x = lo[0]; x <= hi[0]; ++x) {
                const float bmn[3] = {(float)(int32_t)x * HG_CELL, (float)(int32_t)y * HG_CELL,
                                      (float)(int32_t)z * HG_CELL};
                float bc[3], hs[3];
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    const float bmx = bmn[c] + HG_CELL;
                    bc[c] = (bmx + bmn[c]) * .5f;
                    hs[c] = (bmx - bmn[c]) * .5f;
                }
                if (tri_box(bc, hs, tv)) {
                    if (EMIT) {
                        keys[out + k] = hg_hash3((int32_t)x, (int32_t)y, (int32_t)z);
                        vals[out + k] = g;
                    }
                    ++k;
                }
            }
    if (!EMIT) counts[g] = k;
}

__global__ __launch_bounds__(BLOCK) void k_hash_ranges(const uint32_t* __restrict__ keys, uint32_t m,
                                                       uint32_t* __restrict__ bstart, uint32_t* __restrict__ bend) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= m) return;
    const uint32_t k = keys[i];
    if (i == 0 || keys[i - 1] != k) bstart[k] = i;
    if (i == m - 1 || keys[i + 1] != k) bend[k] = i + 1;
}

// bmBoxRayIntersectNoZero (CudaComon.cuh:176-187), the reference's _min/_max (second argument on NaN)
__device__ __forceinline__ float hg_box_exit(const float* bmn, const float* bmx, const vec3f o, const vec3f inv) {
    const float oa[3] = {o.x, o.y, o.z}, ia[3] = {inv.x, inv.y, inv.z};
    float tn[3], tf[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float t0 = (bmn[c] - oa[c]) * ia[c], t1 = (bmx[c] - oa[c]) * ia[c];
        tn[c] = rmin(t0, t1);
        tf[c] = rmax(t0, t1);
    }
    const float ftmin = rmax(tn[0], rmax(tn[1], tn[2]));
    const float ftmax = rmin(tf[0], rmin(tf[1], tf[2]));
    return (__builtin_isinf(ftmin) || ftmin < 0.f) ? ftmax : ftmin;
}

struct HashView {
    const uint32_t* bstart;
    const uint32_t* bend;
    const uint32_t* faces;  // sorted pair values: triangle ids per bucket
};

__global__ __launch_bounds__(BLOCK) void k_hash_march(const TraceParams p, const HashView hv) {
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const uint32_t x = blockIdx.x * 16 + (w & 1) * 8 + (lane & 7);
    const uint32_t y = blockIdx.y * 16 + (w >> 1) * 8 + (lane >> 3);
    if (x >= p.width || y >= p.height) return;
    const float rx = p.rx[x], ry = p.ry[y];
    const float d = 1.f / sqrtf(p.z2 + rx * rx + ry * ry);
    const vec3f r = v3(rx * d, ry * d, p.zoom * d);
    const float* m = p.orient;
    const vec3f dir = v3((m[0] * r.x + m[3] * r.y) + m[6] * r.z, (m[1] * r.x + m[4] * r.y) + m[7] * r.z,
                         (m[2] * r.x + m[5] * r.y) + m[8] * r.z);
    const vec3f inv = v3(1.f / dir.x, 1.f / dir.y, 1.f / dir.z);
    const vec3f eye = v3(p.eye[0], p.eye[1], p.eye[2]);
    vec3f pp = eye;
    float dclosest = FLT_MAXF, tu = 0.f, tvv = 0.f;
    uint32_t fclosest = NO_TRI;
    for (int it = 0; it < HG_ITERS; ++it) {
        const int32_t cx = hg_map(pp.x), cy = hg_map(pp.y), cz = hg_map(pp.z);
        const uint32_t b = hg_hash3(cx, cy, cz);
        const uint32_t c0 = hv.bstart[b];
        uint32_t cnt = hv.bend[b] - c0;
        if (cnt) {
            cnt = min(cnt, HG_CAP);
            for (uint32_t k = 0; k < cnt; ++k) {
                const uint32_t gid = hv.faces[c0 + k];
                const float4 ta = p.tris[3 * (size_t)gid + 0], tb = p.tris[3 * (size_t)gid + 1],
                             tc = p.tris[3 * (size_t)gid + 2];
                // bmTriIntersect (CudaComon.cuh:117-155) from the eye: FLT_MAX on the two rejects
                const vec3f e1 = v3(tb.x, tb.y, tb.z), e2 = v3(tc.x, tc.y, tc.z);
                const vec3f pv = cross(dir, e2);
                const float det = dot(e1, pv);
                const float idet = 1.f / det;
                const vec3f tvec = sub(eye, v3(ta.x, ta.y, ta.z));
                const float u = dot(tvec, pv) * idet;
                if (u < 0 || u > 1) continue;
                const vec3f qv = cross(tvec, e1);
                const float v = dot(dir, qv) * idet;
                if (v < 0 || v + u > 1) continue;
                const float t = dot(e2, qv) * idet;
                if (t < dclosest) {
                    dclosest = t;
                    fclosest = gid;
                    tu = u;
                    tvv = v;
                }
            }
            if (dclosest != FLT_MAXF) break;  // Hash.cu:271
        }
        const float bmn[3] = {(float)cx * HG_CELL, (float)cy * HG_CELL, (float)cz * HG_CELL};
        const float bmx[3] = {bmn[0] + HG_CELL, bmn[1] + HG_CELL, bmn[2] + HG_CELL};
        const float step = hg_box_exit(bmn, bmx, pp, inv) + HG_EPS;
        pp = v3(pp.x + dir.x * step, pp.y + dir.y * step, pp.z + dir.z * step);
    }
    const size_t o = (size_t)y * p.width + x;
    uint32_t packed = MISS_PACKED;
    float nzv = 0.0f, tout = __builtin_inff();
    if (fclosest != NO_TRI) {
        const float* n = p.nrm + 9 * (size_t)fclosest;
        const float ww = 1.f - (tu + tvv);
        const vec3f nn = v3((n[0] * ww + n[3] * tu) + n[6] * tvv, (n[1] * ww + n[4] * tu) + n[7] * tvv,
                            (n[2] * ww + n[5] * tu) + n[8] * tvv);
        const float il = 1.f / sqrtf(dot(nn, nn));
        const float z = nn.z * il;
        const float rr = fabsf(z * 255.f);
        packed = ((rr == rr) ? (uint32_t)rr : 0u) << 16;
        nzv = fabsf(z);
        tout = dclosest;
    }
    p.packed[(size_t)y * p.pitch_u32 + x] = packed;
    p.tri_id[o] = fclosest;
    p.t[o] = tout;
    if (p.nz) p.nz[o] = nzv;
}

}  // namespace

// Leaf depth for the world box: the reference's stop rule on its own halving arithmetic.
int kd_leaf_depth(float wmin, float wmax) {
    float mn[3] = {wmin, wmin, wmin}, mx[3] = {wmax, wmax, wmax};
    for (int d = 0; d < KD_MAX_DEPTH; ++d) {
        const float bs[3] = {mx[0] - mn[0], mx[1] - mn[1], mx[2] - mn[2]};
        const float dmin = std::fmin(bs[0], std::fmin(bs[1], bs[2]));
        if (dmin < KD_MIN_LEAF || d == KD_MAX_DEPTH - 1) return d;
        const int a = d % 3;
        mx[a] = .5f * (mn[a] + mx[a]);  // every node at depth d has the same extents
    }
    return KD_MAX_DEPTH - 1;
}

#define BM_LAUNCH_CHECK()                          \
    do {                                           \
        hipError_t e_ = hipGetLastError();         \
        if (e_ != hipSuccess) return e_;           \
    } while (0)

#ifdef BM_BUILD_DIAG
hipError_t kd_build_diag(unsigned long long* out) { return bdiag_io((const void*)&g_bdiag, out, 9, BDIAG_KERNELS); }
#endif

int kd_split_depth(int leaf_depth, const Tuning& t) {
    const int d = (int)t.get(BM_PARAM_KD_SPLIT, leaf_depth - KD_SPLIT_ABOVE_LEAF);
    return d > 0 && d < leaf_depth ? d : 0;
}

// Whether path_box_grid reproduces path_box's halving recurrence for every node down to leaf_depth. The
// axes halve independently, so each axis's intervals are enumerated (all 2^j at every level j) with the
// device's float operations (host code is compiled without contraction, as the kernels are).
static bool kd_grid_exact(float wmin, float wmax, int leaf_depth, bool off) {
    const int J = (leaf_depth + 2) / 3;
    if (off || J > 14) return false;
    std::vector<float> lo{wmin}, hi{wmax};
    const float ext = wmax - wmin;
    for (int j = 0;; ++j) {
        const float c = std::ldexp(ext, -j);
        for (size_t i = 0; i < lo.size(); ++i) {
            const float m = wmin + (float)i * c;
            if (m != lo[i] || m + c != hi[i]) return false;
        }
        if (j == J) return true;
        std::vector<float> lo2(2 * lo.size()), hi2(2 * lo.size());
        for (size_t i = 0; i < lo.size(); ++i) {
            const float s = .5f * (lo[i] + hi[i]);
            lo2[2 * i] = lo[i];
            hi2[2 * i] = s;
            lo2[2 * i + 1] = s;
            hi2[2 * i + 1] = hi[i];
        }
        lo.swap(lo2);
        hi.swap(hi2);
    }
}

// kd_grid_exact of the last world box asked about, per host thread (the check walks every cell of the
// world interval: ~4k float operations)
static bool kd_grid_exact_cached(float wmin, float wmax, int leaf_depth) {
    thread_local float c_wmin = 0.f, c_wmax = 0.f;
    thread_local int c_depth = -1;
    thread_local bool c_exact = false;
    if (wmin != c_wmin || wmax != c_wmax || leaf_depth != c_depth) {
        c_exact = kd_grid_exact(wmin, wmax, leaf_depth, false);
        c_wmin = wmin;
        c_wmax = wmax;
        c_depth = leaf_depth;
    }
    return c_exact;
}

static KdSplitArgs split_args(const KdBuild& k) {
    return KdSplitArgs{k.n, k.wmin, k.wmax, k.leaf_depth, k.split, k.counts, k.offsets, k.fill, k.keys, k.vals,
                       k.cache, k.queue, k.queue_cap, k.qcount, kd_grid_exact(k.wmin, k.wmax, k.leaf_depth,
                                                                               k.tune && k.tune->get(BM_PARAM_KD_GRID, 1) == 0)
                           ? 1 : 0,
                       k.lq_cap && k.lq_cap < KD_LQ_CAP ? k.lq_cap : KD_LQ_CAP, k.qcount + 1, k.zero_ptr,
                       k.zero_ptr ? k.zero_words : 0u, k.split >= (int)KD_TOP_BITS ? k.topmap : nullptr, k.topcount};
}

template <bool EMIT, bool PAIR, int TB, bool GRID>
static void launch_kd_split_grid(const KdBuild& k, const KdSplitArgs& a, bool top, bool fuse_copy, hipStream_t s) {
    constexpr uint32_t W = kd_w<PAIR>();
    if (top) k_kd_top<EMIT, PAIR, TB, GRID><<<blocks_for(W * k.n, TB), TB, 0, s>>>(k.meshes, k.num_meshes, a);
    // the same lanes in flight as 1024 workgroups of 256
    const uint32_t sub_blocks = std::min<uint32_t>(blocks_for(W * k.queue_cap, TB), 1024u * (256 / TB));
    KdSplitArgs b = a;
    uint32_t grid = sub_blocks;
    if (EMIT && fuse_copy) {  // k_kd_copy's triangles as extra workgroups after the walks'
        b.copy_first = sub_blocks;
        grid += blocks_for(k.n, TB);
    }
    k_kd_sub<EMIT, PAIR, TB, GRID><<<grid, TB, 0, s>>>(k.meshes, k.num_meshes, b);
}
template <bool EMIT, bool PAIR, int TB>
static void launch_kd_split_tb(const KdBuild& k, const KdSplitArgs& a, bool top, bool fuse_copy, hipStream_t s) {
    if (a.grid_exact) launch_kd_split_grid<EMIT, PAIR, TB, true>(k, a, top, fuse_copy, s);
    else launch_kd_split_grid<EMIT, PAIR, TB, false>(k, a, top, fuse_copy, s);
}
// The emit pass's cached-leaf copy inside k_kd_sub's launch (round 6; 0 restores the separate k_kd_copy)
#ifndef BM_KD_FUSE_COPY
#define BM_KD_FUSE_COPY 1
#endif

// The triangles' leaf counters and (for a fused copy) fill counters are zeroed by the count pass's k_kd_top,
// the fill counters otherwise by the emit pass's k_kd_top or k_kd_copy; the queue's count word and overflow flag by a memset (count pass, or an emit pass that walks
// from the root again). BM_PARAM_KD_TB: lanes per workgroup of k_kd_top / k_kd_sub (64 or 256).
template <bool EMIT>
static hipError_t launch_kd_split(const KdBuild& k, hipStream_t s) {
    hipError_t e;
    const KdSplitArgs a = split_args(k);
    const bool fuse_copy = EMIT && k.reuse_queue && BM_KD_FUSE_COPY;  // fill counters: zeroed by the count pass
    if (EMIT && k.reuse_queue) {  // the count pass's queue holds every subtree: no walk from the root
        if (!fuse_copy) k_kd_copy<<<blocks_for(k.n, BLOCK), BLOCK, 0, s>>>(a);
        BM_LAUNCH_CHECK();
    } else if (!(!EMIT && k.qcount_zeroed) && (e = hipMemsetAsync(k.qcount, 0, 8, s)) != hipSuccess) {
        return e;  // count word + overflow flag (the count pass: zeroed by launch_gather already)
    }
    const bool pair = !k.tune || k.tune->get(BM_PARAM_KD_PAIR, 1) != 0;
    const int tb = k.tune ? (int)k.tune->get(BM_PARAM_KD_TB, 64) : 64;
    const bool top = !(EMIT && k.reuse_queue);
    if (tb == 256) {
        if (pair) launch_kd_split_tb<EMIT, true, 256>(k, a, top, fuse_copy, s);
        else launch_kd_split_tb<EMIT, false, 256>(k, a, top, fuse_copy, s);
    } else {
        if (pair) launch_kd_split_tb<EMIT, true, 64>(k, a, top, fuse_copy, s);
        else launch_kd_split_tb<EMIT, false, 64>(k, a, top, fuse_copy, s);
    }
    BM_LAUNCH_CHECK();
    return hipSuccess;
}

static bool use_split(const KdBuild& k) {
    return k.split > 0 && k.split < k.leaf_depth && k.leaf_depth < KD_WALK_STACK && k.queue && k.queue_cap && k.qcount && k.fill;
}

hipError_t launch_kd_count(const KdBuild& k, hipStream_t s) {
    if (k.n == 0) return hipSuccess;
    if (use_split(k)) return launch_kd_split<false>(k, s);
    k_kd_descend<false><<<blocks_for(k.n, BLOCK), BLOCK, 0, s>>>(k.meshes, k.num_meshes, k.n, k.wmin, k.wmax,
                                                                 k.leaf_depth, k.counts, nullptr, nullptr, nullptr,
                                                                 k.cache);
    BM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_exclusive_scan(const uint32_t* in, uint32_t* out, uint32_t n, uint32_t* sums,
                                 uint32_t* grand_total, hipStream_t s, unsigned long long* total64, uint32_t epoch,
                                 const uint32_t* run_keys) {
    if (n == 0) {
        hipError_t e = hipMemsetAsync(grand_total, 0, 4, s);
        if (e == hipSuccess && total64) e = hipMemsetAsync(total64, 0, 8, s);
        return e;
    }
    if (((uintptr_t)(run_keys ? run_keys : in) | (uintptr_t)out) & 15u) return hipErrorInvalidValue;  // 16-B tile accesses
    const uint32_t nt = blocks_for(n, SCAN_TILE);
    // sums: [0] the ticket counter (a fixed word: it resets itself), [2, 2 + 2 nt) the tiles' u64 status
    // words (scan_sums_words)
    unsigned long long* status = reinterpret_cast<unsigned long long*>(sums + 2);
    k_scan1<<<nt, SCAN_BLOCK, 0, s>>>(in, out, n, status, sums, epoch & ((1u << 20) - 1u), nt, grand_total, total64,
                                      run_keys);
    BM_LAUNCH_CHECK();
    return hipSuccess;
}

uint32_t scan_sums_words(uint32_t n) {
    const uint32_t nt = blocks_for(n ? n : 1, SCAN_TILE);
    return 2 + 2 * nt;  // the ticket counter (and a pad word), then the u64 status words
}

hipError_t launch_kd_emit(const KdBuild& k, hipStream_t s) {
    if (k.zeroed) *k.zeroed = false;
    if (k.n == 0) return hipSuccess;
    if (use_split(k)) {
        const hipError_t e = launch_kd_split<true>(k, s);
        if (e == hipSuccess && k.zeroed) *k.zeroed = k.zero_ptr != nullptr;  // k_kd_sub<true> ran
        return e;
    }
    k_kd_descend<true><<<blocks_for(k.n, BLOCK), BLOCK, 0, s>>>(k.meshes, k.num_meshes, k.n, k.wmin, k.wmax,
                                                                k.leaf_depth, k.counts, k.offsets, k.keys, k.vals,
                                                                k.cache);
    BM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_kd_leaves(const uint32_t* keys, uint32_t m, const uint32_t* flags, const uint32_t* leaf_of,
                            uint32_t* leaf_key, uint32_t* leaf_start, uint32_t* leaf_count, uint32_t nl,
                            hipStream_t s, const uint32_t* nl_dev, uint32_t* ubox, const uint32_t* faces,
                            const float4* tri_orig, float4* ftris) {
    if (m == 0 || nl == 0) return ubox ? hipMemsetAsync(ubox, 0, 6 * sizeof(uint32_t), s) : hipSuccess;
    k_kd_leaves<<<blocks_for(m, BLOCK), BLOCK, 0, s>>>(keys, m, flags, leaf_of, leaf_key, leaf_start, nl, ubox, faces,
                                                       tri_orig, ftris);
    BM_LAUNCH_CHECK();
    if (leaf_count) {  // null: k_kd_records counts them (launch_kd_records with m)
        k_kd_leaf_count<<<blocks_for(nl, BLOCK), BLOCK, 0, s>>>(leaf_start, nl, m, leaf_count, nl_dev);
        BM_LAUNCH_CHECK();
    }
    return hipSuccess;
}

hipError_t launch_kd_records(const KdMarch& k, uint32_t m, uint4* nodes, uint4* leaves, uint32_t* node_key,
                             hipStream_t s, uint4* cnodes, uint32_t* ubox, uint32_t* post_host, uint32_t post_seq) {
    if (post_host && !k.num_leaves_dev) return hipErrorInvalidValue;
    if (k.num_leaves == 0) return post_host ? launch_post(k.num_leaves_dev, 1, nullptr, 0, post_host, post_seq, s) : hipSuccess;
    k_kd_records<<<blocks_for(k.num_leaves, BLOCK), BLOCK, 0, s>>>(k.leaf_key, k.leaf_start,
                                                                  const_cast<uint32_t*>(k.leaf_count), m, k.lch,
                                                                  k.rch, k.first, k.last, k.num_leaves, k.leaf_depth,
                                                                  k.wmin, k.wmax, nodes, leaves, node_key,
                                                                  k.num_leaves_dev, cnodes,
                                                                  !k.no_grid && kd_grid_exact_cached(k.wmin, k.wmax, k.leaf_depth)
                                                                      ? 1 : 0, ubox, post_host, post_seq);
    BM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_kd_march(const TraceParams& p, const KdMarch& k, bool count, hipStream_t s) {
    if (p.width == 0 || p.height == 0) return hipSuccess;
    if (k.num_leaves > KD_INDEX_MASK + 1u || k.leaf_depth >= KD_STACK) return hipErrorInvalidValue;
    const int variant = k.march_variant;
    // variant 3 (default): wave-cooperative leaves, child-box steps; 2: the same with one-box steps; 1:
    // lane-per-ray leaves, 64-lane groups; 0: the same in 256-lane groups
    KdView kv{k.nodes, k.leaves, k.node_key, k.leaf_key, k.ftris, k.num_leaves, k.leaf_depth, k.wmin, k.wmax,
              k.ubox, variant == 3 ? k.cnodes : nullptr};
    const dim3 g64((p.width + 7) / 8, (p.height + 7) / 8);
    if (variant >= 2) {
        if (p.diag) k_kd_march_coop<true, true><<<g64, 64, 0, s>>>(p, kv);
        else if (count) k_kd_march_coop<true, false><<<g64, 64, 0, s>>>(p, kv);
        else k_kd_march_coop<false, false><<<g64, 64, 0, s>>>(p, kv);
    } else if (p.diag) {
        k_kd_march<64, true, true><<<g64, 64, 0, s>>>(p, kv);
    } else if (count) {
        k_kd_march<64, true, false><<<g64, 64, 0, s>>>(p, kv);
    } else if (variant == 0) {
        k_kd_march<256><<<dim3((p.width + 15) / 16, (p.height + 15) / 16), 256, 0, s>>>(p, kv);
    } else {
        k_kd_march<64><<<g64, 64, 0, s>>>(p, kv);
    }
    BM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_post(const uint32_t* a, uint32_t na, const uint32_t* b, uint32_t nb, uint32_t* host, uint32_t seq,
                       hipStream_t s) {
    if (na + nb > POST_SEQ_WORD) return hipErrorInvalidValue;
    k_post<<<1, 64, 0, s>>>(a, na, b, nb, host, seq);
    BM_LAUNCH_CHECK();
    return hipSuccess;
}


hipError_t launch_hash_count(const HashBuild& h, hipStream_t s) {
    if (h.n == 0) return hipSuccess;
    k_hash_cells<false><<<blocks_for(h.n, BLOCK), BLOCK, 0, s>>>(h.meshes, h.num_meshes, h.n, h.counts, nullptr,
                                                                 nullptr, nullptr, h.too_large);
    BM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_hash_emit(const HashBuild& h, hipStream_t s) {
    if (h.n == 0) return hipSuccess;
    k_hash_cells<true><<<blocks_for(h.n, BLOCK), BLOCK, 0, s>>>(h.meshes, h.num_meshes, h.n, nullptr, h.offsets,
                                                                h.keys, h.vals, nullptr);
    BM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_hash_ranges(const uint32_t* keys, uint32_t m, uint32_t* bstart, uint32_t* bend, hipStream_t s) {
    hipError_t e;
    if ((e = hipMemsetAsync(bstart, 0, 4 * (size_t)HG_BUCKETS, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(bend, 0, 4 * (size_t)HG_BUCKETS, s)) != hipSuccess) return e;
    if (m == 0) return hipSuccess;
    k_hash_ranges<<<blocks_for(m, BLOCK), BLOCK, 0, s>>>(keys, m, bstart, bend);
    BM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_hash_march(const TraceParams& p, const uint32_t* bstart, const uint32_t* bend,
                             const uint32_t* faces, hipStream_t s) {
    if (p.width == 0 || p.height == 0) return hipSuccess;
    k_hash_march<<<dim3((p.width + 15) / 16, (p.height + 15) / 16), BLOCK, 0, s>>>(p, HashView{bstart, bend, faces});
    BM_LAUNCH_CHECK();
    return hipSuccess;
}

}  // namespace bm
