// bm_gather.hip — the multi-GPU exchange step: screen bands traced on several
// devices land in the root device's render-target planes.
//
// A device's band buffer holds its rows compacted (local row lr <-> global row
// ((lr / band_h) * band_step + band_first) * band_h + lr % band_h, the map of bm_camera_trace_bands).
// k_band_scatter copies band rows into their frame rows, one pixel per lane per plane, so the
// loads and stores of a wave are 256 consecutive bytes of one row. It runs either
//  * on the source device with the root's planes as destination (BM_GATHER_PEER: the stores cross
//    xGMI as posted writes through peer access; no staging copy, no host round trip), or
//  * on the root over the staging buffers an RCCL receive filled (BM_GATHER_RCCL, multi-process),
//    all sources in one launch (blockIdx.z = source).
#include <hip/hip_runtime.h>

#include "bm_internal.h"

namespace bm {

namespace {

struct ScatterArgs {
    BandPlanes src[MAX_BAND_SOURCES];
    FramePlanes dst;
    uint32_t band_h, band_step, planes;
};

__global__ __launch_bounds__(256) void k_band_scatter(const ScatterArgs a) {
    const BandPlanes& s = a.src[blockIdx.z];
    const uint32_t lr = blockIdx.y;
    const uint32_t x = blockIdx.x * 256 + threadIdx.x;
    if (lr >= s.rows || x >= a.dst.width) return;
    const uint32_t gy = ((lr / a.band_h) * a.band_step + s.band_first) * a.band_h + lr % a.band_h;
    if (gy >= a.dst.height) return;
    const size_t si = (size_t)lr * a.dst.width + x, di = (size_t)gy * a.dst.width + x;
    if (a.planes & PLANE_PACKED) a.dst.packed[(size_t)gy * a.dst.pitch_u32 + x] = s.packed[si];
    if (a.planes & PLANE_TRI_ID) a.dst.tri[di] = s.tri[si];
    if (a.planes & PLANE_T) a.dst.t[di] = s.t[si];
    if ((a.planes & PLANE_NZ) && s.nz && a.dst.nz) a.dst.nz[di] = s.nz[si];
    if ((a.planes & PLANE_SHADOW) && s.shadow && a.dst.shadow) a.dst.shadow[di] = s.shadow[si];
}

}  // namespace

hipError_t launch_band_scatter(const BandPlanes* src, uint32_t nsrc, const FramePlanes& dst, uint32_t band_h,
                               uint32_t band_step, uint32_t planes, hipStream_t s) {
    if (nsrc == 0 || nsrc > MAX_BAND_SOURCES || band_h == 0 || band_step == 0) return hipErrorInvalidValue;
    ScatterArgs a{};
    uint32_t rows = 0;
    for (uint32_t i = 0; i < nsrc; ++i) {
        a.src[i] = src[i];
        if (src[i].band_first >= band_step) return hipErrorInvalidValue;
        rows = rows > src[i].rows ? rows : src[i].rows;
    }
    if (rows == 0 || dst.width == 0 || dst.height == 0) return hipSuccess;
    a.dst = dst;
    a.band_h = band_h;
    a.band_step = band_step;
    a.planes = planes;
    k_band_scatter<<<dim3((dst.width + 255) / 256, rows, nsrc), 256, 0, s>>>(a);
    return hipGetLastError();
}

}  // namespace bm
