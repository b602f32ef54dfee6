// L1 -> L2 request size on gfx950: known byte counts against TCP_TCC_READ_REQ_sum / TCP_TCC_WRITE_REQ_sum
// (tools/l2_calib.py runs this under rocprofv3 --pmc and divides). Measurement only; not in the library.
//   k_read16   64 MiB read once, 16 B per lane, coalesced (each wave-instruction 1 KiB contiguous)
//   k_read4    64 MiB read once, 4 B per lane, coalesced (256 B per wave-instruction)
//   k_rec112   the trace's access shape: each lane reads 7 x 16 B of its own 128-B record (random records)
//   k_write16  64 MiB written, 16 B per lane;  k_write4: 4 B per lane (the render-target planes' shape)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void k_read16(const float4* __restrict__ a, float* out, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    float4 v = i < n ? a[i] : make_float4(0, 0, 0, 0);
    const float s = v.x + v.y + v.z + v.w;
    if (s == 1234.5f) out[i & 1023] = s;  // never true for the zero-filled input: keeps the load
}
__global__ void k_read4(const float* __restrict__ a, float* out, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const float s = i < n ? a[i] : 0.f;
    if (s == 1234.5f) out[i & 1023] = s;
}
__global__ void k_rec112(const float4* __restrict__ a, float* out, uint32_t nrec, uint32_t nlanes) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nlanes) return;
    uint32_t h = i * 2654435761u;
    h ^= h >> 13;
    const uint32_t r = h % nrec;  // distinct-ish random records
    const float4* p = a + 8 * (size_t)r;
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
        const float4 v = p[k];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 1234.5f) out[i & 1023] = s;
}
__global__ void k_write16(float4* a, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) a[i] = make_float4(1, 2, 3, 4);
}
__global__ void k_write4(float* a, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) a[i] = 1.f;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main() {
    const size_t bytes = 64u << 20;
    float *a = nullptr, *b = nullptr, *out = nullptr;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMalloc(&out, 4096));
    CK(hipMemset(a, 0, bytes));
    CK(hipMemset(b, 0, bytes));
    const uint32_t n16 = bytes / 16, n4 = bytes / 4, nrec = bytes / 128, nlanes = 1u << 19;
    for (int rep = 0; rep < 3; ++rep) {
        // b is written in between, so a's lines are not all L2-resident at the next read (64 MiB > 32 MiB L2)
        k_read16<<<n16 / 256, 256>>>(reinterpret_cast<const float4*>(a), out, n16);
        k_read4<<<n4 / 256, 256>>>(a, out, n4);
        k_rec112<<<nlanes / 256, 256>>>(reinterpret_cast<const float4*>(a), out, nrec, nlanes);
        k_write16<<<n16 / 256, 256>>>(reinterpret_cast<float4*>(b), n16);
        k_write4<<<n4 / 256, 256>>>(b, n4);
    }
    CK(hipDeviceSynchronize());
    printf("l2_calib: bytes %zu, n16 %u, n4 %u, rec112 lanes %u (112 B each, %u records)\n", bytes, n16, n4, nlanes, nrec);
    CK(hipFree(a));
    CK(hipFree(b));
    CK(hipFree(out));
    return 0;
}
