// Microbenchmark: issue rate of v_pk_mul_f32 vs v_mul_f32 (and v_min_f32, DPP mov) on gfx950.
// 8 independent chains per lane, 4096 iterations, one wave per SIMD and 8 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));
template <int KIND>
__global__ __launch_bounds__(256) void k(float* out, float s) {
    float a[8];
    f2 b[8];
    for (int i = 0; i < 8; ++i) { a[i] = threadIdx.x * 1e-3f + i; b[i] = f2{a[i], a[i] + 1.f}; }
    const f2 ss = {s, s};
    for (int it = 0; it < 4096; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (KIND == 0) a[i] = a[i] * s;
            if (KIND == 1) b[i] = b[i] * ss;
            if (KIND == 2) a[i] = fminf(a[i], s + a[(i + 1) & 7]);
            if (KIND == 3) a[i] = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, a[i]), 0xB1, 0xF, 0xF, true)) * s;
            if (KIND == 4) a[i] = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, a[i]), 0xB1, 0xF, 0xF, true));
            if (KIND == 5) {
                const unsigned u = __builtin_bit_cast(unsigned, a[i]);
                a[i] = __builtin_bit_cast(float, min(u, (unsigned)__builtin_amdgcn_mov_dpp((int)u, 0xB1, 0xF, 0xF, true)) + 1u);
            }
            if (KIND == 6) a[i] = __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, a[i]), 0x80B1));
            if (KIND == 7) a[i] = a[i] > s ? a[(i + 1) & 7] : a[i] * s;
        }
    }
    float r = 0;
    for (int i = 0; i < 8; ++i) r += a[i] + b[i].x + b[i].y;
    out[blockIdx.x * 256 + threadIdx.x] = r;
}
template <int KIND>
void run(const char* name, int blocks) {
    float* o; hipMalloc(&o, blocks * 256 * 4);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    k<KIND><<<blocks, 256>>>(o, 1.0000001f);
    hipEventRecord(e0);
    k<KIND><<<blocks, 256>>>(o, 1.0000001f);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double inst = (double)blocks * 4 * 4096 * 8;  // wave-instructions of the chain op
    int dev; hipGetDevice(&dev); hipDeviceProp_t p; hipGetDeviceProperties(&p, dev);
    const double simds = p.multiProcessorCount * 4.0;
    printf("%-10s blocks %6d: %8.3f ms, %.3f ns per wave-instr per SIMD (%.2f cycles at %d MHz)\n", name, blocks, ms,
           ms * 1e6 / (inst / simds), ms * 1e-3 * p.clockRate * 1e3 / (inst / simds), p.clockRate / 1000);
    hipFree(o);
}
int main() {
    for (int blocks : {256, 2048}) {  // 1 and 8 waves per SIMD (256 CUs)
        run<0>("v_mul", blocks); run<1>("v_pk_mul", blocks); run<2>("v_min+add", blocks); run<3>("dpp*mul", blocks);
        run<4>("mov_dpp", blocks); run<5>("min_dpp+add", blocks); run<6>("swizzle", blocks); run<7>("cmp+cnd+mul", blocks);
    }
    return 0;
}
