// bm_bdiag.h — per-wave timing slots of diagnostic builds (-DBM_BUILD_DIAG; tools/build_diag.py).
// Included inside `namespace bm { namespace {` of each translation unit that times its build kernels
// (bm_build.hip: the LBVH build, kernel rows 0..8; bm_kd.hip: the reference-mode kd build, rows 9..15),
// so each has its own slot buffer; bm_debug_build_diag merges their rows.
#ifdef BM_BUILD_DIAG
// Every wave of a build kernel stores its start and end (s_memrealtime, 100 MHz) into its own slot of
// g_bdiag (no shared words: no contention to distort the times), so that the host can place each
// kernel's waves against the build's event time.
// Slot layout: [kernel k][wave w] -> 8 x u64 (start, end in s_memrealtime ticks; start, end of the
// shader clock counter s_memtime, whose rate against the 100-MHz one gives the wave's clock; four
// checkpoints BDIAG_MARK(0..3) inside the kernel, realtime).
constexpr uint32_t BDIAG_KERNELS = 16, BDIAG_WAVES = 1u << 16, BDIAG_WORDS = 8;
__device__ unsigned long long* g_bdiag;
// The slots exist only after bm_debug_build_diag(NULL) has allocated them: until then (a diagnostic
// library loaded by a program that never resets it) every store is skipped.
struct BDiag {
    unsigned long long* slot;
    __device__ void mark(int i) const {
        if (slot && (threadIdx.x & 63u) == 0) slot[4 + i] = __builtin_amdgcn_s_memrealtime();
    }
    __device__ explicit BDiag(uint32_t k) {
        const uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
        unsigned long long* base = g_bdiag;
        slot = base ? base + BDIAG_WORDS * ((size_t)k * BDIAG_WAVES + min(w, BDIAG_WAVES - 1)) : nullptr;
        if (slot && (threadIdx.x & 63u) == 0) {
            slot[0] = __builtin_amdgcn_s_memrealtime();
            slot[2] = __builtin_amdgcn_s_memtime();
        }
    }
    __device__ ~BDiag() {  // every exit path: the latest one per wave wins
        const unsigned long long m = ballot(1);
        if (slot && (threadIdx.x & 63u) == (uint32_t)__builtin_ctzll(m)) {
            atomicMax(&slot[1], (unsigned long long)__builtin_amdgcn_s_memrealtime());
            atomicMax(&slot[3], (unsigned long long)__builtin_amdgcn_s_memtime());
        }
    }
};
#define BDIAG(k) BDiag bdiag_scope_(k)
#define BDIAG_MARK(i) bdiag_scope_.mark(i)

// out == nullptr zeroes this unit's slots (allocated on first use); otherwise copies kernel rows
// [k0, k1) of them to the same rows of out (BDIAG_KERNELS * BDIAG_WAVES * BDIAG_WORDS u64).
static hipError_t bdiag_io(const void* sym, unsigned long long* out, uint32_t k0, uint32_t k1) {
    static unsigned long long* buf = nullptr;
    const size_t row = (size_t)BDIAG_WAVES * BDIAG_WORDS;
    hipError_t e;
    if (!buf) {
        if ((e = hipMalloc(&buf, BDIAG_KERNELS * row * sizeof(unsigned long long))) != hipSuccess) return e;
        if ((e = hipMemcpyToSymbol(sym, &buf, sizeof(buf))) != hipSuccess) return e;
    }
    if (!out) return hipMemset(buf, 0, BDIAG_KERNELS * row * sizeof(unsigned long long));
    return hipMemcpy(out + k0 * row, buf + k0 * row, (k1 - k0) * row * sizeof(unsigned long long),
                     hipMemcpyDeviceToHost);
}
#else
#define BDIAG(k)
#define BDIAG_MARK(i)
#endif
