// Diagnostic only: calibrates the VALU PMC counters (tools/pmc_summary.py's VALU-issue
// fraction) on kernels of KNOWN instruction count and mix.  Each wave runs ITERS x 8
// independent-chain instructions of one class, at 4 waves per SIMD on every SIMD (1024 blocks
// of 256 threads), so the SIMDs are VALU-issue-bound:
//   mode 0: v_xor_b32 (32-bit integer), 1: v_lshlrev_b64 (64-bit shift), 2: half and half,
//   3: v_bcnt_u32_b32 (32-bit, slow class), 4: v_lshl_add_u64.
// Run under rocprofv3 --pmc (tools/gpu_run.sh step `calib`); the program prints, per mode,
// the known wave-instructions and the event time, and the summary script divides the
// counters by them (what SQ_INSTS_VALU_INT32/INT64 count, what SQ_ACTIVE_INST_VALU counts per
// instruction, cycles per wave-instruction per SIMD at full issue).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define ITERS 20000
#define X8(ins) \
    asm volatile(ins " %0, %8, %0\n\t" ins " %1, %8, %1\n\t" ins " %2, %8, %2\n\t" ins " %3, %8, %3\n\t" \
                 ins " %4, %8, %4\n\t" ins " %5, %8, %5\n\t" ins " %6, %8, %6\n\t" ins " %7, %8, %7"     \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(k))

template <int MODE>
__global__ void __launch_bounds__(256) k_cal(uint64_t* out) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t k = blockIdx.x | 0x10001;
    uint64_t b0 = threadIdx.x, b1 = b0 + 1, b2 = b0 + 2, b3 = b0 + 3;
    const uint64_t c = blockIdx.x | 0x1000000001ull;
    for (int it = 0; it < ITERS; it++) {
        if (MODE == 0) X8("v_xor_b32");
        if (MODE == 3) X8("v_bcnt_u32_b32");
        if (MODE == 1)
            asm volatile("v_lshlrev_b64 %0, 1, %0\n\tv_lshlrev_b64 %1, 1, %1\n\tv_lshlrev_b64 %2, 1, %2\n\t"
                         "v_lshlrev_b64 %3, 1, %3\n\tv_lshlrev_b64 %0, 1, %0\n\tv_lshlrev_b64 %1, 1, %1\n\t"
                         "v_lshlrev_b64 %2, 1, %2\n\tv_lshlrev_b64 %3, 1, %3"
                         : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3));
        if (MODE == 2)
            asm volatile("v_xor_b32 %0, %6, %0\n\tv_lshlrev_b64 %2, 1, %2\n\tv_xor_b32 %1, %6, %1\n\t"
                         "v_lshlrev_b64 %3, 1, %3\n\tv_xor_b32 %0, %6, %0\n\tv_lshlrev_b64 %4, 1, %4\n\t"
                         "v_xor_b32 %1, %6, %1\n\tv_lshlrev_b64 %5, 1, %5"
                         : "+v"(a0), "+v"(a1), "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3) : "v"(k));
        if (MODE == 4)
            asm volatile("v_lshl_add_u64 %0, %0, 0, %4\n\tv_lshl_add_u64 %1, %1, 0, %4\n\t"
                         "v_lshl_add_u64 %2, %2, 0, %4\n\tv_lshl_add_u64 %3, %3, 0, %4\n\t"
                         "v_lshl_add_u64 %0, %0, 0, %4\n\tv_lshl_add_u64 %1, %1, 0, %4\n\t"
                         "v_lshl_add_u64 %2, %2, 0, %4\n\tv_lshl_add_u64 %3, %3, 0, %4"
                         : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3) : "v"(c));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7) ^ b0 ^ b1 ^ b2 ^ b3;
}

template <int MODE>
static void run(uint64_t* o, const char* name) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    k_cal<MODE><<<1024, 256>>>(o);  // warm (code load); the summary uses the LAST dispatch per mode
    hipDeviceSynchronize();
    hipEventRecord(e0, 0);
    k_cal<MODE><<<1024, 256>>>(o);
    hipEventRecord(e1, 0);
    hipDeviceSynchronize();
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double waves = 1024.0 * 4, winst = waves * 8.0 * ITERS;
    printf("{\"mode\": %d, \"op\": \"%s\", \"waves\": %.0f, \"wave_insts\": %.0f, \"ms\": %.4f}\n", MODE, name, waves,
           winst, ms);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}

int main() {
    uint64_t* o;
    if (hipMalloc(&o, (size_t)1024 * 256 * 8) != hipSuccess) return 1;
    run<0>(o, "v_xor_b32");
    run<1>(o, "v_lshlrev_b64");
    run<2>(o, "v_xor_b32 + v_lshlrev_b64 (1:1)");
    run<3>(o, "v_bcnt_u32_b32");
    run<4>(o, "v_lshl_add_u64");
    hipFree(o);
    return 0;
}
