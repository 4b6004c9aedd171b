// Diagnostic only: VALU issue throughput on gfx950 for the integer ops the chess kernels are
// made of, at 1 / 2 / 4 waves per SIMD.  Each wave runs 8 independent dependency chains of one
// opcode (inline asm, so nothing is folded); cycles per wave-instruction per SIMD follow from
// the kernel time at the measured shader clock (s_memtime vs s_memrealtime).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define ITERS 40000
// 8 independent chains of a 2-source op "ins dst, src, dst"
#define OP8(ins)                                                                                        \
    asm volatile(ins " %0, %8, %0\n\t" ins " %1, %8, %1\n\t" ins " %2, %8, %2\n\t" ins " %3, %8, %3\n\t" \
                 ins " %4, %8, %4\n\t" ins " %5, %8, %5\n\t" ins " %6, %8, %6\n\t" ins " %7, %8, %7"     \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)        \
                 : "v"(k))
// 3-source op "ins dst, dst, src, src"
#define OP8_3(ins)                                                                                                     \
    asm volatile(ins " %0, %0, %8, %8\n\t" ins " %1, %1, %8, %8\n\t" ins " %2, %2, %8, %8\n\t" ins " %3, %3, %8, %8\n\t" \
                 ins " %4, %4, %8, %8\n\t" ins " %5, %5, %8, %8\n\t" ins " %6, %6, %8, %8\n\t" ins " %7, %7, %8, %8"     \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)                        \
                 : "v"(k))
// 1-source op "ins dst, dst"
#define OP8_1(ins)                                                                                    \
    asm volatile(ins " %0, %0\n\t" ins " %1, %1\n\t" ins " %2, %2\n\t" ins " %3, %3\n\t" ins " %4, %4\n\t" \
                 ins " %5, %5\n\t" ins " %6, %6\n\t" ins " %7, %7"                                     \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7))

template <int OP>
__global__ void __launch_bounds__(256) k_valu(uint32_t* out, unsigned long long* clk) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t k = blockIdx.x | 0x10001;
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < ITERS; it++) {
        if (OP == 0) OP8("v_and_b32");
        if (OP == 1) OP8("v_lshlrev_b32");
        if (OP == 2) OP8_3("v_alignbit_b32");
        if (OP == 3) OP8_3("v_perm_b32");
        if (OP == 4) OP8_3("v_bfi_b32");
        if (OP == 5) OP8_3("v_bfe_u32");
        if (OP == 6) OP8("v_bcnt_u32_b32");
        if (OP == 7) OP8_1("v_bfrev_b32");
        if (OP == 8) OP8_1("v_ffbl_b32");
        if (OP == 9) OP8("v_mul_lo_u32");
        if (OP == 10) OP8("v_mul_hi_u32");
        if (OP == 11) OP8_3("v_and_or_b32");
        if (OP == 12) OP8_3("v_or3_b32");
        if (OP == 13) OP8_3("v_lshl_or_b32");
        if (OP == 14) OP8_3("v_xad_u32");
        if (OP == 15) OP8("v_lshrrev_b32");
        if (OP == 16) OP8_1("v_not_b32");
        if (OP == 17) OP8_3("v_add3_u32");
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

template <int OP>
__global__ void __launch_bounds__(256) k_valu64(uint64_t* out, unsigned long long* clk) {
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    uint64_t c = blockIdx.x | 0x1000000001ull;
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < ITERS; it++) {
        if (OP == 0)
            asm volatile("v_lshlrev_b64 %0, 1, %0\n\tv_lshlrev_b64 %1, 1, %1\n\tv_lshlrev_b64 %2, 1, %2\n\t"
                         "v_lshlrev_b64 %3, 1, %3\n\tv_lshlrev_b64 %0, 1, %0\n\tv_lshlrev_b64 %1, 1, %1\n\t"
                         "v_lshlrev_b64 %2, 1, %2\n\tv_lshlrev_b64 %3, 1, %3"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3));
        if (OP == 1)
            asm volatile("v_lshl_add_u64 %0, %0, 0, %4\n\tv_lshl_add_u64 %1, %1, 0, %4\n\t"
                         "v_lshl_add_u64 %2, %2, 0, %4\n\tv_lshl_add_u64 %3, %3, 0, %4\n\t"
                         "v_lshl_add_u64 %0, %0, 0, %4\n\tv_lshl_add_u64 %1, %1, 0, %4\n\t"
                         "v_lshl_add_u64 %2, %2, 0, %4\n\tv_lshl_add_u64 %3, %3, 0, %4"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(c));
        if (OP == 2)
            asm volatile("v_mov_b64 %0, %1\n\tv_mov_b64 %1, %2\n\tv_mov_b64 %2, %3\n\tv_mov_b64 %3, %0\n\t"
                         "v_mov_b64 %0, %1\n\tv_mov_b64 %1, %2\n\tv_mov_b64 %2, %3\n\tv_mov_b64 %3, %0"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3));
        if (OP == 3)
            asm volatile("v_lshrrev_b64 %0, 3, %0\n\tv_lshrrev_b64 %1, 3, %1\n\tv_lshrrev_b64 %2, 3, %2\n\t"
                         "v_lshrrev_b64 %3, 3, %3\n\tv_lshrrev_b64 %0, 3, %0\n\tv_lshrrev_b64 %1, 3, %1\n\t"
                         "v_lshrrev_b64 %2, 3, %2\n\tv_lshrrev_b64 %3, 3, %3"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3));
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3;
    if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

// Kernel time (HIP events) x the measured clock / wave-instructions per SIMD.  (The in-kernel
// span of one wave is NOT a throughput measure: the oldest wave on a SIMD wins VALU
// arbitration and runs nearly unimpeded while younger ones wait.)
static double measure(void (*launch)(int, unsigned long long*), int wps) {
    unsigned long long* clk;
    hipMalloc(&clk, 16);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    launch(wps, clk);
    hipDeviceSynchronize();
    hipEventRecord(e0, 0);
    launch(wps, clk);
    hipEventRecord(e1, 0);
    hipDeviceSynchronize();
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h[2];
    hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost);
    hipFree(clk);
    double ghz = (double)h[0] / ((double)h[1] * 10.0);  // s_memrealtime ticks at 100 MHz
    return ms * 1e-3 * ghz * 1e9 / (8.0 * ITERS * wps);
}

static uint32_t* o32;
static uint64_t* o64;
#define L32(OPN) [](int wps, unsigned long long* clk) { k_valu<OPN><<<256 * wps, 256>>>(o32, clk); }
#define L64(OPN) [](int wps, unsigned long long* clk) { k_valu64<OPN><<<256 * wps, 256>>>(o64, clk); }

int main() {
    hipMalloc(&o32, (size_t)1024 * 4 * 64 * 4 * 8);
    hipMalloc(&o64, (size_t)1024 * 4 * 64 * 8 * 8);
    struct { const char* n; void (*f)(int, unsigned long long*); } ops[] = {
        {"v_and_b32", L32(0)}, {"v_lshlrev_b32", L32(1)}, {"v_lshrrev_b32", L32(15)}, {"v_alignbit_b32", L32(2)},
        {"v_perm_b32", L32(3)}, {"v_bfi_b32", L32(4)}, {"v_bfe_u32", L32(5)}, {"v_bcnt_u32_b32", L32(6)},
        {"v_bfrev_b32", L32(7)}, {"v_ffbl_b32", L32(8)}, {"v_mul_lo_u32", L32(9)}, {"v_mul_hi_u32", L32(10)},
        {"v_and_or_b32", L32(11)}, {"v_or3_b32", L32(12)}, {"v_lshl_or_b32", L32(13)}, {"v_xad_u32", L32(14)},
        {"v_not_b32", L32(16)}, {"v_add3_u32", L32(17)},
        {"v_lshlrev_b64", L64(0)}, {"v_lshrrev_b64", L64(3)}, {"v_lshl_add_u64", L64(1)}, {"v_mov_b64", L64(2)},
    };
    printf("%-16s %8s %8s %8s   (cycles per wave-instruction per SIMD; waves/SIMD)\n", "op", "1", "2", "4");
    for (auto& o : ops) {
        double c[3];
        int k = 0;
        for (int w = 1; w <= 4; w *= 2) c[k++] = measure(o.f, w);
        printf("%-16s %8.2f %8.2f %8.2f\n", o.n, c[0], c[1], c[2]);
    }
    return 0;
}
