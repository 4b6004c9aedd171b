// Diagnostic only: what does a cold instruction cache cost a launch?  The same VALU work
// (8 independent v_xor chains, 4-B VOP2 encodings) as a small loop (code stays in one I-cache
// line group) vs fully unrolled straight-line code of 12 / 24 / 48 KiB, launched back to back
// (every launch starts with caches invalidated, like the step kernel's launches).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define X8 asm volatile("v_xor_b32 %0, %8, %0\n\tv_xor_b32 %1, %8, %1\n\tv_xor_b32 %2, %8, %2\n\tv_xor_b32 %3, %8, %3\n\t" \
                        "v_xor_b32 %4, %8, %4\n\tv_xor_b32 %5, %8, %5\n\tv_xor_b32 %6, %8, %6\n\tv_xor_b32 %7, %8, %7"     \
                        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)          \
                        : "v"(k))

// ITER bodies of 16 instructions (64 B); UNROLL: straight line, else a loop
template <int ITER, bool UNROLL>
__global__ void __launch_bounds__(256) k(uint32_t* out) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t k = blockIdx.x | 0x10001;
    if (UNROLL) {
#pragma unroll
        for (int it = 0; it < ITER; it++) { X8; X8; }
    } else {
#pragma unroll 1
        for (int it = 0; it < ITER; it++) { X8; X8; }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

template <int ITER, bool UNROLL>
static void run(const char* name, uint32_t* out, int threads) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int it = 0; it < 300; it++) {
        if (it == 100) hipEventRecord(e0, 0);
        k<ITER, UNROLL><<<threads / 256, 256>>>(out);
    }
    hipEventRecord(e1, 0);
    hipDeviceSynchronize();
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    printf("%-26s %7d threads  %5d instr/wave  %7.2f us/launch\n", name, threads, ITER * 16, ms * 1000 / 200);
}

int main() {
    uint32_t* out;
    hipMalloc(&out, (size_t)262144 * 4);
    for (int t = 65536; t <= 131072; t *= 2) {
        run<1, false>("empty-ish (16 instr)", out, t);
        run<192, false>("loop 12 KiB of work", out, t);
        run<192, true>("straight 12 KiB", out, t);
        run<384, false>("loop 24 KiB of work", out, t);
        run<384, true>("straight 24 KiB", out, t);
        run<768, false>("loop 48 KiB of work", out, t);
        run<768, true>("straight 48 KiB", out, t);
    }
    return 0;
}
