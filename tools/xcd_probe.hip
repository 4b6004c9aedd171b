// Diagnostic only: does an XCD-stable board mapping make the step kernel's entry loads hit
// L2?  Back-to-back launches, each reading what the previous one wrote (SoA, 7 x u64 + 5 x
// u32 per board, 256 boards per workgroup).  mode 0: block b -> board block b (the step
// kernel's mapping; a block's XCD changes between dispatches).  mode 1: block b -> board block
// (b & ~7) | XCC_ID, the same XCD every launch IF the dispatcher deals blocks strictly round
// robin -- checked: every board block must be visited once per launch (coverage counter).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

__device__ __forceinline__ unsigned long long stamp() {
    __builtin_amdgcn_sched_barrier(0);
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}

__global__ void __launch_bounds__(256) k(uint64_t* bb, uint32_t* m, int n, unsigned long long* out, int mode,
                                         unsigned* cover) {
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    const int b = blockIdx.x;
    const int blk = mode ? ((b & ~7) | (int)(xcc & 7)) : b;
    const int i = blk * 256 + threadIdx.x;
    if (threadIdx.x == 0) atomicAdd(&cover[blk], 1u);
    unsigned long long t0 = stamp();
    uint64_t v[7];
    uint32_t w[5];
#pragma unroll
    for (int j = 0; j < 7; j++) v[j] = bb[(size_t)j * n + i];
#pragma unroll
    for (int j = 0; j < 5; j++) w[j] = m[(size_t)j * n + i];
#pragma unroll
    for (int j = 0; j < 7; j++) asm volatile("" : "+v"(v[j]));
#pragma unroll
    for (int j = 0; j < 5; j++) asm volatile("" : "+v"(w[j]));
    unsigned long long t1 = stamp();
    uint64_t x = 0;
#pragma unroll
    for (int j = 0; j < 7; j++) x ^= v[j] * (j + 3);
    uint32_t y = 0;
#pragma unroll
    for (int j = 0; j < 5; j++) y ^= w[j] + j;
#pragma unroll
    for (int j = 0; j < 7; j++) bb[(size_t)j * n + i] = v[j] + x;
#pragma unroll
    for (int j = 0; j < 5; j++) m[(size_t)j * n + i] = w[j] + y;
    if ((threadIdx.x & 63) == 0) out[i >> 6] = t1 - t0;
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 65536, nb = n / 256, iters = 200;
    uint64_t* bb;
    uint32_t* m;
    unsigned long long* out;
    unsigned* cover;
    hipMalloc(&bb, (size_t)7 * n * 8);
    hipMalloc(&m, (size_t)5 * n * 4);
    hipMalloc(&out, (size_t)(n / 64) * 8);
    hipMalloc(&cover, (size_t)nb * 4);
    hipMemset(bb, 1, (size_t)7 * n * 8);
    hipMemset(m, 1, (size_t)5 * n * 4);
    std::vector<unsigned long long> h(n / 64);
    std::vector<unsigned> c(nb);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int rep = 0; rep < 2; rep++)
        for (int mode = 0; mode < 2; mode++) {
            hipMemset(cover, 0, (size_t)nb * 4);
            for (int it = 0; it < iters; it++) {
                if (it == iters / 2) hipEventRecord(e0, 0);
                k<<<nb, 256>>>(bb, m, n, out, mode, cover);
            }
            hipEventRecord(e1, 0);
            hipDeviceSynchronize();
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            hipMemcpy(h.data(), out, h.size() * 8, hipMemcpyDeviceToHost);
            hipMemcpy(c.data(), cover, c.size() * 4, hipMemcpyDeviceToHost);
            int bad = 0;
            for (unsigned x : c) bad += x != (unsigned)iters;
            std::sort(h.begin(), h.end());
            printf("mode %d (%s): median entry-load wait %llu cycles (p90 %llu), %.2f us/launch, blocks visited != %d times: %d\n",
                   mode, mode ? "XCD-stable" : "block id  ", h[h.size() / 2], h[h.size() * 9 / 10], ms * 1000 / (iters / 2),
                   iters, bad);
        }
    return 0;
}
