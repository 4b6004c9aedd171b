// Diagnostic only: which property of the paired step kernel makes its entry loads slow?
// Variants of the SoA entry-load probe (tools/lat_probe.hip): block shape, duplicate loads by
// a partner wave, LDS allocation, register footprint, and a long ALU tail.
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

template <int PAIR, int LDSB, int TAIL, int REGS>
__global__ void __launch_bounds__(PAIR ? 128 : 256) k(uint64_t* bb, uint32_t* m, int n, unsigned long long* out) {
    __shared__ uint64_t lds[LDSB ? 2112 : 1];
    int role = PAIR ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) : 0;
    int i = PAIR ? blockIdx.x * 64 + (threadIdx.x & 63) : blockIdx.x * blockDim.x + threadIdx.x;
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
    if (REGS) {  // hold ~140 VGPRs live
        uint64_t r[64];
#pragma unroll
        for (int j = 0; j < 64; j++) { r[j] = x * (j + 1); asm volatile("" : "+v"(r[j])); }
#pragma unroll
        for (int j = 0; j < 64; j++) x ^= r[j];
    }
    if (TAIL) {  // ~3000 dependent integer ops
        for (int j = 0; j < 1000; j++) { x = (x << 1) ^ (x >> 3) ^ (uint64_t)j; asm volatile("" : "+v"(x)); }
    }
    if (LDSB) { lds[threadIdx.x] = x; __syncthreads(); x ^= lds[(threadIdx.x + 1) & 127]; }
    if (role == 0) {
#pragma unroll
        for (int j = 0; j < 7; j++) bb[(size_t)j * n + i] = v[j] + x;
#pragma unroll
        for (int j = 0; j < 5; j++) m[(size_t)j * n + i] = w[j] + (uint32_t)x;
    }
    if ((threadIdx.x & 63) == 0) out[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = t1 - t0;
}

static unsigned long long median(std::vector<unsigned long long> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

template <int PAIR, int LDSB, int TAIL, int REGS>
static void run(const char* name, uint64_t* bb, uint32_t* m, int n, unsigned long long* out) {
    int waves = PAIR ? n / 32 : n / 64;
    std::vector<unsigned long long> h(waves);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int it = 0; it < 200; it++) {
        if (it == 100) hipEventRecord(e0, 0);
        if (PAIR) k<PAIR, LDSB, TAIL, REGS><<<n / 64, 128>>>(bb, m, n, out);
        else k<PAIR, LDSB, TAIL, REGS><<<n / 256, 256>>>(bb, m, n, out);
    }
    hipEventRecord(e1, 0);
    hipDeviceSynchronize();
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    hipMemcpy(h.data(), out, h.size() * 8, hipMemcpyDeviceToHost);
    printf("%-34s median entry-load wait %5llu cycles, %6.2f us/launch\n", name, median(h), ms * 1000 / 100);
}

int main(int argc, char** argv) {
    int n = argc > 1 ? atoi(argv[1]) : 65536;
    uint64_t* bb;
    uint32_t* m;
    unsigned long long* out;
    hipMalloc(&bb, (size_t)7 * n * 8);
    hipMalloc(&m, (size_t)5 * n * 4);
    hipMalloc(&out, (size_t)(n / 32) * 8);
    hipMemset(bb, 1, (size_t)7 * n * 8);
    hipMemset(m, 1, (size_t)5 * n * 4);
    run<0, 0, 0, 0>("base (256-thread blocks)", bb, m, n, out);
    run<1, 0, 0, 0>("pair (2 waves load each board)", bb, m, n, out);
    run<1, 1, 0, 0>("pair + 17 KB LDS", bb, m, n, out);
    run<1, 1, 0, 1>("pair + LDS + ~140 VGPRs", bb, m, n, out);
    run<1, 1, 1, 1>("pair + LDS + VGPRs + 3k-op tail", bb, m, n, out);
    run<0, 0, 1, 0>("base + 3k-op tail", bb, m, n, out);
    return 0;
}
