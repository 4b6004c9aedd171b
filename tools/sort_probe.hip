// Diagnostic only: hipCUB radix sort of (u32 key, u32 value) pairs by the top B key bits, at the
// perft transposition pass's size (2^26 records per chunk) -- is a sorted (bucketed) pass cheaper
// than one random CAS per record (k_dedup_bin: ~12 ms per chunk)?
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <cstdio>
#include <cstdint>
__global__ void fill(uint32_t* k, uint32_t* v, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t x = (uint64_t)i * 0x9E3779B97F4A7C15ull;
    x ^= x >> 31; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 29;
    k[i] = (uint32_t)(x >> 32);
    v[i] = (uint32_t)i;
}
int main() {
    const int n = 68000000;
    uint32_t *k0, *k1, *v0, *v1;
    hipMalloc(&k0, 4ull * n); hipMalloc(&k1, 4ull * n); hipMalloc(&v0, 4ull * n); hipMalloc(&v1, 4ull * n);
    fill<<<(n + 255) / 256, 256>>>(k0, v0, n);
    for (int bits : {12, 16, 20, 32}) {
        size_t tb = 0;
        hipcub::DeviceRadixSort::SortPairs(nullptr, tb, k0, k1, v0, v1, n, 32 - bits, 32);
        void* tmp; hipMalloc(&tmp, tb);
        hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
        for (int r = 0; r < 3; r++) {
            hipEventRecord(a);
            hipcub::DeviceRadixSort::SortPairs(tmp, tb, k0, k1, v0, v1, n, 32 - bits, 32);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b);
            printf("bits %d: %.3f ms (%.2f Gpairs/s)\n", bits, ms, n / ms / 1e6);
        }
        hipFree(tmp);
    }
    return 0;
}
