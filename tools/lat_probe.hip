// Diagnostic only: entry-load latency of one launch, by layout, in back-to-back launches
// (each launch reads what the previous one wrote, like the step kernel).
//   SoA: 12 separate arrays (7 x u64 + 5 x u32), one load each
//   AoS: one 96-B record per board, 6 x 16-B loads
// Per wave: s_memtime before the loads and after their s_waitcnt; median over waves.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <vector>

__device__ __forceinline__ unsigned long long stamp() {
    __builtin_amdgcn_sched_barrier(0);
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}

__global__ void __launch_bounds__(256) k_soa(uint64_t* bb, uint32_t* m, int n, unsigned long long* out,
                                             ulonglong2* htab, int salt, int layout) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
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
    if (htab) {  // the step kernel's 3-fold window: one random 64-B line per board read + written
        uint32_t pos = (uint32_t)((x ^ (uint64_t)salt * 0x9E3779B97F4A7C15ull) >> 20) & 1023;
        size_t ent;
        switch (layout) {
            case 0: ent = (size_t)i * 1024 + pos; break;                                 // board-major
            case 1: ent = ((size_t)(i >> 6) * 1024 + pos) * 64 + (i & 63); break;        // wave-blocked
            case 2: ent = (size_t)i * 256 + (pos & 255); break;                          // 256 entries
            default: ent = (size_t)i * 1024 + pos; break;                                // nontemporal
        }
        ulonglong2* e = htab + ent * 4;
        ulonglong2 a, b, c, d;
        typedef unsigned long long v2u64 __attribute__((ext_vector_type(2)));
        v2u64* ev = reinterpret_cast<v2u64*>(e);
        if (layout == 3) {
            v2u64 t0 = __builtin_nontemporal_load(ev), t1 = __builtin_nontemporal_load(ev + 1);
            v2u64 t2 = __builtin_nontemporal_load(ev + 2), t3 = __builtin_nontemporal_load(ev + 3);
            a = make_ulonglong2(t0.x, t0.y); b = make_ulonglong2(t1.x, t1.y);
            c = make_ulonglong2(t2.x, t2.y); d = make_ulonglong2(t3.x, t3.y);
        } else {
            a = e[0]; b = e[1]; c = e[2]; d = e[3];
        }
        asm volatile("" : "+v"(a.x), "+v"(b.x), "+v"(c.x), "+v"(d.x));
        a.x += 1;
        if (layout == 3) {
            v2u64 t0 = {a.x, a.y}, t1 = {b.x, b.y}, t2 = {c.x, c.y}, t3 = {d.x, d.y};
            __builtin_nontemporal_store(t0, ev); __builtin_nontemporal_store(t1, ev + 1);
            __builtin_nontemporal_store(t2, ev + 2); __builtin_nontemporal_store(t3, ev + 3);
        } else {
            e[0] = a; e[1] = b; e[2] = c; e[3] = d;
        }
    }
    if ((threadIdx.x & 63) == 0) out[i >> 6] = t1 - t0;
}

__global__ void __launch_bounds__(256) k_aos(ulonglong2* rec, int n, unsigned long long* out) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long t0 = stamp();
    ulonglong2 r[6];
#pragma unroll
    for (int j = 0; j < 6; j++) r[j] = rec[(size_t)i * 6 + j];
#pragma unroll
    for (int j = 0; j < 6; j++) asm volatile("" : "+v"(r[j].x), "+v"(r[j].y));
    unsigned long long t1 = stamp();
    uint64_t x = 0;
#pragma unroll
    for (int j = 0; j < 6; j++) x ^= r[j].x * (j + 3) + r[j].y;
#pragma unroll
    for (int j = 0; j < 6; j++) rec[(size_t)i * 6 + j] = make_ulonglong2(r[j].x + x, r[j].y ^ x);
    if ((threadIdx.x & 63) == 0) out[i >> 6] = t1 - t0;
}

static unsigned long long median(std::vector<unsigned long long> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main(int argc, char** argv) {
    int n = argc > 1 ? atoi(argv[1]) : 65536;
    uint64_t* bb;
    uint32_t* m;
    ulonglong2* rec;
    unsigned long long* out;
    hipMalloc(&bb, (size_t)7 * n * 8);
    hipMalloc(&m, (size_t)5 * n * 4);
    hipMalloc(&rec, (size_t)6 * n * 16);
    hipMalloc(&out, (size_t)(n / 64) * 8);
    ulonglong2* htab = nullptr;
    if (hipMalloc(&htab, (size_t)n * 1024 * 64) != hipSuccess) htab = nullptr;
    else hipMemset(htab, 0, (size_t)n * 1024 * 64);
    hipMemset(bb, 1, (size_t)7 * n * 8);
    hipMemset(m, 1, (size_t)5 * n * 4);
    hipMemset(rec, 1, (size_t)6 * n * 16);
    std::vector<unsigned long long> h(n / 64);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char* names[] = {"SoA 12 arrays", "AoS 6x16B", "SoA + table board-major", "SoA + table wave-blocked",
                           "SoA + table 256 entries", "SoA + table nontemporal"};
    for (int mode = 0; mode < 6; mode++) {
        for (int it = 0; it < 200; it++) {
            if (it == 100) hipEventRecord(e0, 0);
            if (mode == 0) k_soa<<<n / 256, 256>>>(bb, m, n, out, nullptr, it, 0);
            else if (mode == 1) k_aos<<<n / 256, 256>>>(rec, n, out);
            else k_soa<<<n / 256, 256>>>(bb, m, n, out, htab, it, mode - 2);
        }
        hipEventRecord(e1, 0);
        hipDeviceSynchronize();
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        hipMemcpy(h.data(), out, h.size() * 8, hipMemcpyDeviceToHost);
        printf("%-26s n=%d: median entry-load wait %llu cycles, %.2f us/launch\n", names[mode], n, median(h),
               ms * 1000 / 100);
    }
    return 0;
}
