// Diagnostic only: what one launch costs the host's wall clock, by parts.
// For each variant: [t0; launch (optionally between two event records); wait; t1], median over
// reps, with the kernel's own first-wave-start -> last-wave-end span (s_memrealtime, 100 MHz).
// Variants: grid shape / LDS / VGPR footprint of k_env_rollout4's launch (512 x 512, 59 KB),
// dirty bytes left in L2 at the end (the trace and state of a 20-ply launch: ~11 MB), plain vs
// non-temporal stores, and the wait: hipStreamSynchronize, a hipStreamQuery spin, or a spin on a
// host-mapped word the last workgroup writes.
//   hipcc --offload-arch=gfx950 -O3 -o tools/_region_anatomy tools/region_anatomy.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

struct Args {
    uint64_t* dirty;       // bytes to write per lane (u64 words), or null
    int words;             // u64 words per lane
    int nt;                // non-temporal stores
    unsigned long long* span;  // [0] min start, [1] max end (s_memrealtime)
    unsigned* done_ctr;    // workgroups finished
    volatile unsigned* host_flag;  // host-mapped: the last workgroup writes the launch id
    unsigned id;
    int spin_cycles;       // per-wave busy work (s_sleep loop) before the end
};

template <int LDS_BYTES>
__global__ void __launch_bounds__(512) k_probe(Args a) {
    __shared__ uint64_t lds[LDS_BYTES / 8 > 0 ? LDS_BYTES / 8 : 1];
    const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
    if (LDS_BYTES > 0) lds[threadIdx.x % (LDS_BYTES / 8)] = threadIdx.x;
    for (int k = 0; k < a.spin_cycles; k += 64) __builtin_amdgcn_s_sleep(1);
    const size_t gt = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (a.dirty && ((gt >> 6) & 3) == 1) {  // one wave of four writes, as Q1 does: one board per lane
        const size_t n = (size_t)gridDim.x * blockDim.x / 4;
        const size_t i = (gt >> 8) * 64 + (gt & 63);
        for (int w = 0; w < a.words; w++) {
            uint64_t v = i ^ ((uint64_t)w << 40) ^ (LDS_BYTES > 0 ? lds[(threadIdx.x + w) % (LDS_BYTES / 8)] : 0);
            if (a.nt) __builtin_nontemporal_store(v, a.dirty + (size_t)w * n + i);
            else a.dirty[(size_t)w * n + i] = v;
        }
    }
    if (threadIdx.x == 0) atomicMin(a.span, t_start);
    __syncthreads();
    if (threadIdx.x == 0) {
        atomicMax(a.span + 1, (unsigned long long)__builtin_amdgcn_s_memrealtime());
        __threadfence_system();
        const unsigned prev = atomicAdd(a.done_ctr, 1u);
        if (prev == gridDim.x - 1) {
            *a.done_ctr = 0;
            __threadfence_system();
            *a.host_flag = a.id;
        }
    }
}

using clk = std::chrono::steady_clock;
static double us(clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); }

int main() {
    hipStream_t st;
    CHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    uint64_t* dirty;
    const int max_words = 22;  // 20 trace words + state ~ 11.5 MB at 65 536 lanes
    CHK(hipMalloc(&dirty, (size_t)8 * max_words * 65536));
    unsigned long long* span;
    CHK(hipMalloc(&span, 16));
    unsigned* ctr;
    CHK(hipMalloc(&ctr, 4));
    CHK(hipMemset(ctr, 0, 4));
    unsigned* hflag;
    CHK(hipHostMalloc(&hflag, 4, hipHostMallocMapped | hipHostMallocCoherent));
    unsigned* dflag;
    CHK(hipHostGetDevicePointer((void**)&dflag, hflag, 0));
    *hflag = 0;
    struct V { const char* name; int blocks, threads, lds, words, nt, wait, events, spin; };
    // wait: 0 hipStreamSynchronize, 1 hipStreamQuery spin, 2 host-flag spin (then a sync off the clock)
    const V vs[] = {
        {"empty 512x512 nolds sync", 512, 512, 0, 0, 0, 0, 0, 0},
        {"empty 512x512 nolds query", 512, 512, 0, 0, 0, 1, 0, 0},
        {"empty 512x512 nolds flag", 512, 512, 0, 0, 0, 2, 0, 0},
        {"empty 512x512 lds59k query", 512, 512, 1, 0, 0, 1, 0, 0},
        {"empty 512x512 lds59k query events", 512, 512, 1, 0, 0, 1, 1, 0},
        {"empty 256x1024 lds59k query", 256, 1024, 1, 0, 0, 1, 0, 0},
        {"dirty11MB 512x512 lds59k query", 512, 512, 1, max_words, 0, 1, 0, 0},
        {"dirty11MB nt 512x512 lds59k query", 512, 512, 1, max_words, 1, 1, 0, 0},
        {"dirty11MB 512x512 lds59k flag", 512, 512, 1, max_words, 0, 2, 0, 0},
        {"spin80us 512x512 lds59k query", 512, 512, 1, 0, 0, 1, 0, 160000},
        {"spin80us dirty11MB 512x512 lds59k query", 512, 512, 1, max_words, 0, 1, 0, 160000},
        {"spin80us dirty11MB 512x512 lds59k flag", 512, 512, 1, max_words, 0, 2, 0, 160000},
    };
    unsigned id = 1;
    for (const V& v : vs) {
        std::vector<double> wall, span_us, enq, ev;
        for (int r = 0; r < 25; r++) {
            unsigned long long init[2] = {~0ull, 0ull};
            CHK(hipMemcpy(span, init, 16, hipMemcpyHostToDevice));
            CHK(hipDeviceSynchronize());
            Args a{v.words ? dirty : nullptr, v.words, v.nt, span, ctr, dflag, id, v.spin};
            const auto t0 = clk::now();
            if (v.events) CHK(hipEventRecord(e0, st));
            if (v.lds) k_probe<59008><<<v.blocks, v.threads, 0, st>>>(a);
            else k_probe<0><<<v.blocks, v.threads, 0, st>>>(a);
            if (v.events) CHK(hipEventRecord(e1, st));
            const auto t1 = clk::now();
            if (v.wait == 0) {
                CHK(hipStreamSynchronize(st));
            } else if (v.wait == 1) {
                while (hipStreamQuery(st) == hipErrorNotReady) {}
            } else {
                while (__atomic_load_n(hflag, __ATOMIC_ACQUIRE) != id) {
                    if (us(t0, clk::now()) > 2e6) { printf("flag never written\n"); return 1; }
                }
            }
            const auto t2 = clk::now();
            CHK(hipStreamSynchronize(st));
            id++;
            unsigned long long sp[2];
            CHK(hipMemcpy(sp, span, 16, hipMemcpyDeviceToHost));
            if (r < 3) continue;  // warm
            wall.push_back(us(t0, t2));
            enq.push_back(us(t0, t1));
            span_us.push_back((double)(sp[1] - sp[0]) / 100.0);
            if (v.events) {
                float ms = 0;
                CHK(hipEventElapsedTime(&ms, e0, e1));
                ev.push_back(ms * 1e3);
            }
        }
        auto med = [](std::vector<double> x) { if (x.empty()) return -1.0; std::sort(x.begin(), x.end()); return x[x.size() / 2]; };
        printf("{\"variant\": \"%s\", \"wall_us\": %.2f, \"enqueue_us\": %.2f, \"kernel_span_us\": %.2f, \"event_us\": %.2f}\n",
               v.name, med(wall), med(enq), med(span_us), med(ev));
    }
    return 0;
}
