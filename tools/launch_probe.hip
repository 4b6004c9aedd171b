// Diagnostic only: the per-launch floor of back-to-back dependent launches on one stream, by
// grid shape, plain launches vs one captured hipGraph of the same launches.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

__global__ void k_empty(uint32_t* out) {
    if (threadIdx.x == 0 && out[blockIdx.x] == 0xFFFFFFFFu) out[blockIdx.x] = 1;  // keep a memory op
}

static float run(int blocks, int threads, bool graph, hipStream_t st, uint32_t* out) {
    const int N = 400;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipGraphExec_t ge = nullptr;
    if (graph) {
        hipGraph_t g;
        (void)hipStreamBeginCapture(st, hipStreamCaptureModeGlobal);
        for (int i = 0; i < N; i++) k_empty<<<blocks, threads, 0, st>>>(out);
        (void)hipStreamEndCapture(st, &g);
        (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
        (void)hipGraphLaunch(ge, st);
    } else {
        for (int i = 0; i < N; i++) k_empty<<<blocks, threads, 0, st>>>(out);
    }
    (void)hipStreamSynchronize(st);
    (void)hipEventRecord(e0, st);
    if (graph) (void)hipGraphLaunch(ge, st);
    else for (int i = 0; i < N; i++) k_empty<<<blocks, threads, 0, st>>>(out);
    (void)hipEventRecord(e1, st);
    (void)hipStreamSynchronize(st);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms * 1000 / N;
}

int main() {
    uint32_t* out;
    (void)hipMalloc(&out, 1 << 20);
    (void)hipMemset(out, 0, 1 << 20);
    hipStream_t st;
    (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    int shapes[][2] = {{1, 64}, {256, 64}, {256, 256}, {1024, 128}, {2048, 64}, {4096, 64}};
    for (auto& s : shapes)
        printf("%5d blocks x %3d threads: %6.2f us/launch plain, %6.2f us/launch graph\n", s[0], s[1],
               run(s[0], s[1], false, st, out), run(s[0], s[1], true, st, out));
    return 0;
}
