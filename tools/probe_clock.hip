// Diagnostic micro-probe (not product code): shader clock under a latency-bound load,
// dependent global-load latency, and the duration of an empty / tiny kernel.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>

__global__ void k_empty() {}

__global__ void k_chain(float *out, unsigned long long *stamps, int n)
{
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    float x = threadIdx.x * 1e-3f;
    for (int i = 0; i < n; ++i) x = fmaf(x, 0.999f, 0.001f);
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) { stamps[0] = t1 - t0; stamps[1] = r1 - r0; }
}

__global__ void k_chase(const int *next, int *out, unsigned long long *stamps, int hops)
{
    unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    int p = 0;
    for (int i = 0; i < hops; ++i) p = next[p];
    unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    out[0] = p;
    stamps[2] = r1 - r0;
}

int main()
{
    float *out; unsigned long long *st; int *next, *o;
    hipMalloc(&out, 4096); hipMalloc(&st, 64); hipMalloc(&o, 64);
    const int n = 1 << 20;  // 4 MB ring, stride 64 KB + 4
    std::vector<int> h(n);
    for (int i = 0; i < n; ++i) h[i] = (i + 16411) % n;
    hipMalloc(&next, n * 4); hipMemcpy(next, h.data(), n * 4, hipMemcpyHostToDevice);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(a);
        for (int i = 0; i < 2000; ++i) hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, 0);
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        printf("empty kernel (256 WGs) back-to-back eager: %.2f us/launch\n", ms * 1000 / 2000);
    }
    // graph of 2000 empty kernels
    hipStream_t s; hipStreamCreate(&s);
    hipGraph_t g; hipGraphExec_t ge;
    hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
    for (int i = 0; i < 2000; ++i) hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, s);
    hipStreamEndCapture(s, &g); hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(a, s); hipGraphLaunch(ge, s); hipEventRecord(b, s); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        printf("empty kernel (256 WGs) in graph: %.2f us/launch\n", ms * 1000 / 2000);
    }
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k_chain, dim3(1), dim3(64), 0, 0, out, st, 200000);
        hipDeviceSynchronize();
        unsigned long long hs[3]; hipMemcpy(hs, st, 24, hipMemcpyDeviceToHost);
        printf("chain: %llu shader cycles / %llu x10ns -> clock %.0f MHz\n", hs[0], hs[1], hs[0] / (hs[1] * 10e-3));
    }
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k_chase, dim3(1), dim3(1), 0, 0, next, o, st, 4000);
        hipDeviceSynchronize();
        unsigned long long hs[3]; hipMemcpy(hs, st, 24, hipMemcpyDeviceToHost);
        printf("dependent load latency (4 MB ring): %.1f ns/hop\n", hs[2] * 10.0 / 4000);
    }
    return 0;
}
