// Barrier / hand-off probe for the C2 chain's structure decision.
// A persistent launch of G workgroups (256 threads, one per CU; XCD-aware: workgroup w runs on
// XCD w % 8) runs `iters` rounds of: publish a record (R floats, write-through sc1 stores,
// drained), arrive on a counter, wait for every workgroup's arrival (bounded poll of sc1 loads),
// then read the first 16 floats of every workgroup's record (sc1 loads) — the hand-off a
// weight-stationary chain would pay at each of its per-minibatch sync points (head partials,
// dW1 / norm partials).  Two counter forms: flat (one agent-scope counter) and XCD-hierarchical
// (a counter per XCD, the last arriver of an XCD adds to a top counter).  Prints µs per round
// from HIP events around the launch, for G in {32, 64, 128, 256}.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe/barrier_probe tools/probe/barrier_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__device__ __forceinline__ void store_wt(float *p, float4 v)
{
    typedef float xf4 __attribute__((ext_vector_type(4)));
    xf4 x = {v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(x) : "memory");
}

__device__ __forceinline__ uint32_t load_relaxed(const uint32_t *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ctr: [0] top, [8 + 16 x] per-XCD counters (own 64-B lines), [512] error
template <bool HIER>
__global__ __launch_bounds__(256) void k_probe(int iters, uint32_t *ctr, float *recs, int R, float *sink,
                                               uint64_t timeout)
{
    const int G = gridDim.x, w = blockIdx.x, tid = threadIdx.x;
    const int xcd = w & 7;
    const int per_xcd = G / 8;
    __shared__ int s_fail;
    if (tid == 0) s_fail = 0;
    float acc = 0.f;
    for (int it = 1; it <= iters; ++it) {
        // publish R floats (write-through), drained before the arrival
        for (int i = tid * 4; i < R; i += 1024)
            store_wt(recs + (size_t)w * R + i, make_float4((float)it, (float)w, (float)i, 1.f));
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            uint32_t target;
            uint32_t *poll;
            if (HIER) {
                const uint32_t old = __hip_atomic_fetch_add(ctr + 8 + 16 * xcd, 1u, __ATOMIC_RELAXED,
                                                            __HIP_MEMORY_SCOPE_AGENT);
                if (old + 1 == (uint32_t)(per_xcd * it))   // last of this XCD: carry the XCD up
                    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                poll = ctr;
                target = 8u * it;
            } else {
                __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                poll = ctr;
                target = (uint32_t)G * it;
            }
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            while (load_relaxed(poll) < target) {
                __builtin_amdgcn_s_sleep(1);
                if (__builtin_amdgcn_s_memrealtime() - t0 > timeout) {
                    s_fail = 1;
                    __hip_atomic_fetch_or(ctr + 512, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
            }
        }
        __syncthreads();
        if (s_fail) break;
        // read 16 floats of every workgroup's record (L1 bypass)
        if (tid < G * 4) {
            const uint32_t *src = reinterpret_cast<const uint32_t *>(recs + (size_t)(tid >> 2) * R + 4 * (tid & 3));
#pragma unroll
            for (int j = 0; j < 4; ++j) acc += __uint_as_float(load_relaxed(src + j));
        }
    }
    if (tid == 0 || acc == -1.f) sink[w] = acc;
}

int main()
{
    uint32_t *ctr;
    float *recs, *sink;
    CK(hipMalloc(&ctr, 4096));
    CK(hipMalloc(&recs, 256 * 4096 * sizeof(float)));
    CK(hipMalloc(&sink, 256 * sizeof(float)));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int iters = 2000;
    printf("{\"probe\": \"barrier\", \"iters\": %d, \"rows\": [\n", iters);
    bool first = true;
    for (int hier = 0; hier < 2; ++hier)
        for (int G : {32, 64, 128, 256})
            for (int R : {64, 1024}) {
                float best = 1e30f;
                for (int rep = 0; rep < 3; ++rep) {
                    CK(hipMemset(ctr, 0, 4096));
                    CK(hipDeviceSynchronize());
                    CK(hipEventRecord(a));
                    if (hier)
                        hipLaunchKernelGGL(k_probe<true>, dim3(G), dim3(256), 0, 0, iters, ctr, recs, R, sink,
                                           (uint64_t)200000000);
                    else
                        hipLaunchKernelGGL(k_probe<false>, dim3(G), dim3(256), 0, 0, iters, ctr, recs, R, sink,
                                           (uint64_t)200000000);
                    CK(hipEventRecord(b));
                    CK(hipEventSynchronize(b));
                    float ms;
                    CK(hipEventElapsedTime(&ms, a, b));
                    uint32_t err = 0;
                    CK(hipMemcpy(&err, ctr + 512, 4, hipMemcpyDeviceToHost));
                    if (err) { printf("timeout G=%d\n", G); return 2; }
                    best = ms < best ? ms : best;
                }
                printf("%s  {\"hier\": %d, \"G\": %d, \"record_floats\": %d, \"us_per_round\": %.3f}", first ? "" : ",\n",
                       hier, G, R, 1000.f * best / iters);
                first = false;
            }
    printf("\n]}\n");
    return 0;
}
