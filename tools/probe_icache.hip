// Diagnostic micro-probe (not product code): cost of executing straight-line code once
// (instruction-cache misses) vs the same instruction count in a warm loop.
#include <hip/hip_runtime.h>
#include <stdio.h>

#define REP_BODY "v_add_f32 %0, %0, 1.0\n"
template <int KB>
__global__ void k_straight(float *out)
{
    float x = threadIdx.x;
    // each v_add_f32 with inline constant is 4 bytes (VOP2) -> 256 per KB
    if constexpr (KB >= 1) asm volatile(".rept 256*" "1" "\n" REP_BODY ".endr" : "+v"(x));
    if constexpr (KB >= 4) asm volatile(".rept 256*" "3" "\n" REP_BODY ".endr" : "+v"(x));
    if constexpr (KB >= 16) asm volatile(".rept 256*" "12" "\n" REP_BODY ".endr" : "+v"(x));
    if constexpr (KB >= 32) asm volatile(".rept 256*" "16" "\n" REP_BODY ".endr" : "+v"(x));
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__global__ void k_loop(float *out, int n)
{
    float x = threadIdx.x;
    for (int i = 0; i < n; ++i) asm volatile(".rept 64\n" REP_BODY ".endr" : "+v"(x));
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

template <typename F>
static void timeit(const char *name, F launch)
{
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int w = 0; w < 5; ++w) launch();
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a);
    for (int i = 0; i < 500; ++i) launch();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    printf("%-40s %8.2f us/launch\n", name, ms * 1000 / 500);
}

int main()
{
    float *out;
    (void)hipMalloc(&out, 1 << 24);
    timeit("straight 1KB, 1 WG", [&] { hipLaunchKernelGGL(k_straight<1>, dim3(1), dim3(256), 0, 0, out); });
    timeit("straight 4KB, 1 WG", [&] { hipLaunchKernelGGL(k_straight<4>, dim3(1), dim3(256), 0, 0, out); });
    timeit("straight 16KB, 1 WG", [&] { hipLaunchKernelGGL(k_straight<16>, dim3(1), dim3(256), 0, 0, out); });
    timeit("straight 32KB, 1 WG", [&] { hipLaunchKernelGGL(k_straight<32>, dim3(1), dim3(256), 0, 0, out); });
    timeit("straight 32KB, 256 WG", [&] { hipLaunchKernelGGL(k_straight<32>, dim3(256), dim3(256), 0, 0, out); });
    timeit("loop = 32KB of adds, 1 WG", [&] { hipLaunchKernelGGL(k_loop, dim3(1), dim3(256), 0, 0, out, 128); });
    timeit("loop = 32KB of adds, 256 WG", [&] { hipLaunchKernelGGL(k_loop, dim3(256), dim3(256), 0, 0, out, 128); });
    // alternate two different 16 KB kernels (cache thrash between launches)
    timeit("alt straight 16KB / 32KB, 1 WG", [&] {
        hipLaunchKernelGGL(k_straight<16>, dim3(1), dim3(256), 0, 0, out);
        hipLaunchKernelGGL(k_straight<32>, dim3(1), dim3(256), 0, 0, out);
    });
    return 0;
}
