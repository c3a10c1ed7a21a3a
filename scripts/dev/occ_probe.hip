// occ_probe.hip — residency of 512-thread workgroups by dynamic LDS size on the MI355X: the
// runtime's occupancy answer and a timing census (2,048 blocks that each sleep a fixed time:
// the kernel takes 2048 / (256 x resident per CU) sleeps). Development probe, not product code.
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ __launch_bounds__(512) void sleeper(int spin, unsigned* sink) {
    extern __shared__ unsigned char lds[];
    if (threadIdx.x == 0) lds[0] = 1;
    __syncthreads();
    for (int i = 0; i < spin; ++i) __builtin_amdgcn_s_sleep(127);
    if (threadIdx.x == 0 && lds[0] == 7) sink[0] = 1;
}

int main() {
    unsigned* sink;
    hipMalloc(&sink, 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const size_t sizes[] = {20000, 60000, 67664, 72000, 76240, 79000, 81920, 90000};
    for (size_t s : sizes) {
        int n = 0;
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, sleeper, 512, s);
        hipLaunchKernelGGL(sleeper, dim3(2048), dim3(512), s, 0, 200, sink);  // warm-up
        hipEventRecord(a);
        hipLaunchKernelGGL(sleeper, dim3(2048), dim3(512), s, 0, 200, sink);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0.f;
        hipEventElapsedTime(&ms, a, b);
        printf("dynamic LDS %6zu B: occupancy API %d blocks/CU, 2048 sleeping blocks %.3f ms\n", s, n, ms);
    }
    return 0;
}
