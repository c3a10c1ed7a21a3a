// Developer probe: what each DPP control used by the tile kernels returns per lane (gfx950).
// hipcc --offload-arch=gfx950 -O2 scripts/dev/dpp_probe.hip -o /tmp/dpp_probe && /tmp/dpp_probe
#include <hip/hip_runtime.h>
#include <cstdio>
template <int C> __device__ int d(int old, int x) { return __builtin_amdgcn_update_dpp(old, x, C, 0xf, 0xf, false); }
__global__ void k(int* o) {
    const int x = 1000 + threadIdx.x;
    int i = 0;
    o[64 * i++ + threadIdx.x] = d<0xB1>(-1, x);
    o[64 * i++ + threadIdx.x] = d<0x0F>(-1, x);
    o[64 * i++ + threadIdx.x] = d<0x141>(-1, x);
    o[64 * i++ + threadIdx.x] = d<0x150>(-1, x);
    o[64 * i++ + threadIdx.x] = d<0x15F>(-1, x);
    o[64 * i++ + threadIdx.x] = d<0x101>(-1, x);
    o[64 * i++ + threadIdx.x] = d<0x108>(-1, x);
    const int hm = d<0x141>(-1, x);
    o[64 * i++ + threadIdx.x] = d<0xFF>(-1, hm);
    o[64 * i++ + threadIdx.x] = d<0x00>(-1, hm);
}
int main() {
    int* dv; hipMalloc(&dv, 64 * 9 * 4);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dv);
    int h[64 * 9]; hipMemcpy(h, dv, sizeof h, hipMemcpyDeviceToHost);
    const char* nm[] = {"quad[1032]", "quad[3300]", "half_mirror", "newbcast0", "newbcast15", "row_shl1", "row_shl8", "hm+quad3333", "hm+quad0000"};
    for (int r = 0; r < 9; ++r) { printf("%-12s", nm[r]); for (int l = 0; l < 64; ++l) printf(" %d", h[64 * r + l] < 0 ? -1 : h[64 * r + l] - 1000); printf("\n"); }
    return 0;
}
