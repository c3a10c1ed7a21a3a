// Issue-rate probe: N independent chains per lane of one VALU instruction kind, many waves per
// SIMD; prints cycles per instruction per SIMD (s_memtime around the loop). Build:
//   hipcc --offload-arch=gfx950 -O3 scripts/dev/rate_probe.hip -o scripts/dev/rate_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int KIND>
__global__ void probe(uint64_t* out, unsigned long long* cyc, int iters) {
    uint64_t a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13, a6 = a0 * 17, a7 = a0 * 19;
    const uint64_t b = blockIdx.x + 12345;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#define OP(x)                                                                                      \
        if (KIND == 0) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(x) : "v"(b));           \
        else if (KIND == 1) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(*(uint32_t*)&x) : "v"((uint32_t)b)); \
        else asm volatile("v_alignbit_b32 %0, %0, %1, 31" : "+v"(*(uint32_t*)&x) : "v"((uint32_t)b));
        OP(a0) OP(a1) OP(a2) OP(a3) OP(a4) OP(a5) OP(a6) OP(a7)
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    if (threadIdx.x == 0) atomicAdd(cyc, (unsigned long long)(t1 - t0));
}

int main() {
    uint64_t* out; unsigned long long* cyc;
    const int cus = 256, waves = 16, iters = 4096;  // 16 waves per CU = 4 per SIMD
    hipMalloc(&out, (size_t)cus * waves * 64 * 8);
    hipMalloc(&cyc, 8);
    const char* names[3] = {"v_lshl_add_u64", "v_sub_u32", "v_alignbit_b32"};
    for (int kind = 0; kind < 3; ++kind) {
        for (int rep = 0; rep < 2; ++rep) {
            hipMemset(cyc, 0, 8);
            if (kind == 0) hipLaunchKernelGGL(probe<0>, dim3(cus), dim3(64 * waves), 0, 0, out, cyc, iters);
            if (kind == 1) hipLaunchKernelGGL(probe<1>, dim3(cus), dim3(64 * waves), 0, 0, out, cyc, iters);
            if (kind == 2) hipLaunchKernelGGL(probe<2>, dim3(cus), dim3(64 * waves), 0, 0, out, cyc, iters);
            unsigned long long c = 0;
            hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
            // per block (CU): cycles / (waves per SIMD * instructions per wave) = cycles per instr per SIMD
            const double per_block = (double)c / cus;
            printf("%-16s %.2f cycles per wave-instruction per SIMD\n", names[kind], per_block / ((double)iters * 8 * (waves / 4)));
        }
    }
    return 0;
}
