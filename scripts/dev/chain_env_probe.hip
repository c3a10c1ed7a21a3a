// chain_env_probe.hip — the EMA recurrence (3 dependent fp64 ops per bar, no FMA) on 8 lanes of
// wave 0, each value stored to LDS in pairs as helper B does, with 15 neighbour waves doing
// (0) nothing, (1) fp64 FMA chains, (2) 64-bit integer VALU, (3) LDS ds_read_b128 streams,
// (4) LDS ds_write_b64 streams, (5) DPP scans: chain cycles per bar. Development probe only.
#include <hip/hip_runtime.h>

#include <cstdio>

template <int STORE, int OTHERS>
__global__ __launch_bounds__(1024) void chain(const int* close, int nbars, int iters, double* out,
                                              unsigned long long* cyc) {
    __shared__ double lds[2 * 65 * 8 + 16 * 1024];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (wave == 0) {
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
        double a = 2.0 / (10.0 * (lane + 1) + 1.0), e = (double)close[0];
        int cn = close[lane];
        if (lane < 8) {
            for (int t0b = 0; t0b < nbars; t0b += 64) {
                const int cl = cn;
                cn = close[(t0b + 64 + lane) % nbars];
                double* E = lds + ((t0b >> 6) & 1) * 65 * 8 + lane * 65;
#pragma unroll
                for (int b = 0; b < 64; ++b) {
                    const double cd = (double)__builtin_amdgcn_readlane(cl, b);
                    e = e + a * (cd - e);
                    if (STORE) E[b] = e;
                }
            }
        }
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();
        out[lane] = e + lds[lane];
        if (lane == 0) cyc[0] = t1 - t0;
    } else if (OTHERS == 1) {
        double x = lane * 1.0001, y = 1.0 + wave * 1e-3;
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int u = 0; u < 16; ++u) x = x * y + 1e-9;
        }
        out[64 + threadIdx.x] = x;
    } else if (OTHERS == 2) {
        unsigned long long x = lane * 0x9E3779B97F4A7C15ull + wave, y = 0xBF58476D1CE4E5B9ull;
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int u = 0; u < 16; ++u) x = (x ^ (x >> 31)) * y + (unsigned long long)u;
        }
        out[64 + threadIdx.x] = (double)x;
    } else if (OTHERS == 3) {
        const int4* p = reinterpret_cast<const int4*>(lds + 2 * 65 * 8);
        int4 acc = {0, 0, 0, 0};
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const int4 v = p[((lane + u * 64 + i) & 1023) ^ wave];
                acc.x ^= v.x; acc.y += v.y; acc.z ^= v.z; acc.w += v.w;
            }
        }
        out[64 + threadIdx.x] = acc.x + acc.y + acc.z + acc.w;
    } else if (OTHERS == 4) {
        double* p = lds + 2 * 65 * 8 + wave * 512;
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int u = 0; u < 16; ++u) p[(lane + u * 8) & 511] = (double)(i + u);
        }
    } else if (OTHERS == 5) {
        long long x = lane + wave;
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                x += __builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);
                x += __builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);
                x += __builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);
                x += __builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);
            }
        }
        out[64 + threadIdx.x] = (double)x;
    }
}

template <int S, int O>
void run(const int* dc, int nbars, double* dout, unsigned long long* dcyc, const char* what) {
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL((chain<S, O>), dim3(1), dim3(O ? 1024 : 64), 0, 0, dc, nbars, 4000, dout, dcyc);
        (void)hipDeviceSynchronize();
    }
    unsigned long long cyc = 0;
    (void)hipMemcpy(&cyc, dcyc, 8, hipMemcpyDeviceToHost);
    printf("stores %d, neighbours %-22s: %.1f per bar\n", S, what, (double)cyc / nbars);
}

int main() {
    const int nbars = 64 * 1024;
    int* dc;
    double* dout;
    unsigned long long* dcyc;
    (void)hipMalloc(&dc, nbars * 4);
    (void)hipMalloc(&dout, 2048 * 8);
    (void)hipMalloc(&dcyc, 16);
    int* hc = new int[nbars];
    for (int i = 0; i < nbars; ++i) hc[i] = 1000000 + (i * 7919) % 5000;
    (void)hipMemcpy(dc, hc, nbars * 4, hipMemcpyHostToDevice);
    run<0, 0>(dc, nbars, dout, dcyc, "none");
    run<1, 0>(dc, nbars, dout, dcyc, "none");
    run<1, 1>(dc, nbars, dout, dcyc, "fp64 FMA");
    run<1, 2>(dc, nbars, dout, dcyc, "64-bit integer");
    run<1, 3>(dc, nbars, dout, dcyc, "LDS ds_read_b128");
    run<1, 4>(dc, nbars, dout, dcyc, "LDS ds_write_b64");
    run<1, 5>(dc, nbars, dout, dcyc, "DPP scans");
    run<0, 2>(dc, nbars, dout, dcyc, "64-bit integer");
    run<0, 3>(dc, nbars, dout, dcyc, "LDS ds_read_b128");
    return 0;
}
