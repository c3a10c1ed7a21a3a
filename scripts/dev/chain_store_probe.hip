// chain_store_probe.hip — where the EMA chain's per-bar LDS store goes: the recurrence (3
// dependent fp64 ops per bar, no FMA) on 8 lanes, 15 neighbour waves on 64-bit integer VALU,
// store placement: 0 none, 1 right after the value (compiler order), 2 the previous bar's value
// after this bar's subtract, 3 after its multiply, 4 pairs (ds_write2) after every second
// subtract. sched_barrier keeps the order. Development probe only.
#include <hip/hip_runtime.h>

#include <cstdio>

#define SB() __builtin_amdgcn_sched_barrier(0)

template <int MODE, int OTHERS>
__global__ __launch_bounds__(1024) void chain(const int* close, int nbars, int iters, double* out,
                                              unsigned long long* cyc) {
    __shared__ double lds[2 * 65 * 8 + 128];
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
                double prev = e, prev2 = e;
#pragma unroll
                for (int b = 0; b < 64; ++b) {
                    const double cd = (double)__builtin_amdgcn_readlane(cl, b);
                    if (MODE == 1) {
                        e = e + a * (cd - e);
                        E[b] = e;
                    } else if (MODE == 0) {
                        e = e + a * (cd - e);
                    } else {
                        const double d = cd - e;
                        SB();
                        if (MODE == 2 && b > 0) E[b - 1] = prev;
                        if (MODE == 4 && b > 1 && (b & 1) == 0) { E[b - 2] = prev2; E[b - 1] = prev; }
                        SB();
                        const double m = a * d;
                        SB();
                        if (MODE == 3 && b > 0) E[b - 1] = prev;
                        SB();
                        prev2 = prev;
                        e = e + m;
                        prev = e;
                    }
                }
                if (MODE >= 2) {
                    if (MODE == 4) E[62] = prev2;
                    E[63] = prev;
                }
            }
        }
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();
        out[lane] = e + lds[lane];
        if (lane == 0) cyc[0] = t1 - t0;
    } else if (OTHERS) {
        unsigned long long x = lane * 0x9E3779B97F4A7C15ull + wave, y = 0xBF58476D1CE4E5B9ull;
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int u = 0; u < 16; ++u) x = (x ^ (x >> 31)) * y + (unsigned long long)u;
        }
        out[64 + threadIdx.x] = (double)x;
    }
}

template <int M, int O>
void run(const int* dc, int nbars, double* dout, unsigned long long* dcyc) {
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL((chain<M, O>), dim3(1), dim3(O ? 1024 : 64), 0, 0, dc, nbars, 4000, dout, dcyc);
        (void)hipDeviceSynchronize();
    }
    unsigned long long cyc = 0;
    (void)hipMemcpy(&cyc, dcyc, 8, hipMemcpyDeviceToHost);
    double h[8];
    (void)hipMemcpy(h, dout, 64, hipMemcpyDeviceToHost);
    printf("mode %d neighbours %d: %.1f per bar (check %.6f)\n", M, O, (double)cyc / nbars, h[3]);
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
    run<0, 0>(dc, nbars, dout, dcyc);
    run<1, 0>(dc, nbars, dout, dcyc);
    run<2, 0>(dc, nbars, dout, dcyc);
    run<3, 0>(dc, nbars, dout, dcyc);
    run<4, 0>(dc, nbars, dout, dcyc);
    run<0, 1>(dc, nbars, dout, dcyc);
    run<1, 1>(dc, nbars, dout, dcyc);
    run<2, 1>(dc, nbars, dout, dcyc);
    run<3, 1>(dc, nbars, dout, dcyc);
    run<4, 1>(dc, nbars, dout, dcyc);
    return 0;
}
