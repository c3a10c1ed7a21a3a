// chain_ilp_probe.hip — the EMA recurrence e = e + a (c - e) (three dependent fp64 ops per bar,
// -ffp-contract=off), 8 spans on one wave: one chain per lane (8 lanes) vs two chains per lane
// (4 lanes, spans q and q + 4 interleaved: ILP 2) vs four per lane (2 lanes), alone and next to
// 15 waves issuing fp64 work: chain cycles per bar. Development probe, not product code.
#include <hip/hip_runtime.h>

#include <cstdio>

template <int PER, int OTHERS>  // PER chains per lane (1, 2, 4); OTHERS: 0 none, 1 fp64 VALU
__global__ __launch_bounds__(1024) void chain(const int* close, int nbars, int busy_iters,
                                              double* out, unsigned long long* cyc) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (wave == 0) {
        double e[PER], a[PER];
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int q = lane + u * (8 / PER);
            a[u] = 2.0 / (10.0 * (q + 1) + 1.0);
            e[u] = (double)close[0];
        }
        int cn = close[lane];
        if (lane < 8 / PER) {
            for (int t0b = 0; t0b < nbars; t0b += 64) {
                const int cl = cn;
                cn = close[(t0b + 64 + lane) % nbars];
#pragma unroll
                for (int b = 0; b < 64; ++b) {
                    const double cd = (double)__builtin_amdgcn_readlane(cl, b);
#pragma unroll
                    for (int u = 0; u < PER; ++u) e[u] = e[u] + a[u] * (cd - e[u]);
                }
            }
        }
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();
        double s = 0;
#pragma unroll
        for (int u = 0; u < PER; ++u) s += e[u];
        out[lane] = s;
        if (lane == 0) cyc[0] = t1 - t0;
    } else if (OTHERS == 1) {
        double x = lane * 1.0001, y = 1.0 + wave * 1e-3;
        for (int i = 0; i < busy_iters; ++i) {
#pragma unroll
            for (int u = 0; u < 16; ++u) x = x * y + 1e-9;
        }
        out[64 + threadIdx.x] = x;
    }
}

template <int PER, int O>
void run(const int* dc, int nbars, double* dout, unsigned long long* dcyc) {
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL((chain<PER, O>), dim3(1), dim3(O ? 1024 : 64), 0, 0, dc, nbars, 3000, dout, dcyc);
        (void)hipDeviceSynchronize();
    }
    unsigned long long cyc[2] = {0, 0};
    (void)hipMemcpy(cyc, dcyc, 16, hipMemcpyDeviceToHost);
    printf("%d chains per lane, neighbours %d: %.1f cycles per bar (all 8 spans)\n", PER, O,
           (double)cyc[0] / nbars);
}

int main() {
    const int nbars = 64 * 1536;
    int* dc;
    double* dout;
    unsigned long long* dcyc;
    (void)hipMalloc(&dc, nbars * 4);
    (void)hipMalloc(&dout, 2048 * 8);
    (void)hipMalloc(&dcyc, 16);
    int* hc = new int[nbars];
    for (int i = 0; i < nbars; ++i) hc[i] = 1000000 + (i * 7919) % 5000;
    (void)hipMemcpy(dc, hc, nbars * 4, hipMemcpyHostToDevice);
    run<1, 0>(dc, nbars, dout, dcyc);
    run<2, 0>(dc, nbars, dout, dcyc);
    run<4, 0>(dc, nbars, dout, dcyc);
    run<1, 1>(dc, nbars, dout, dcyc);
    run<2, 1>(dc, nbars, dout, dcyc);
    run<4, 1>(dc, nbars, dout, dcyc);
    return 0;
}
