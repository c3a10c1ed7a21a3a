// chain_probe.hip — the EMA recurrence e = e + a (c - e) (three dependent fp64 ops per bar,
// -ffp-contract=off) on one wave (8 spans), with the chain values stored to LDS in several
// ways, alone and next to 15 waves issuing fp64 work or LDS reads: chain cycles per bar, and
// the neighbours' cycles for a fixed amount of work (how much the chain's variant slows them).
// Development probe, not product code.
#include <hip/hip_runtime.h>

#include <cstdio>

// MODE: 0 no store; 1 store per bar (8 lanes); 2 8 lanes, 4 stores per 8 bars from registers;
// 3 8 copies on 64 lanes, one store per 8 bars; 4 2 copies on 16 lanes, one 16-byte store per
// 4 bars; 5 4 copies on 32 lanes, one store per 4 bars
template <int MODE, int OTHERS>  // OTHERS: 0 none, 1 fp64 VALU, 2 LDS reads
__global__ __launch_bounds__(1024) void chain(const int* close, int nbars, int busy_iters,
                                              double* out, unsigned long long* cyc) {
    __shared__ __attribute__((aligned(16))) double E[2][8 * 66];
    __shared__ int4 junk[1024];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    junk[threadIdx.x] = int4{lane, wave, 1, 2};
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (wave == 0) {
        const int q = lane & 7, j = lane >> 3;
        const double alpha = 2.0 / (10.0 * (q + 1) + 1.0);
        double e = (double)close[0];
        int cn = close[lane];
        for (int t0b = 0; t0b < nbars; t0b += 64) {
            const int cl = cn;
            cn = close[(t0b + 64 + lane) % nbars];
            double* Eq = &E[(t0b >> 6) & 1][q * 66];
            if ((MODE <= 2 && lane < 8) || MODE == 3 || (MODE == 4 && lane < 16) || (MODE == 5 && lane < 32)) {
                double acc = 0.0;
                double2 acc2{0.0, 0.0};
                double hist[8];
#pragma unroll
                for (int b = 0; b < 64; ++b) {
                    const double cd = (double)__builtin_amdgcn_readlane(cl, b);
                    e = e + alpha * (cd - e);
                    if (MODE == 1) Eq[b] = e;
                    if (MODE == 2) {
                        hist[b & 7] = e;
                        if ((b & 7) == 7) {
#pragma unroll
                            for (int u = 0; u < 8; ++u) Eq[b - 7 + u] = hist[u];
                        }
                    }
                    if (MODE == 3) {
                        if (j == (b & 7)) acc = e;
                        if ((b & 7) == 7) Eq[b - 7 + j] = acc;
                    }
                    if (MODE == 4) {
                        if ((b & 3) == 2 * j) acc2.x = e;
                        if ((b & 3) == 2 * j + 1) acc2.y = e;
                        if ((b & 3) == 3) *reinterpret_cast<double2*>(&Eq[b - 3 + 2 * j]) = acc2;
                    }
                    if (MODE == 5) {
                        if (j == (b & 3)) acc = e;
                        if ((b & 3) == 3) Eq[b - 3 + j] = acc;
                    }
                }
            }
        }
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();
        out[lane] = e + E[0][lane] + E[1][lane];
        if (lane == 0) cyc[0] = t1 - t0;
    } else if (OTHERS == 1) {
        double x = lane * 1.0001, y = 1.0 + wave * 1e-3;
        for (int i = 0; i < busy_iters; ++i) {
#pragma unroll
            for (int u = 0; u < 16; ++u) x = x * y + 1e-9;
        }
        out[64 + threadIdx.x] = x;
        if (lane == 0 && wave == 1) cyc[1] = __builtin_amdgcn_s_memtime() - t0;
    } else if (OTHERS == 2) {
        int acc = 0;
        for (int i = 0; i < busy_iters; ++i) {
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int4 v = junk[(threadIdx.x + 37 * u + i) & 1023];
                acc += v.x ^ v.w;
            }
        }
        out[64 + threadIdx.x] = acc;
        if (lane == 0 && wave == 1) cyc[1] = __builtin_amdgcn_s_memtime() - t0;
    }
}

template <int M, int O>
void run(const char* what, const int* dc, int nbars, double* dout, unsigned long long* dcyc) {
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL((chain<M, O>), dim3(1), dim3(O ? 1024 : 64), 0, 0, dc, nbars, O == 1 ? 3000 : 2000, dout, dcyc);
        (void)hipDeviceSynchronize();
    }
    unsigned long long cyc[2] = {0, 0};
    (void)hipMemcpy(cyc, dcyc, 16, hipMemcpyDeviceToHost);
    printf("mode %d others %d %-44s chain %.1f cycles/bar, neighbour %llu kcycles\n", M, O, what,
           (double)cyc[0] / nbars, O ? cyc[1] / 1000 : 0ULL);
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
#define RUN3(M, txt) run<M, 0>(txt, dc, nbars, dout, dcyc); run<M, 1>(txt, dc, nbars, dout, dcyc); run<M, 2>(txt, dc, nbars, dout, dcyc);
    RUN3(0, "no store")
    RUN3(1, "store per bar, 8 lanes")
    RUN3(2, "8 lanes, stores grouped per 8 bars")
    RUN3(3, "8 copies / 64 lanes, 1 store per 8 bars")
    RUN3(4, "2 copies / 16 lanes, 16-B store per 4 bars")
    RUN3(5, "4 copies / 32 lanes, 1 store per 4 bars")
    return 0;
}
