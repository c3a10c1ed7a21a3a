// k_gen.hip — synthetic OHLCV straight into HBM (spec §1 / SURVEY A.1), one wave per symbol.
//
// The SplitMix64 stream is in counter form, so every draw is a pure function of
// (seed, symbol, draw index); only the multiplicative walk is sequential along the bar axis.
// Output rows are int32 ticks at SymDesc::off in each column (column pointers may be null).
#include "internal.h"

namespace bt {

__device__ __forceinline__ uint64_t sm64(uint64_t s0, uint64_t k) {
    uint64_t z = s0 + (k + 1) * 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

// One wave per symbol, 64 bars per chunk: lane = bar draws the chunk's moves and the high/low
// offsets (the 64-bit modular reductions are most of the cost), then the closes are chained
// through the chunk on the wave-uniform `prev` (one multiply, one division by a constant per bar)
// and lane j takes bar j's open and close.
__global__ __launch_bounds__(256) void gen_kernel(const SymDesc* __restrict__ syms, int32_t n_sym,
                                                  uint64_t seed, int32_t freq, int32_t* o,
                                                  int32_t* h, int32_t* l, int32_t* c) {
    const int s = (int)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
    const int lane = (int)(threadIdx.x & 63);
    if (s >= n_sym) return;  // wave-uniform
    const SymDesc sd = syms[s];
    const uint64_t s0 = seed ^ ((uint64_t)(int64_t)sd.id * 0x9E3779B97F4A7C15ULL);
    const int64_t m = freq == BT_DAILY ? 17320 : 866;
    const uint64_t span = (uint64_t)(2 * m + 1);
    const uint64_t r = (uint64_t)(m / 4 + 1);
    int64_t prev = 1000000 + (int64_t)(sm64(s0, 0) % 9000001ULL);
    for (int t0 = 0; t0 < sd.bars; t0 += 64) {
        const int t = t0 + lane;
        const uint64_t base = 1 + 7 * (uint64_t)t;
        int64_t x = 0;
        if (t > 0 && t < sd.bars)
            x = (int64_t)(sm64(s0, base) % span) + (int64_t)(sm64(s0, base + 1) % span) +
                (int64_t)(sm64(s0, base + 2) % span) + (int64_t)(sm64(s0, base + 3) % span) - 4 * m;
        int64_t hr = 0, lr = 0;
        if ((h || l) && t < sd.bars) {
            hr = (int64_t)(sm64(s0, base + 4) % r);
            lr = (int64_t)(sm64(s0, base + 5) % r);
        }
        const int n = min(64, sd.bars - t0);
        uint32_t cl_l = 0, op_l = 0;  // this lane's bar
        for (int j = 0; j < n; ++j) {
            const int64_t xj = (int64_t)(((uint64_t)__builtin_amdgcn_readlane((uint32_t)((uint64_t)x >> 32), j) << 32) |
                                         __builtin_amdgcn_readlane((uint32_t)x, j));
            int64_t cl = prev;
            if (t0 + j > 0) {
                cl = prev + (xj * prev) / 1000000;  // truncation toward zero
                cl = cl < 10000 ? 10000 : cl;
                cl = cl > 2146435072LL ? 2146435072LL : cl;  // 2^31 - 2^20
            }
            if (lane == j) {
                op_l = (uint32_t)prev;
                cl_l = (uint32_t)cl;
            }
            prev = cl;
        }
        if (t < sd.bars) {
            const int64_t cl = (int32_t)cl_l, op = (int32_t)op_l;
            const size_t i = (size_t)sd.off + t;
            if (c) c[i] = (int32_t)cl;
            if (o) o[i] = (int32_t)op;
            if (h || l) {
                const int64_t hi = op > cl ? op : cl, lo = op < cl ? op : cl;
                int64_t ll = lo - lr;
                ll = ll < 10000 ? 10000 : ll;
                if (h) h[i] = (int32_t)(hi + hr);
                if (l) l[i] = (int32_t)ll;
            }
        }
    }
}

hipError_t launch_gen(const SymDesc* syms, int32_t n_sym, uint64_t seed, int32_t freq,
                      int32_t* o, int32_t* h, int32_t* l, int32_t* c, hipStream_t st) {
    if (n_sym <= 0) return hipSuccess;
    hipLaunchKernelGGL(gen_kernel, dim3((n_sym + 3) / 4), dim3(256), 0, st, syms, n_sym, seed,
                       freq, o, h, l, c);
    return hipGetLastError();
}

}  // namespace bt
