// k_topk.hip — per-GPU top-k of (symbol, param) results by Sharpe.
//
// Radix select on the 64-bit order key (orderable Sharpe), two 12-bit digits:
//   hist(bits 63..52) -> select -> hist(bits 51..40 | prefix) -> select
//   -> collect: records whose 24-bit prefix is above the selected one (< k of them) and the
//      candidates that share it -> finish: one block sorts them in LDS by
//      (key desc, sym asc, param asc) and writes the k result records.
// Six small launches (the finish block also resets the selection state), no host round trip; the host reads the count and k records in one copy. The order
// is exact and deterministic (atomics only decide collection order, which the sort removes).
// If more than kCap records tie on the 24-bit prefix (a tie-heavy grid), the finish block
// completes the exact selection on the device itself (topk_finish_ties), so the result never
// depends on a host fallback: single-GPU reads and the multi-GPU exchange (comm.cpp) get the same
// k records.
#include "internal.h"

namespace bt {

namespace {
constexpr int kBins = 4096;
// key counts up to which the histogram passes use global atomics only (topk_hist_global)
constexpr int64_t kHistGlobalMax = 1 << 18;
}

// state: [0] prefix, [1] mask of decided bits, [2] records still needed from the prefix group
__global__ __launch_bounds__(256) void topk_hist(const uint64_t* __restrict__ key, int64_t n, int shift,
                                                 const unsigned long long* __restrict__ state,
                                                 unsigned int* __restrict__ hist) {
    __shared__ unsigned int h[kBins];
    for (int i = threadIdx.x; i < kBins; i += blockDim.x) h[i] = 0;
    __syncthreads();
    const uint64_t prefix = state[0], mask = state[1];
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t k = key[i];
        if ((k & mask) == prefix) atomicAdd(&h[(k >> shift) & (kBins - 1)], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kBins; i += blockDim.x)
        if (h[i]) atomicAdd(&hist[i], h[i]);
}

// The same histogram without LDS: every matching key adds to the global bins directly. Used (up
// to kHistGlobalMax keys) behind a strategy kernel whose two blocks per CU fill the LDS (EMA+OLS
// in 128-bar stages: 2 x 80.2 KB), so that the chain's first kernel never takes LDS from a CU
// and both blocks can always be placed, whichever is dispatched first when a run ends: a 16-KB
// histogram block placed first split a CU's free LDS so that its second block waited for the
// first to finish, and the kernel ran up to 1.9x longer (profiles/r06/topk_lds_race.txt). Not
// by default: beside the Bollinger kernel (26 KB spare per CU) the global atomics on its 128k
// keys' few hot bins made the kernel 7 % slower.
__global__ __launch_bounds__(256) void topk_hist_global(const uint64_t* __restrict__ key, int64_t n,
                                                        int shift,
                                                        const unsigned long long* __restrict__ state,
                                                        unsigned int* __restrict__ hist) {
    const uint64_t prefix = state[0], mask = state[1];
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t k = key[i];
        if ((k & mask) == prefix) atomicAdd(&hist[(k >> shift) & (kBins - 1)], 1u);
    }
}

// One block of 256 threads; thread t owns bins 4095-16t .. 4080-16t (counted from the top).
// The owner of the k-th record is found by a block scan of the 256 partial sums; it resolves
// the bin from its own 16 counts. `need0` > 0 on the first digit (state[2] is set from it).
__global__ __launch_bounds__(256) void topk_select(unsigned int* __restrict__ hist, int shift,
                                                   unsigned long long* __restrict__ state,
                                                   unsigned long long need0) {
    __shared__ unsigned long long part[256];
    const int t = threadIdx.x;
    const int top = kBins - 1 - 16 * t;
    unsigned int c[16];
    unsigned long long s = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        c[j] = hist[top - j];
        s += c[j];
    }
    part[t] = s;
    __syncthreads();
    // inclusive Hillis-Steele scan over the 256 partial sums (bins from the top)
    for (int d = 1; d < 256; d <<= 1) {
        const unsigned long long v = t >= d ? part[t - d] : 0ULL;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    const unsigned long long need = need0 ? need0 : state[2];
    const unsigned long long incl = part[t], excl = incl - s;
    // owner: the first group whose inclusive count reaches `need` (the last group if the
    // histogram holds fewer records than need: then every record is taken)
    const bool owner = (excl < need && incl >= need) || (t == 255 && incl < need);
    __syncthreads();
    if (owner) {
        unsigned long long cum = excl;
        int bin = top - 15;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            if (cum + c[j] >= need) {
                bin = top - j;
                break;
            }
            cum += c[j];
        }
        state[0] |= (unsigned long long)bin << shift;
        state[1] |= (unsigned long long)(kBins - 1) << shift;
        state[2] = need - cum;
    }
    for (int i = t; i < kBins; i += blockDim.x) hist[i] = 0;  // ready for the next digit
}

__global__ __launch_bounds__(256) void topk_collect(const uint64_t* __restrict__ key, int64_t n,
                                                    const unsigned long long* __restrict__ state,
                                                    unsigned int* __restrict__ counts,
                                                    unsigned long long* __restrict__ above,
                                                    unsigned long long* __restrict__ cand, int cap) {
    const uint64_t prefix = state[0], mask = state[1];
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t m = key[i] & mask;
        if (m > prefix) {
            const unsigned int j = atomicAdd(&counts[0], 1u);
            if ((int)j < cap) above[j] = (unsigned long long)i;
        } else if (m == prefix) {
            const unsigned int j = atomicAdd(&counts[1], 1u);
            if ((int)j < cap) cand[j] = (unsigned long long)i;
        }
    }
}

// (sym id, param) of record idx, the tie-break order (ascending) as one 64-bit word.
__device__ __forceinline__ uint64_t sym_param(const SymDesc* __restrict__ syms, int32_t P,
                                              unsigned long long idx) {
    // 32-bit division whenever the index fits (a 64-bit one is a long software sequence)
    const bool small = idx < (1ULL << 32);
    const int s = small ? (int)((uint32_t)idx / (uint32_t)P) : (int)(idx / (unsigned long long)P);
    const int p = (int)(idx - (unsigned long long)s * (unsigned long long)P);
    return ((uint64_t)(uint32_t)syms[s].id << 32) | (uint32_t)p;
}

// One block of 256 threads over a 4096-bin histogram h counted from the top bin: the bin that
// holds the need-th record and how many records lie in the bins above it (the last bin and the
// total when h holds fewer than need). Same owner search as topk_select; `part` is 256 slots of
// shared scratch. Every thread returns the result.
__device__ void block_select(const unsigned int* h, unsigned long long need, unsigned long long* part,
                             int* bin_out, unsigned long long* above_out) {
    const int t = threadIdx.x;
    const int top = kBins - 1 - 16 * t;
    unsigned long long s = 0;
    for (int j = 0; j < 16; ++j) s += h[top - j];
    part[t] = s;
    __syncthreads();
    for (int d = 1; d < 256; d <<= 1) {
        const unsigned long long v = t >= d ? part[t - d] : 0ULL;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    const unsigned long long incl = part[t], excl = incl - s;
    const bool owner = (excl < need && incl >= need) || (t == 255 && incl < need);
    __syncthreads();
    if (owner) {
        unsigned long long cum = excl;
        int bin = top - 15;
        for (int j = 0; j < 16; ++j) {
            if (cum + h[top - j] >= need) {
                bin = top - j;
                break;
            }
            cum += h[top - j];
        }
        *bin_out = bin;
        *above_out = cum;
    }
    __syncthreads();
}

// The degenerate case of topk_finish: more than `cap` records share the selected 24-bit key
// prefix (a tie-heavy grid, e.g. flat prices where every Sharpe is 0). This block finishes the
// exact selection itself over the whole key array — the remaining 40 key bits by radix select
// (digits of 12, 12, 12 and 4 bits), then, among the records equal to the selected key, the
// (sym id, param) tie-break by a radix select on its complement — and gathers the indices of the
// min(k, n) best records into ix (at most k <= kTopkMax <= cap of them). Slow (a dozen passes of
// one block over the keys) but bounded, and only tie-heavy grids take it. Returns the count.
__device__ int topk_finish_ties(const uint64_t* __restrict__ key, int64_t nrec,
                                const SymDesc* __restrict__ syms, int32_t P, uint64_t prefix,
                                uint64_t mask, unsigned long long need, int32_t k,
                                unsigned int* h, uint64_t* ix, unsigned long long* part) {
    __shared__ int sh_bin;
    __shared__ unsigned long long sh_above;
    __shared__ unsigned int sh_n, sh_eq;
    const int t = threadIdx.x;
    // 1. the rest of the key: prefix/mask grow to all 64 bits; need = records wanted at that key
    for (int pass = 0; pass < 4; ++pass) {
        const int shift = pass < 3 ? 28 - 12 * pass : 0;
        const uint64_t dmask = pass < 3 ? (uint64_t)(kBins - 1) : 15ULL;
        for (int i = t; i < kBins; i += blockDim.x) h[i] = 0;
        __syncthreads();
        for (int64_t i = t; i < nrec; i += blockDim.x) {
            const uint64_t kx = key[i];
            if ((kx & mask) == prefix) atomicAdd(&h[(kx >> shift) & dmask], 1u);
        }
        __syncthreads();
        block_select(h, need, part, &sh_bin, &sh_above);
        prefix |= (uint64_t)sh_bin << shift;
        mask |= dmask << shift;
        need -= sh_above;
    }
    // 2. among key == prefix, the `need` smallest (sym id, param): the largest complements
    uint64_t tpre = 0, tmask = 0;
    for (int pass = 0; pass < 6; ++pass) {
        const int shift = pass < 5 ? 52 - 12 * pass : 0;
        const uint64_t dmask = pass < 5 ? (uint64_t)(kBins - 1) : 15ULL;
        for (int i = t; i < kBins; i += blockDim.x) h[i] = 0;
        __syncthreads();
        for (int64_t i = t; i < nrec; i += blockDim.x) {
            if (key[i] != prefix) continue;
            const uint64_t c = ~sym_param(syms, P, (unsigned long long)i);
            if ((c & tmask) == tpre) atomicAdd(&h[(c >> shift) & dmask], 1u);
        }
        __syncthreads();
        block_select(h, need, part, &sh_bin, &sh_above);
        tpre |= (uint64_t)sh_bin << shift;
        tmask |= dmask << shift;
        need -= sh_above;
    }
    // 3. gather: every key above the selected one, the tied keys whose tie-break ranks above
    // the selected (sym id, param), and `need` records equal to both (more than one only when
    // the caller's symbol ids repeat)
    if (t == 0) {
        sh_n = 0;
        sh_eq = 0;
    }
    __syncthreads();
    for (int64_t i = t; i < nrec; i += blockDim.x) {
        const uint64_t kx = key[i];
        bool take = kx > prefix;
        if (kx == prefix) {
            const uint64_t c = ~sym_param(syms, P, (unsigned long long)i);
            take = c > tpre || (c == tpre && atomicAdd(&sh_eq, 1u) < need);
        }
        if (take) {
            const unsigned int j = atomicAdd(&sh_n, 1u);
            if ((int)j < k) ix[j] = (uint64_t)i;
        }
    }
    __syncthreads();
    const int got = (int)sh_n;
    return got < k ? got : k;
}

__global__ __launch_bounds__(256) void topk_finish(
    const uint64_t* __restrict__ key, const bt_summary* __restrict__ sum,
    const SymDesc* __restrict__ syms, int64_t nrec, int32_t P,
    unsigned long long* __restrict__ state, unsigned int* __restrict__ counts,
    const unsigned long long* __restrict__ above, const unsigned long long* __restrict__ cand,
    int cap, int32_t k, bt_topk_rec* __restrict__ out, int32_t* __restrict__ out_n) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ unsigned long long part[256];
    uint64_t* kk = reinterpret_cast<uint64_t*>(smem);  // order key (desc)
    uint64_t* ss = kk + cap;                            // (sym id, param) (asc)
    uint64_t* ix = ss + cap;                            // record index (payload)
    const int n_above = (int)counts[0], n_cand = (int)counts[1];
    int n = n_above + n_cand;
    const bool ties = n > cap;
    // the tie histogram borrows the cap key slots (cap = kTopkCap, engine.cpp)
    static_assert(kTopkCap * sizeof(uint64_t) >= kBins * sizeof(unsigned int),
                  "topk_finish_ties' histogram must fit the key slots");
    if (ties) {  // the histogram (16 KB) borrows the key slots, filled only after the gather
        // state[2]: records still wanted from the prefix group (k minus those above it)
        n = topk_finish_ties(key, nrec, syms, P, state[0], state[1], state[2], k,
                             reinterpret_cast<unsigned int*>(kk), ix, part);
    }
    int m = 1;
    while (m < n) m <<= 1;
    for (int i = threadIdx.x; i < m; i += blockDim.x) {
        if (i < n) {
            const unsigned long long idx = ties ? ix[i] : (i < n_above ? above[i] : cand[i - n_above]);
            kk[i] = key[idx];
            ss[i] = sym_param(syms, P, idx);
            ix[i] = idx;
        } else {  // padding sorts last
            kk[i] = 0;
            ss[i] = ~0ULL;
            ix[i] = 0;
        }
    }
    __syncthreads();
    for (int size = 2; size <= m; size <<= 1) {  // bitonic: best first
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int i = threadIdx.x; i < m; i += blockDim.x) {
                const int j = i ^ stride;
                if (j > i) {
                    const bool up = (i & size) == 0;
                    const bool i_first = kk[i] > kk[j] || (kk[i] == kk[j] && ss[i] < ss[j]);
                    if (i_first != up) {
                        uint64_t t = kk[i];
                        kk[i] = kk[j];
                        kk[j] = t;
                        t = ss[i];
                        ss[i] = ss[j];
                        ss[j] = t;
                        t = ix[i];
                        ix[i] = ix[j];
                        ix[j] = t;
                    }
                }
            }
            __syncthreads();
        }
    }
    const int take = n < k ? n : k;
    for (int i = threadIdx.x; i < take; i += blockDim.x) {
        const bt_summary& r = sum[ix[i]];
        out[i] = bt_topk_rec{r.sharpe, (int32_t)(ss[i] >> 32), (int32_t)(uint32_t)ss[i], r.pnl};
    }
    __syncthreads();  // every read of state / counts is done: reset them for the next chain
    if (threadIdx.x == 0) {
        out_n[0] = take;
        state[0] = state[1] = state[2] = 0;
        counts[0] = counts[1] = 0;
    }
}


__global__ void topk_init(unsigned long long* state, unsigned int* counts, unsigned int* hist) {
    for (int i = threadIdx.x; i < kBins; i += blockDim.x) hist[i] = 0;
    if (threadIdx.x == 0) {
        state[0] = state[1] = state[2] = 0;
        counts[0] = counts[1] = 0;
    }
}

hipError_t launch_topk_init(const TopkWork& w, hipStream_t st) {
    hipLaunchKernelGGL(topk_init, dim3(1), dim3(256), 0, st, w.state, w.counts, w.hist);
    return hipGetLastError();
}

// The chain assumes the state left by topk_init or by the previous chain's finish; the
// histogram is left zeroed by topk_select.
hipError_t launch_topk(const uint64_t* key, const bt_summary* sum, const SymDesc* syms, int64_t n,
                       int32_t P, int32_t k, const TopkWork& w, hipStream_t st, bool lds_free_hist) {
    if (n <= 0 || k <= 0) return hipSuccess;
    const unsigned long long need = (unsigned long long)(k < n ? k : n);
    // few blocks, many keys per thread: each block adds its LDS histogram's non-empty bins to the
    // global one with device-scope atomics that pile up on the few bins a Sharpe distribution
    // fills (1,024 blocks made the chain ~0.34 ms per config-2 step, overlapped with the next kernel)
    int64_t blocks = (n + 8191) / 8192;
    if (blocks > 256) blocks = 256;
    for (int shift = 52; shift >= 40; shift -= 12) {
        if (lds_free_hist && n <= kHistGlobalMax)
            hipLaunchKernelGGL(topk_hist_global, dim3((unsigned)blocks), dim3(256), 0, st, key, n, shift,
                               (const unsigned long long*)w.state, w.hist);
        else
            hipLaunchKernelGGL(topk_hist, dim3((unsigned)blocks), dim3(256), 0, st, key, n, shift,
                               (const unsigned long long*)w.state, w.hist);
        hipLaunchKernelGGL(topk_select, dim3(1), dim3(256), 0, st, w.hist, shift, w.state,
                           shift == 52 ? need : 0ULL);
    }
    hipLaunchKernelGGL(topk_collect, dim3((unsigned)blocks), dim3(256), 0, st, key, n,
                       (const unsigned long long*)w.state, w.counts, w.above, w.cand, w.cap);
    // one small block (256 threads, the sort's 2,048 slots in 48 KB of LDS): it finds room on a CU
    // beside the next step's strategy kernel sooner than a 1,024-thread block
    hipLaunchKernelGGL(topk_finish, dim3(1), dim3(256), (size_t)w.cap * 24, st, key, sum, syms,
                       n, P, w.state, w.counts, w.above, w.cand, w.cap, k, w.out, w.out_n);
    return hipGetLastError();
}

}  // namespace bt
