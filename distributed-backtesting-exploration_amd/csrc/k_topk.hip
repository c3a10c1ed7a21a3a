// k_topk.hip — per-GPU top-k of (symbol, param) results by Sharpe.
//
// Radix select on the 64-bit order key (orderable Sharpe): eight 8-bit digit passes find the
// k-th largest key K exactly, then one pass collects every record with key > K (< k of them)
// and every record with key == K. The host orders those few candidates by
// (sharpe desc, sym asc, param asc); ties at K are resolved there, so the result is exact and
// deterministic regardless of atomics order.
#include "internal.h"

namespace bt {

__global__ __launch_bounds__(256) void topk_hist(const uint64_t* __restrict__ key, int64_t n,
                                                 int shift, const unsigned long long* state,
                                                 unsigned int* hist) {
    __shared__ unsigned int h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t prefix = state[0];
    const uint64_t hi_mask = shift >= 56 ? 0ULL : ~((1ULL << (shift + 8)) - 1);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t k = key[i];
        if ((k & hi_mask) == (prefix & hi_mask)) atomicAdd(&h[(k >> shift) & 255], 1u);
    }
    __syncthreads();
    if (h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], h[threadIdx.x]);
}

// One wave: find the digit holding the `need`-th largest key among the current prefix group.
__global__ void topk_select(int shift, unsigned long long* state, unsigned int* hist) {
    if (threadIdx.x == 0) {
        uint64_t need = state[1];
        uint64_t cum = 0;
        int d = 255;
        for (; d > 0; --d) {
            if (cum + hist[d] >= need) break;
            cum += hist[d];
        }
        state[0] |= (uint64_t)d << shift;
        state[1] = need - cum;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 256; i += blockDim.x) hist[i] = 0;
}

__global__ __launch_bounds__(256) void topk_collect(const uint64_t* __restrict__ key, int64_t n,
                                                    const unsigned long long* state,
                                                    unsigned int* counts,
                                                    unsigned long long* above,
                                                    unsigned long long* equal) {
    const uint64_t K = state[0];
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t k = key[i];
        if (k > K) above[atomicAdd(&counts[0], 1u)] = (unsigned long long)i;
        else if (k == K) equal[atomicAdd(&counts[1], 1u)] = (unsigned long long)i;
    }
}

__global__ void topk_init(unsigned long long* state, unsigned int* counts, unsigned int* hist,
                          unsigned long long need) {
    for (int i = threadIdx.x; i < 256; i += blockDim.x) hist[i] = 0;
    if (threadIdx.x == 0) {
        state[0] = 0;
        state[1] = need;
        counts[0] = counts[1] = 0;
    }
}

hipError_t launch_topk(const uint64_t* key, int64_t n, int32_t k, const TopkWork& w,
                       hipStream_t st) {
    if (n <= 0 || k <= 0) return hipSuccess;
    const unsigned long long need = (unsigned long long)(k < n ? k : n);
    hipLaunchKernelGGL(topk_init, dim3(1), dim3(256), 0, st, w.state, w.counts, w.hist, need);
    int64_t blocks = (n + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    for (int shift = 56; shift >= 0; shift -= 8) {
        hipLaunchKernelGGL(topk_hist, dim3((unsigned)blocks), dim3(256), 0, st, key, n, shift,
                           (const unsigned long long*)w.state, w.hist);
        hipLaunchKernelGGL(topk_select, dim3(1), dim3(64), 0, st, shift, w.state, w.hist);
    }
    hipLaunchKernelGGL(topk_collect, dim3((unsigned)blocks), dim3(256), 0, st, key, n,
                       (const unsigned long long*)w.state, w.counts, w.above, w.equal);
    return hipGetLastError();
}

}  // namespace bt
