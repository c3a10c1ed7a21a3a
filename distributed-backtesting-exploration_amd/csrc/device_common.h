// device_common.h — device helpers shared by the strategy kernels.
#pragma once
#include "internal.h"

namespace bt {

constexpr uint64_t kFnvOff = 0xCBF29CE484222325ULL;
constexpr uint64_t kFnvPrime = 0x100000001B3ULL;
constexpr int kDstLevels = 6;      // log2(kTile)
constexpr int kKeyStride = kTile + 1;  // +1 double per key row: conflict-free ds_read_b64

typedef __int128 i128;

// Price-path aggregate over a run of closes, in order: max, min, max drawdown (max over
// i<=j of c_i - c_j), max draw-up (max over i<=j of c_j - c_i). Prices < 2^31, so every
// field fits int32.
struct Agg {
    int32_t mx, mn, dd, du;
};

__device__ __forceinline__ Agg agg_one(int32_t x) { return Agg{x, x, 0, 0}; }

// Field-wise select (keeps both operands in registers: a ternary on the struct can become a
// two-element private array indexed at run time, i.e. scratch memory).
__device__ __forceinline__ Agg agg_sel(bool c, const Agg& a, const Agg& b) {
    return Agg{c ? a.mx : b.mx, c ? a.mn : b.mn, c ? a.dd : b.dd, c ? a.du : b.du};
}

// a happens before b
__device__ __forceinline__ Agg agg_merge(const Agg& a, const Agg& b) {
    Agg r;
    r.mx = max(a.mx, b.mx);
    r.mn = min(a.mn, b.mn);
    r.dd = max(max(a.dd, b.dd), a.mx - b.mn);
    r.du = max(max(a.du, b.du), b.mx - a.mn);
    return r;
}

// Disjoint sparse table over one tile of closes (kTile entries, kDstLevels levels).
// D[L*kTile + pos]: for level L (blocks of 2^(L+1)), the aggregate from pos to the block
// middle (left half) or from the middle+1 to pos (right half). Any range [a, b] inside the
// tile is then one merge of two entries: O(1) per trade, independent of trade length.
__device__ __forceinline__ void dst_build(Agg* D, const int32_t* cT, int tid, int nthreads) {
    for (int idx = tid; idx < kDstLevels * kTile; idx += nthreads) {
        const int L = idx / kTile, pos = idx % kTile;
        const int half = 1 << L;
        const int mid = (pos & ~(2 * half - 1)) + half - 1;
        Agg a;
        if (pos <= mid) {  // suffix pos..mid, built right-to-left
            a = agg_one(cT[mid]);
            for (int q = mid - 1; q >= pos; --q) {
                const int32_t x = cT[q];
                a.dd = max(a.dd, x - a.mn);
                a.du = max(a.du, a.mx - x);
                a.mx = max(a.mx, x);
                a.mn = min(a.mn, x);
            }
        } else {  // prefix mid+1..pos, built left-to-right
            a = agg_one(cT[mid + 1]);
            for (int q = mid + 2; q <= pos; ++q) {
                const int32_t x = cT[q];
                a.dd = max(a.dd, a.mx - x);
                a.du = max(a.du, x - a.mn);
                a.mx = max(a.mx, x);
                a.mn = min(a.mn, x);
            }
        }
        D[idx] = a;
    }
}

// Aggregate of closes cT[a..b], 0 <= a <= b < kTile.
__device__ __forceinline__ Agg dst_query(const Agg* D, const int32_t* cT, int a, int b) {
    if (a == b) return agg_one(cT[a]);
    const int L = 31 - __builtin_clz((unsigned)(a ^ b));
    return agg_merge(D[L * kTile + a], D[L * kTile + b]);
}

// Branch-free form: for a == b level 0 holds the single bar (D[0][a] == one(c_a)), and
// merging it with itself leaves max/min unchanged and gives drawdown/draw-up 0.
__device__ __forceinline__ Agg dst_query_bf(const Agg* D, int a, int b) {
    const unsigned x = (unsigned)(a ^ b);
    const int L = x ? 31 - __builtin_clz(x) : 0;
    return agg_merge(D[L * kTile + a], D[L * kTile + b]);
}

// Per-lane trade accounting state (spec §4), updated only at trade events.
// S1/S2 (spec §4) of an open trade are folded in at the entry (-side*Q1[e], -Q2[e]) and the
// exit (+side*Q1[x], +Q2[x]), so no per-trade prefix value has to stay live in registers.
struct Acct {
    int32_t pos, e, ce, ntr, expo;
    int64_t R, peak, mdd;
    i128 s1, s2;
    uint64_t h;
    Agg agg;  // closes [e, current tile start - 1] while a trade spans tiles
};

__device__ __forceinline__ void acct_init(Acct& a) {
    a.pos = 0;
    a.e = 0;
    a.ce = 0;
    a.ntr = 0;
    a.expo = 0;
    a.R = a.peak = a.mdd = 0;
    a.s1 = a.s2 = 0;
    a.h = kFnvOff;
    a.agg = Agg{0, 0, 0, 0};
}

// Close the open trade at bar x (tile offset bx) at price px; `st` = aggregate of the trade's
// MTM path (closes e..x for a close fill; closes e..x-1 plus the fill for an SL/TP fill).
__device__ __forceinline__ void acct_close(Acct& a, int x, int64_t px, const Agg& st, i128 q1x,
                                           i128 q2x, bt_trade* tr, int cap) {
    int64_t emin, emax, path, pnl;
    if (a.pos > 0) {
        emin = a.R + ((int64_t)st.mn - a.ce);
        emax = a.R + ((int64_t)st.mx - a.ce);
        path = st.dd;
        pnl = px - a.ce;
        a.s1 += q1x;
    } else {
        emin = a.R + ((int64_t)a.ce - st.mx);
        emax = a.R + ((int64_t)a.ce - st.mn);
        path = st.du;
        pnl = (int64_t)a.ce - px;
        a.s1 -= q1x;
    }
    a.s2 += q2x;
    a.mdd = max(a.mdd, max(a.peak - emin, path));
    a.peak = max(a.peak, emax);
    a.R += pnl;
    a.expo += x - a.e;
    const uint64_t w = (uint64_t)(uint32_t)a.e | ((uint64_t)(uint32_t)x << 31) |
                       ((uint64_t)(a.pos > 0) << 62);
    a.h = (a.h ^ w) * kFnvPrime;
    if (tr != nullptr && a.ntr < cap) {
        bt_trade r;
        r.entry_bar = a.e;
        r.exit_bar = x;
        r.side = a.pos;
        r.pad = 0;
        r.entry_px = a.ce;
        r.exit_px = px;
        tr[a.ntr] = r;
    }
    a.ntr++;
    a.pos = 0;
}

__device__ __forceinline__ void acct_open(Acct& a, int t, int side, int32_t ce, i128 q1, i128 q2) {
    a.pos = side;
    a.e = t;
    a.ce = ce;
    if (side > 0) a.s1 -= q1;
    else a.s1 += q1;
    a.s2 -= q2;
}

__device__ __forceinline__ void acct_write(const Acct& a, int bars, double sqrt_ann, size_t gi,
                                           const Out& out) {
    const uint64_t s1lo = (uint64_t)a.s1, s2lo = (uint64_t)a.s2;
    const int64_t s1hi = (int64_t)(a.s1 >> 64), s2hi = (int64_t)(a.s2 >> 64);
    const double sh = sharpe_fx(s1lo, s1hi, s2lo, s2hi, bars, sqrt_ann);
    bt_summary r;
    r.n_trades = a.ntr;
    r.status = 0;
    r.pnl = a.R;
    r.mdd = a.mdd;
    r.exposure = a.expo;
    r.sharpe = sh;
    r.hash = a.h;
    out.sum[gi] = r;
    out.key[gi] = order_key(sh);
    if (out.sums != nullptr) out.sums[gi] = bt_sums{s1lo, s1hi, s2lo, s2hi};
}

// Wave-wide inclusive scans (wave64).
__device__ __forceinline__ int64_t wave_scan_i64(int64_t x, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int64_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    return x;
}

__device__ __forceinline__ i128 wave_scan_i128(i128 x, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t lo = __shfl_up((unsigned long long)(uint64_t)x, d, 64);
        const int64_t hi = __shfl_up((long long)(int64_t)(x >> 64), d, 64);
        if (lane >= d) x += (i128)(((unsigned __int128)(uint64_t)hi << 64) | lo);
    }
    return x;
}

__device__ __forceinline__ i128 wave_bcast_i128(i128 x, int src) {
    const uint64_t lo = __shfl((unsigned long long)(uint64_t)x, src, 64);
    const uint64_t hi = __shfl((unsigned long long)(uint64_t)(x >> 64), src, 64);
    return (i128)(((unsigned __int128)hi << 64) | lo);
}

// q_t and q2_t of spec §3 for one bar.
__device__ __forceinline__ void fixed_ret(int32_t c, int32_t cp, int64_t& q, int64_t& q2) {
    const double ret = (double)((int64_t)c - cp) / (double)cp;
    q = (int64_t)rint(ret * 72057594037927936.0);
    const double rr = ret * ret;
    q2 = (int64_t)rint(rr * 72057594037927936.0);
}

__device__ __forceinline__ void wave_add_trades(const Out& out, int ntr) {
    unsigned long long v = (unsigned long long)ntr;
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) v += __shfl_down(v, d, 64);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(out.n_trades, v);
}

}  // namespace bt
