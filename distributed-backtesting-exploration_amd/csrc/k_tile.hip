// k_tile.hip — EMA + rolling-OLS (config 3) and Bollinger + SL/TP (config 4) backtests in the
// same tile pipeline as the SMA kernel: one workgroup per symbol, one lane per parameter.
//
// Hot path of BASELINE.json north_star (configs 3 and 4), replacing the sleep in
// process_incoming_job (/root/reference/src/worker/process.rs:21-25). Spec:
// docs/oracle_spec.md §3-§5; checked bit-for-bit against oracle/oracle.c (orc_ema_ols, orc_boll).
//
// Every signal condition of these strategies factors into per-indicator conditions, so a whole
// 64-bar tile of them is a handful of 64-bit words shared by all lanes:
//   EMA+OLS (n, w): enter long  = [c*1e4 < e_n*(1e4-b)] & [N_w >= 0]
//                   enter short = [c*1e4 > e_n*(1e4+b)] & [N_w <= 0] (and not long)
//                   exit long = [c >= e_n], exit short = [c <= e_n]
//   Bollinger (w, k, sl, tp): enter long = [z_w < -k], short = [z_w > k];
//                   signal exit long = [D_w >= 0], short = [D_w <= 0]; SL/TP hits depend on the
//                   entry price and are found by binary lifting over per-tile min-low /
//                   max-high sparse tables.
// Workgroup = parameter waves + 2 helper waves, one barrier per tile:
//   helper A, tile k+2: closes (loaded one tile ahead) -> returns, drawdown sparse table, prefix
//            rings (and, for Bollinger, the low/high sparse tables);
//   helper B, tile k+1: indicator condition words (EMA: one sequential fp64 chain per span, lane
//            = span, then ballots with lane = bar; OLS numerator and Bollinger D, Q from the
//            prefix rings in exact (wrapping) integer arithmetic, ballots with lane = bar);
//   parameter waves, tile k: each lane ANDs its words and walks only its position changes
//            (ctz), O(1) accounting per change (tile_common.h).
#include <algorithm>

#include "tile_common.h"

namespace bt {

namespace {

constexpr int kEStride = kTile + 1;  // ema buffer row stride (doubles): conflict-free columns

struct TileLds {
    size_t r1, r2, ct, ql, dst, stl, sth, ebuf, words, win, total;
};

// kind 0 = EMA+OLS (na spans, nb windows), 1 = Bollinger (na windows, nb ks)
__host__ __device__ inline TileLds tile_lds_layout(int kind, int ring, int na, int nb) {
    TileLds L{};
    size_t o = 0;
    auto take = [&](size_t bytes) { size_t r = o; o += (bytes + 15) & ~size_t(15); return r; };
    L.r1 = take((size_t)ring * 8);
    L.r2 = take((size_t)ring * (kind == 0 ? 8 : 16));
    L.ct = take((size_t)kTileStages * kTile * 4);
    L.ql = take((size_t)kTileStages * 2 * kTile * 8);
    L.dst = take((size_t)kTileStages * kDstLevels * kTile * sizeof(Agg));
    if (kind == 1) {
        L.stl = take((size_t)kTileStages * kDstLevels * kTile * 4);
        L.sth = take((size_t)kTileStages * kDstLevels * kTile * 4);
        L.words = take((size_t)2 * (2 * na * nb + 2 * na) * 8);
        L.win = take((size_t)na * 4);
    } else {
        L.ebuf = take((size_t)na * kEStride * 8);
        L.words = take((size_t)2 * (4 * na + 2 * nb) * 8);
        L.win = take((size_t)nb * 4);
    }
    L.total = o;
    return L;
}

__device__ __forceinline__ int32_t ldc(const int32_t* __restrict__ row, int B, int t, int32_t pad) {
    return t < B ? row[t] : pad;
}

// First in-tile bar >= a whose low is <= X (64 if none): binary lifting over
// ST[k][i] = min(low[i .. i + 2^k)).
__device__ __forceinline__ int first_le(const int32_t* ST, int a, int64_t X) {
    int pos = a;
#pragma unroll
    for (int k = kDstLevels - 1; k >= 0; --k) {
        const int len = 1 << k;
        const int32_t v = ST[k * kTile + min(pos, kTile - 1)];
        pos += (pos + len <= kTile && (int64_t)v > X) ? len : 0;
    }
    // the skips sum to at most 63: from bar 0 a tile without a hit stops on bar 63
    return (pos < kTile && (int64_t)ST[pos] > X) ? kTile : pos;
}

// First in-tile bar >= a whose high is >= X: ST[k][i] = max(high[i .. i + 2^k)).
__device__ __forceinline__ int first_ge(const int32_t* ST, int a, int64_t X) {
    int pos = a;
#pragma unroll
    for (int k = kDstLevels - 1; k >= 0; --k) {
        const int len = 1 << k;
        const int32_t v = ST[k * kTile + min(pos, kTile - 1)];
        pos += (pos + len <= kTile && (int64_t)v < X) ? len : 0;
    }
    return (pos < kTile && (int64_t)ST[pos] < X) ? kTile : pos;
}

}  // namespace

// ----------------------------------------------------------------------------- EMA + OLS
template <bool PARITY>
__global__ __launch_bounds__(1024) void ema_tile_kernel(const SymDesc* __restrict__ syms,
                                                        const int32_t* __restrict__ close,
                                                        Grid g, Out out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int nsp = g.na, nol = g.nb, R = g.ring, RM = g.ring - 1;
    const TileLds LL = tile_lds_layout(0, R, nsp, nol);
    uint64_t* r1 = reinterpret_cast<uint64_t*>(smem + LL.r1);  // sum_{i<x} c_i
    uint64_t* r2 = reinterpret_cast<uint64_t*>(smem + LL.r2);  // sum_{i<x} i*c_i (mod 2^64)
    int32_t* cts = reinterpret_cast<int32_t*>(smem + LL.ct);
    int64_t* qls = reinterpret_cast<int64_t*>(smem + LL.ql);
    Agg* dst = reinterpret_cast<Agg*>(smem + LL.dst);
    double* ebuf = reinterpret_cast<double*>(smem + LL.ebuf);
    uint64_t* words = reinterpret_cast<uint64_t*>(smem + LL.words);
    int32_t* win = reinterpret_cast<int32_t*>(smem + LL.win);

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int npw = (int)(blockDim.x >> 6) - 2;
    const bool helperA = wave == npw, helperB = wave == npw + 1;
    const SymDesc sd = syms[blockIdx.x];
    const int B = sd.bars, ntiles = (B + kTile - 1) / kTile, P = g.n_params;
    const int j = blockIdx.y * npw * 64 + tid;
    const bool active = wave < npw && j < P;
    const int pj = active ? j : 0;
    const int i_n = pj / nol, i_w = pj % nol;
    const int warm = max(g.a[i_n], g.b[i_w]) - 1;
    const int32_t* crow = close + sd.off;
    const int nword = 4 * nsp + 2 * nol;

    for (int o = tid; o < nol; o += blockDim.x) win[o] = g.b[o];
    if (tid == 0) r1[0] = r2[0] = 0;
    double alpha = 0.0, ema = 0.0;
    if (helperB && lane < nsp) alpha = 2.0 / ((double)g.a[lane] + 1.0);
    const double lo_mult = (double)(10000 - g.band_bps), hi_mult = (double)(10000 + g.band_bps);
    __syncthreads();

    TileCarry cy{0, 0};
    uint64_t cy2 = 0;
    int32_t cpre = 0;

    auto scanA = [&](int T, int32_t c) {
        const int s = T % kTileStages, t0 = T * kTile, t = t0 + lane;
        const int64_t pre = tile_scan(c, B, t0, lane, cts + s * kTile, qls + s * 2 * kTile,
                                      dst + s * kDstLevels * kTile, cy);
        r1[(t + 1) & RM] = (uint64_t)pre;
        const int64_t inc2 = wave_iscan_i64((int64_t)t * c);  // c = 0 past the end
        r2[(t + 1) & RM] = cy2 + (uint64_t)inc2;
        cy2 += (uint64_t)lane63_i64(inc2);
    };

    auto flagsB = [&](int T) {
        const int s = T % kTileStages, t1 = T * kTile, t = t1 + lane;
        const int32_t cl = cts[s * kTile + lane];
        uint64_t* W = words + (T & 1) * nword;
        // EMA chains, lane = span: e_t = e_{t-1} + alpha (c_t - e_{t-1}), three roundings
        if (lane < nsp) {
            if (t1 > 0 && t1 + kTile <= B) {
#pragma unroll
                for (int b = 0; b < kTile; ++b) {
                    const double cd = (double)__builtin_amdgcn_readlane(cl, b);
                    ema = ema + alpha * (cd - ema);
                    ebuf[lane * kEStride + b] = ema;
                }
            } else {
#pragma unroll 1
                for (int b = 0; b < kTile; ++b) {
                    const double cd = (double)__builtin_amdgcn_readlane(cl, b);
                    if (t1 + b < B) ema = (t1 + b == 0) ? cd : ema + alpha * (cd - ema);
                    ebuf[lane * kEStride + b] = ema;
                }
            }
        }
        // lane = bar from here on
        const double cd = (double)cl;
        const double lhs = cd * 10000.0;
#pragma unroll 1
        for (int sp = 0; sp < nsp; ++sp) {
            const double e = ebuf[sp * kEStride + lane];
            const uint64_t wa = __ballot(lhs < e * lo_mult), wb = __ballot(lhs > e * hi_mult);
            const uint64_t wx = __ballot(cd >= e), wy = __ballot(cd <= e);
            if (lane == 0) {
                W[4 * sp + 0] = wa;
                W[4 * sp + 1] = wb;
                W[4 * sp + 2] = wx;
                W[4 * sp + 3] = wy;
            }
        }
        // OLS centred numerator N = 2 T - (w-1) S over [t-w+1, t], exact modulo 2^64
        const uint64_t P1t = r1[(t + 1) & RM], P2t = r2[(t + 1) & RM];
#pragma unroll 1
        for (int o = 0; o < nol; ++o) {
            const int Wn = win[o];
            const int jj = t + 1 - Wn;
            const bool valid = jj >= 0 && t < B;
            const uint64_t S = P1t - r1[jj & RM];
            const uint64_t Tq = (P2t - r2[jj & RM]) - (uint64_t)(int64_t)jj * S;
            const int64_t N = (int64_t)(2 * Tq - (uint64_t)(Wn - 1) * S);
            const uint64_t wp = __ballot(valid && N >= 0), wn = __ballot(valid && N <= 0);
            if (lane == 0) {
                W[4 * nsp + 2 * o] = wp;
                W[4 * nsp + 2 * o + 1] = wn;
            }
        }
    };

    // prologue: scan tiles 0, 1; flag tile 0
    if (helperA) {
        const int32_t c0 = ldc(crow, B, lane, 0), c1 = ldc(crow, B, kTile + lane, 0);
        cpre = ldc(crow, B, 2 * kTile + lane, 0);
        scanA(0, c0);
        __syncthreads();
        if (ntiles > 1) scanA(1, c1);
    } else {
        __syncthreads();
        if (helperB) flagsB(0);
    }
    __syncthreads();

    TradeAcct a;
    acct_init(a);
    const size_t gi = (size_t)blockIdx.x * P + pj;
    bt_trade* tr = (PARITY && active) ? out.trades + gi * out.trade_cap : nullptr;
    const int cap = out.trade_cap;

    for (int k = 0; k < ntiles; ++k) {
        const int t0 = k * kTile;
        if (helperA && k + 2 < ntiles) {
            scanA(k + 2, cpre);
            cpre = ldc(crow, B, t0 + 3 * kTile + lane, 0);
        }
        if (helperB && k + 1 < ntiles) flagsB(k + 1);
        if (active) {
            const int s = k % kTileStages;
            const int32_t* cT = cts + s * kTile;
            const int64_t* ql = qls + s * 2 * kTile;
            const Agg* D = dst + s * kDstLevels * kTile;
            const uint64_t* W = words + (k & 1) * nword;
            const uint64_t vm = bar_range_mask(t0, warm, B - 2);
            const uint64_t Aw = W[4 * i_n] & W[4 * nsp + 2 * i_w] & vm;
            const uint64_t Bw = W[4 * i_n + 1] & W[4 * nsp + 2 * i_w + 1] & vm & ~Aw;
            const uint64_t Xw = W[4 * i_n + 2] & vm, Yw = W[4 * i_n + 3] & vm;
            const int bl = B - 1 - t0;
            const uint64_t fb = (bl >= 0 && bl < kTile) ? (1ULL << bl) : 0ULL;
            int cur = 0;
            while (cur < kTile) {  // one position change per iteration, in bar order
                const uint64_t el = ~0ULL << cur;
                const uint64_t m = (a.pos == 0 ? (Aw | Bw) : ((a.pos > 0 ? Xw : Yw) | fb)) & el;
                if (m == 0) break;
                const int b = __builtin_ctzll(m);
                const int t = t0 + b;
                const int32_t cx = cT[b];
                const uint64_t qx = (uint64_t)ql[b], q2x = (uint64_t)ql[kTile + b];
                if (a.pos == 0) {
                    const int np = ((Aw >> b) & 1) ? 1 : -1;
                    a.ps1 += np > 0 ? (uint64_t)0 - qx : qx;
                    a.ps2 -= q2x;
                    acct_open(a, t, b, cx);
                    a.pos = np;
                } else {
                    const Agg st = agg_merge(a.agg, dst_query_bf(D, a.sb, b));
                    acct_close<PARITY>(a, t, cx, st, tr, cap);
                    a.ps1 += a.pos > 0 ? qx : (uint64_t)0 - qx;
                    a.ps2 += q2x;
                    a.pos = 0;
                }
                cur = b + 1;
            }
            acct_tile_end(a, D, ql);
        }
        __syncthreads();
    }
    if (active) acct_write(a, B, g.sqrt_ann, gi, out);
    wave_add_trades(out, active ? a.ntr : 0);
}

// ----------------------------------------------------------------------------- Bollinger
template <bool PARITY>
__global__ __launch_bounds__(1024) void boll_tile_kernel(const SymDesc* __restrict__ syms,
                                                         const int32_t* __restrict__ high,
                                                         const int32_t* __restrict__ low,
                                                         const int32_t* __restrict__ close,
                                                         Grid g, Out out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int nw = g.na, nk = g.nb, R = g.ring, RM = g.ring - 1;
    const TileLds LL = tile_lds_layout(1, R, nw, nk);
    uint64_t* r1 = reinterpret_cast<uint64_t*>(smem + LL.r1);                    // sum c
    unsigned __int128* r2 = reinterpret_cast<unsigned __int128*>(smem + LL.r2);  // sum c^2
    int32_t* cts = reinterpret_cast<int32_t*>(smem + LL.ct);
    int64_t* qls = reinterpret_cast<int64_t*>(smem + LL.ql);
    Agg* dst = reinterpret_cast<Agg*>(smem + LL.dst);
    int32_t* stl = reinterpret_cast<int32_t*>(smem + LL.stl);
    int32_t* sth = reinterpret_cast<int32_t*>(smem + LL.sth);
    uint64_t* words = reinterpret_cast<uint64_t*>(smem + LL.words);
    int32_t* win = reinterpret_cast<int32_t*>(smem + LL.win);

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int npw = (int)(blockDim.x >> 6) - 2;
    const bool helperA = wave == npw, helperB = wave == npw + 1;
    const SymDesc sd = syms[blockIdx.x];
    const int B = sd.bars, ntiles = (B + kTile - 1) / kTile, P = g.n_params;
    const int j = blockIdx.y * npw * 64 + tid;
    const bool active = wave < npw && j < P;
    const int pj = active ? j : 0;
    // param = ((iw * nk + ik) * nsl + isl) * ntp + itp
    const int itp = pj % g.nd, isl = (pj / g.nd) % g.nc, ik = (pj / (g.nd * g.nc)) % nk,
              iw = pj / (g.nd * g.nc * nk);
    const int w = g.a[iw];
    const int64_t sl_bps = g.c[isl], tp_bps = g.d[itp];
    const int32_t* crow = close + sd.off;
    const int32_t* hrow = high + sd.off;
    const int32_t* lrow = low + sd.off;
    const int nword = 2 * nw * nk + 2 * nw;
    const i128 kd2 = (i128)((int64_t)g.k_den * g.k_den);

    for (int o = tid; o < nw; o += blockDim.x) win[o] = g.a[o];
    if (tid == 0) {
        r1[0] = 0;
        r2[0] = 0;
    }
    __syncthreads();

    TileCarry cy{0, 0};
    unsigned __int128 cy2 = 0;
    int32_t cpre = 0, hpre = 0, lpre = 0;

    auto scanA = [&](int T, int32_t c, int32_t hv, int32_t lv) {
        const int s = T % kTileStages, t0 = T * kTile, t = t0 + lane;
        const int64_t pre = tile_scan(c, B, t0, lane, cts + s * kTile, qls + s * 2 * kTile,
                                      dst + s * kDstLevels * kTile, cy);
        r1[(t + 1) & RM] = (uint64_t)pre;
        // sum of c^2 in 128 bits: scan the 32-bit halves of c^2 < 2^62 separately
        const uint64_t c2 = (uint64_t)((int64_t)c * c);
        const int64_t slo = wave_iscan_i64((int64_t)(c2 & 0xFFFFFFFFu));
        const int64_t shi = wave_iscan_i64((int64_t)(c2 >> 32));
        const unsigned __int128 inc2 = ((unsigned __int128)(uint64_t)shi << 32) + (uint64_t)slo;
        r2[(t + 1) & RM] = cy2 + inc2;
        cy2 += ((unsigned __int128)(uint64_t)lane63_i64(shi) << 32) + (uint64_t)lane63_i64(slo);
        // low / high sparse tables for SL/TP first-passage search
        int32_t* SL = stl + s * kDstLevels * kTile;
        int32_t* SH = sth + s * kDstLevels * kTile;
        int32_t mn = lv, mx = hv;
        SL[lane] = mn;
        SH[lane] = mx;
#pragma unroll
        for (int m = 1; m < kDstLevels; ++m) {
            const int d = 1 << (m - 1);
            mn = min(mn, __shfl_down(mn, d, 64));
            mx = max(mx, __shfl_down(mx, d, 64));
            SL[m * kTile + lane] = mn;
            SH[m * kTile + lane] = mx;
        }
    };

    auto flagsB = [&](int T) {
        const int s = T % kTileStages, t = T * kTile + lane;
        const int64_t c = cts[s * kTile + lane];
        uint64_t* W = words + (T & 1) * nword;
        const uint64_t P1t = r1[(t + 1) & RM];
        const unsigned __int128 P2t = r2[(t + 1) & RM];
#pragma unroll 1
        for (int o = 0; o < nw; ++o) {
            const int Wn = win[o];
            const int jj = t + 1 - Wn;
            const bool valid = jj >= 0 && t < B;
            const int64_t S1 = (int64_t)(P1t - r1[jj & RM]);
            const i128 S2 = (i128)(P2t - r2[jj & RM]);
            const int64_t Dv = (int64_t)Wn * c - S1;
            const i128 Q = (i128)Wn * S2 - (i128)S1 * (i128)S1;
            const i128 lhs = (i128)Dv * (i128)Dv * kd2;
#pragma unroll 1
            for (int q = 0; q < nk; ++q) {
                const int64_t kn = g.b[q];
                const i128 rhs = (i128)(kn * kn) * Q;
                const bool big = valid && lhs > rhs;
                const uint64_t zl = __ballot(big && Dv < 0), zh = __ballot(big && Dv > 0);
                if (lane == 0) {
                    W[2 * (o * nk + q)] = zl;
                    W[2 * (o * nk + q) + 1] = zh;
                }
            }
            const uint64_t dp = __ballot(valid && Dv >= 0), dn = __ballot(valid && Dv <= 0);
            if (lane == 0) {
                W[2 * nw * nk + 2 * o] = dp;
                W[2 * nw * nk + 2 * o + 1] = dn;
            }
        }
    };

    if (helperA) {
        const int32_t c0 = ldc(crow, B, lane, 0), c1 = ldc(crow, B, kTile + lane, 0);
        const int32_t h0 = ldc(hrow, B, lane, INT32_MIN), h1 = ldc(hrow, B, kTile + lane, INT32_MIN);
        const int32_t l0 = ldc(lrow, B, lane, INT32_MAX), l1 = ldc(lrow, B, kTile + lane, INT32_MAX);
        cpre = ldc(crow, B, 2 * kTile + lane, 0);
        hpre = ldc(hrow, B, 2 * kTile + lane, INT32_MIN);
        lpre = ldc(lrow, B, 2 * kTile + lane, INT32_MAX);
        scanA(0, c0, h0, l0);
        __syncthreads();
        if (ntiles > 1) scanA(1, c1, h1, l1);
    } else {
        __syncthreads();
        if (helperB) flagsB(0);
    }
    __syncthreads();

    TradeAcct a;
    acct_init(a);
    int64_t lv_sl = 0, lv_tp = 0;  // SL / TP levels of the open trade (ticks)
    const size_t gi = (size_t)blockIdx.x * P + pj;
    bt_trade* tr = (PARITY && active) ? out.trades + gi * out.trade_cap : nullptr;
    const int cap = out.trade_cap;

    for (int k = 0; k < ntiles; ++k) {
        const int t0 = k * kTile;
        if (helperA && k + 2 < ntiles) {
            scanA(k + 2, cpre, hpre, lpre);
            const int tn = t0 + 3 * kTile + lane;
            cpre = ldc(crow, B, tn, 0);
            hpre = ldc(hrow, B, tn, INT32_MIN);
            lpre = ldc(lrow, B, tn, INT32_MAX);
        }
        if (helperB && k + 1 < ntiles) flagsB(k + 1);
        if (active) {
            const int s = k % kTileStages;
            const int32_t* cT = cts + s * kTile;
            const int64_t* ql = qls + s * 2 * kTile;
            const Agg* D = dst + s * kDstLevels * kTile;
            const int32_t* SL = stl + s * kDstLevels * kTile;
            const int32_t* SH = sth + s * kDstLevels * kTile;
            const uint64_t* W = words + (k & 1) * nword;
            const uint64_t vm = bar_range_mask(t0, w - 1, B - 2);
            const uint64_t ZL = W[2 * (iw * nk + ik)] & vm, ZH = W[2 * (iw * nk + ik) + 1] & vm;
            const uint64_t DP = W[2 * nw * nk + 2 * iw] & vm, DN = W[2 * nw * nk + 2 * iw + 1] & vm;
            const int bl = B - 1 - t0;
            int cur = 0;
            while (cur < kTile) {
                const uint64_t el = ~0ULL << cur;
                if (a.pos == 0) {  // entry at the first flagged bar
                    const uint64_t m = (ZL | ZH) & el;
                    if (m == 0) break;
                    const int b = __builtin_ctzll(m);
                    const int np = ((ZL >> b) & 1) ? 1 : -1;
                    const int32_t cx = cT[b];
                    const uint64_t qx = (uint64_t)ql[b], q2x = (uint64_t)ql[kTile + b];
                    a.ps1 += np > 0 ? (uint64_t)0 - qx : qx;
                    a.ps2 -= q2x;
                    acct_open(a, t0 + b, b, cx);
                    a.pos = np;
                    const int64_t ce = cx;
                    lv_sl = np > 0 ? ce * (10000 - sl_bps) / 10000 : ce * (10000 + sl_bps) / 10000;
                    lv_tp = np > 0 ? ce * (10000 + tp_bps) / 10000 : ce * (10000 - tp_bps) / 10000;
                    cur = b + 1;
                } else {  // exit: first of SL/TP (intrabar, from entry+1), forced, signal
                    const bool lg = a.pos > 0;
                    const uint64_t sig = (lg ? DP : DN) & el;
                    int x = sig ? __builtin_ctzll(sig) : kTile;
                    if (bl >= cur && bl < kTile) x = min(x, bl);
                    const int xsl = lg ? first_le(SL, cur, lv_sl) : first_ge(SH, cur, lv_sl);
                    const int xtp = lg ? first_ge(SH, cur, lv_tp) : first_le(SL, cur, lv_tp);
                    const int xs = min(xsl, xtp);
                    int32_t px;
                    Agg st;
                    if (xs < kTile && xs <= x) {  // SL wins a tie with TP; both beat the close
                        x = xs;
                        px = (int32_t)(xsl <= xtp ? lv_sl : lv_tp);
                        const Agg before = x > a.sb ? dst_query_bf(D, a.sb, x - 1) : kAggId;
                        st = agg_merge(agg_merge(a.agg, before), agg_one(px));
                    } else if (x < kTile) {
                        px = cT[x];
                        st = agg_merge(a.agg, dst_query_bf(D, a.sb, x));
                    } else {
                        break;
                    }
                    const uint64_t qx = (uint64_t)ql[x], q2x = (uint64_t)ql[kTile + x];
                    acct_close<PARITY>(a, t0 + x, px, st, tr, cap);
                    a.ps1 += lg ? qx : (uint64_t)0 - qx;
                    a.ps2 += q2x;
                    a.pos = 0;
                    cur = x + 1;
                }
            }
            acct_tile_end(a, D, ql);
        }
        __syncthreads();
    }
    if (active) acct_write(a, B, g.sqrt_ann, gi, out);
    wave_add_trades(out, active ? a.ntr : 0);
}

// ----------------------------------------------------------------------------- launchers
static int tile_param_waves(int P) { return std::min((P + 63) / 64, 1024 / 64 - 2); }

size_t ema_lds_bytes(const Grid& g) { return tile_lds_layout(0, g.ring, g.na, g.nb).total; }
size_t boll_lds_bytes(const Grid& g) { return tile_lds_layout(1, g.ring, g.na, g.nb).total; }

hipError_t launch_ema_ols(const SymDesc* syms, int32_t n_sym, const int32_t* close, const Grid& g,
                          const Out& out, bool parity, hipStream_t st) {
    if (n_sym <= 0) return hipSuccess;
    const int pw = tile_param_waves(g.n_params);
    const dim3 grid(n_sym, (g.n_params + 64 * pw - 1) / (64 * pw));
    const dim3 block(64 * (pw + 2));
    const size_t lds = ema_lds_bytes(g);
    if (parity)
        hipLaunchKernelGGL(ema_tile_kernel<true>, grid, block, lds, st, syms, close, g, out);
    else
        hipLaunchKernelGGL(ema_tile_kernel<false>, grid, block, lds, st, syms, close, g, out);
    return hipGetLastError();
}

hipError_t launch_boll(const SymDesc* syms, int32_t n_sym, const int32_t* high, const int32_t* low,
                       const int32_t* close, const Grid& g, const Out& out, bool parity,
                       hipStream_t st) {
    if (n_sym <= 0) return hipSuccess;
    const int pw = tile_param_waves(g.n_params);
    const dim3 grid(n_sym, (g.n_params + 64 * pw - 1) / (64 * pw));
    const dim3 block(64 * (pw + 2));
    const size_t lds = boll_lds_bytes(g);
    if (parity)
        hipLaunchKernelGGL(boll_tile_kernel<true>, grid, block, lds, st, syms, high, low, close, g, out);
    else
        hipLaunchKernelGGL(boll_tile_kernel<false>, grid, block, lds, st, syms, high, low, close, g, out);
    return hipGetLastError();
}

}  // namespace bt
