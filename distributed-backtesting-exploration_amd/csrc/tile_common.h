// tile_common.h — pieces shared by the tile-pipelined strategy kernels (k_tile.hip):
// the per-tile close scan (returns, drawdown sparse table) and the per-lane trade accounting
// that runs only at position changes. Spec: docs/oracle_spec.md §3-§4.
#pragma once
#include "device_common.h"

namespace bt {

// s_setprio takes an immediate: a wave-uniform priority through a scalar switch (folds to one
// instruction for a constant)
__device__ __forceinline__ void set_prio(int p) {
    switch (p) {
        case 0: __builtin_amdgcn_s_setprio(0); break;
        case 1: __builtin_amdgcn_s_setprio(1); break;
        case 2: __builtin_amdgcn_s_setprio(2); break;
        default: __builtin_amdgcn_s_setprio(3); break;
    }
}

constexpr int kTileStages = 3;  // tile buffers in flight: scanned (k+2), flagged (k+1), walked (k)


struct TileCarry {
    int64_t P;       // sum of closes before the tile
    int32_t prevc;   // close of the bar before the tile
    uint32_t tv;     // total variation of the closes up to the tile, saturated at 2^31 (narrow
                     // accounts, Acct32)
};

// Level fills (Bollinger SL/TP, HL = true): a trade closed by its stop-loss or take-profit fills
// at the level price px, not at a close, so the equity path the narrow bound needs is the close
// path with px inserted before c_t at every such exit. That adds at most 2 dist(px, [min(c_(t-1),
// c_t), max(c_(t-1), c_t)]) to the total variation, and the distance is bounded by the bar data
// alone: a long stop at bar t fills at XL >= l_t (the low touched it) with XL <= c_(t-1) (else
// l_(t-1) <= c_(t-1) < XL had stopped it a bar earlier, or t-1 is the entry bar, c = ce >= XL), so
// dist <= min(c_(t-1), c_t) - l_t; a long take-profit likewise <= h_t - max(c_(t-1), c_t); shorts
// mirror. Bars with l > c or h < c (the parser does not order OHLC) break the "a bar earlier"
// step by at most l_(t-1) - c_(t-1) or c_(t-1) - h_(t-1). So each bar adds twice
//   max(0, min(c_(t-1), c_t) - l_t) + max(0, h_t - max(c_(t-1), c_t)) + max(0, l_t - c_t)
//   + max(0, c_t - h_t)
// to TV (each term clamped at 2^24; synthetic bars: about twice the h/l offsets, ~1 % of TV).
__device__ __forceinline__ uint32_t level_fill_slack(int32_t c, int32_t cp, int32_t hv, int32_t lv) {
    const int64_t mlo = min(c, cp), mhi = max(c, cp), C = c, H = hv, L = lv;
    auto cl = [](int64_t x) { return (uint32_t)min(max(x, (int64_t)0), (int64_t)1 << 24); };
    return cl(mlo - L) + cl(H - mhi) + cl(L - C) + cl(C - H);
}

// One whole wave, lane = bar t0 + lane, c = its close (0 past the end): writes the tile's
// closes cT[64], the in-tile prefixes of the fixed-point returns ql[0..63] (q) and
// ql[64..127] (q2), and the disjoint sparse table D[6][64] of the close path. Returns the
// inclusive prefix sum of closes up to this lane's bar (exact int64); `also` (optional) is
// replaced by its own inclusive wave prefix. AC: 64-bit scans as DPP add-with-carry pairs
// (device_common.h wave_iscan_i64_ac). With HL, the bar's high
// and low (hv, lv) add their level-fill slack to the narrow bound's total variation.
template <bool HL = false, bool AC = false>
__device__ __forceinline__ int64_t tile_scan(int32_t c, int B, int t0, int lane, int32_t* cT,
                                             int64_t* ql, Agg* D, TileCarry& cy,
                                             bool with_dst = true, int32_t* narrow = nullptr,
                                             int32_t hv = 0, int32_t lv = 0, int64_t* also = nullptr) {
    const int t = t0 + lane;
    const bool valid = t < B;
    const int32_t cp = (int32_t)__builtin_amdgcn_update_dpp((uint32_t)cy.prevc, (uint32_t)c,
                                                            0x138, 0xf, 0xf, false);  // wave_shr:1
    // the closes' prefix (AC: with the add-with-carry scans, paired with the caller's `also`)
    int64_t inc = (int64_t)c;
    if (AC && also != nullptr)
        wave_iscan2_i64_ac(inc, *also);
    else if (AC)
        inc = wave_iscan_i64_ac(inc);
    else
        inc = wave_iscan_i64(inc);
    if (!AC && also != nullptr) *also = wave_iscan_i64(*also);
    const int64_t pre = cy.P + inc;
    cT[lane] = c;
    int64_t q = 0, q2 = 0;
    uint32_t dv = 0;  // |c_t - c_(t-1)| (+ the level-fill slack, HL)
    if (valid && t >= 1) {
        fixed_ret(c, cp, q, q2);
        dv = (uint32_t)abs(c - cp);
    }
    if (HL && narrow != nullptr && valid)  // dv < 2^31, twice the slack <= 2^27: no wrap
        dv += 2 * level_fill_slack(c, t >= 1 ? cp : c, hv, lv);
    if (AC) {
        wave_iscan2_i64_ac(q, q2);
    } else {
        q = wave_iscan_i64(q);
        q2 = wave_iscan_i64(q2);
    }
    ql[lane] = q;
    ql[kTile + lane] = q2;
    if (narrow != nullptr) {  // the tile's total variation and the narrow flag (Acct32)
        const bool big = __ballot(dv >= (1u << 25)) != 0;
        const uint32_t tvt = __builtin_amdgcn_readlane(wave_iscan_u32(min(dv, 1u << 25)), 63);
        cy.tv = big ? (1u << 31) : min(cy.tv + tvt, 1u << 31);
        if (lane == 0) *narrow = cy.tv < (1u << 30);
    }
    cy.P += lane63_i64(inc);
    cy.prevc = (int32_t)__builtin_amdgcn_readlane((uint32_t)c, 63);
    if (with_dst) dst_build(c, lane, D);  // (profiling ablation only: false skips the table)
    return pre;
}

// Per-lane trade accounting (spec §4), touched only when the position changes.
//  * drawdown via gap = peak - realized (int64 >= 0): a closed trade whose MTM path has range
//    [lo, hi] and internal drawdown `path` gives mdd = max(mdd, gap - lo, path) and
//    gap' = max(gap, hi) - pnl;
//  * S1/S2 via per-tile partial sums of the in-tile return prefixes QL (uint64, exact modulo
//    2^64, folded into int128 at the tile end): a position change at bar b from pos to np adds
//    (pos - np) * QL[b] to ps1 and (|pos| - |np|) * QL2[b] to ps2; an open position at the tile
//    end adds pos * QL[63] and QL2[63].
//  * bar segments (SEG): the entering gap g and mdd m are unknown, so the drawdown is kept as
//    gap = max(g + A, Bq), mdd = max(m, g + C, D): a trade (lo, hi, path, pnl) maps
//    C' = max(C, A - lo), D' = max(D, Bq - lo, path), A' = A - pnl, Bq' = max(Bq, hi) - pnl.
//    A starts at 0 with R and moves by -pnl as R moves by +pnl, so A = -R is not stored.
constexpr int64_t kNegInf = -(1LL << 60);  // "minus infinity" of the max-plus forms

// A 96-bit signed accumulator (two VGPRs fewer than int128): the Sharpe sums are bounded by
// 2^22 bars x 2^56 < 2^78 (spec §3), and 2^95 leaves room to spare.
struct I96 {
    uint64_t lo;
    int32_t hi;
    __device__ __forceinline__ void clear() { lo = 0; hi = 0; }
    __device__ __forceinline__ void add(int64_t x) {
        const uint64_t n = lo + (uint64_t)x;
        hi += (int32_t)(n < lo) - (int32_t)(x < 0);  // carry out of the low word, sign of x
        lo = n;
    }
    __device__ __forceinline__ int64_t hi64() const { return (int64_t)hi; }
    __device__ __forceinline__ uint64_t lo64() const { return lo; }
};

struct TradeAcct {
    int32_t pos, e, ce, sb, ntr, expo;  // sb: in-tile bar where the open trade's path resumes
    int64_t R, gap, mdd;
    int64_t Bq, C, D;                   // SEG walks only (A = -R)
    uint64_t ps1, ps2, h;
    I96 s1, s2;
    Agg agg;  // closes [e, tile start - 1] of the open trade (kAggId when e is in this tile)
};

__device__ __forceinline__ void acct_init(TradeAcct& a) {
    a.pos = a.e = a.ce = a.sb = a.ntr = a.expo = 0;
    a.R = a.gap = a.mdd = 0;
    a.Bq = a.C = a.D = kNegInf;
    a.ps1 = a.ps2 = 0;
    a.h = 0;
    a.s1.clear();
    a.s2.clear();
    a.agg = kAggId;
}

// Close the open trade (a.pos, a.e, a.ce) at global bar t for price px, given the trade's
// adverse / favourable excursions lo / hi and internal drawdown `path` (all relative to the
// entry close, in the trade's direction), its pnl and its hash term mix(w).
// Narrow accounts (unsplit runs): while the closes' total variation TV (through the tile's last
// bar) is below 2^30, gap and mdd — differences of equity or price values, |.| <= TV, and the
// recursion's intermediates <= 2 TV — are exact in int32 (k_sma.hip SmaAcct has the argument).
// Bar segments (SEG) keep the wide max-plus forms.
struct Acct32 {
    int32_t g, m;        // gap, mdd
};

template <bool PARITY, bool SEG = false, bool NARROW = false>
__device__ __forceinline__ void acct_fold(TradeAcct& a, Acct32& n, int t, int32_t px, int32_t lo,
                                          int32_t hi, int32_t path, int32_t pnl, uint64_t mix,
                                          bt_trade* tr, int cap) {
    if (NARROW && !SEG) {  // (a SEG instantiation of a narrow path is never taken)
        n.m = max(n.m, max(n.g - lo, path));
        n.g = max(n.g, hi) - pnl;
    } else if (SEG) {
        const int64_t A0 = -a.R, B0 = a.Bq;  // A = -R (see TradeAcct)
        a.C = max(a.C, A0 - (int64_t)lo);
        a.D = max(a.D, max(B0 - (int64_t)lo, (int64_t)path));
        a.Bq = max(B0, (int64_t)hi) - pnl;
    } else {
        a.mdd = max(a.mdd, max(a.gap - (int64_t)lo, (int64_t)path));
        a.gap = max(a.gap, (int64_t)hi) - pnl;
    }
    a.R += pnl;
    a.expo += t - a.e;
    a.h += mix;
    if (PARITY && a.ntr < cap) {
        bt_trade r;
        r.entry_bar = a.e;
        r.exit_bar = t;
        r.side = a.pos;
        r.pad = 0;
        r.entry_px = a.ce;
        r.exit_px = px;
        tr[a.ntr] = r;
    }
    a.ntr++;
}

// Hash term of a trade (spec §4): w = entry | exit << 31 | (side > 0) << 62.
__device__ __forceinline__ uint64_t trade_term(int e, int t, bool lg) {
    return trade_mix_et((uint32_t)e, (uint32_t)t, lg);
}

// Close the open trade at global bar t for price px; `st` aggregates the trade's whole price
// path in order, exit point included.
template <bool PARITY, bool SEG = false, bool NARROW = false>
__device__ __forceinline__ void acct_close(TradeAcct& a, Acct32& n, int t, int32_t px, const Agg& st,
                                           bt_trade* tr, int cap) {
    const bool lg = a.pos > 0;
    const int32_t lo = lg ? st.mn - a.ce : a.ce - st.mx;  // |.| < 2^31
    const int32_t hi = lg ? st.mx - a.ce : a.ce - st.mn;
    const int32_t path = lg ? st.dd : st.du;
    const int32_t pnl = lg ? px - a.ce : a.ce - px;
    acct_fold<PARITY, SEG, NARROW>(a, n, t, px, lo, hi, path, pnl, trade_term(a.e, t, lg), tr, cap);
}

template <bool PARITY, bool SEG = false>
__device__ __forceinline__ void acct_close(TradeAcct& a, int t, int32_t px, const Agg& st,
                                           bt_trade* tr, int cap) {
    Acct32 unused{0, 0};
    acct_close<PARITY, SEG, false>(a, unused, t, px, st, tr, cap);
}

// Unsplit runs' close with the width of gap / mdd chosen at run time: `narrow` (wave-uniform, a
// scalar branch, so the caller keeps one copy of its loop) keeps both in the low words of the
// int64 fields — both are >= 0 and, while the closes' total variation allows (Acct32), < 2^31,
// so the high words stay 0.
template <bool PARITY>
__device__ __forceinline__ void acct_close_rt(TradeAcct& a, bool narrow, int t, int32_t px,
                                              const Agg& st, bt_trade* tr, int cap) {
    const bool lg = a.pos > 0;
    const int32_t lo = lg ? st.mn - a.ce : a.ce - st.mx;
    const int32_t hi = lg ? st.mx - a.ce : a.ce - st.mn;
    const int32_t path = lg ? st.dd : st.du;
    const int32_t pnl = lg ? px - a.ce : a.ce - px;
    if (narrow) {
        const int32_t g = (int32_t)a.gap, m = (int32_t)a.mdd;
        a.mdd = (uint32_t)max(m, max(g - lo, path));
        a.gap = (uint32_t)(max(g, hi) - pnl);
    } else {
        a.mdd = max(a.mdd, max(a.gap - (int64_t)lo, (int64_t)path));
        a.gap = max(a.gap, (int64_t)hi) - pnl;
    }
    a.R += pnl;
    a.expo += t - a.e;
    a.h += trade_term(a.e, t, lg);
    if (PARITY && a.ntr < cap) {
        bt_trade r;
        r.entry_bar = a.e;
        r.exit_bar = t;
        r.side = a.pos;
        r.pad = 0;
        r.entry_px = a.ce;
        r.exit_px = px;
        tr[a.ntr] = r;
    }
    a.ntr++;
}

__device__ __forceinline__ void acct_open(TradeAcct& a, int t, int b, int32_t px) {
    a.e = t;
    a.ce = px;
    a.sb = b;
    a.agg = kAggId;
}

// Tile end: carry the open trade's path, fold the tile's return partials into int128.
__device__ __forceinline__ void acct_tile_end(TradeAcct& a, const Agg* D, const int64_t* ql) {
    if (a.pos != 0) {
        a.agg = agg_merge(a.agg, dst_query_bf(D, a.sb, kTile - 1));
        a.sb = 0;
        const uint64_t q63 = (uint64_t)ql[kTile - 1];
        a.ps1 += a.pos > 0 ? q63 : (uint64_t)0 - q63;
        a.ps2 += (uint64_t)ql[2 * kTile - 1];
    }
    a.s1.add((int64_t)a.ps1);
    a.s2.add((int64_t)a.ps2);
    a.ps1 = a.ps2 = 0;
}

__device__ __forceinline__ void acct_write(const TradeAcct& a, int bars, double sqrt_ann,
                                           size_t gi, const Out& out) {
    const uint64_t s1lo = a.s1.lo64(), s2lo = a.s2.lo64();
    const int64_t s1hi = a.s1.hi64(), s2hi = a.s2.hi64();
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

// ---- bar segments (SegRec / SegArgs in internal.h; used by both tile kernels)
// Tiles of one block: scanned from T_scan (every window of the first walked bar complete),
// walked from T_walk, accounted from T_acct, up to T_end (exclusive). Speculative segments
// s >= 1 walk `burn` tiles before their first bar; the fix pass (fix_seg = s) walks segment s
// from its first bar.
struct SegRange {
    int seg, T_scan, T_walk, T_acct, T_end;
};

// Boundaries balance the walked tiles: segment 0 (no burn-in) is `burn` tiles longer than the
// others, so every segment walks about (ntiles + (G - 1) burn) / G tiles.
__device__ __forceinline__ int seg_start(int s, int G, int ntiles, int burn) {
    if (s <= 0) return 0;
    if (s >= G) return ntiles;
    const int x = (ntiles - burn) / G;
    return x > 0 ? burn + s * x : (int)((int64_t)s * ntiles / G);
}

__device__ __forceinline__ SegRange seg_range(const SegArgs& sg, int fix_seg, int ntiles, int wmax) {
    SegRange r;
    r.seg = fix_seg > 0 ? fix_seg : (int)blockIdx.z;
    r.T_acct = seg_start(r.seg, sg.G, ntiles, sg.burn_tiles);
    r.T_end = seg_start(r.seg + 1, sg.G, ntiles, sg.burn_tiles);
    r.T_walk = (fix_seg > 0 || r.seg == 0) ? r.T_acct : max(0, r.T_acct - sg.burn_tiles);
    r.T_scan = max(0, r.T_walk - (wmax - 1 + kTile - 1) / kTile);
    if (r.T_acct >= r.T_end) r.T_scan = r.T_walk = r.T_acct = r.T_end;  // no bars: state passes through
    return r;
}

// Do a lane's speculative start and the true state entering its segment differ? Two walks in
// the same state at a bar (flat, or in the trade entered at the same bar) agree from then on.
__device__ __forceinline__ bool seg_start_differs(const SegRec* mine, const SegRec* prev) {
    const int tp = prev->end_pos, te = prev->end_e;
    return !(mine->start_pos == tp && (tp == 0 || mine->start_e == te));
}

// The true state entering the segment (fix pass).
__device__ __forceinline__ void seg_inject(TradeAcct& a, const SegRec* prev) {
    a.pos = prev->end_pos;
    a.e = prev->end_e;
    a.ce = prev->end_ce;
    a.agg = Agg{prev->end_agg[0], prev->end_agg[1], prev->end_agg[2], prev->end_agg[3]};
    a.sb = 0;
}

// First accounted tile: the sums restart (the burn-in's are dropped); the state carries on.
__device__ __forceinline__ void seg_reset_sums(TradeAcct& a) {
    a.R = 0;
    a.Bq = a.C = a.D = kNegInf;
    a.ntr = a.expo = 0;
    a.h = 0;
    a.s1.clear();
    a.s2.clear();
    a.ps1 = a.ps2 = 0;
}

// The state at the segment's first accounted bar, stored when the walk reaches it (the Bollinger
// kernel keeps no register for it across the walk); seg_write_rest then leaves it in place.
__device__ __forceinline__ void seg_write_start(SegRec* mine, int start_pos, int start_e) {
    *reinterpret_cast<int2*>(&mine->start_pos) = make_int2(start_pos, start_e);
}

__device__ __forceinline__ void seg_write_rest(const TradeAcct& a, SegRec* mine) {
    *reinterpret_cast<int2*>(&mine->ntr) = make_int2(a.ntr, a.expo);
    SegRec r;
    r.end_pos = a.pos;
    r.end_e = a.e;
    r.end_ce = a.ce;
    r.pad = 0;
    r.end_agg[0] = a.agg.mx;
    r.end_agg[1] = a.agg.mn;
    r.end_agg[2] = a.agg.dd;
    r.end_agg[3] = a.agg.du;
    r.R = a.R;
    r.A = -a.R;
    r.B = a.Bq;
    r.C = a.C;
    r.D = a.D;
    r.h = a.h;
    r.s1lo = a.s1.lo64();
    r.s1hi = a.s1.hi64();
    r.s2lo = a.s2.lo64();
    r.s2hi = a.s2.hi64();
    // bytes 16..127 of the record (16-B aligned: records are 128 B)
    const int4* src = reinterpret_cast<const int4*>(&r) + 1;
    int4* dst = reinterpret_cast<int4*>(mine) + 1;
#pragma unroll
    for (int i = 0; i < 7; ++i) dst[i] = src[i];
}

__device__ __forceinline__ void seg_write(const TradeAcct& a, int start_pos, int start_e, SegRec* mine) {
    SegRec r;
    r.ntr = a.ntr;
    r.expo = a.expo;
    r.start_pos = start_pos;
    r.start_e = start_e;
    r.end_pos = a.pos;
    r.end_e = a.e;
    r.end_ce = a.ce;
    r.pad = 0;
    r.end_agg[0] = a.agg.mx;
    r.end_agg[1] = a.agg.mn;
    r.end_agg[2] = a.agg.dd;
    r.end_agg[3] = a.agg.du;
    r.R = a.R;
    r.A = -a.R;
    r.B = a.Bq;
    r.C = a.C;
    r.D = a.D;
    r.h = a.h;
    r.s1lo = a.s1.lo64();
    r.s1hi = a.s1.hi64();
    r.s2lo = a.s2.lo64();
    r.s2hi = a.s2.hi64();
    *mine = r;
}

// Diagnostic s_memtime stamps (Grid::ablate & 64 builds only): per role (0 = parameter waves,
// 1 = helper A, 2 = helper B) the cycles spent working and waiting at the tile barrier.
// dbg[8 * role + {0, 1, 2..5, 6, 7}] = work, barrier, marked segments / counts, condition-word
// task cycles, waves; dbg[64 + role] = level-task cycles.
struct StampAcc {
    uint64_t prev = 0, w = 0, b = 0, x[4] = {0, 0, 0, 0};
    uint64_t task[2] = {0, 0};  // cycles inside condition-word (0) and level (1) tasks
    __device__ __forceinline__ void begin() { prev = __builtin_amdgcn_s_memtime(); }
    __device__ __forceinline__ void mark(int i) {  // work segment i (counted into w as well)
        const uint64_t now = __builtin_amdgcn_s_memtime();
        x[i] += now - prev;
        w += now - prev;
        prev = now;
    }
    __device__ __forceinline__ void count(int i) { x[i] += 1; }
    __device__ __forceinline__ void work() {
        const uint64_t now = __builtin_amdgcn_s_memtime();
        w += now - prev;
        prev = now;
    }
    __device__ __forceinline__ void barrier() {
        const uint64_t now = __builtin_amdgcn_s_memtime();
        b += now - prev;
        prev = now;
    }
    __device__ __forceinline__ void flush(unsigned long long* dbg, int role, int lane) {
        if (lane == 0 && dbg != nullptr) {
            atomicAdd(&dbg[8 * role + 0], (unsigned long long)w);
            atomicAdd(&dbg[8 * role + 1], (unsigned long long)b);
            for (int i = 0; i < 4; ++i) atomicAdd(&dbg[8 * role + 2 + i], (unsigned long long)x[i]);
            atomicAdd(&dbg[8 * role + 7], 1ULL);
            atomicAdd(&dbg[8 * role + 6], (unsigned long long)task[0]);
            atomicAdd(&dbg[64 + role], (unsigned long long)task[1]);
        }
    }
};

// Decision-bar mask of a tile: bits for bars t0+b with lo <= t0+b <= hi.
__device__ __forceinline__ uint64_t bar_range_mask(int t0, int lo, int hi) {
    const int a = lo - t0, b = hi - t0;
    if (b < 0 || a > 63 || a > b) return 0;
    const uint64_t top = b >= 63 ? ~0ULL : ((1ULL << (b + 1)) - 1);
    const uint64_t bot = a <= 0 ? ~0ULL : (~0ULL << a);
    return top & bot;
}

}  // namespace bt
