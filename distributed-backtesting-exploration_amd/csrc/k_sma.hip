// k_sma.hip — SMA-crossover backtest: one workgroup per symbol, one lane per parameter pair.
//
// Hot path of BASELINE.json north_star (config 2), replacing the sleep in
// process_incoming_job (/root/reference/src/worker/process.rs:21-25). Spec: docs/oracle_spec.md
// §3-§5 (SMA). Checked bit-for-bit against oracle/oracle.c::orc_sma.
//
// HBM is read once (4 B of close per bar per symbol); everything else lives in LDS, one 64-bar
// tile at a time, in a three-stage software pipeline with ONE workgroup barrier per tile:
//   stage 1, tile k+2 (a dedicated helper wave): exact int64 prefix of close appended to a ring
//            of doubles (exact below 2^53); fixed-point returns q, q2 (spec §3) and their
//            in-tile int64 prefixes + int128 tile base; the closes' total variation (narrow
//            accounts, SmaAcct).
//   stage 2, tile k+1 (all waves, helper included, tasks grabbed from an LDS counter): the
//            tile's disjoint sparse table (DST) of the close path (max, min, drawdown, draw-up),
//            built by log-doubling shuffles, and (lane = bar, window wave-uniform) int32 SMA
//            keys K[w][b] = floor(window_sum / w) for every window of the grid (one f64
//            multiply, no division).
//   stage 3, tile k (parameter waves, lane = (fast, slow) pair): per bar one subtract whose
//            sign bit is shifted into the 64-bit word L (fast key < slow key), and a running
//            unsigned min that detects equal keys; without equal keys G (fast > slow) = ~L.
//            Keys are monotone in the exact SMA, so a strict key order is the exact order; equal
//            keys (rare: ~1e-4 of lane-tiles on config 2) are settled exactly (F*s vs L*f in
//            int64, products < 2^59). The whole tile's position path then follows
//            bit-parallel: a set/reset latch is an add-with-carry (LONG = carries of
//            ~L + G + [pos == +1]). Each lane walks only its flips (ctz): per trade O(1) work —
//            PnL, MTM drawdown from the DST, Sharpe sums as int128 prefix differences, hash.
#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "tile_common.h"

namespace bt {

namespace {

constexpr int kKS = kTile + 4;        // int32 key row stride: rows 16-B aligned for b128 reads
constexpr int kStages = 3;            // tile buffers in flight (cT, Q)
constexpr int kDstStages = 2;         // drawdown tables: built in interval k - 1, read in k
constexpr int kKeyGrab = 4;           // windows per key task (one LDS atomic per group)
// Key-row pairs in flight in the 16-wave (ONE_TRIP) compare: 2, 4, 8 and 16 are within 0.5 %
// of each other on config 5's shard (round 4); the whole 10,000-symbol workload ran 3 % slower
// with 16 and no VGPR cap, so 2.
constexpr int kCmpDepth1 = 2;

struct SmaLds {                       // byte offsets into dynamic LDS
    size_t ring, keys, invw, win, dst, ct, ql, nar, ctr, total;
};

__host__ __device__ inline SmaLds sma_lds_layout(int ring, int nw) {
    SmaLds L;
    size_t o = 0;
    auto take = [&](size_t bytes) { size_t r = o; o += (bytes + 15) & ~size_t(15); return r; };
    L.ring = take((size_t)ring * 8);
    const int nwp = (nw + kKeyGrab - 1) / kKeyGrab * kKeyGrab;  // key rows: whole groups
    L.keys = take((size_t)2 * nwp * kKS * 4);
    L.invw = take((size_t)nwp * 8);
    L.win = take((size_t)nwp * 4);
    L.dst = take((size_t)kDstStages * kDstLevels * kTile * sizeof(Agg));
    L.ct = take((size_t)kStages * kTile * 4);
    L.ql = take((size_t)kStages * 2 * kTile * 8);
    L.nar = take((size_t)kStages * 4);    // per tile stage: accounts fit int32 (SmaAcct)
    L.ctr = take(4);
    L.total = o;
    return L;
}

// Stage 1 for one tile, executed by one whole wave (lane = bar of the tile).
struct ScanCarry {
    int64_t P;          // sum of closes before the tile
    int32_t prevc;      // close of the bar before the tile
    uint32_t tv;        // total variation of the closes up to the tile, saturated at 2^31
                        // (SmaAcct narrow tiles)
};

__device__ __forceinline__ int32_t load_close(const int32_t* __restrict__ crow, int B, int t) {
    return t < B ? crow[t] : 0;
}

// c = close of bar t0 + lane (0 past the end), loaded one tile ahead by the caller so the HBM
// latency is off the pipeline's critical path. The tile's drawdown table is a stage-2 task
// (stage_keys), built from the closes stored here.
__device__ __forceinline__ void stage_ring(int32_t c, int B, int t0, int lane, int R, double* ring,
                                           int32_t* cT, int64_t* ql, int32_t* narrow,
                                           ScanCarry& cy) {
    const int t = t0 + lane;
    const bool valid = t < B;
    // previous bar's close: DPP wave_shr:1, lane 0 takes the carry
    const int32_t cp = (int32_t)__builtin_amdgcn_update_dpp((uint32_t)cy.prevc, (uint32_t)c,
                                                            0x138, 0xf, 0xf, false);
    const int64_t inc = wave_iscan_i64((int64_t)c);
    ring[(t + 1) & (R - 1)] = (double)(cy.P + inc);
    cT[lane] = c;
    int64_t q = 0, q2 = 0;
    uint32_t dv = 0;  // |c_t - c_(t-1)| (prices in [1, 2^31): the difference fits int32)
    if (valid && t >= 1) {
        fixed_ret(c, cp, q, q2);
        dv = (uint32_t)abs(c - cp);
    }
    ql[lane] = wave_iscan_i64(q);              // in-tile prefix: |.| <= 64 * 2^56 < 2^63
    ql[kTile + lane] = wave_iscan_i64(q2);
    // the tile's total variation: a sum of 64 terms clamped to 2^25 fits uint32, and a clamped
    // term alone puts TV past the narrow bound
    const bool big = __ballot(dv >= (1u << 25)) != 0;
    const uint32_t tvt = __builtin_amdgcn_readlane(wave_iscan_u32(min(dv, 1u << 25)), 63);
    cy.tv = big ? (1u << 31) : min(cy.tv + tvt, 1u << 31);  // both terms < 2^31: no wrap
    if (lane == 0) *narrow = cy.tv < (1u << 30);
    cy.P += lane63_i64(inc);
    cy.prevc = (int32_t)__builtin_amdgcn_readlane((uint32_t)c, 63);
}

// Stage 2 for one tile: int32 floor keys for every window. lane = bar, so the window length
// and its reciprocal are wave-uniform and the top of the ring is read once per tile.
// Windows are handed out dynamically, kKeyGrab per grab: every wave of the block (helper
// included) grabs window groups from an LDS counter after its other work for the tile, so waves
// with few flips to walk compute more keys. Round r owns counter values [r*per, (r+1)*per) with
// per = kKeyGrab * (ceil(nw / kKeyGrab) + nwaves): the group grabs plus exactly one failing grab
// per wave (the barrier separates rounds). The next group's atomic is in flight while the
// current group computes (its result is read only at the end of the iteration), and the group's
// ring reads are issued together.
// Bars without a full window (or past the series end) get key -1 on fast rows and -2 on slow
// rows: their difference is never 0, so they never look like ties to the compare stage (they
// are outside every lane's decision mask anyway).
__device__ __forceinline__ uint32_t grab_issue(uint32_t* ctr, int lane) {
    uint32_t v = 0;
    if (lane == 0) v = atomicAdd(ctr, (uint32_t)kKeyGrab);
    return v;
}

// floor(F / W) for the exact window sum F (an integer < 2^53 held as a double, F/W < 2^31):
// one multiply by an UPWARD-biased reciprocal iw = RN(RN(1/W) * (1 + 2^-47)) and a truncating
// conversion, no fix-up. Three roundings of at most 2^-53 relative each leave the computed
// product p = F/W * (1 + e) with 2^-47 * (1 - 3/64) < e < 2^-47 * (1 + 3/64): the bias is never
// undone, so p >= F/W, and p - F/W < 2^31 * 2^-46.9 = 2^-15.9 < 1/W for every W < 62,000
// (the LDS ring caps SMA windows near 16,000), while F/W = n + r/W sits at least 1/W below
// n + 1. Hence trunc(p) == floor(F/W) exactly (tests/test_oracle_golden.py::
// test_biased_reciprocal_floor checks all W <= 16,384 at and around multiples of W).
__device__ __forceinline__ int32_t floor_key(double F, double iw) {
    return (int32_t)(F * iw);
}

// Counter values of one stage-2 round: the drawdown-table task, the key groups, and one failing
// grab per wave.
__host__ __device__ inline uint32_t key_round_len(int nwp, int nwaves) {
    return (uint32_t)kKeyGrab * ((uint32_t)nwp / kKeyGrab + 1 + (uint32_t)nwaves);
}

// Stage 2 of round r (tile r): the tile's drawdown table (device_common.h dst_build) from the
// closes stage 1 left in LDS (cTr), into Dr, as the round's first task, then the key groups.
// The table is a task rather than a fixed role: on the half-empty seventh parameter wave of a
// config-2 block it set the tile (that wave's compare and walk plus the table's DPP chain).
__device__ __forceinline__ void stage_keys(int t0, int B, int nw, int nwp, int nf, int wmax, int R,
                                           double* ring, const int32_t* win,
                                           const double* invw, int32_t* K, uint32_t* ctr,
                                           uint32_t round, int nwaves, int lane,
                                           const int32_t* cTr, Agg* Dr) {
    const int t = t0 + lane;
    const double top = ring[(t + 1) & (R - 1)];
    // wave-uniform: every bar of the tile has a full window for every window length
    const bool full = t0 + 1 - wmax >= 0 && t0 + kTile <= B;
    const uint32_t base = round * key_round_len(nwp, nwaves);
    uint32_t w = __builtin_amdgcn_readlane(grab_issue(ctr, lane), 0) - base;
#pragma unroll 1
    while (w < (uint32_t)(nwp + kKeyGrab)) {
        const uint32_t vn = grab_issue(ctr, lane);  // next group, read at the end
        if (w == 0) {  // the table task (counter value 0 of the round)
            dst_build<true>(cTr[lane], lane, Dr);
            w = __builtin_amdgcn_readlane(vn, 0) - base;
            continue;
        }
        w -= kKeyGrab;
        // w is a multiple of kKeyGrab: the group's lengths and reciprocals are aligned 16-B
        // reads; rows nw..nwp-1 are padding (length 1) whose keys nobody reads
        int Wv[kKeyGrab];
        double Iv[kKeyGrab], Fv[kKeyGrab];
#pragma unroll
        for (int q = 0; q < kKeyGrab; q += 4) {
            const int4 W4 = *reinterpret_cast<const int4*>(win + w + q);
            Wv[q] = W4.x; Wv[q + 1] = W4.y; Wv[q + 2] = W4.z; Wv[q + 3] = W4.w;
        }
#pragma unroll
        for (int q = 0; q < kKeyGrab; q += 2) {
            const double2 I2 = *reinterpret_cast<const double2*>(invw + w + q);
            Iv[q] = I2.x; Iv[q + 1] = I2.y;
        }
#pragma unroll
        for (int q = 0; q < kKeyGrab; ++q) {
            Wv[q] = __builtin_amdgcn_readfirstlane(Wv[q]);
            Fv[q] = top - ring[(t + 1 - Wv[q]) & (R - 1)];  // exact (< 2^53)
        }
        int32_t* Kw = K + w * kKS + lane;
        if (full) {
#pragma unroll
            for (int q = 0; q < kKeyGrab; ++q) Kw[q * kKS] = floor_key(Fv[q], Iv[q]);
        } else {
            const bool tin = t < B;
#pragma unroll
            for (int q = 0; q < kKeyGrab; ++q) {
                const int32_t kq = floor_key(Fv[q], Iv[q]);
                Kw[q * kKS] = (tin && t + 1 - Wv[q] >= 0) ? kq : ((int)(w + q) < nf ? -1 : -2);
            }
        }
        w = __builtin_amdgcn_readlane(vn, 0) - base;
    }
}

// Four bars, 10 VALU: d = x - y (no overflow: keys are in [-2, 2^31)); the sign bit of d is
// [x < y] and is shifted into L by v_alignbit ({l, d} >> 31 == l << 1 | d >> 31); z keeps the
// unsigned minimum of every d, which is 0 iff some bar has equal keys. With no equal keys,
// [x > y] is simply ~[x < y]; a tile with an equal pair takes the exact path.
__device__ __forceinline__ void cmp4(uint32_t& l, uint32_t& z, const int4& x, const int4& y) {
    const uint32_t d0 = (uint32_t)(x.x - y.x), d1 = (uint32_t)(x.y - y.y);
    const uint32_t d2 = (uint32_t)(x.z - y.z), d3 = (uint32_t)(x.w - y.w);
    l = __builtin_amdgcn_alignbit(l, d0, 31);
    l = __builtin_amdgcn_alignbit(l, d1, 31);
    l = __builtin_amdgcn_alignbit(l, d2, 31);
    l = __builtin_amdgcn_alignbit(l, d3, 31);
    z = min(min(z, d0), d1);   // one v_min3_u32 per two bars
    z = min(min(z, d2), d3);
}

// Equality word for the rare tiles with equal keys (same bit order as cmp4).
__device__ __forceinline__ uint64_t eq_word(const int32_t* k1, const int32_t* k2) {
    uint64_t e = 0;
#pragma unroll 1
    for (int b = 0; b < kTile; ++b) e |= (uint64_t)(k1[b] == k2[b]) << b;
    return e;
}

}  // namespace

// Per-lane trade accounting (spec §4), touched only at position flips.
//  * drawdown via gap = peak - realized (int64 >= 0): a closed trade with MTM range
//    [R+lo, R+hi] and path drawdown `path` gives mdd = max(mdd, gap - lo, path) and
//    gap' = max(gap, hi) - pnl;
//  * S1/S2 via per-tile partial sums of the in-tile return prefix (uint64, exact modulo 2^64;
//    each tile's true total is a masked sum of <= 64 q's, |.| < 2^63), folded into int128 at
//    the tile end: entry at bar b adds -side*QL[b], exit adds +side*QL[b], an open position
//    at the tile end adds +side*QL[63].
//  * narrow tiles: every quantity the drawdown recursion touches (gap, mdd, a trade's lo, hi,
//    path and pnl, the realized sum) is a difference of equity or price values at two bars, so
//    its magnitude is at most the total variation TV = sum |c_t - c_(t-1)| of the closes so far,
//    and gap - lo, max(gap, hi) - pnl at most 2 TV. While TV (through the tile's last bar) is
//    below 2^30, the walk keeps gap / mdd / realized pnl in int32 (g32, m32, r32), exactly; at
//    the first wider tile they move into the int64 fields for good.
struct SmaAcct {
    int32_t pos, e, ce, sb, ntr, e0;     // sb: in-tile bar where the open trade's path resumes;
                                         // e0: first entry bar
    int32_t g32, m32, r32;               // narrow tiles: gap, mdd, realized pnl
    int64_t R, gap, mdd;
    uint64_t ps1, ps2, h;
    I96 s1, s2;
    Agg agg;  // closes [e, tile start - 1] of the open trade (kAggId when e is in this tile)
    // bar segments (SEG) only: the drawdown as max-plus forms of the unknown entering gap and mdd
    // (tile_common.h TradeAcct), and the trade open at the segment start, whose entry lies in an
    // earlier segment: `carried` while it is open, then its exit bar x1, fill px1 and path agg1
    // from the segment start (closed by the combine pass, internal.h SmaSegRec)
    int64_t Bq, C, D;                    // A = -R: both start at 0, R moves by +pnl, A by -pnl
    int32_t carried, x1, px1;
    Agg agg1;
};

// SMA positions: flat until the first decision, then every flip reverses (fast > slow is
// long, fast < slow short), and the forced exit at bar B-1 goes flat. So a tile's flips are at
// most one entry from flat, then reversals (a branch-free loop), then at most the forced exit.

// Closes the open trade at in-tile bar b (fill cx = close of bar t = t0 + b).
// MERGE = false: the trade opened in this tile (a.agg is the identity), so seg is its whole path.
// SEG: a close of the carried trade (only possible with MERGE: the first close of a tile) is
// recorded for the combine pass instead of accounted.
template <bool PARITY, bool MERGE = true, bool SEG = false, bool NARROW = false>
__device__ __forceinline__ void sma_close(SmaAcct& a, const Agg& seg, int t, int32_t cx,
                                          bt_trade* tr, int cap) {
    const Agg st = MERGE ? agg_merge(a.agg, seg) : seg;   // seg: closes [sb, b] of this tile
    if (SEG && MERGE && a.carried) {
        a.x1 = t;
        a.px1 = cx;
        a.agg1 = st;
        a.carried = 0;
        a.ntr++;
        return;
    }
    const bool lg = a.pos > 0;
    const int32_t lo = lg ? st.mn - a.ce : a.ce - st.mx;   // |.| < 2^31
    const int32_t hi = lg ? st.mx - a.ce : a.ce - st.mn;
    const int32_t path = lg ? st.dd : st.du;
    const int32_t pnl = lg ? cx - a.ce : a.ce - cx;
    if (SEG) {
        const int64_t A0 = -a.R, B0 = a.Bq;  // A = -R (SmaAcct)
        a.C = max(a.C, A0 - (int64_t)lo);
        a.D = max(a.D, max(B0 - (int64_t)lo, (int64_t)path));
        a.Bq = max(B0, (int64_t)hi) - pnl;
    } else if (NARROW) {  // |.| <= 2 TV < 2^31 (SmaAcct)
        a.m32 = max(a.m32, max(a.g32 - lo, path));
        a.g32 = max(a.g32, hi) - pnl;
    } else {
        a.mdd = max(a.mdd, max(a.gap - (int64_t)lo, (int64_t)path));
        a.gap = max(a.gap, (int64_t)hi) - pnl;
    }
    if (NARROW)
        a.r32 += pnl;
    else
        a.R += pnl;
    a.h += trade_mix_et((uint32_t)a.e, (uint32_t)t, lg);
    if (PARITY && a.ntr < cap) {
        bt_trade r;
        r.entry_bar = a.e;
        r.exit_bar = t;
        r.side = a.pos;
        r.pad = 0;
        r.entry_px = a.ce;
        r.exit_px = cx;
        tr[a.ntr] = r;
    }
    a.ntr++;
}

template <bool RESET_AGG = true>
__device__ __forceinline__ void sma_open(SmaAcct& a, int b, int t, int32_t cx, int np) {
    a.e = t;
    a.ce = cx;
    a.sb = b;
    if (RESET_AGG) a.agg = kAggId;
    a.pos = np;
}

// One reversal at the lowest flip of F. FIRST: the lane's first reversal of the tile, whose
// closing trade may carry a path from earlier tiles (a.agg); every later reversal of the tile
// closes a trade opened at the previous flip, so it skips the merge and leaves a.agg alone
// (already the identity).
template <bool PARITY, bool ONE_TRIP, bool FIRST, bool SEG, bool NARROW>
__device__ __forceinline__ void sma_reverse(SmaAcct& a, uint64_t& F, uint64_t& alt, int t0,
                                            const int32_t* cT, const int64_t* ql, const Agg* D,
                                            bt_trade* tr, int cap) {
    const int b = __builtin_ctzll(F);
    F &= F - 1;
    Agg seg;
    int32_t cx;
    uint64_t qb;
    if (ONE_TRIP) {
        // all four LDS reads of the iteration issued before one wait: pays at low occupancy
        // (config 5's one 16-wave block per CU: 157.7 -> 152.1 ms), costs ~1 % at config 2's
        // six waves per SIMD, where the compiler's two round trips are hidden anyway
        const Agg* Dr = dst_rowp(D, a.sb, b);
        const Agg d1 = Dr[a.sb], d2 = Dr[b];
        cx = cT[b];
        qb = (uint64_t)ql[b];
        asm volatile("" ::"v"(d1.mx), "v"(d1.mn), "v"(d1.dd), "v"(d1.du), "v"(d2.mx),
                     "v"(d2.mn), "v"(d2.dd), "v"(d2.du), "v"(cx), "v"((uint32_t)qb),
                     "v"((uint32_t)(qb >> 32)));
        seg = agg_merge(d1, d2);
    } else {
        seg = dst_query_bf(D, a.sb, b);  // issued first: addresses need only b
        cx = cT[b];
        qb = (uint64_t)ql[b];
    }
    alt = qb - alt;
    sma_close<PARITY, FIRST, SEG, NARROW>(a, seg, t0 + b, cx, tr, cap);
    sma_open<FIRST>(a, b, t0 + b, cx, -a.pos);
}

// The tile's flips F (bar order). Sharpe partials: a close adds +pos * QL[b], an open subtracts
// np * QL[b] (a reversal adds 2 pos QL[b]); the squared sum changes only on the first entry
// (-Q2L[b]) and the forced exit (+Q2L[b]).
template <bool PARITY, bool ONE_TRIP, bool SEG, bool NARROW>
__device__ __forceinline__ void sma_flips(SmaAcct& a, uint64_t F, int t0, int bl, uint64_t LONG,
                                          const int32_t* cT, const int64_t* ql, const Agg* D,
                                          bt_trade* tr, int cap) {
    const uint64_t FX = (bl >= 0 && bl < 64) ? (F & (1ULL << bl)) : 0ULL;  // forced exit
    F ^= FX;
    if (a.pos == 0 && F != 0) {  // the entry from flat (once per lane)
        const int b = __builtin_ctzll(F);
        F &= F - 1;
        const int np = ((LONG >> b) & 1) ? 1 : -1;
        const uint64_t qx = (uint64_t)ql[b];
        a.ps1 += np > 0 ? (uint64_t)0 - qx : qx;
        a.ps2 -= (uint64_t)ql[kTile + b];
        a.e0 = t0 + b;
        sma_open(a, b, t0 + b, cT[b], np);
    }
    // reversals; a wave iterates max(flips per lane) times. The k-th reversal closes side
    // p_k = (-1)^(k-1) p_1 and adds 2 p_k QL[b_k]: an alternating sum, carried as
    // alt_k = QL[b_k] - alt_(k-1), so that sum = 2 p_n alt_n = -2 pos alt after the loop
    uint64_t alt = 0;
    if (F) sma_reverse<PARITY, ONE_TRIP, true, SEG, NARROW>(a, F, alt, t0, cT, ql, D, tr, cap);
    while (F) sma_reverse<PARITY, ONE_TRIP, false, SEG, NARROW>(a, F, alt, t0, cT, ql, D, tr, cap);
    a.ps1 += a.pos > 0 ? (uint64_t)0 - (alt << 1) : alt << 1;
    if (FX) {  // flat after bar B-1 (only set when a position is open before it)
        const int b = bl;
        const uint64_t qx = (uint64_t)ql[b];
        sma_close<PARITY, true, SEG, NARROW>(a, dst_query_bf(D, a.sb, b), t0 + b, cT[b], tr, cap);
        a.ps1 += a.pos > 0 ? qx : (uint64_t)0 - qx;
        a.ps2 += (uint64_t)ql[kTile + b];
        a.pos = 0;
    }
}

// The kernel body. SEG: one bar segment per block (blockIdx.z = segment, or with fix_seg >= 1 the
// fix pass of that boundary), results into SmaSegRec records (internal.h) that sma_seg_combine
// folds. A segment s >= 1 scans the ring alone over the windows' lookback (the prefix sums only),
// walks `burn` tiles before its first bar starting flat (an SMA position is the sign of the last
// strict crossover comparison, so one decided bar sets it), and carries the trade open at its
// first bar symbolically (SmaAcct::carried). The fix pass re-walks a segment whose lanes started
// in a position other than the previous segment's last one (a burn-in of tied comparisons only).
template <bool PARITY, bool STAMPS, bool ONE_TRIP, bool SEG>
__device__ __forceinline__ void sma_body(const SymDesc* __restrict__ syms,
                                         const int32_t* __restrict__ close, const Grid& g,
                                         const Out& out, int dedicated, const SegArgs& sg,
                                         int fix_seg) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int nf = g.na, ns = g.nb, nw = nf + ns;
    const int R = g.ring;
    const SmaLds LL = sma_lds_layout(R, nw);
    double* ring = reinterpret_cast<double*>(smem + LL.ring);
    int32_t* keys = reinterpret_cast<int32_t*>(smem + LL.keys);
    double* invw = reinterpret_cast<double*>(smem + LL.invw);
    int32_t* win = reinterpret_cast<int32_t*>(smem + LL.win);
    Agg* dst = reinterpret_cast<Agg*>(smem + LL.dst);
    int32_t* cts = reinterpret_cast<int32_t*>(smem + LL.ct);
    int64_t* qls = reinterpret_cast<int64_t*>(smem + LL.ql);
    int32_t* nars = reinterpret_cast<int32_t*>(smem + LL.nar);
    uint32_t* ctr = reinterpret_cast<uint32_t*>(smem + LL.ctr);

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // the last wave runs stage 1; with `dedicated` it is a helper with no parameter lanes,
    // otherwise (a grid that fills all 16 waves of one block) it also walks 64 parameters
    const int nwaves = (int)blockDim.x >> 6;
    const bool helper = (tid >> 6) == nwaves - 1;
    const int nparam_threads = dedicated ? (int)blockDim.x - 64 : (int)blockDim.x;
    const SymDesc sd = syms[blockIdx.x];
    const int B = sd.bars;
    const int ntiles = (B + kTile - 1) / kTile;
    const int P = g.n_params;
    // lanes run over the fast windows first (lane j -> fast j % nf, slow j / nf): a wave then
    // holds few slow windows, and the slow window sets most of a pair's flip rate, so the flip
    // loop (a wave iterates max-over-lanes flips) wastes fewer lanes (config 2: 2.51 -> 2.11
    // iterations per wave-tile). Results stay in param order p = fast * ns + slow.
    const int j = blockIdx.y * nparam_threads + tid;
    const bool active = tid < nparam_threads && j < P;
    const int kf = active ? j % nf : 0;
    const int ks = nf + (active ? j / nf : 0);
    const int p = (kf * ns) + (ks - nf);
    const int32_t* crow = close + sd.off;

    // tiles of this block: ring-only lookback from T_scan, walked from T_walk, accounted from
    // T_acct, up to T_end (exclusive); all tiles without SEG
    SegRange sr{0, 0, 0, 0, ntiles};
    SmaSegRec* mine = nullptr;
    size_t ipos = 0, npos = 0;  // this lane's slot in the position planes, their size
    if (SEG) {
        sr = seg_range(sg, fix_seg, ntiles, g.wmax);
        const size_t per_seg = (size_t)gridDim.x * P;
        ipos = sr.seg * per_seg + (size_t)blockIdx.x * P + p;
        npos = (size_t)sg.G * per_seg;
        mine = reinterpret_cast<SmaSegRec*>(sg.rec) + ipos;
        if (fix_seg > 0) {  // re-walk only if some lane started in a position other than the true one
            // (the int8 planes: 2 B per lane instead of a line of each record)
            if (!__syncthreads_or(active && sg.pos[ipos] != sg.pos[npos + ipos - per_seg])) return;
            if (tid == 0) atomicAdd(sg.refixed, 1ULL);
        }
    }
    const int T_scan = sr.T_scan, T_walk = sr.T_walk, T_acct = sr.T_acct, T_end = sr.T_end;

    const int nwp = (nw + kKeyGrab - 1) / kKeyGrab * kKeyGrab;
    const uint32_t key_round = key_round_len(nwp, nwaves);
    for (int w = tid; w < nwp; w += blockDim.x) {
        const int W = w < nf ? g.a[w] : (w < nw ? g.b[w - nf] : 1);
        win[w] = W;
        invw[w] = key_recip(W);
    }
    if (tid == 0) {
        ring[(T_scan * kTile) & (R - 1)] = 0.0;  // prefix base: sums over scanned bars
        *ctr = (uint32_t)T_walk * key_round;     // key rounds are numbered by tile
    }
    __syncthreads();
    const int warm = max(win[kf], win[ks]) - 1;  // first decision bar of this lane
    // both window lengths in one register (each < 2^16), for the rare exact tie settle
    const uint32_t fsw = (uint32_t)win[kf] | ((uint32_t)win[ks] << 16);

    ScanCarry cy{0, (T_scan > 0 && T_scan * kTile - 1 < B) ? crow[T_scan * kTile - 1] : 0};
    // SEG lookback: the prefix ring over the windows before the first walked bar (config 5: 100
    // tiles). The loop is bound by the load latency, so kLookAhead tiles' closes are in flight
    // while one is summed (one in flight made the lookback ~5 % of a segment block)
    if (SEG && helper && T_scan < T_walk) {
        constexpr int kLookAhead = 8;
        int32_t cn[kLookAhead];
#pragma unroll
        for (int u = 0; u < kLookAhead; ++u) cn[u] = load_close(crow, B, (T_scan + u) * kTile + lane);
#pragma unroll 1
        for (int T0 = T_scan; T0 < T_walk; T0 += kLookAhead) {
#pragma unroll
            for (int u = 0; u < kLookAhead; ++u) {
                const int T = T0 + u;
                if (T < T_walk) {  // wave-uniform
                    const int32_t c = cn[u];
                    cn[u] = load_close(crow, B, (T + kLookAhead) * kTile + lane);
                    const int64_t inc = wave_iscan_i64((int64_t)c);
                    ring[(T * kTile + lane + 1) & (R - 1)] = (double)(cy.P + inc);
                    cy.P += lane63_i64(inc);
                    cy.prevc = (int32_t)__builtin_amdgcn_readlane((uint32_t)c, 63);
                }
            }
        }
    }
    // prologue: stage 1 for the first two walked tiles; stage 2 for the first. The helper keeps
    // the closes of the tile after next in flight (cpre) across the barrier.
    int32_t cpre = 0;
    if (helper) {
        const int b0 = T_walk * kTile;
        const int32_t c0 = load_close(crow, B, b0 + lane), c1 = load_close(crow, B, b0 + kTile + lane);
        cpre = load_close(crow, B, b0 + 2 * kTile + lane);
        const int s0 = T_walk % kStages, s1 = (T_walk + 1) % kStages;
        if (T_walk < T_end) stage_ring(c0, B, b0, lane, R, ring, cts + s0 * kTile, qls + s0 * 2 * kTile, nars + s0, cy);
        __syncthreads();
        if (T_walk + 1 < T_end)
            stage_ring(c1, B, b0 + kTile, lane, R, ring, cts + s1 * kTile, qls + s1 * 2 * kTile, nars + s1, cy);
    } else {
        __syncthreads();
    }
    if (T_walk < T_end)
        stage_keys(T_walk * kTile, B, nw, nwp, nf, g.wmax, R, ring, win, invw,
                   keys + (T_walk & 1) * nwp * kKS, ctr, (uint32_t)T_walk, nwaves, lane,
                   cts + (T_walk % kStages) * kTile, dst + (T_walk % kDstStages) * kDstLevels * kTile);
    __syncthreads();

    SmaAcct a;
    a.pos = a.e = a.ce = a.sb = a.ntr = a.e0 = 0;
    a.g32 = a.m32 = a.r32 = 0;
    a.R = a.gap = a.mdd = 0;
    a.ps1 = a.ps2 = 0;
    a.h = 0;
    a.s1.clear();
    a.s2.clear();
    a.agg = kAggId;
    a.Bq = a.C = a.D = kNegInf;
    a.carried = a.x1 = a.px1 = 0;
    a.agg1 = kAggId;
    int32_t start_pos = 0;
    // the true position entering (the previous segment's end)
    if (SEG && fix_seg > 0 && active) a.pos = sg.pos[npos + ipos - (size_t)gridDim.x * P];
    // SEG: at the first accounted bar keep the position, drop the burn-in's accounts, and carry
    // the open trade (its entry lies before the segment) symbolically from here
    auto enter_acct = [&]() {
        start_pos = a.pos;
        a.carried = a.pos != 0;
        a.agg = kAggId;
        a.sb = 0;
        a.R = 0;
        a.Bq = a.C = a.D = kNegInf;
        a.ntr = 0;
        a.h = 0;
        a.s1.clear();
        a.s2.clear();
        a.ps1 = a.ps2 = 0;
        a.e0 = -1;
        a.x1 = -1;
        a.px1 = 0;
        a.agg1 = kAggId;
    };
    if (SEG && T_walk == T_acct) enter_acct();
    bt_trade* tr = nullptr;
    // the result index; recomputed after the walk (result_index) so that neither it nor kf / ks
    // stay live through the tile loop for it
    auto result_index = [&]() -> size_t {
        int le = lane;
        asm volatile("" : "+v"(le));  // opaque: not merged with the value computed above
        const int je = blockIdx.y * nparam_threads + wave * 64 + le;
        return (size_t)blockIdx.x * P + (size_t)((je % nf) * ns + je / nf);
    };
    const size_t gi = (size_t)blockIdx.x * P + p;
    if (PARITY && active) tr = out.trades + gi * out.trade_cap;
    const int cap = out.trade_cap;

    // profiling stamps (diagnostic only: Grid::ablate & 64); wave-uniform sums in SGPRs
    constexpr bool stamps = STAMPS;  // separate diagnostic instantiation
    uint64_t st_acc[7] = {0, 0, 0, 0, 0, 0, 0};
    uint64_t st_prev = 0;
#define BT_STAMP(i)                                             \
    if (stamps) {                                               \
        const uint64_t now_ = __builtin_amdgcn_s_memtime();     \
        st_acc[i] += now_ - st_prev;                            \
        st_prev = now_;                                         \
    }
    if (stamps) st_prev = __builtin_amdgcn_s_memtime();

    // One tile (interval k of the pipeline). NARROW: the accounts run in int32 (SmaAcct) — the
    // tiles of a symbol whose closes' total variation through the tile end is below 2^30, a
    // prefix of its tiles (TV only grows): a loop over them, then a loop over the rest with
    // int64 accounts, so each walk keeps its own registers.
    auto tile_step = [&](auto narrow_tag, const int k) __attribute__((always_inline)) {
        constexpr bool NARROW = decltype(narrow_tag)::value;
        const int t0 = k * kTile;
        // ---- stage 1 (helper, tile k+2), then stage 3 (parameter waves, tile k), then stage 2
        // (tile k+1) on every wave, balanced dynamically
        if (helper && k + 2 < T_end && !BT_ABL(g, 1)) {
            // stage 1 is a dependent DPP/fp64 chain on one wave: issue it first
            if (!BT_ABL(g, 32)) __builtin_amdgcn_s_setprio(2);
            const int s = (k + 2) % kStages;
            stage_ring(cpre, B, t0 + 2 * kTile, lane, R, ring, cts + s * kTile,
                       qls + s * 2 * kTile, nars + s, cy);
            cpre = load_close(crow, B, t0 + 3 * kTile + lane);
            __builtin_amdgcn_s_setprio(0);
        }
        BT_STAMP(0)
        // ---- stage 3 (tile k)
        if (SEG && active && k == T_acct && k != T_walk) enter_acct();
        if (active) {
            // blocks of more than 8 waves (one per CU): compare and walk at raised priority over
            // the keys / scan work of other waves (config 5 156.4 -> 151.0 ms; config 2's 8-wave
            // blocks are ~1 % slower with it)
            if (ONE_TRIP) __builtin_amdgcn_s_setprio(1);
            const int s = k % kStages;
            const int32_t* cT = cts + s * kTile;
            const int64_t* ql = qls + s * 2 * kTile;
            const Agg* D = dst + (k % kDstStages) * kDstLevels * kTile;
            const int32_t* K = keys + (k & 1) * nwp * kKS;
            const int4* k1 = reinterpret_cast<const int4*>(K + kf * kKS);
            const int4* k2 = reinterpret_cast<const int4*>(K + ks * kKS);
            uint32_t l0 = 0, l1 = 0, z = ~0u;
            if (!BT_ABL(g, 4)) {
                // all reads at immediate offsets from one address per row
#pragma unroll
                for (int v = 0; v < 16; ++v) {
                    if (v < 8) cmp4(l0, z, k1[v], k2[v]);
                    else cmp4(l1, z, k1[v], k2[v]);
                    // keep the schedule to two int4 pairs in flight at config 2's 80-VGPR budget;
                    // a one-block-per-CU 16-wave block (ONE_TRIP, up to 128 VGPRs, 4 waves per
                    // SIMD to hide LDS latency) keeps kCmpDepth1 pairs in flight
                    if (ONE_TRIP ? ((v % kCmpDepth1) == kCmpDepth1 - 1) : (v & 1))
                        __builtin_amdgcn_sched_barrier(0);
                }
            }
            BT_STAMP(2)
            uint64_t L = ((uint64_t)__builtin_bitreverse32(l1) << 32) | __builtin_bitreverse32(l0);
            const int lastdec = B - 2 - t0;  // decisions only at t <= B-2, from the warm bar on
            const int wb = warm - t0;
            const int bl = B - 1 - t0;       // forced exit: flat after bar B-1
            uint64_t LONG, F;
            if (z != 0 && wb <= 0 && lastdec >= 63) {
                // every bar decides and no keys are equal: the position after bar b is simply
                // long iff fast > slow (LONG = G = ~L), and the flips are its changes
                LONG = ~L;
                F = (LONG ^ ((LONG << 1) | (uint64_t)(a.pos == 1))) | (uint64_t)(a.pos == 0);
            } else {
                uint64_t vm = lastdec >= 63 ? ~0ULL : (lastdec < 0 ? 0ULL : ((1ULL << (lastdec + 1)) - 1));
                vm &= wb <= 0 ? ~0ULL : (wb >= 64 ? 0ULL : (~0ULL << wb));
                uint64_t G, T = 0;
                if (z != 0) {
                    G = ~L & vm;
                } else {  // some bar has equal floor keys: settle those exactly
                    const uint64_t E = eq_word(K + kf * kKS, K + ks * kKS);
                    G = ~(L | E) & vm;
                    T = E & vm;
                }
                L &= vm;
                while (T) {
                    const int b = __builtin_ctzll(T);
                    T &= T - 1;
                    const int t = t0 + b;
                    // window sums are exact in the ring (< 2^53) and < 2^31 w; F s and L f
                    // are < 2^31 f s < 2^59 for any windows the LDS ring can hold (< 2^14),
                    // so the tie is settled in int64 for every grid the engine accepts
                    const double top = ring[(t + 1) & (R - 1)];
                    const int fw = (int)(fsw & 0xffffu), sw = (int)(fsw >> 16);
                    const int64_t Fs = (int64_t)(top - ring[(t + 1 - fw) & (R - 1)]) * sw;
                    const int64_t Lf = (int64_t)(top - ring[(t + 1 - sw) & (R - 1)]) * fw;
                    G |= (uint64_t)(Fs > Lf) << b;
                    L |= (uint64_t)(Fs < Lf) << b;
                }
                // set/reset latches via add-with-carry: carry into bit b+1 == position after bar b
                uint64_t SHORT;
                {
                    const uint64_t A = ~L;
                    const uint64_t s1 = A + G;
                    uint64_t cout = s1 < A;
                    const uint64_t sum = s1 + (uint64_t)(a.pos == 1);
                    cout |= sum < s1;
                    LONG = ((sum ^ A ^ G) >> 1) | (cout << 63);
                }
                {
                    const uint64_t A = ~G;
                    const uint64_t s1 = A + L;
                    uint64_t cout = s1 < A;
                    const uint64_t sum = s1 + (uint64_t)(a.pos == -1);
                    cout |= sum < s1;
                    SHORT = ((sum ^ A ^ L) >> 1) | (cout << 63);
                }
                if (bl < 64) {
                    const uint64_t keep = bl <= 0 ? 0ULL : ((1ULL << bl) - 1);
                    LONG &= keep;
                    SHORT &= keep;
                }
                const uint64_t pL = (LONG << 1) | (uint64_t)(a.pos == 1);
                const uint64_t pS = (SHORT << 1) | (uint64_t)(a.pos == -1);
                F = (LONG ^ pL) | (SHORT ^ pS);
            }
            BT_STAMP(3)
            uint64_t Fw = F;
            if (BT_ABL(g, 8)) {  // profiling: drop the trade events (keep F live)
                asm volatile("" ::"v"((uint32_t)Fw), "v"((uint32_t)(Fw >> 32)));
                Fw = 0;
            }
            sma_flips<PARITY, ONE_TRIP, SEG, NARROW>(a, Fw, t0, bl, LONG, cT, ql, D, tr, cap);
            BT_STAMP(4)
            if (a.pos != 0) {  // open at the tile end: path so far, returns to the tile end
                a.agg = agg_merge(a.agg, dst_query_bf(D, a.sb, kTile - 1));
                a.sb = 0;
                const uint64_t q63 = (uint64_t)ql[kTile - 1];
                a.ps1 += a.pos > 0 ? q63 : (uint64_t)0 - q63;
                a.ps2 += (uint64_t)ql[2 * kTile - 1];
            }
            // fold the return partials into int128 every second tile (and at the last): over
            // 128 bars |sum pos q| and sum q2 stay below 2^63 (|q|, q2 <= 2^56 by spec §3, and not
            // all 128 can reach it: that needs |ret| = 1 at every bar, i.e. 128 doublings or a
            // zero price), so the uint64 partials are exact as int64
            if ((k & 1) || k + 1 == T_end) {
                a.s1.add((int64_t)a.ps1);
                a.s2.add((int64_t)a.ps2);
                a.ps1 = a.ps2 = 0;
            }
            BT_STAMP(5)
            if (ONE_TRIP) __builtin_amdgcn_s_setprio(0);
        }
        if (k + 1 < T_end && !BT_ABL(g, 2))
            stage_keys(t0 + kTile, B, nw, nwp, nf, g.wmax, R, ring, win, invw, keys + ((k + 1) & 1) * nwp * kKS,
                       ctr, (uint32_t)(k + 1), nwaves, lane, cts + ((k + 1) % kStages) * kTile,
                       dst + ((k + 1) % kDstStages) * kDstLevels * kTile);
        BT_STAMP(1)
        __syncthreads();
        BT_STAMP(6)
    };
    int k = T_walk;
    if (!SEG && k < T_end) {
        bool nar = __builtin_amdgcn_readfirstlane(nars[k % kStages]) != 0;
        while (nar) {
            // the flag of tile k + 1: written by stage 1 two intervals ago, rewritten (tile k + 4)
            // only in interval k + 2
            const int32_t nn = k + 1 < T_end ? nars[(k + 1) % kStages] : 0;
            tile_step(std::true_type{}, k);
            nar = __builtin_amdgcn_readfirstlane(nn) != 0;
            ++k;
        }
        a.gap = (uint32_t)a.g32;  // >= 0
        a.mdd = (uint32_t)a.m32;
        a.R = a.r32;
    }
    for (; k < T_end; ++k) tile_step(std::false_type{}, k);
#undef BT_STAMP
    if (stamps && lane == 0) {
        unsigned long long* d = out.dbg + (helper ? 8 : 0);
        for (int i = 0; i < 7; ++i) atomicAdd(&d[i], (unsigned long long)st_acc[i]);
        atomicAdd(&d[7], 1ULL);
    }
    if (SEG) {
        if (active) {
            SmaSegRec r;
            r.ntr = a.ntr;
            r.e0 = a.e0;
            r.start_pos = start_pos;
            r.end_pos = a.pos;
            r.end_e = a.carried ? -1 : a.e;
            r.end_ce = a.ce;
            r.x1 = a.x1;
            r.px1 = a.px1;
            const Agg g1 = a.x1 >= 0 ? a.agg1 : a.agg;  // carried through: its path so far
            r.agg1[0] = g1.mx;
            r.agg1[1] = g1.mn;
            r.agg1[2] = g1.dd;
            r.agg1[3] = g1.du;
            r.end_agg[0] = a.agg.mx;
            r.end_agg[1] = a.agg.mn;
            r.end_agg[2] = a.agg.dd;
            r.end_agg[3] = a.agg.du;
            r.R = a.R;
            r.B = a.Bq;
            r.C = a.C;
            r.D = a.D;
            r.h = a.h;
            r.s1lo = a.s1.lo;
            r.s1hi = a.s1.hi;
            r.s2lo = a.s2.lo;
            r.s2hi = a.s2.hi;
            *mine = r;
            sg.pos[ipos] = (int8_t)start_pos;
            sg.pos[npos + ipos] = (int8_t)a.pos;
        }
        return;
    }
    if (active) {
        const uint64_t s1lo = a.s1.lo, s2lo = a.s2.lo;
        const int64_t s1hi = a.s1.hi64(), s2hi = a.s2.hi64();
        const double sh = sharpe_fx(s1lo, s1hi, s2lo, s2hi, B, g.sqrt_ann);
        bt_summary r;
        r.n_trades = a.ntr;
        r.status = 0;
        r.pnl = a.R;
        r.mdd = a.mdd;
        // bars held: trades are back to back from the first entry to the forced exit at B-1
        r.exposure = a.ntr > 0 ? B - 1 - a.e0 : 0;
        r.sharpe = sh;
        r.hash = a.h;
        const size_t go = result_index();
        out.sum[go] = r;
        out.key[go] = order_key(sh);
        if (out.sums != nullptr) out.sums[go] = bt_sums{s1lo, s1hi, s2lo, s2hi};
    }
    wave_add_trades(out, active ? a.ntr : 0);
}

template <bool PARITY, bool STAMPS, bool ONE_TRIP>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(6))) void sma_kernel(
    const SymDesc* __restrict__ syms, const int32_t* __restrict__ close, Grid g, Out out,
    int dedicated) {
    sma_body<PARITY, STAMPS, ONE_TRIP, false>(syms, close, g, out, dedicated, SegArgs{}, 0);
}

// Bar segments (SMA_SEG): its own kernel, for one-block-per-CU shapes (up to 128 VGPRs).
template <bool ONE_TRIP>
__global__ __launch_bounds__(1024) void sma_seg_kernel(const SymDesc* __restrict__ syms,
                                                       const int32_t* __restrict__ close, Grid g,
                                                       Out out, int dedicated, SegArgs sg,
                                                       int fix_seg) {
    sma_body<false, false, ONE_TRIP, true>(syms, close, g, out, dedicated, sg, fix_seg);
}

// Folds the segments of every (symbol, param) in order (internal.h SmaSegRec): the trade open
// across a boundary is closed here, with its entry from the segment that opened it and its path
// merged over the segments it spans; the other trades' sums add and their drawdown forms compose.
// The block's 256 records of a segment are read as one contiguous 32 KB run, 16 B per lane and
// load (a streaming read, instead of eight 16-B loads per lane strided by the 128-B record),
// through LDS.
__global__ __launch_bounds__(256) void sma_seg_combine(const SymDesc* __restrict__ syms, int n_sym,
                                                       int P, const SmaSegRec* __restrict__ rec,
                                                       int G, double sqrt_ann, Out out) {
    __shared__ int4 stage[256 * sizeof(SmaSegRec) / sizeof(int4)];
    const size_t i0 = (size_t)blockIdx.x * blockDim.x;
    const size_t i = i0 + threadIdx.x;
    const size_t n = (size_t)n_sym * P;
    const size_t nb = min((size_t)blockDim.x, n - i0);  // records of this block (per segment)
    constexpr int kPer = sizeof(SmaSegRec) / sizeof(int4);  // 16-B chunks per record
    int ntr = 0;
    {
        const int s = i < n ? (int)(i / P) : 0;
        int32_t pos = 0, e = 0, ce = 0, e0 = -1;
        Agg agg = kAggId;
        int64_t R = 0, gap = 0, mdd = 0;
        uint64_t h = 0;
        i128 s1 = 0, s2 = 0;
        for (int q = 0; q < G; ++q) {
            __syncthreads();  // the previous segment's records are consumed
            const int4* src = reinterpret_cast<const int4*>(rec + (size_t)q * n + i0);
            for (int c = threadIdx.x; c < (int)nb * kPer; c += blockDim.x) stage[c] = src[c];
            __syncthreads();
            if (i >= n) continue;
            const SmaSegRec& r = reinterpret_cast<const SmaSegRec*>(stage)[threadIdx.x];
            ntr += r.ntr;
            R += r.R;
            h += r.h;
            s1 += (i128)(((unsigned __int128)(uint64_t)(int64_t)r.s1hi << 64) | r.s1lo);
            s2 += (i128)(((unsigned __int128)(uint64_t)(int64_t)r.s2hi << 64) | r.s2lo);
            if (e0 < 0) e0 = r.e0;
            const Agg a1 = Agg{r.agg1[0], r.agg1[1], r.agg1[2], r.agg1[3]};
            if (pos != 0) {
                if (r.x1 >= 0) {  // the carried trade closes in this segment, before its others
                    const Agg st = agg_merge(agg, a1);
                    const bool lg = pos > 0;
                    const int32_t lo = lg ? st.mn - ce : ce - st.mx;
                    const int32_t hi = lg ? st.mx - ce : ce - st.mn;
                    const int32_t path = lg ? st.dd : st.du;
                    const int32_t pnl = lg ? r.px1 - ce : ce - r.px1;
                    mdd = max(mdd, max(gap - (int64_t)lo, (int64_t)path));
                    gap = max(gap, (int64_t)hi) - pnl;
                    R += pnl;
                    h += trade_mix_et((uint32_t)e, (uint32_t)r.x1, lg);
                } else {
                    agg = agg_merge(agg, a1);
                }
            }
            mdd = max(mdd, max(gap + r.C, r.D));
            gap = max(gap - r.R, r.B);  // A = -R
            if (r.end_pos == 0) {
                pos = 0;
            } else if (r.end_e >= 0) {  // a trade opened in this segment is open at its end
                pos = r.end_pos;
                e = r.end_e;
                ce = r.end_ce;
                agg = Agg{r.end_agg[0], r.end_agg[1], r.end_agg[2], r.end_agg[3]};
            }
        }
        if (i < n) {
            const int B = syms[s].bars;
            const uint64_t s1lo = (uint64_t)s1, s2lo = (uint64_t)s2;
            const int64_t s1hi = (int64_t)(s1 >> 64), s2hi = (int64_t)(s2 >> 64);
            const double sh = sharpe_fx(s1lo, s1hi, s2lo, s2hi, B, sqrt_ann);
            bt_summary r;
            r.n_trades = ntr;
            r.status = 0;
            r.pnl = R;
            r.mdd = mdd;
            r.exposure = ntr > 0 ? B - 1 - e0 : 0;
            r.sharpe = sh;
            r.hash = h;
            out.sum[i] = r;
            out.key[i] = order_key(sh);
            if (out.sums != nullptr) out.sums[i] = bt_sums{s1lo, s1hi, s2lo, s2hi};
        }
    }
    wave_add_trades(out, ntr);
}

size_t sma_lds_bytes(const Grid& g) { return sma_lds_layout(g.ring, g.na + g.nb).total; }

// Block shape: one block per symbol when the parameters fit (<= 15 parameter waves + a helper,
// or exactly 16 waves with the scan folded into the last parameter wave), otherwise the fewest
// equal y-blocks; each y-block recomputes the tile scan and keys, so splits are avoided.
SmaShape sma_shape(int P) {
    const int need = (P + 63) / 64;
    SmaShape s;
    if (need == 16) {
        s.pw = 16;
        s.dedicated = 0;
    } else {
        const int nby = (need + 14) / 15;
        s.pw = (need + nby - 1) / nby;
        s.dedicated = 1;
    }
    s.block = 64 * (s.pw + s.dedicated);
    s.gy = (P + 64 * s.pw - 1) / (64 * s.pw);
    return s;
}

// Bar segments for a shard of one-block-per-CU symbols (16-wave blocks: config 5) that fills the
// GPU only a few times over: block times vary with each symbol's trade count, so the launch ends
// with the CU whose few blocks took longest (config 5's 1,250-symbol 8-GPU shard: 4.9 blocks per
// CU, 121 us per symbol against 107 at 10,000 symbols). Cutting each symbol into G segments gives
// G times as many, shorter blocks. A segment costs its burn-in tiles and a ring-only lookback
// over the longest window (about a twentieth of a tile each): G is kept where that stays under 2 %
// of a segment. Shapes of several blocks per CU (config 2) keep G = 1.
int32_t sma_auto_segments(int32_t n_sym, int32_t n_params, int32_t max_bars, int32_t wmax,
                          int32_t burn_tiles) {
    if (n_sym <= 0) return 1;
    const SmaShape sh = sma_shape(n_params);
    if (sh.block <= 512) return 1;
    // enough segment blocks for ~kSegRounds rounds of one block per CU (config 5's 1,250-symbol
    // shard, 4.9 rounds unsplit, round 4: G = 3 / 4 / 5 / 6 / 8 -> 135.0 / 133.5-134.0 /
    // 132.4-132.5 / 132.0 / 132.5 ms; each segment adds one 128-B record per parameter)
    constexpr double kSegRounds = 28.0;
    const double rounds = (double)n_sym * sh.gy / device_cus();
    if (rounds >= kSegRounds) return 1;
    int G = std::min(8, (int)std::ceil(kSegRounds / rounds));
    const int ntiles = (max_bars + kTile - 1) / kTile;
    const int lookback = (wmax - 1 + kTile - 1) / kTile;
    while (G > 1 && burn_tiles + 0.05 * lookback > 0.02 * ntiles / G) --G;
    return G;
}

namespace {

template <bool ONE_TRIP>
hipError_t launch_sma_variant(const SymDesc* syms, int32_t n_sym, const int32_t* close,
                              const Grid& g, const Out& out, bool parity, const SegArgs& seg,
                              hipStream_t st, const SmaShape& sh, size_t lds) {
    const dim3 grid(n_sym, sh.gy), block(sh.block);
    if (seg.G > 1 && !parity) {
        // speculative segments, the fix pass of each boundary in order (a block returns at once
        // when every lane started in the true position), then the fold
        const dim3 sgrid(n_sym, sh.gy, seg.G), fgrid(n_sym, sh.gy, 1);
        for (int s = 0; s < seg.G; ++s)
            hipLaunchKernelGGL((sma_seg_kernel<ONE_TRIP>), s == 0 ? sgrid : fgrid, block, lds, st, syms,
                               close, g, out, sh.dedicated, seg, s);
        const size_t n = (size_t)n_sym * g.n_params;
        hipLaunchKernelGGL(sma_seg_combine, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, syms, n_sym,
                           g.n_params, reinterpret_cast<const SmaSegRec*>(seg.rec), seg.G, g.sqrt_ann, out);
    } else if (parity) {
        hipLaunchKernelGGL((sma_kernel<true, false, ONE_TRIP>), grid, block, lds, st, syms, close, g, out,
                           sh.dedicated);
    } else {
        hipLaunchKernelGGL((sma_kernel<false, false, ONE_TRIP>), grid, block, lds, st, syms, close, g, out,
                           sh.dedicated);
    }
    return hipGetLastError();
}

}  // namespace

hipError_t launch_sma(const SymDesc* syms, int32_t n_sym, const int32_t* close, const Grid& g,
                      const Out& out, bool parity, const SegArgs& seg, hipStream_t st) {
    if (n_sym <= 0) return hipSuccess;
    const SmaShape sh = sma_shape(g.n_params);
    size_t lds = sma_lds_bytes(g);
    // blocks of more than 8 waves (config 5: one 16-wave block per CU) hide little LDS latency:
    // their reversal loop issues all of an iteration's reads before one wait
    bool one_trip = sh.block > 512;
#ifdef BT_PROFILING
    if (BT_ABL(g, 128)) lds = std::max(lds, (size_t)(g.ablate & 256 ? 80 : 60) * 1024);  // occupancy probe
    if (const char* v = getenv("BT_ONE_TRIP")) one_trip = atoi(v) != 0;  // tuning aid
    if (BT_ABL(g, 64)) {
        const dim3 grid(n_sym, sh.gy), block(sh.block);
        hipLaunchKernelGGL((sma_kernel<false, true, false>), grid, block, lds, st, syms, close, g, out,
                           sh.dedicated);
        return hipGetLastError();
    }
#endif
    if (one_trip) return launch_sma_variant<true>(syms, n_sym, close, g, out, parity, seg, st, sh, lds);
    return launch_sma_variant<false>(syms, n_sym, close, g, out, parity, seg, st, sh, lds);
}

}  // namespace bt
