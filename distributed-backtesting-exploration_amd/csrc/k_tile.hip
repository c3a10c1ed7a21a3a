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
#include <cstdlib>

#include <type_traits>

#include "tile_common.h"

namespace bt {

namespace {

// wave priorities (s_setprio) of the pacing roles; BT_PRIO overrides them in the profiling build
// (scripts/gpu_prio_sweep.sh). Round 3 sweep + release A/B: the accountant one level below the
// finder, 7.23 -> 7.03 ms on config 4 at 500 symbols and 3.95 -> 3.83 at 250. The EMA chain at
// the top priority since it alone sets the 128-bar stage (round 6: helper A's tables moved to
// tasks and the chain wave out of the task rounds): config 3 2.565 -> 2.483 ms at 500 symbols,
// 1.598 -> 1.511 at 250 (at the base priority before, -0.5 to -1 %)
#ifndef BT_EMA_CHAIN_PRIO
#define BT_EMA_CHAIN_PRIO 3
#endif
#ifndef BT_EMA_WALK_PRIO
#define BT_EMA_WALK_PRIO 2
#endif
#ifndef BT_BOLL_WALK_PRIO
#define BT_BOLL_WALK_PRIO 2
#endif
#ifndef BT_BOLL_ACCT_PRIO
#define BT_BOLL_ACCT_PRIO 1
#endif
constexpr int kEmaChainPrio = BT_EMA_CHAIN_PRIO, kEmaWalkPrio = BT_EMA_WALK_PRIO;
constexpr int kBollWalkPrio = BT_BOLL_WALK_PRIO, kBollAcctPrio = BT_BOLL_ACCT_PRIO;
constexpr int kEStride = kTile + 1;  // ema buffer row stride (doubles): conflict-free columns
// Bollinger tile buffers: scanned (k+2), flagged (k+1), walked (k) and accounted (k-1, by the
// accountant wave of a split walk)
constexpr int kBollStages = 4;
// EMA+OLS runs stages of TS tiles per barrier (ema_tile_kernel): closes, returns and narrow
// flags of three stages in flight (scanned st+2, flagged st+1, walked st), drawdown tables, chain
// values and condition words of two (built / chained / flagged st+1 or st+2, read a stage later)
__host__ __device__ constexpr int ema_ct_slots(int ts) { return 3 * ts; }
__host__ __device__ constexpr int ema_slots(int ts) { return 2 * ts; }
// drawdown tables: 64-bar stages build them in the scan (three stages of buffers, as the closes),
// 128-bar stages a stage later (two)
__host__ __device__ constexpr int ema_dst_slots(int ts) { return ts == 1 ? ema_ct_slots(1) : ema_slots(ts); }
constexpr int kEmaTS = 2;  // 128-bar stages where the LDS allows (ema_stage_tiles)

// Trade records per lane and tile: an entry needs a bar after the previous exit and an exit a bar
// after its entry, so a tile holds at most 32 entries plus the exit of a position carried in.
constexpr int kRecCap = 33;

// EMA+OLS walk accounts in int32 while the closes' total variation allows (unsplit runs)
#ifndef BT_EMA_NARROW
#define BT_EMA_NARROW 1
#endif
constexpr bool kEmaNarrow = BT_EMA_NARROW;

// the Bollinger walkers' (unsplit parameter waves') gap / mdd in int32 while the closes' total
// variation allows (unsplit runs; tile_common.h acct_close_rt)
#ifndef BT_BOLL_WALK_NARROW
#define BT_BOLL_WALK_NARROW 1
#endif
constexpr bool kBollWalkNarrow = BT_BOLL_WALK_NARROW;

// Bollinger per-stage low/high staging (int32): lows[64], highs[64], 8 block minima of the lows
// then 8 block maxima of the highs, per bar the minimum low / maximum high from that bar to the
// end of its 8-bar block, and per bar the minimum low / maximum high from that bar to the end of
// the tile (SL/TP first-passage search)
constexpr int kLH = 6 * kTile + 16;
constexpr int kLhBx = 2 * kTile, kLhSuf = 2 * kTile + 16, kLhTs = 4 * kTile + 16;

struct TileLds {
    size_t r1, r2, ct, ql, dst, stl, sth, ebuf, words, win, lev, levp, levf, lvb, rec, nrec, nar, ctr, total;
};

// kind 0 = EMA+OLS (na spans, nb windows, ts tiles per stage), 1 = Bollinger (na windows, nb ks,
// nlev SL/TP levels per side: nsl + ntp)
__host__ __device__ inline TileLds tile_lds_layout(int kind, int ring, int na, int nb, int nlev = 0,
                                                  int ts = kEmaTS) {
    TileLds L{};
    size_t o = 0;
    auto take = [&](size_t bytes) { size_t r = o; o += (bytes + 15) & ~size_t(15); return r; };
    // tile buffers: Bollinger kBollStages (one per 64-bar pipeline stage); EMA ema_ct_slots
    // for closes / returns / narrow flags and ema_slots for tables, chain values and words
    const int ns = kind == 1 ? kBollStages : ema_ct_slots(ts), nd = kind == 1 ? kBollStages : ema_dst_slots(ts);
    L.r1 = take((size_t)ring * 8);
    L.r2 = take((size_t)ring * (kind == 0 ? 8 : 16));
    L.ct = take((size_t)ns * kTile * 4);
    L.ql = take((size_t)ns * 2 * kTile * 8);
    L.dst = take((size_t)nd * kDstLevels * kTile * sizeof(Agg));
    if (kind == 1) {
        L.stl = take((size_t)ns * kLH * 4);  // lows, highs, block and in-block suffix extrema
        L.ebuf = take((size_t)nb * 8);                              // k_num^2 as doubles
        L.words = take((size_t)2 * (na * nb + 2 * na) * 8);
        L.win = take((size_t)na * 4);
        L.lev = take((size_t)2 * 2 * nlev * kTile);  // first-passage bars, [tile & 1][side][level][bar]
        L.levp = take((size_t)3 * 2 * nlev * kTile * 4);  // the levels (int32), [tile % 3][side][level][bar]
        L.levf = take((size_t)2 * nlev * 8);         // level factors per side
        L.lvb = take((size_t)(nlev + 1) * 4);        // distinct SL/TP bps, then their count
        // the finder's trade records [tile & 1][record][lane] and records per lane [tile & 1][lane]
        L.rec = take((size_t)2 * kRecCap * kTile * 2);
        L.nrec = take((size_t)2 * kTile);
        L.nar = take((size_t)ns * 4);  // per tile stage: the accountant's sums fit int32 (Acct32)
    } else {
        L.ebuf = take((size_t)ema_slots(ts) * na * kEStride * 8);
        L.words = take((size_t)ema_slots(ts) * (4 * na + 2 * nb) * 8);
        L.win = take((size_t)nb * 4);
        L.nar = take((size_t)ns * 4);  // per tile stage: the walk's accounts fit int32 (Acct32)
    }
    L.ctr = take(4);
    L.total = o;
    return L;
}

__device__ __forceinline__ int32_t ldc(const int32_t* __restrict__ row, int B, int t, int32_t pad) {
    return t < B ? row[t] : pad;
}

// Task counter: round r owns counter values [r * (n + nwaves), (r + 1) * (n + nwaves)):
// n successful grabs plus exactly one failing grab per wave (the barrier separates rounds).
// grab_issue returns the atomic's VGPR; the caller reads lane 0 only when it needs the value,
// so the next grab's round trip overlaps the current task.
__device__ __forceinline__ uint32_t grab_issue(uint32_t* ctr, int lane) {
    uint32_t v = 0;
    if (lane == 0) v = atomicAdd(ctr, 1u);
    return v;
}
__device__ __forceinline__ uint32_t grab_value(uint32_t v) { return __builtin_amdgcn_readlane(v, 0); }

// Prefix rings: entry x (the sum over bars < x) lives at x mod R, with R a multiple of 64 of at
// least the longest window + 3 tiles (engine.cpp), so windows up to the spec's 4,096 bars fit
// in LDS. Position of x = T*64 + lane + 1, and of x - W given that position (0 < W < R).
__device__ __forceinline__ int ring_pos(int T, int lane, int R) {
    const int p = (T % (R / kTile)) * kTile + lane + 1;
    return p == R ? 0 : p;
}
__device__ __forceinline__ int ring_back(int p, int W, int R) {
    const int q = p - W;
    return q < 0 ? q + R : q;
}

// x^2 for x < 2^64, unsigned 128-bit, from three 32 x 32 -> 64 products (the generic
// 64 x 64 -> 128 multiply takes four and sign terms): x^2 = l^2 + 2 h l 2^32 + h^2 2^64.
__device__ __forceinline__ unsigned __int128 sq_u64(uint64_t x) {
    const uint32_t l = (uint32_t)x, h = (uint32_t)(x >> 32);
    const uint64_t ll = (uint64_t)l * l, hl = (uint64_t)h * l, hh = (uint64_t)h * h;
    const uint64_t mid_lo = hl << 33, mid_hi = hl >> 31;  // 2 h l 2^32 = mid_hi 2^64 + mid_lo
    const uint64_t lo = ll + mid_lo;
    const uint64_t hi = hh + mid_hi + (lo < ll ? 1 : 0);
    return ((unsigned __int128)hi << 64) | lo;
}

// a * w for a < 2^96 and a 32-bit w (sums of squared prices: < 2^75), exact below 2^128.
__device__ __forceinline__ unsigned __int128 mul_u128_u32(unsigned __int128 a, uint32_t w) {
    const uint64_t lo = (uint64_t)a;
    const uint32_t hi = (uint32_t)(a >> 64);
    const uint64_t p0 = (uint64_t)(uint32_t)lo * w, p1 = (lo >> 32) * (uint64_t)w;
    const uint64_t r_lo = p0 + (p1 << 32);
    const uint64_t r_hi = (uint64_t)hi * w + (p1 >> 32) + (r_lo < p0 ? 1 : 0);
    return ((unsigned __int128)r_hi << 64) | r_lo;
}

// f(integral_constant<int, i>) for i = 0 .. N-1, unrolled.
template <int N, int I = 0, class F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<N, I + 1>(f);
    }
}

// Lane mask of a condition (the builtin on the bool itself: HIP's __ballot(int) materialises the
// condition in a VGPR and compares it again).
__device__ __forceinline__ uint64_t ballot(bool c) { return __builtin_amdgcn_ballot_w64(c); }

// A lane mask as an opaque 64-bit scalar: a mask reassigned in a branch then merges as a scalar
// value instead of a per-lane boolean rebuilt in a VGPR.
__device__ __forceinline__ uint64_t sgpr64(uint64_t x) {
    asm volatile("" : "+s"(x));
    return x;
}

// Lane mask of a > b (fp64) straight from the compare's scalar destination (inactive lanes 0).
__device__ __forceinline__ uint64_t vcmp_gt_f64(double a, double b) {
    uint64_t m;
    asm volatile("v_cmp_gt_f64_e64 %0, %1, %2" : "=s"(m) : "v"(a), "v"(b));
    return m;
}

// Lane masks of 0 <= a, a <= 0 (fp64, int64) and w <= x (int32, w wave-uniform), likewise straight from
// the compare (a ballot of a bool that is not itself a compare costs two VALU more: the bool is
// materialised in a VGPR and compared again).
__device__ __forceinline__ uint64_t vcmp_ge0_f64(double a) {
    uint64_t m;
    asm volatile("v_cmp_le_f64_e64 %0, 0, %1" : "=s"(m) : "v"(a));
    return m;
}
__device__ __forceinline__ uint64_t vcmp_le0_f64(double a) {
    uint64_t m;
    asm volatile("v_cmp_ge_f64_e64 %0, 0, %1" : "=s"(m) : "v"(a));
    return m;
}
__device__ __forceinline__ uint64_t vcmp_ge0_i64(int64_t a) {
    uint64_t m;
    asm volatile("v_cmp_le_i64_e64 %0, 0, %1" : "=s"(m) : "v"(a));
    return m;
}
__device__ __forceinline__ uint64_t vcmp_le0_i64(int64_t a) {
    uint64_t m;
    asm volatile("v_cmp_ge_i64_e64 %0, 0, %1" : "=s"(m) : "v"(a));
    return m;
}
__device__ __forceinline__ uint64_t vcmp_le_i32(int32_t w, int32_t x) {
    uint64_t m;
    asm volatile("v_cmp_le_i32_e64 %0, %1, %2" : "=s"(m) : "s"(w), "v"(x));
    return m;
}

// `bit` if the lane mask m is not empty, else 0, in two scalar instructions (the compiler turns
// the same test into a VGPR bool and a readfirstlane when the result is a zero-extended flag)
template <uint32_t bit>
__device__ __forceinline__ uint32_t any_bit(uint64_t m) {
    uint32_t r;
    asm volatile("s_cmp_lg_u64 %1, 0\n\ts_cselect_b32 %0, %2, 0" : "=s"(r) : "s"(m), "i"(bit) : "scc");
    return r;
}

// v_writelane: lane L of v takes the wave-uniform x.
template <int L>
__device__ __forceinline__ void writelane(uint32_t& v, uint32_t x) {
    asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(v) : "s"(x), "i"(L));
}

// Bits [cur, 63] of a tile word (none for cur >= 64).
__device__ __forceinline__ uint64_t bits_from(int cur) { return cur < kTile ? (~0ULL << cur) : 0ULL; }

// State after every bar of a tile of a set/reset latch (set S and reset R disjoint), q = the
// state before bar 0: an add with carry, whose carry out of bit b is S_b | (~R_b & carry into b).
__device__ __forceinline__ uint64_t latch64(uint64_t S, uint64_t R, uint64_t q) {
    const uint64_t A = ~R;
    const uint64_t s1 = A + S;
    uint64_t cout = s1 < A;
    const uint64_t sum = s1 + q;
    cout |= sum < s1;
    return ((sum ^ A ^ S) >> 1) | (cout << 63);
}

}  // namespace

// profiling stamps: the hardware placement (SE / CU / SIMD, XCD) of wave hw_wave < 8 of the
// first kDbgBlocks blocks (internal.h)
__device__ __forceinline__ void stamp_place(unsigned long long* dbg, int hw_wave, int lane) {
    if (dbg == nullptr || lane != 0 || hw_wave >= 8 || blockIdx.x >= (unsigned)kDbgBlocks || blockIdx.y != 0 ||
        blockIdx.z != 0)
        return;
    const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
    const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);  // XCC_ID
    dbg[kDbgSlots + blockIdx.x * 8 + hw_wave] = ((unsigned long long)xcc << 32 | hw) | (1ull << 40);
}

// ----------------------------------------------------------------------------- EMA + OLS
// Workgroup = parameter waves + helper A + helper B, one barrier per tile:
//   helper A, tile k+2: closes -> returns, drawdown sparse table, prefix rings;
//   helper B, tile k+2: the EMA chains (one sequential fp64 chain per span, lane = span);
//   every wave, tile k+1, after its own work: condition words, one task per span (4 ballots
//           over the EMA values) or per OLS window (exact numerator sign), grabbed from an LDS
//           counter;
//   parameter waves, tile k: the position after every bar from two coupled set/reset latches
//           over the condition words (latch64), then one trade per loop iteration over the
//           latches' edges, O(1) accounting per trade.
// SEG: bar segments as in boll_tile_kernel; besides the lanes' trade states a segment's start
// must agree on the EMA chains: a speculative segment starts each chain at its first scanned bar
// from an estimate of the true value (a truncated weighted sum of the closes before it, summed in
// parallel) and records the values entering its first accounted bar; fp64 chains from different
// starts meet bit for bit once the start's error has decayed below rounding (from the estimate:
// <= 4 spans of bars; from e = c: ~16), after which they are identical. The fix pass compares
// them too and re-walks from the true values.
template <bool PARITY, bool STAMPS, bool SEG, int TS>
__global__ __launch_bounds__(1024) void ema_tile_kernel(const SymDesc* __restrict__ syms,
                                                        const int32_t* __restrict__ close,
                                                        Grid g, Out out, int nextra, int lpw,
                                                        SegArgs sg, int fix_seg) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int nsp = g.na, nol = g.nb, R = g.ring;
    const TileLds LL = tile_lds_layout(0, R, nsp, nol, 0, TS);
    static_assert(TS == 1 || TS == 2, "64- or 128-bar stages");
    constexpr int CT = ema_ct_slots(TS), SL = ema_slots(TS), DS = ema_dst_slots(TS);
    // drawdown tables: built by the scan from its registers (64-bar stages, DSCAN), or as the
    // first tasks of the round that flags their stage (128-bar stages, DSTT: helper A then has
    // only the scans; config 3's task waves were idle ~2.5k cycles per tile while helper A paced
    // at ~3.9k with the tables)
    constexpr bool DSCAN = TS == 1, DSTT = TS == 2;
    uint64_t* r1 = reinterpret_cast<uint64_t*>(smem + LL.r1);  // sum_{i<x} c_i
    uint64_t* r2 = reinterpret_cast<uint64_t*>(smem + LL.r2);  // sum_{i<x} i*c_i (mod 2^64)
    int32_t* cts = reinterpret_cast<int32_t*>(smem + LL.ct);
    int64_t* qls = reinterpret_cast<int64_t*>(smem + LL.ql);
    Agg* dst = reinterpret_cast<Agg*>(smem + LL.dst);
    double* ebuf = reinterpret_cast<double*>(smem + LL.ebuf);  // [2][nsp][kEStride]
    uint64_t* words = reinterpret_cast<uint64_t*>(smem + LL.words);
    int32_t* win = reinterpret_cast<int32_t*>(smem + LL.win);
    int32_t* nars = reinterpret_cast<int32_t*>(smem + LL.nar);
    uint32_t* ctr = reinterpret_cast<uint32_t*>(smem + LL.ctr);

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // waves: [0, npw) parameters, npw helper A, npw + 1 helper B, then `nextra` task-only waves
    const int nwaves = (int)(blockDim.x >> 6), npw = nwaves - 2 - nextra;
    const bool helperA = wave == npw, helperB = wave == npw + 1;
    const SymDesc sd = syms[blockIdx.x];
    const int B = sd.bars, ntiles = (B + kTile - 1) / kTile, P = g.n_params;
    // lpw parameter lanes per parameter wave (64, or fewer for shorter max-over-lanes walks)
    const int j = (blockIdx.y * npw + wave) * lpw + lane;
    const bool active = wave < npw && lane < lpw && j < P;
    const int pj = active ? j : 0;
    const int i_n = pj / nol, i_w = pj % nol;
    const int warm = max(g.a[i_n], g.b[i_w]) - 1;
    const int32_t* crow = close + sd.off;
    // tasks per stage: the drawdown tables of its tiles (DSTT), then one per span / OLS window
    const int nword = 4 * nsp + 2 * nol, ntask = max(nsp, nol) + (DSTT ? TS : 0);
    const int estage = nsp * kEStride;

    SegRange sr{0, 0, 0, 0, ntiles};
    double* ema_mine = nullptr;        // this (segment, symbol)'s chain record
    const double* ema_prev = nullptr;  // the previous segment's
    // this lane's record of segment sq, its address recomputed where it is used from an opaque
    // copy of the parameter index (a pointer kept live across the walk costs a VGPR pair, and the
    // split kernel runs at the 128-VGPR edge)
    auto seg_rec = [&](int sq) {
        int pje = pj;
        asm volatile("" : "+v"(pje));
        return sg.rec + (size_t)sq * gridDim.x * P + (size_t)blockIdx.x * P + pje;
    };
    if (SEG) {
        sr = seg_range(sg, fix_seg, ntiles, g.wmax);
        ema_mine = sg.ema + ((size_t)sr.seg * gridDim.x + blockIdx.x) * kEmaSegStride;
        if (sr.seg > 0) ema_prev = ema_mine - (size_t)gridDim.x * kEmaSegStride;
        if (fix_seg > 0) {  // re-walk if a lane's state or a span's chain value is not the true one
            const bool lane_differs = active && seg_start_differs(seg_rec(sr.seg), seg_rec(sr.seg - 1));
            const bool chain_differs = helperB && lane < nsp && ema_mine[lane] != ema_prev[64 + lane];
            if (!__syncthreads_or(lane_differs || chain_differs)) return;
            if (tid == 0) atomicAdd(sg.refixed, 1ULL);
        }
    }
    if (STAMPS) stamp_place(out.dbg, wave, lane);
    const int T_scan = sr.T_scan, T_walk = sr.T_walk, T_acct = sr.T_acct, T_end = sr.T_end;
    // the chains start at bar 0 with e = c there; a speculative segment's chains continue from
    // an estimate of the true values entering its first scanned bar, and the fix pass starts
    // them at its first bar from the true values
    const bool chain_injected = SEG && fix_seg > 0;
    const bool chain_est = SEG && fix_seg == 0 && T_scan > 0;
    const int chain_b0 = (chain_injected || chain_est) ? -1 : 0;
    const int chain_T0 = chain_injected ? T_acct : T_scan;

    // The estimate: e_ts = sum_{i<M} a (1-a)^i c_{ts-i} + (1-a)^M c_{ts-M+1}, the closed form of
    // the recurrence truncated after e^-36 of the weight (exact in real arithmetic when M reaches
    // bar 0). Every wave sums a strided share of the M bars, four spans at a time; the per-wave
    // sums go to ebuf (free until the first chain tile) and helper B adds them in wave order, so
    // the estimate is deterministic. Its rounding (~1e-14 relative) dies out in ~4 spans of
    // bars; the chains then meet the true ones bit for bit, and the fix pass catches any that
    // do not.
    int est_M = 0;
    if (chain_est) {
        const int ts = T_scan * kTile - 1;
        int maxspan = 1;
        for (int q = 0; q < nsp; ++q) maxspan = max(maxspan, g.a[q]);
        est_M = (int)min((int64_t)ts + 1, (int64_t)18 * ((int64_t)maxspan + 1) + 1);
        const int nchunk = (est_M + kTile - 1) / kTile;
        for (int q0 = 0; q0 < nsp; q0 += 4) {
            double acc[4], w[4], r[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int q = min(q0 + u, nsp - 1);
                const double a = 2.0 / ((double)g.a[q] + 1.0), lb = log2(1.0 - a);
                acc[u] = 0.0;
                w[u] = q0 + u < nsp ? a * exp2(lb * (double)(wave * kTile + lane)) : 0.0;
                r[u] = exp2(lb * (double)(kTile * nwaves));
            }
            for (int ch = wave; ch < nchunk; ch += 8 * nwaves) {
                int32_t cv[8];
#pragma unroll
                for (int v = 0; v < 8; ++v) {
                    const int i = (ch + v * nwaves) * kTile + lane;
                    cv[v] = i < est_M ? crow[ts - i] : 0;
                }
#pragma unroll
                for (int v = 0; v < 8; ++v) {
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        acc[u] = __builtin_fma(w[u], (double)cv[v], acc[u]);
                        w[u] *= r[u];
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                double s = acc[u];
#pragma unroll
                for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
                if (lane == 0 && q0 + u < nsp) ebuf[wave * nsp + q0 + u] = s;
            }
        }
    }

    for (int o = tid; o < nol; o += blockDim.x) win[o] = g.b[o];
    if (tid == 0) {
        // prefix entry x (sum over scanned bars < x) sits at x mod R: the scan's base is 0
        r1[(T_scan * kTile) % R] = 0;
        r2[(T_scan * kTile) % R] = 0;
        // task rounds are numbered by stage (flags), from 0
        *ctr = 0;
    }
    double alpha = 0.0, ema = 0.0;
    if (helperB && lane < nsp) {
        alpha = 2.0 / ((double)g.a[lane] + 1.0);
        if (chain_injected) ema = ema_prev[64 + lane];
    }
    const int winreg = lane < nol ? g.b[lane] : 1;  // OLS window lengths, lane = window
    const double lo_mult = (double)(10000 - g.band_bps), hi_mult = (double)(10000 + g.band_bps);
    __syncthreads();
    if (chain_est && helperB && lane < nsp) {
        double s = 0.0;
        for (int w2 = 0; w2 < nwaves; ++w2) s += ebuf[w2 * nsp + lane];
        const double tail = (double)crow[T_scan * kTile - est_M];
        ema = s + exp2(log2(1.0 - alpha) * (double)est_M) * tail;
    }

    TileCarry cy{0, (T_scan > 0 && T_scan * kTile - 1 < B) ? crow[T_scan * kTile - 1] : 0};
    uint64_t cy2 = 0;

    // Stages of TS tiles (TS = 2: 128 bars per barrier): stage st holds tiles T_scan + TS st ..
    // T_scan + TS st + TS - 1 (those past T_end absent). Per stage, one barrier:
    //   helper A: scans stage st + 2 (closes, returns, prefix rings; at TS = 1 the drawdown
    //             tables too);
    //   helper B: chains stage st + 2;
    //   the other waves: the tasks of stage st + 1 (DSTT: its tables, a stage after the scan,
    //             so they need two stages of buffers, not three: 80 KB per block at TS = 2; then
    //             one task per span / window over all its tiles);
    //   parameter waves: walk stage st, tile by tile.
    // Buffers by tile T: closes, returns, narrow flags T % CT (written st + 2, read st + 1 and st);
    // tables, chain values, words T % SL.
    const int nstage = (T_end - T_scan + TS - 1) / TS;
    auto scan = [&](int T, int32_t c) {
        const int s = T % CT, t0 = T * kTile, t = t0 + lane;
        int64_t inc2 = (int64_t)t * c;  // c = 0 past the end; scanned with the closes
        const int64_t pre = tile_scan<false, true>(c, B, t0, lane, cts + s * kTile, qls + s * 2 * kTile,
                                      dst + (T % DS) * kDstLevels * kTile, cy, DSCAN && !BT_ABL(g, 512),
                                      (SEG || !kEmaNarrow) ? nullptr : nars + s, 0, 0, &inc2);
        const int pt = ring_pos(T, lane, R);
        r1[pt] = (uint64_t)pre;
        r2[pt] = cy2 + (uint64_t)inc2;
        cy2 += (uint64_t)lane63_i64(inc2);
    };
    // drawdown sparse table of tile T from its staged closes (lane = bar; 0 past the end, as the
    // scan saw them)
    auto dbuild = [&](int T) {
        if (BT_ABL(g, 512)) return;  // (profiling ablation: no table)
        dst_build(cts[(T % CT) * kTile + lane], lane, dst + (T % DS) * kDstLevels * kTile);
    };

    // EMA chains of tile T, lane = span, from the tile's closes cl (lane = bar) that helper B
    // loads itself (no dependency on helper A's scan of the same tile):
    // e_t = e_{t-1} + alpha (c_t - e_{t-1}), three roundings, e_0 = c_0
    auto chain = [&](int T, int32_t cl) {
        if (SEG && T < chain_T0) return;  // fix pass: bars before the segment are not needed
        const int t1 = T * kTile;
        double* E = ebuf + (T % SL) * estage + lane * kEStride;
        // three dependent fp64 operations per bar; raising its priority over the walk no longer
        // pays (the walk, tasks, scan and chain all set the tile together: DESIGN.md §4.2)
        if (!BT_ABL(g, 32)) set_prio(BT_PRIO(g, 16, kEmaChainPrio));
        // the tile's closes as doubles, staged in span 0's row (lane = bar): each bar's close is
        // then one broadcast LDS read issued ahead of the chain instead of a readlane and a
        // conversion on it; span 0 overwrites bar b only after every span has read it (one
        // wave, LDS in program order)
        const double* CD = ebuf + (T % SL) * estage;
        if (nsp > 0) ebuf[(T % SL) * estage + lane] = (double)cl;
        if (lane < nsp && !BT_ABL(g, 256)) {  // profiling: 256 drops the chain, 128 its math
            if (BT_ABL(g, 128)) {
#pragma unroll
                for (int b = 0; b < kTile; ++b) E[b] = (double)__builtin_amdgcn_readlane(cl, b);
            } else if ((chain_b0 < t1 || chain_b0 >= t1 + kTile) && t1 + kTile <= B) {
                // 8 bars' closes read one chunk ahead (the reads precede, in program order, the
                // chain's stores that may alias them; opaque LDS pointers with immediate offsets
                // measured 6 % slower: DESIGN.md Appendix A)
                double* Ev = E;
                const double* Cv = CD;
                double nx[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) nx[u] = Cv[u];
#pragma unroll
                for (int c = 0; c < kTile / 8; ++c) {
                    double cur[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) cur[u] = nx[u];
                    if (c + 1 < kTile / 8) {
#pragma unroll
                        for (int u = 0; u < 8; ++u) nx[u] = Cv[8 * (c + 1) + u];
                    }
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        ema = ema + alpha * (cur[u] - ema);
                        Ev[8 * c + u] = ema;
                    }
                }
            } else {
#pragma unroll 1
                for (int b = 0; b < kTile; ++b) {
                    const double cd = (double)__builtin_amdgcn_readlane(cl, b);
                    if (t1 + b < B) ema = (t1 + b == chain_b0) ? cd : ema + alpha * (cd - ema);
                    E[b] = ema;
                }
            }
            // the values entering the first accounted bar, stored when the chain reaches them (a
            // register kept across the walk for them costs two VGPRs at the split kernel's edge);
            // a fix pass leaves the start record alone (other blockIdx.y blocks of the symbol
            // compare it with the previous segment's end, chain_differs, and may not have yet)
            if (SEG && fix_seg == 0 && T + 1 == T_acct) ema_mine[lane] = ema;
        }
        __builtin_amdgcn_s_setprio(0);
    };

    // with task-only waves present the parameter waves only walk: the walk is the per-tile
    // critical path (config 3: ~3.7k of ~4.9k cycles per tile on the parameter wave)
    const bool walk_only = nextra >= 2;
    // ... and helper B (the chain, which sets the stage with task waves idle) takes none either:
    // its grab after the chain would only find the round empty
    const bool chain_only = walk_only;
    const bool no_tasks = (walk_only && wave < npw) || (chain_only && helperB);
    const int ngrab = nwaves - (walk_only ? npw : 0) - (chain_only ? 1 : 0);

    // condition words of stage st (its TS tiles), tasks grabbed dynamically (round st), lane =
    // bar. Task o pairs span o with OLS window o (either may be absent) over every tile of the
    // stage: all LDS reads of the task are issued together, and the window length comes from a
    // register (winreg, lane = window), so a task costs one dependent LDS round trip after its
    // grab. A stage's tiles past T_end are computed on stale rows and not stored.
    auto flags = [&](int st) {
        if (no_tasks) return;
        const int T0 = T_scan + TS * st;
        const int nt = min(TS, T_end - T0);  // tiles of the stage (wave-uniform)
        double cd[TS], lhs[TS];
        uint64_t* Wd[TS];
        const double* Er[TS];
        int pt[TS];
        uint64_t P1[TS], P2[TS], tin[TS];
#pragma unroll
        for (int u = 0; u < TS; ++u) {
            const int T = T0 + u, t = T * kTile + lane;
            cd[u] = (double)cts[(T % CT) * kTile + lane];
            lhs[u] = cd[u] * 10000.0;
            Wd[u] = words + (T % SL) * nword;
            Er[u] = ebuf + (T % SL) * estage;
            pt[u] = ring_pos(T, lane, R);
            P1[u] = r1[pt[u]];
            P2[u] = r2[pt[u]];
            tin[u] = ballot(t < B);  // bars of the tile inside the series
        }
        const uint32_t base = (uint32_t)st * (uint32_t)(ntask + ngrab);
        uint32_t o = grab_value(grab_issue(ctr, lane)) - base;
        if (DSTT) {  // the round's first TS tasks: the tiles' drawdown tables
#pragma unroll 1
            while (o < (uint32_t)TS) {
                const uint32_t vn = grab_issue(ctr, lane);
                if ((int)o < nt) dbuild(T0 + (int)o);
                o = grab_value(vn) - base;
            }
            o -= TS;
        }
#pragma unroll 1
        while (o < (uint32_t)(ntask - (DSTT ? TS : 0))) {
            const uint32_t vn = grab_issue(ctr, lane);  // next task, read at the end
            const bool hs = (int)o < nsp, ho = (int)o < nol;  // wave-uniform
            const int Wn = nol <= 64 ? __builtin_amdgcn_readlane(winreg, (int)o & 63) : win[o];
            // unconditional reads at clamped / valid addresses (a task without a span or a window
            // leaves them unused): no select on the task's kind, which the compiler builds as a
            // VGPR bool
            const int erow = min((int)o, nsp - 1) * kEStride + lane;
            double e[TS];
            uint64_t r1j[TS], r2j[TS];
#pragma unroll
            for (int u = 0; u < TS; ++u) {
                const int pj = ring_back(pt[u], Wn, R);
                e[u] = Er[u][erow];
                r1j[u] = r1[pj];
                r2j[u] = r2[pj];
            }
            if (hs) {  // span: entry / exit conditions against the EMA
#pragma unroll
                for (int u = 0; u < TS; ++u) {
                    const uint64_t wa = __ballot(lhs[u] < e[u] * lo_mult), wb = __ballot(lhs[u] > e[u] * hi_mult);
                    const uint64_t wx = __ballot(cd[u] >= e[u]), wy = __ballot(cd[u] <= e[u]);
                    if (lane == 0 && u < nt) {
                        Wd[u][4 * o + 0] = wa;
                        Wd[u][4 * o + 1] = wb;
                        Wd[u][4 * o + 2] = wx;
                        Wd[u][4 * o + 3] = wy;
                    }
                }
            }
            if (ho) {  // OLS window: N = 2 T - (w-1) S over [t-w+1, t], exact modulo 2^64
                // 2 (sum i c_i - jj S) - (w - 1) S with one multiply, jj = t + 1 - w; masks
                // straight from the compares (a ballot of `valid && N >= 0` is a VGPR bool
                // compared again)
#pragma unroll
                for (int u = 0; u < TS; ++u) {
                    const int t = (T0 + u) * kTile + lane;
                    const uint64_t S = P1[u] - r1j[u];
                    const int64_t N = (int64_t)(2 * (P2[u] - r2j[u]) - (uint64_t)(int64_t)(2 * (t + 1 - Wn) + Wn - 1) * S);
                    const uint64_t vm = vcmp_le_i32(Wn, t + 1) & tin[u];  // jj >= 0 && t < B
                    const uint64_t wp = vcmp_ge0_i64(N) & vm, wn = vcmp_le0_i64(N) & vm;
                    if (lane == 0 && u < nt) {
                        Wd[u][4 * nsp + 2 * o] = wp;
                        Wd[u][4 * nsp + 2 * o + 1] = wn;
                    }
                }
            }
            o = grab_value(vn) - base - (DSTT ? TS : 0);
        }
    };

    // prologue: scan + chain stages 0 and 1; tables and words of stage 0
    int32_t cpre[TS];  // closes of the helpers' next stage, loaded a stage ahead
    if (helperA || helperB) {
        const int b0 = T_scan * kTile;
        int32_t c0[2 * TS];
#pragma unroll
        for (int u = 0; u < 2 * TS; ++u) c0[u] = ldc(crow, B, b0 + u * kTile + lane, 0);
#pragma unroll
        for (int u = 0; u < TS; ++u) cpre[u] = ldc(crow, B, b0 + (2 * TS + u) * kTile + lane, 0);
#pragma unroll
        for (int u = 0; u < 2 * TS; ++u) {
            if (T_scan + u < T_end) {
                if (helperA) scan(T_scan + u, c0[u]); else chain(T_scan + u, c0[u]);
            }
        }
    }
    __syncthreads();
    if (nstage > 0) flags(0);
    __syncthreads();

    TradeAcct a;
    acct_init(a);
    if (SEG && fix_seg > 0 && active) seg_inject(a, seg_rec(sr.seg - 1));
    const size_t gi = (size_t)blockIdx.x * P + pj;
    bt_trade* tr = (PARITY && active) ? out.trades + gi * out.trade_cap : nullptr;
    const int cap = out.trade_cap;

    StampAcc sa;
    // the walk of tile k (parameter waves)
    auto walk = [&](int k) {
        const int t0 = k * kTile;
        if (SEG && k == T_acct && active) {
            // first accounted tile: the state the (speculative) walk reached goes to the record
            // now; the burn-in's sums are dropped
            seg_write_start(seg_rec(sr.seg), a.pos, a.e);
            seg_reset_sums(a);
        }
        if (active && k >= T_walk && !BT_ABL(g, 8)) {
            set_prio(BT_PRIO(g, 18, kEmaWalkPrio));  // the walk is the per-tile critical path
            const int s = k % CT;
            const int32_t* cT = cts + s * kTile;
            const int64_t* ql = qls + s * 2 * kTile;
            const Agg* D = dst + (k % DS) * kDstLevels * kTile;
            const uint64_t* W = words + (k % SL) * nword;
            const uint64_t vm = bar_range_mask(t0, warm, B - 2);
            const uint64_t Aw = W[4 * i_n] & W[4 * nsp + 2 * i_w] & vm;
            const uint64_t Bw = W[4 * i_n + 1] & W[4 * nsp + 2 * i_w + 1] & vm & ~Aw;
            const uint64_t Xw = W[4 * i_n + 2] & vm, Yw = W[4 * i_n + 3] & vm;
            const int bl = B - 1 - t0;
            const uint64_t fb = bl < kTile ? (1ULL << bl) : 0ULL;  // forced exit (bl >= 0)
            // positions after every bar at once (replaces a per-trade search for the next entry
            // and exit bar): a long latch (set A, reset X or the forced exit) and a short one (set
            // B, reset Y); A and X are disjoint, B and Y too (band >= 0 and e > 0, so a close under
            // the lower band is under the EMA, fp64 rounding being monotone).
            // They are coupled only through "an entry needs a flat position": an entry bit
            // survives if the other side was not held before that bar. Bit b of the coupled masks
            // depends only on bits < b, so iterating to the fixpoint settles one more bar per pass
            // at least (one or two passes in practice).
            {
                const uint64_t RL = Xw | fb, RS = Yw | fb;
                const uint64_t lin = a.pos > 0, sin = a.pos < 0;
                uint64_t Ap = Aw, Bp = Bw, Lw, Sw;
#pragma unroll 1
                for (;;) {
                    Lw = latch64(Ap, RL, lin);
                    Sw = latch64(Bp, RS, sin);
                    const uint64_t An = Aw & ~((Sw << 1) | sin), Bn = Bw & ~((Lw << 1) | lin);
                    if (An == Ap && Bn == Bp) break;
                    Ap = An;
                    Bp = Bn;
                }
                const uint64_t Lb = (Lw << 1) | lin, Sb = (Sw << 1) | sin;
                const uint64_t EL = Lw & ~Lb;
                const uint64_t Ev0 = EL | (Sw & ~Sb), Xv0 = (Lb & ~Lw) | (Sb & ~Sw);
                // the trades of the tile; NARROW: gap and mdd in int32 while the closes' total
                // variation allows (tile_common.h Acct32; fills are at closes), one copy of the
                // loop per width, chosen per tile (wave-uniform)
                auto trades = [&](auto narrow_tag) {
                    constexpr bool NARROW = decltype(narrow_tag)::value;
                    Acct32 n32{(int32_t)a.gap, (int32_t)a.mdd};  // <= TV < 2^30 if NARROW
                    uint64_t Ev = Ev0, Xv = Xv0;
                    if (a.pos != 0 && Xv) {  // the position carried in closes first
                        const int x = __builtin_ctzll(Xv);
                        Xv &= Xv - 1;
                        const int32_t cx = cT[x];
                        const uint64_t qx = (uint64_t)ql[x], q2x = (uint64_t)ql[kTile + x];
                        const bool lg = a.pos > 0;
                        acct_close<PARITY, SEG, NARROW>(a, n32, t0 + x, cx,
                                                        agg_merge(a.agg, dst_query_w(D, a.sb, x)), tr, cap);
                        a.ps1 += lg ? qx : (uint64_t)0 - qx;
                        a.ps2 += q2x;
                        a.pos = 0;
                    }
#pragma unroll 1
                    while (Ev) {
                        if (STAMPS) sa.count(3);
                        // entry and exit bars are both known: every LDS read of the trade is
                        // issued together (an entry left open reads the tile's last bar, unused)
                        const int b = __builtin_ctzll(Ev);
                        Ev &= Ev - 1;
                        const bool hx = Xv != 0;
                        const int x = hx ? __builtin_ctzll(Xv) : kTile - 1;
                        Xv &= Xv - 1;
                        const int32_t cb = cT[b], cx = cT[x];
                        const uint64_t qb = (uint64_t)ql[b], q2b = (uint64_t)ql[kTile + b];
                        const uint64_t qx = (uint64_t)ql[x], q2x = (uint64_t)ql[kTile + x];
                        // whole 16-B entries, kept live: the side's drawdown or draw-up is then
                        // not re-read in a divergent branch (the compiler sank those reads once
                        // the accounting changed shape: config 3 +2 %)
                        const Agg st = dst_query_w(D, b, x);
                        const int np = ((EL >> b) & 1) ? 1 : -1;
                        a.ps1 += np > 0 ? (uint64_t)0 - qb : qb;
                        a.ps2 -= q2b;
                        acct_open(a, t0 + b, b, cb);
                        a.pos = np;
                        if (!hx) break;  // open at the tile end
                        acct_close<PARITY, SEG, NARROW>(a, n32, t0 + x, cx, st, tr, cap);
                        a.ps1 += np > 0 ? qx : (uint64_t)0 - qx;
                        a.ps2 += q2x;
                        a.pos = 0;
                    }
                    if (NARROW) {
                        a.gap = (uint32_t)n32.g;  // >= 0
                        a.mdd = (uint32_t)n32.m;
                    }
                };
                if (!SEG && kEmaNarrow && __builtin_amdgcn_readfirstlane(nars[s]))
                    trades(std::true_type{});
                else
                    trades(std::false_type{});
            }
            if (STAMPS) sa.mark(1);
            acct_tile_end(a, D, ql);
            __builtin_amdgcn_s_setprio(0);
        }
    };

    if (STAMPS) sa.begin();
    for (int st = 0; st < nstage; ++st) {
        const int k0 = T_scan + TS * st;
        if (helperA || helperB) {
#pragma unroll
            for (int u = 0; u < TS; ++u) {
                const int T = k0 + 2 * TS + u;
                if (T < T_end) {
                    if (helperA) scan(T, cpre[u]); else chain(T, cpre[u]);
                }
                cpre[u] = ldc(crow, B, (T + TS) * kTile + lane, 0);
            }
        }
        if (STAMPS) sa.mark(0);
#pragma unroll
        for (int u = 0; u < TS; ++u)
            if (k0 + u < T_end) walk(k0 + u);
        if (st + 1 < nstage && !BT_ABL(g, 2)) flags(st + 1);
        if (STAMPS) sa.mark(2);
        __syncthreads();
        if (STAMPS) sa.barrier();
    }
    if (STAMPS) sa.flush(out.dbg, wave < npw ? 0 : (helperA ? 1 : (helperB ? 2 : 3)), lane);
    if (SEG) {
        if (active) {
            // a segment with no bars never reached its first accounted tile: the state passes
            // through (flat, or the fix pass's injected one)
            if (T_acct >= T_end) seg_write_start(seg_rec(sr.seg), a.pos, a.e);
            seg_write_rest(a, seg_rec(sr.seg));
        }
        if (helperB && lane < nsp) {
            // a speculative segment whose chain never reached its first accounted bar records 0
            if (fix_seg == 0 && !(T_acct >= T_scan + 1 && T_acct <= T_end)) ema_mine[lane] = 0.0;
            ema_mine[64 + lane] = ema;  // after the segment's last bar
        }
        return;
    }
    if (active) acct_write(a, B, g.sqrt_ann, gi, out);
    wave_add_trades(out, active ? a.ntr : 0);
}

// ----------------------------------------------------------------------------- Bollinger
// Workgroup = parameter waves + one helper wave + task-only waves, one barrier per tile:
//   helper, tile k+2: closes/highs/lows -> returns, drawdown sparse table, prefix rings, the raw
//           lows/highs and their 8-bar block / in-block / tile suffix extrema;
//   every wave, tile k+1, after its own work: tasks grabbed from an LDS counter — per window the
//           condition words (z tests in fp64 with an exact int128 fallback), per side the SL/TP
//           first-passage tables of the tile's entry bars;
//   parameter waves, tile k: one trade per loop iteration (entry at the first z signal, exit at
//           the first of SL/TP / signal / forced), O(1) accounting per trade.
constexpr int kMaxK = 8;             // z thresholds tested per unrolled pass of a window task
// SL/TP levels per level task (searched together); 1, 2 or 4 levels per task and level tasks
// queued before the window tasks measured within noise or slower (config 4: 7.91-8.06 ms)
constexpr int kLevPassLog = 1, kLevPass = 1 << kLevPassLog;
// Parameter waves take tasks after their walk too: with the level tables the tasks, not the walk,
// set the tile time (config 4 at 500 symbols: task waves ~11.6k busy cycles per tile, parameter
// waves ~6.1k busy and ~6.5k at the barrier; 8.51 -> 7.96 ms)
constexpr bool kWalkOnly = false;

// 8-bit mask of v_j > X over a (4+4)-int32 group, bit j = element j: the sign bit of X - v_j
// (no overflow: prices, padding and levels all lie in [0, 2^31)) shifted in by v_alignbit,
// two VALU per element.
__device__ __forceinline__ uint32_t gt8(const int4& a, const int4& b, int32_t X) {
    uint32_t m = 0;
    m = __builtin_amdgcn_alignbit(m, (uint32_t)(X - b.w), 31);
    m = __builtin_amdgcn_alignbit(m, (uint32_t)(X - b.z), 31);
    m = __builtin_amdgcn_alignbit(m, (uint32_t)(X - b.y), 31);
    m = __builtin_amdgcn_alignbit(m, (uint32_t)(X - b.x), 31);
    m = __builtin_amdgcn_alignbit(m, (uint32_t)(X - a.w), 31);
    m = __builtin_amdgcn_alignbit(m, (uint32_t)(X - a.z), 31);
    m = __builtin_amdgcn_alignbit(m, (uint32_t)(X - a.y), 31);
    m = __builtin_amdgcn_alignbit(m, (uint32_t)(X - a.x), 31);
    return m;
}

__device__ __forceinline__ int4 ld4(const int32_t* p) { return *reinterpret_cast<const int4*>(p); }

// Keep loaded values live here: the loads above are issued together and not sunk into the
// divergent branches that consume them.
__device__ __forceinline__ void pin4(const int4& v) {
    asm volatile("" ::"v"(v.x), "v"(v.y), "v"(v.z), "v"(v.w));
}

// SL/TP first passage from in-tile bar cur (< 64) of an open trade: xlo = first bar whose low
// is <= XL, xhi = first bar whose high is > XH1 (64 if none). LH: one stage of the staging
// (kLH layout). Two dependent LDS round trips for both searches together: round 1 reads the
// suffix extrema of `cur` within its 8-bar block and the 8 block extrema (one hit test for the
// rest of the block, 8 for the later blocks), round 2 the 8 bars of the block that holds the
// first hit (`cur`'s own block from `cur` on, or the first later block that qualifies).
__device__ __forceinline__ void sltp_search(const int32_t* LH, int cur, int32_t XL, int32_t XH1,
                                            int& xlo, int& xhi) {
    const int cb = cur >> 3;
    const int32_t sl = LH[kLhSuf + cur], sh = LH[kLhSuf + kTile + cur];
    const int32_t tl = LH[kLhTs + cur], th = LH[kLhTs + kTile + cur];
    const int4 n0 = ld4(LH + kLhBx), n1 = ld4(LH + kLhBx + 4);
    const int4 x0 = ld4(LH + kLhBx + 8), x1 = ld4(LH + kLhBx + 12);
    asm volatile("" ::"v"(sl), "v"(sh), "v"(tl), "v"(th));
    pin4(n0); pin4(n1); pin4(x0); pin4(x1);
    xlo = xhi = kTile;
    // the tile-suffix extrema tell at once whether a level is touched in [cur, 63]: a wave
    // whose lanes all miss (mostly its last iteration of the tile, carrying open trades past
    // its end) skips the block tests and round 2
    if (!__ballot(tl <= XL || th > XH1)) return;
    const uint32_t after = (0xFEu << cb) & 0xFFu;
    const bool inL = sl <= XL, inH = sh > XH1;
    const uint32_t laL = ~gt8(n0, n1, XL) & after, laH = gt8(x0, x1, XH1) & after;
    // block to scan per side (cb when the hit is in cur's block; unused when there is none)
    const int fL = inL ? cb : (laL ? __builtin_ctz(laL) : cb);
    const int fH = inH ? cb : (laH ? __builtin_ctz(laH) : cb);
    const int4 a0 = ld4(LH + 8 * fL), a1 = ld4(LH + 8 * fL + 4);
    const int4 b0 = ld4(LH + kTile + 8 * fH), b1 = ld4(LH + kTile + 8 * fH + 4);
    pin4(a0); pin4(a1); pin4(b0); pin4(b1);
    const uint32_t from = (0xFFu << (cur & 7)) & 0xFFu;
    const uint32_t mL = (~gt8(a0, a1, XL) & (fL == cb ? from : 0xFFu)) | 0x100u;
    const uint32_t mH = (gt8(b0, b1, XH1) & (fH == cb ? from : 0xFFu)) | 0x100u;
    xlo = (inL || laL) ? 8 * fL + __builtin_ctz(mL) : kTile;
    xhi = (inH || laH) ? 8 * fH + __builtin_ctz(mH) : kTile;
}

// First bar in [cur, 63] whose low is <= XL (first_low) or whose high is > XH1 (first_high), 64
// if none; one lane's search (the level tasks run it with lane = entry bar): the tile suffix
// decides whether there is a hit at all, then the in-block suffix and the block extrema find its
// block, then that block's 8 bars.
__device__ __forceinline__ int first_low(const int32_t* LH, int cur, int32_t XL) {
    if (cur >= kTile || LH[kLhTs + cur] > XL) return kTile;
    const int cb = cur >> 3;
    const uint32_t la = ~gt8(ld4(LH + kLhBx), ld4(LH + kLhBx + 4), XL) & ((0xFEu << cb) & 0xFFu);
    const int f = LH[kLhSuf + cur] <= XL ? cb : __builtin_ctz(la | 0x100u);
    const uint32_t m = ~gt8(ld4(LH + 8 * f), ld4(LH + 8 * f + 4), XL) & (f == cb ? (0xFFu << (cur & 7)) & 0xFFu : 0xFFu);
    return 8 * f + __builtin_ctz(m | 0x100u);
}
__device__ __forceinline__ int first_high(const int32_t* LH, int cur, int32_t XH1) {
    if (cur >= kTile || LH[kLhTs + kTile + cur] <= XH1) return kTile;
    const int cb = cur >> 3;
    const uint32_t la = gt8(ld4(LH + kLhBx + 8), ld4(LH + kLhBx + 12), XH1) & ((0xFEu << cb) & 0xFFu);
    const int f = LH[kLhSuf + kTile + cur] > XH1 ? cb : __builtin_ctz(la | 0x100u);
    const uint32_t m = gt8(ld4(LH + kTile + 8 * f), ld4(LH + kTile + 8 * f + 4), XH1) & (f == cb ? (0xFFu << (cur & 7)) & 0xFFu : 0xFFu);
    return 8 * f + __builtin_ctz(m | 0x100u);
}

// SL/TP levels floor(ce * f / 10000) for 0 < ce < 2^31, 0 < f < 2^15 (spec §4), with the
// per-lane factor g = fl(f * fl(1e-4)) precomputed: y = fl(ce * g) is within 3 * 2^-53 relative
// (< 2^-18.7 absolute, y < 2^32.7) of ce * f / 10000 = n + r / 10000 (0 <= r <= 9999), so the
// 2^-16 offset keeps y + 2^-16 inside (n, n + 1) and truncation is the exact floor
// (tests/test_oracle_golden.py::test_sltp_level_floor checks every f against integer division).
__device__ __forceinline__ double level_y(double ce, double g) { return ce * g + 0x1p-16; }

// SEG: one bar segment per block (blockIdx.z = segment; or, with fix_seg >= 1, the fix pass of
// boundary fix_seg: the block re-walks that segment from the previous segment's end states if
// any lane's speculative start differs, and otherwise returns at once). Results go to SegRec
// records (internal.h) that seg_combine folds.
template <bool PARITY, bool STAMPS, bool SEG>
__global__ __launch_bounds__(1024) void boll_tile_kernel(const SymDesc* __restrict__ syms,
                                                         const int32_t* __restrict__ high,
                                                         const int32_t* __restrict__ low,
                                                         const int32_t* __restrict__ close,
                                                         Grid g, Out out, int nextra, int lpw,
                                                         SegArgs sg, int fix_seg, int split_grp,
                                                         uint32_t wave_map) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int nw = g.na, nk = g.nb, R = g.ring;
    const int nsl = g.nc, ntp = g.nd, nlev = nsl + ntp;
    // a split walk: parameter group split_grp (>= 0) finds its trades, an accountant wave keeps
    // their accounts
    const bool split = split_grp >= 0;
    const TileLds LL = tile_lds_layout(1, R, nw, nk, nlev);
    // prefix rings as exact doubles (every prefix < 2^53 for series up to kMaxBars = 2^22 bars):
    // sum c, and sum c^2 split at bit 31 into sum (c^2 >> 31) and sum (c^2 & (2^31 - 1)), so
    // a window's S1 and the two halves of S2 are exact double differences and S2 = hi 2^31 + lo
    // rounds once, with no int64 / int128 arithmetic or conversion per window task
    double* r1 = reinterpret_cast<double*>(smem + LL.r1);     // sum c
    double2* r2 = reinterpret_cast<double2*>(smem + LL.r2);   // {sum c^2 >> 31, sum c^2 & 2^31-1}
    int32_t* cts = reinterpret_cast<int32_t*>(smem + LL.ct);
    int64_t* qls = reinterpret_cast<int64_t*>(smem + LL.ql);
    Agg* dst = reinterpret_cast<Agg*>(smem + LL.dst);
    int32_t* lhs_ = reinterpret_cast<int32_t*>(smem + LL.stl);
    uint64_t* words = reinterpret_cast<uint64_t*>(smem + LL.words);
    int32_t* win = reinterpret_cast<int32_t*>(smem + LL.win);
    double* kn2d = reinterpret_cast<double*>(smem + LL.ebuf);
    // SL/TP first passage precomputed per entry bar (level tasks in flags): for every bar b of a
    // tile and every level the grid uses, the first bar in (b, 63] whose low touches the level
    // (low side: 1e4 - sl for longs' SL, 1e4 - tp for shorts' TP) or whose high does (high side:
    // 1e4 + tp, 1e4 + sl), 64 if none; the walk of a trade entered in the tile reads it
    uint8_t* levt = reinterpret_cast<uint8_t*>(smem + LL.lev);
    // ... and the level of each (side, level, entry bar): low side floor(c_b (1e4 - bps) / 1e4)
    // (lows <= it touch), high side that level minus one (highs > it touch; INT32_MAX when the
    // level reaches 2^31): a trade entered in the tile reads both with its entry close
    int32_t* levp = reinterpret_cast<int32_t*>(smem + LL.levp);
    double* levf = reinterpret_cast<double*>(smem + LL.levf);
    int32_t* lvb = reinterpret_cast<int32_t*>(smem + LL.lvb);
    // split walk: the finder records its lanes' trades per tile, the accountant folds them a
    // tile later
    uint16_t* recs = reinterpret_cast<uint16_t*>(smem + LL.rec);
    uint8_t* nrec = reinterpret_cast<uint8_t*>(smem + LL.nrec);
    int32_t* nars = reinterpret_cast<int32_t*>(smem + LL.nar);
    uint32_t* ctr = reinterpret_cast<uint32_t*>(smem + LL.ctr);

    // wave_map: role of hardware wave w < 8 (4 bits each; the roles below are logical wave
    // indices), so the heavy roles land on different SIMDs next to light ones
    const int tid = threadIdx.x, lane = tid & 63, hw_wave = tid >> 6;
    const int wave = hw_wave < 8 ? (int)((wave_map >> (4 * hw_wave)) & 15u) : hw_wave;
    if (STAMPS) stamp_place(out.dbg, hw_wave, lane);
    // waves: [0, npw) parameter groups, npw the helper, npw + 1 the accountant of a split walk,
    // then `nextra` task-only waves. Without a split every parameter wave walks and accounts its
    // lanes' trades (walker); with one, parameter wave split_grp (the group of the busiest z
    // threshold, whose per-lane trade chain sets the tile time) only finds its trades (finder)
    // and the accountant wave keeps their accounts, one tile behind.
    const int nwaves = (int)(blockDim.x >> 6), npw = nwaves - 1 - nextra - (split ? 1 : 0);
    const bool helper = wave == npw;
    const bool accountant = split && wave == npw + 1;
    const bool finder = split && wave == split_grp;
    const int grp = accountant ? split_grp : wave;
    const SymDesc sd = syms[blockIdx.x];
    const int B = sd.bars, ntiles = (B + kTile - 1) / kTile, P = g.n_params;
    const int j = (blockIdx.y * npw + grp) * lpw + lane;
    const bool active = (wave < npw || accountant) && lane < lpw && j < P;
    const bool keeps = active && !finder;       // keeps accounts (walker or accountant)
    const bool walks = active && !accountant;   // walks the condition words (walker or finder)
    // lanes run k-major (lane j -> (ik, iw, isl, itp)) while results keep the param order
    // ((iw * nk + ik) * nsl + isl) * ntp + itp: a wave then holds one z threshold, and the
    // threshold sets most of a lane's trade rate, so the walk (a wave iterates the maximum
    // over its lanes' trades per tile) wastes fewer lanes: 20.2 -> 17.8 iterations per
    // block-tile on config 4 (oracle trade lists of 3 symbols)
    const int jl = active ? j : 0;
    const int itp = jl % g.nd, isl = (jl / g.nd) % g.nc, iw = (jl / (g.nd * g.nc)) % nw,
              ik = jl / (g.nd * g.nc * nw);
    const int pj = ((iw * nk + ik) * g.nc + isl) * g.nd + itp;
    // an opaque copy for the result write after the walk (not recomputed there from the index's
    // parts, which would keep two sign-extended pairs live across the walk)
    int pj_out = pj;
    asm volatile("" : "+v"(pj_out));
    const int w = g.a[iw];
    const int32_t sl_bps = g.c[isl], tp_bps = g.d[itp];
    const int32_t* crow = close + sd.off;
    const int32_t* hrow = high + sd.off;
    const int32_t* lrow = low + sd.off;
    // condition words of a tile: per (window, k) the |z| > k word, then per window the D >= 0
    // and D <= 0 words (the walk forms [z < -k] = |z| > k and not D >= 0, [z > k] likewise)
    const int nword = nw * nk + 2 * nw;
    const int winreg = lane < nw ? g.a[lane] : 1;  // window lengths, lane = window (no LDS trip)
    const int64_t kd2 = (int64_t)g.k_den * g.k_den;
    const double kd2d = (double)kd2;

    // tiles of this block: scanned from T_scan (every window of the first walked bar complete),
    // walked from T_walk, accounted from T_acct, up to T_end (exclusive)
    SegRange sr{0, 0, 0, 0, ntiles};
    const SegRec* prev = nullptr;
    SegRec* mine = nullptr;
    if (SEG) {
        sr = seg_range(sg, fix_seg, ntiles, g.wmax);
        const size_t per_seg = (size_t)gridDim.x * P;
        mine = sg.rec + sr.seg * per_seg + (size_t)blockIdx.x * P + pj;
        if (sr.seg > 0) prev = mine - per_seg;
        if (fix_seg > 0) {  // re-walk only if some lane's speculative start is not the true one
            if (!__syncthreads_or(keeps && seg_start_differs(mine, prev))) return;
            if (tid == 0) atomicAdd(sg.refixed, 1ULL);
        }
    }
    const int T_scan = sr.T_scan, T_walk = sr.T_walk, T_acct = sr.T_acct, T_end = sr.T_end;

    for (int o = tid; o < nw; o += blockDim.x) win[o] = g.a[o];
    for (int o = tid; o < nk; o += blockDim.x) kn2d[o] = (double)((int64_t)g.b[o] * g.b[o]);
    // tasks per tile: one per window (condition words), then per side one per kLevPass levels
    // (first-passage tables)
    auto task_count = [&](int nu) { return nw + 2 * ((nu + kLevPass - 1) / kLevPass); };
    if (tid == 0) {
        // prefix entry x (sum over scanned bars < x) sits at x mod R: the scan's base is 0
        r1[(T_scan * kTile) % R] = 0.0;
        r2[(T_scan * kTile) % R] = double2{0.0, 0.0};
        // the distinct SL/TP distances (a level 1e4 -+ bps is shared by every SL and TP of that
        // bps: config 4's {50, 100} and {50, 100, 200, 400} make 4 levels per side, not 6) and
        // their factors (level_y)
        int nu = 0;
        for (int o = 0; o < nlev; ++o) {
            const int32_t v = o < nsl ? g.c[o] : g.d[o - nsl];
            bool seen = false;
            for (int u = 0; u < nu; ++u) seen |= lvb[u] == v;
            if (!seen) {
                levf[nu] = (double)(10000 - v) * 1e-4;
                levf[nlev + nu] = (double)(10000 + v) * 1e-4;
                lvb[nu++] = v;
            }
        }
        lvb[nlev] = nu;
        // task rounds are numbered by tile (flags): the counter starts at round T_scan
        const int ngrab0 = nwaves - (kWalkOnly && nextra >= 2 ? npw : 0);
        *ctr = (uint32_t)T_scan * (uint32_t)(task_count(nu) + ngrab0);
    }
    __syncthreads();
    const int nu = lvb[nlev], ntask = task_count(nu);
    // this lane's rows of the first-passage tables: long SL / short TP below (1e4 - bps), long
    // TP / short SL above (1e4 + bps)
    int usl = 0, utp = 0;
    for (int u = 0; u < nu; ++u) {
        usl = lvb[u] == sl_bps ? u : usl;
        utp = lvb[u] == tp_bps ? u : utp;
    }
    const int lev_lo_long = usl, lev_lo_short = utp, lev_hi_long = utp, lev_hi_short = usl;

    TileCarry cy{0, (T_scan > 0 && T_scan * kTile - 1 < B) ? crow[T_scan * kTile - 1] : 0};
    int64_t cy2h = 0, cy2l = 0;  // sums of c^2 >> 31 and c^2 & (2^31 - 1) before the tile
    int32_t cpre = 0, hpre = 0, lpre = 0;

    auto scan = [&](int T, int32_t c, int32_t hv, int32_t lv) {
        const int s = T % kBollStages, t0 = T * kTile;
        const int64_t pre = tile_scan<true>(c, B, t0, lane, cts + s * kTile, qls + s * 2 * kTile,
                                            dst + s * kDstLevels * kTile, cy, true,
                                            (SEG && fix_seg > 0) ? nullptr : nars + s, hv, lv);
        const int pt = ring_pos(T, lane, R);
        r1[pt] = (double)pre;  // exact: < 2^31 x 2^22 bars
        // sum of c^2 (< 2^62) as its parts above and below bit 31, each prefix < 2^53
        const uint64_t c2 = (uint64_t)((int64_t)c * c);
        const int64_t slo = wave_iscan_i64((int64_t)(c2 & 0x7FFFFFFFu));
        const int64_t shi = wave_iscan_i64((int64_t)(c2 >> 31));
        r2[pt] = double2{(double)(cy2h + shi), (double)(cy2l + slo)};
        cy2h += lane63_i64(shi);
        cy2l += lane63_i64(slo);
        // raw lows / highs and their 8-bar block extrema
        int32_t* LH = lhs_ + s * kLH;
        LH[lane] = lv;
        LH[kTile + lane] = hv;
        // 8-bar block extrema: xor 1, xor 2 inside quads, then the other quad of the 8
        int32_t mn = lv, mx = hv;
        mn = min(mn, dpp<0xB1>(0, mn));
        mx = max(mx, dpp<0xB1>(0, mx));
        mn = min(mn, dpp<0x4E>(0, mn));
        mx = max(mx, dpp<0x4E>(0, mx));
        mn = min(mn, dpp<0x141>(0, mn));
        mx = max(mx, dpp<0x141>(0, mx));
        if ((lane & 7) == 0) {
            LH[kLhBx + (lane >> 3)] = mn;
            LH[kLhBx + 8 + (lane >> 3)] = mx;
        }
        // min low / max high from each bar to the end of its 8-bar block (suffix within the
        // block: row_shl, masked at the block end) ...
        int32_t smn = lv, smx = hv;
        auto blk = [&](auto dtag) {
            constexpr int d = decltype(dtag)::value;
            const int32_t on = dpp<0x100 + d>(INT32_MAX, smn), ox = dpp<0x100 + d>(INT32_MIN, smx);
            const bool in = (lane & 7) + d < 8;
            smn = in ? min(smn, on) : smn;
            smx = in ? max(smx, ox) : smx;
        };
        blk(std::integral_constant<int, 1>{});
        blk(std::integral_constant<int, 2>{});
        blk(std::integral_constant<int, 4>{});
        LH[kLhSuf + lane] = smn;
        LH[kLhSuf + kTile + lane] = smx;
        // ... and to the end of the tile (one test tells whether a level is touched at all): in
        // each 16-lane row by row_shl, then the later rows' totals (their lane 0) by readlane
        int32_t tmn = lv, tmx = hv;
        auto row = [&](auto dtag) {
            constexpr int d = decltype(dtag)::value;
            tmn = min(tmn, dpp<0x100 + d>(INT32_MAX, tmn));
            tmx = max(tmx, dpp<0x100 + d>(INT32_MIN, tmx));
        };
        row(std::integral_constant<int, 1>{});
        row(std::integral_constant<int, 2>{});
        row(std::integral_constant<int, 4>{});
        row(std::integral_constant<int, 8>{});
        {
            const int32_t n3 = (int32_t)__builtin_amdgcn_readlane((uint32_t)tmn, 48);
            const int32_t n2 = min((int32_t)__builtin_amdgcn_readlane((uint32_t)tmn, 32), n3);
            const int32_t n1 = min((int32_t)__builtin_amdgcn_readlane((uint32_t)tmn, 16), n2);
            const int32_t x3 = (int32_t)__builtin_amdgcn_readlane((uint32_t)tmx, 48);
            const int32_t x2 = max((int32_t)__builtin_amdgcn_readlane((uint32_t)tmx, 32), x3);
            const int32_t x1 = max((int32_t)__builtin_amdgcn_readlane((uint32_t)tmx, 16), x2);
            const int r = lane >> 4;
            tmn = min(tmn, r == 0 ? n1 : r == 1 ? n2 : r == 2 ? n3 : INT32_MAX);
            tmx = max(tmx, r == 0 ? x1 : r == 1 ? x2 : r == 2 ? x3 : INT32_MIN);
        }
        LH[kLhTs + lane] = tmn;
        LH[kLhTs + kTile + lane] = tmx;
    };

    StampAcc sa;
    // with two or more task-only waves the parameter waves only walk (at raised priority)
    const bool walk_only = kWalkOnly && nextra >= 2;
    const bool no_tasks = walk_only && wave < npw;
    const int ngrab = nwaves - (walk_only ? npw : 0);

    // condition words of tile T, windows grabbed dynamically (round T), lane = bar
    auto flags = [&](int T) {
        if (no_tasks) return;
        const int s = T % kBollStages, t = T * kTile + lane;
        const int64_t c = cts[s * kTile + lane];
        uint64_t* Wd = words + (T & 1) * nword;
        const int ptop = ring_pos(T, lane, R);
        const double P1t = r1[ptop];
        const double2 P2t = r2[ptop];
        const double cdw = (double)c;
        const uint64_t tin = ballot(t < B);  // bars of the tile inside the series
        const uint32_t base = (uint32_t)T * (uint32_t)(ntask + ngrab);
        uint32_t o = grab_value(grab_issue(ctr, lane)) - base;
        // window tasks (counter values [0, nw)) first, then level tasks: a wave's grabs only
        // grow, so two loops, each body one kind of task
#pragma unroll 1
        while (o < (uint32_t)nw) {
            const uint32_t vn = grab_issue(ctr, lane);  // next task, read at the end
            const int ow = (int)o;
            const uint64_t tt0 = STAMPS ? __builtin_amdgcn_s_memtime() : 0;
            const int Wn = nw <= 64 ? __builtin_amdgcn_readlane(winreg, ow & 63) : win[ow];
            const int jj = t + 1 - Wn;
            const bool valid = jj >= 0 && t < B;
            const int pj = ring_back(ptop, Wn, R);
            // window sums: S1 = sum c < 2^47 (prices < 2^31, windows <= 2^16) and the two parts
            // of S2 = sum c^2: exact differences of the exact prefix doubles; D = W c - S1 is
            // exact too (W c < 2^47)
            const double2 q2 = r2[pj];
            const double S1d = P1t - r1[pj];
            const double dH = P2t.x - q2.x, dL = P2t.y - q2.y;
            const double wlen = (double)Wn;
            const double Dd = wlen * cdw - S1d;
            // Q = W S2 - S1^2 in fp64 with a proven bracket: S1 is exact, S2 = dH 2^31 + dL
            // (< 2^79) rounds once, the product, the square and the difference once each, and
            // S1^2 <= W S2, so |Qd - Q| < 2^-50 pd (pd = W S2 rounded). Qd -/+ 2^-48 pd then
            // brackets Q with room for the roundings of the bracket and of the k^2 products below.
            const double S2d = dH * 0x1p31 + dL;
            const double pd = wlen * S2d;
            const double Qd = pd - S1d * S1d;
            // with lh's own margin folded in (lh is within 2^-51 of L; 2^-47 covers both)
            const double QH = (Qd + pd * 0x1p-48) * (1.0 + 0x1p-47);
            const double QL = (Qd - pd * 0x1p-48) * (1.0 - 0x1p-47);
            // fp64 fast path: |z| > k <=> L = D^2 kd^2 > R = kn^2 Q. D is exact and lh is within
            // 2^-51 of L; after rounding lh > kn^2 QH proves L > R and kn^2 QL > lh proves L < R.
            // A valid lane with neither (both sides zero included, or a window so flat that Q is
            // inside the bracket) is settled exactly in int128 with its whole wave.
            const double lh = (Dd * Dd) * kd2d;
            const uint64_t vm = vcmp_le_i32(Wn, t + 1) & tin;  // ballot(valid)
            const uint64_t dp = vcmp_ge0_f64(Dd) & vm, dn = vcmp_le0_f64(Dd) & vm;
            // z tests of one k: lanes 2 qq, 2 qq + 1 of `zw` collect its |z| > k word (v_writelane,
            // lane = dword of Wd[ow nk + q]; the walk splits it by the sign of D), one store per
            // pass of kMaxK values; a
            // lane the fp64 bracket cannot settle marks the k in `unc` (wave-uniform), and the
            // pass then settles those k exactly in int128, once, outside the unrolled tests
            auto ztest = [&](auto qtag, double kn2, uint32_t& zw, uint32_t& unc) {
                constexpr int qq = decltype(qtag)::value;
                const uint64_t big = vcmp_gt_f64(lh, kn2 * QH) & vm;
                const uint64_t small = vcmp_gt_f64(kn2 * QL, lh);
                unc |= any_bit<1u << qq>(vm & ~big & ~small);
                writelane<2 * qq>(zw, (uint32_t)big);
                writelane<2 * qq + 1>(zw, (uint32_t)(big >> 32));
            };
            auto settle = [&](int q0, uint32_t unc, uint32_t& zw) {  // rare
                // the exact integers behind the doubles, re-read from the rings (nothing stays live
                // across the tests for this rare path); lanes outside the window are masked by
                // `valid`, their values are never used
                const double2 r2x = r2[pj];
                const double S1e = P1t - r1[pj];
                const uint64_t S1x = valid ? (uint64_t)S1e : 0;
                const int64_t Dv = valid ? (int64_t)((double)Wn * cdw - S1e) : 0;
                const unsigned __int128 S2x =
                    valid ? ((unsigned __int128)(uint64_t)(P2t.x - r2x.x) << 31) + (uint64_t)(P2t.y - r2x.y) : 0;
                const unsigned __int128 Q = mul_u128_u32(S2x, (uint32_t)Wn) - sq_u64(S1x);
#pragma unroll 1
                while (unc) {
                    const int qq = __builtin_amdgcn_readfirstlane(__builtin_ctz(unc));
                    unc &= unc - 1;
                    const int64_t kn = g.b[q0 + qq];
                    const uint64_t big = sgpr64(ballot(valid && (i128)Dv * (i128)Dv * (i128)kd2 > (i128)(kn * kn) * (i128)Q));
                    const int d = lane - 2 * qq;  // lane 2 qq + d holds dword d of big
                    if (d >= 0 && d < 2) zw = (uint32_t)(big >> (32 * d));
                }
            };
            {  // first pass: k_num^2 from the kernel arguments
                uint32_t zw = 0, unc = 0;
                static_for<kMaxK>([&](auto qtag) {
                    constexpr int qq = decltype(qtag)::value;
                    if (qq < nk) ztest(qtag, g.kn2[qq], zw, unc);
                });
                if (unc) settle(0, unc, zw);
                if (lane < 2 * min(nk, kMaxK)) reinterpret_cast<uint32_t*>(Wd + ow * nk)[lane] = zw;
            }
#pragma unroll 1
            for (int q0 = kMaxK; q0 < nk; q0 += kMaxK) {  // grids of more than 8 k values
                uint32_t zw = 0, unc = 0;
                static_for<kMaxK>([&](auto qtag) {
                    constexpr int qq = decltype(qtag)::value;
                    if (q0 + qq < nk) ztest(qtag, kn2d[q0 + qq], zw, unc);
                });
                if (unc) settle(q0, unc, zw);
                if (lane < 2 * min(nk - q0, kMaxK)) reinterpret_cast<uint32_t*>(Wd + ow * nk + q0)[lane] = zw;
            }
            if (lane == 0) {
                Wd[nw * nk + 2 * ow] = dp;
                Wd[nw * nk + 2 * ow + 1] = dn;
            }
            if (STAMPS) sa.task[0] += __builtin_amdgcn_s_memtime() - tt0;
            o = grab_value(vn) - base;
        }
#pragma unroll 1
        while (o < (uint32_t)ntask) {  // level task: lane = entry bar b, first passage from b + 1
            const uint32_t vn = grab_issue(ctr, lane);
            const int ol = (int)o - nw;
            const uint64_t tt0 = STAMPS ? __builtin_amdgcn_s_memtime() : 0;
            const int side = ol & 1, i = ol >> 1 << kLevPassLog;
            const int32_t* LH = lhs_ + s * kLH;
            const double cd = (double)c;
            uint8_t* tab = levt + ((T & 1) * 2 + side) * nlev * kTile;
            int32_t* ptab = levp + ((T % 3) * 2 + side) * nlev * kTile;
            // kLevPass levels: independent searches, all stored after all
            {
                int x[kLevPass];
                int32_t X[kLevPass];
#pragma unroll
                for (int u = 0; u < kLevPass; ++u) {
                    const double y = level_y(cd, levf[side * nlev + min(i + u, nu - 1)]);
                    X[u] = side == 0 ? (int32_t)y : (y >= 2147483648.0 ? INT32_MAX : (int32_t)y - 1);
                    x[u] = side == 0 ? first_low(LH, lane + 1, X[u]) : first_high(LH, lane + 1, X[u]);
                }
#pragma unroll
                for (int u = 0; u < kLevPass; ++u) {
                    tab[min(i + u, nu - 1) * kTile + lane] = (uint8_t)x[u];
                    ptab[min(i + u, nu - 1) * kTile + lane] = X[u];
                }
            }
            if (STAMPS) sa.task[1] += __builtin_amdgcn_s_memtime() - tt0;
            o = grab_value(vn) - base;
        }
    };

    if (helper) {
        const int b0 = T_scan * kTile;
        const int32_t c0 = ldc(crow, B, b0 + lane, 0), c1 = ldc(crow, B, b0 + kTile + lane, 0);
        const int32_t h0 = ldc(hrow, B, b0 + lane, 0), h1 = ldc(hrow, B, b0 + kTile + lane, 0);
        const int32_t l0 = ldc(lrow, B, b0 + lane, INT32_MAX), l1 = ldc(lrow, B, b0 + kTile + lane, INT32_MAX);
        cpre = ldc(crow, B, b0 + 2 * kTile + lane, 0);
        hpre = ldc(hrow, B, b0 + 2 * kTile + lane, 0);
        lpre = ldc(lrow, B, b0 + 2 * kTile + lane, INT32_MAX);
        if (T_scan < T_end) scan(T_scan, c0, h0, l0);
        __syncthreads();
        if (T_scan + 1 < T_end) scan(T_scan + 1, c1, h1, l1);
    } else {
        __syncthreads();
    }
    if (T_scan < T_end) flags(T_scan);
    __syncthreads();

    TradeAcct a;
    acct_init(a);
    // open trade: lows <= XL hit the low-side level, highs > XHm1 the high-side level (the
    // walker's and finder's copy; the accountant keeps its own for the fill prices)
    int32_t XL = 0, XHm1 = 0;
    int fpos = 0;  // finder: position carried between tiles (its only state besides the levels)
    // low-side level: long SL / short TP (< ce); high-side: long TP / short SL (may reach 2^31:
    // no high can exceed it then)
    auto set_levels = [&](int32_t cx, int np) {
        const double cd = (double)cx;
        // level factors (10000 -+ bps) * 1e-4 of the trade's sides (level_y)
        const double yl = level_y(cd, levf[np > 0 ? usl : utp]);
        const double yh = level_y(cd, levf[nlev + (np > 0 ? utp : usl)]);
        XL = (int32_t)yl;
        XHm1 = yh >= 2147483648.0 ? INT32_MAX : (int32_t)yh - 1;
    };
    // SEG: this lane's record; the state at the first accounted bar goes there when the walk
    // reaches it (seg_write_start), the rest at the end. The address is recomputed at both
    // points from an opaque copy of the parameter index (kept live, a pointer costs a VGPR pair)
    auto seg_rec = [&]() {
        int pje = pj;
        asm volatile("" : "+v"(pje));
        return sg.rec + (size_t)sr.seg * gridDim.x * P + (size_t)blockIdx.x * P + pje;
    };
    if (SEG && fix_seg > 0 && active) {  // the true state entering the segment
        seg_inject(a, prev);
        if (a.pos != 0) set_levels(a.ce, a.pos);
        fpos = a.pos;
    }
    const size_t gi = (size_t)blockIdx.x * P + pj;
    bt_trade* tr = (PARITY && keeps) ? out.trades + gi * out.trade_cap : nullptr;
    const int cap = out.trade_cap;

    // Close the open trade at in-tile bar x (exit kind: SL/TP fill at px, else the close at x),
    // given D / ql of its tile and the trade's sparse-table query index qi (the bar before a
    // fill, the exit bar of a signal exit): the path is the carried aggregate (kAggId for a
    // trade opened in this tile), the tile's closes [a.sb, qi] and the fill price.
    // FIRST: the tile's first record, the only one that can close a position carried in (path
    // a.agg, and qi < a.sb for a fill at the tile's first bar); every later record closes the
    // trade it opened (a.agg = kAggId, qi >= a.sb), whose path is the tile's closes alone.
    auto close_trade = [&](auto narrow_tag, auto first_tag, Acct32& n32, int t0, int x, int qi,
                           int32_t px, const Agg& seg, int64_t qx, int64_t q2x) {
        constexpr bool NARROW = decltype(narrow_tag)::value;
        constexpr bool FIRST = decltype(first_tag)::value;
        const bool lg = a.pos > 0;
        const Agg sp = (FIRST && qi < a.sb) ? kAggId : seg;
        const Agg st = agg_merge(FIRST ? agg_merge(a.agg, sp) : sp, agg_one(px));
        acct_close<PARITY, SEG, NARROW>(a, n32, t0 + x, px, st, tr, cap);
        a.ps1 += lg ? (uint64_t)qx : (uint64_t)0 - (uint64_t)qx;
        a.ps2 += (uint64_t)q2x;
        a.pos = 0;
    };

    if (STAMPS) sa.begin();
    // a split walk's accountant folds tile k - 1 in step k: one step more
    for (int k = T_scan; k < T_end + (split ? 1 : 0); ++k) {
        const int t0 = k * kTile;
        if (helper && k + 2 < T_end) {
            scan(k + 2, cpre, hpre, lpre);
            const int tn = t0 + 3 * kTile + lane;
            cpre = ldc(crow, B, tn, 0);
            hpre = ldc(hrow, B, tn, 0);
            lpre = ldc(lrow, B, tn, INT32_MAX);
        }
        if (STAMPS) sa.mark(0);
        // the tile whose accounts this lane advances in this step
        const int ka = accountant ? k - 1 : k;
        if (SEG && ka == T_acct && keeps) {
            // first accounted tile: keep the state the (speculative) walk reached, drop the
            // burn-in's sums (a trade open here is closed and accounted in this segment)
            seg_write_start(seg_rec(), a.pos, a.e);
            seg_reset_sums(a);
        }
        if (walks && k >= T_walk && k < T_end && !BT_ABL(g, 8)) {
            set_prio(BT_PRIO(g, 16, kBollWalkPrio));  // the walk is the per-tile critical path
            const int s = k % kBollStages;
            const int32_t* cT = cts + s * kTile;
            const int64_t* ql = qls + s * 2 * kTile;
            const Agg* D = dst + s * kDstLevels * kTile;
            const int32_t* LO = lhs_ + s * kLH;
            const uint64_t* W = words + (k & 1) * nword;
            const uint64_t vm = bar_range_mask(t0, w - 1, B - 2);
            const uint64_t Zb = W[iw * nk + ik] & vm;
            const uint64_t dpw = W[nw * nk + 2 * iw], dnw = W[nw * nk + 2 * iw + 1];
            const uint64_t ZL = Zb & ~dpw, ZH = Zb & ~dnw;  // z < -k (D < 0), z > k (D > 0)
            // signal exits with the forced exit at bar B-1 folded in (in this tile iff bl < 64)
            const int bl = B - 1 - t0;
            const uint64_t fb = bl < kTile ? (1ULL << bl) : 0ULL;
            const uint64_t DP = (dpw & vm) | fb;
            const uint64_t DN = (dnw & vm) | fb;
            const uint8_t* TL = levt + (k & 1) * 2 * nlev * kTile;  // first-passage tables
            const uint8_t* TH = TL + nlev * kTile;
            const int32_t* PL = levp + (k % 3) * 2 * nlev * kTile;  // levels
            const int32_t* PH = PL + nlev * kTile;
            if (!finder) {
                int cur = 0;
                // gap / mdd in int32 this tile (unsplit runs; acct_close_rt)
                const bool nar = !SEG && kBollWalkNarrow && __builtin_amdgcn_readfirstlane(nars[s]);
                // walker: one trade (entry and/or exit) per call, in bar order; false when the
                // tile is done. Only the first trade of the tile can start open (path carried in
                // a.agg). Two LDS round trips per trade: everything the entry bar decides (close,
                // returns, both sides' first passages and levels), then everything the exit bar
                // decides (close, returns, the path's sparse-table entries), each issued together
                // before any branch.
                auto trade = [&](auto first_tag) -> bool {
                    constexpr bool FIRST = decltype(first_tag)::value;
                    if (STAMPS) sa.count(3);
                    int xlo = kTile, xhi = kTile;
                    bool entered = false;
                    if (!FIRST || a.pos == 0) {
                        const uint64_t m = (ZL | ZH) & bits_from(cur);
                        if (m == 0) return false;
                        const int b = __builtin_ctzll(m);
                        const int np = ((ZL >> b) & 1) ? 1 : -1;
                        const int rl = (np > 0 ? lev_lo_long : lev_lo_short) * kTile + b;
                        const int rh = (np > 0 ? lev_hi_long : lev_hi_short) * kTile + b;
                        const int32_t cx = cT[b];
                        const int64_t qx = ql[b], q2x = ql[kTile + b];
                        const int32_t pl = PL[rl], ph = PH[rh];
                        xlo = TL[rl];
                        xhi = TH[rh];
                        asm volatile("" ::"v"(cx), "v"(qx), "v"(q2x), "v"(pl), "v"(ph), "v"(xlo), "v"(xhi));
                        entered = true;
                        a.ps1 += np > 0 ? (uint64_t)0 - (uint64_t)qx : (uint64_t)qx;
                        a.ps2 -= (uint64_t)q2x;
                        acct_open(a, t0 + b, b, cx);
                        a.pos = np;
                        XL = pl;
                        XHm1 = ph;
                        cur = b + 1;
                    }
                    if (cur >= kTile) return false;
                    // exit: first of SL/TP (intrabar, from entry + 1; SL wins a same-bar tie),
                    // the signal exit and the forced exit at B-1 (SL/TP beat both on the same bar)
                    const bool lg = a.pos > 0;
                    const uint64_t sig = (lg ? DP : DN) & (~0ULL << cur);  // cur < 64 here
                    int x = sig ? __builtin_ctzll(sig) : kTile;
                    // a position carried into the tile searches with its levels; a trade entered
                    // in it has its first passages from the tables
                    if (FIRST && !entered) sltp_search(LO, cur, XL, XHm1, xlo, xhi);
                    const int xs = min(xlo, xhi);
                    const bool hit = xs < kTile && xs <= x;
                    if (hit) x = xs;
                    // one path for both exit kinds (no divergence): the trade's closes up to the
                    // bar before an SL/TP fill or up to a signal exit's bar, then the fill price
                    // (for a signal exit that is the last close again, which leaves the aggregate
                    // unchanged). With no exit in the tile (x = 64) the reads are clamped, issued
                    // and unused.
                    const int xc = min(x, kTile - 1);
                    const int qi = hit ? x - 1 : xc;  // >= a.sb - 1 (exits follow the entry bar)
                    // qi < a.sb only for a fill at the first bar of the tile of a carried
                    // position; a trade opened in this tile exits after its entry bar a.sb
                    const Agg seg = dst_query_w(D, a.sb, FIRST ? max(qi, a.sb) : qi);
                    const int32_t cxx = cT[xc];
                    const int64_t qx = ql[xc], q2x = ql[kTile + xc];
                    asm volatile("" ::"v"(cxx), "v"(qx), "v"(q2x));
                    if (!hit && x >= kTile) return false;
                    // fill price: the touched level (XHm1 + 1 = the upper level below 2^31)
                    const bool low = xlo < xhi || (xlo == xhi && lg);
                    const int32_t px = hit ? (low ? XL : XHm1 + 1) : cxx;
                    const Agg sp = (FIRST && qi < a.sb) ? kAggId : seg;
                    const Agg st = agg_merge(FIRST ? agg_merge(a.agg, sp) : sp, agg_one(px));
                    if (SEG || !kBollWalkNarrow)
                        acct_close<PARITY, SEG>(a, t0 + x, px, st, tr, cap);
                    else
                        acct_close_rt<PARITY>(a, nar, t0 + x, px, st, tr, cap);
                    a.ps1 += lg ? (uint64_t)qx : (uint64_t)0 - (uint64_t)qx;
                    a.ps2 += (uint64_t)q2x;
                    a.pos = 0;
                    cur = x + 1;
                    return true;
                };
                if (trade(std::true_type{})) {
#pragma unroll 1
                    while (trade(std::false_type{})) {
                    }
                }
                if (STAMPS) sa.mark(1);
                acct_tile_end(a, D, ql);
            } else {
                // finder: the same walk without the accounts; each trade leaves a 16-bit record
                // [tile & 1][record][lane]: bits 0-5 entry bar, 6 entered in this tile, 7 long,
                // 8-13 exit bar, 14-15 exit kind (0 still open, 1 signal / forced exit at the
                // close, 2 low-level fill, 3 high-level fill)
                uint16_t* RB = recs + (k & 1) * kRecCap * kTile + lane;
                int nr = 0, fcur = 0;
                // one trade per call, false when the lane's tile is done; the first call of the
                // tile is peeled (FIRST: only it can start open and search with the carried
                // levels), so the loop's body has no branch on it
                auto find = [&](auto first_tag) -> bool {
                    constexpr bool FIRST = decltype(first_tag)::value;
                    if (STAMPS) sa.count(3);
                    int xlo = kTile, xhi = kTile;
                    bool entered = false;
                    uint32_t rec;
                    if (!FIRST || fpos == 0) {
                        const uint64_t m = (ZL | ZH) & bits_from(fcur);
                        if (m == 0) return false;
                        const int b = __builtin_ctzll(m);
                        const int np = ((ZL >> b) & 1) ? 1 : -1;
                        const int rl = (np > 0 ? lev_lo_long : lev_lo_short) * kTile + b;
                        const int rh = (np > 0 ? lev_hi_long : lev_hi_short) * kTile + b;
                        const int32_t pl = PL[rl], ph = PH[rh];
                        xlo = TL[rl];
                        xhi = TH[rh];
                        asm volatile("" ::"v"(pl), "v"(ph), "v"(xlo), "v"(xhi));
                        entered = true;
                        fpos = np;
                        XL = pl;
                        XHm1 = ph;
                        fcur = b + 1;
                        rec = (uint32_t)b | 64u | (np > 0 ? 128u : 0u);
                    } else {
                        rec = fpos > 0 ? 128u : 0u;
                    }
                    // one record store per trade; an entry at the tile's last bar or with no exit
                    // in the tile leaves an open record, a carried position with no exit none
                    bool emit = true, more = false;
                    int x = kTile;
                    if (fcur < kTile) {
                        const bool lg = fpos > 0;
                        const uint64_t sig = (lg ? DP : DN) & (~0ULL << fcur);
                        x = sig ? __builtin_ctzll(sig) : kTile;
                        if (FIRST && !entered) sltp_search(LO, fcur, XL, XHm1, xlo, xhi);
                        const int xs = min(xlo, xhi);
                        const bool hit = xs < kTile && xs <= x;
                        if (hit) x = xs;
                        if (hit || x < kTile) {
                            const bool low = xlo < xhi || (xlo == xhi && lg);
                            rec |= ((uint32_t)x << 8) | ((hit ? (low ? 2u : 3u) : 1u) << 14);
                            more = true;
                        } else {
                            emit = entered;
                        }
                    }
                    if (emit) {
                        RB[nr * kTile] = (uint16_t)rec;
                        ++nr;
                    }
                    if (!more) return false;
                    fpos = 0;
                    fcur = x + 1;
                    return true;
                };
                if (find(std::true_type{})) {
#pragma unroll 1
                    while (find(std::false_type{})) {
                    }
                }
                nrec[(k & 1) * kTile + lane] = (uint8_t)nr;
                if (STAMPS) sa.mark(1);
            }
            __builtin_amdgcn_s_setprio(0);
        }
        // (profiling: 4096 drops the accountant's records, an upper bound on what a cheaper
        // accountant can gain)
        if (accountant && active && ka >= T_walk && ka < T_end && !BT_ABL(g, 8) && !BT_ABL(g, 4096)) {
            // accountant: the finder's records of tile ka, in order (the tile's buffers stay
            // until step ka + 2: four stages, levels in three)
            set_prio(BT_PRIO(g, 18, kBollAcctPrio));
            const int s = ka % kBollStages, ta = ka * kTile;
            const int32_t* cT = cts + s * kTile;
            const int64_t* ql = qls + s * 2 * kTile;
            const Agg* D = dst + s * kDstLevels * kTile;
            const int32_t* PL = levp + (ka % 3) * 2 * nlev * kTile;
            const int32_t* PH = PL + nlev * kTile;
            const uint16_t* RB = recs + (ka & 1) * kRecCap * kTile + lane;
            const int n = nrec[(ka & 1) * kTile + lane];
            // the records' accounts in int32 while the closes' total variation allows (Acct32);
            // one copy of the loop per width, chosen per tile (wave-uniform)
            auto records = [&](auto narrow_tag) {
                constexpr bool NARROW = decltype(narrow_tag)::value;
                // gap, mdd (SEG: the forms) within 2 TV < 2^31 if NARROW
                Acct32 n32{(int32_t)a.gap, (int32_t)a.mdd};
                // one record per call; the tile's first is peeled (FIRST: only it can be the exit
                // of a position carried in), so every later record enters at b
                auto record = [&](auto first_tag, int i) {
                    constexpr bool FIRST = decltype(first_tag)::value;
                    if (STAMPS) sa.count(3);
                    const uint32_t rec = RB[i * kTile];
                    const int b = (int)(rec & 63u), x = (int)((rec >> 8) & 63u), kind = (int)(rec >> 14);
                    if (!FIRST || (rec & 64u)) {  // entry at b
                        const int np = (rec & 128u) ? 1 : -1;
                        const int rl = (np > 0 ? lev_lo_long : lev_lo_short) * kTile + b;
                        const int rh = (np > 0 ? lev_hi_long : lev_hi_short) * kTile + b;
                        const int32_t cx = cT[b];
                        const int64_t qx = ql[b], q2x = ql[kTile + b];
                        const int32_t pl = PL[rl], ph = PH[rh];
                        asm volatile("" ::"v"(cx), "v"(qx), "v"(q2x), "v"(pl), "v"(ph));
                        a.ps1 += np > 0 ? (uint64_t)0 - (uint64_t)qx : (uint64_t)qx;
                        a.ps2 -= (uint64_t)q2x;
                        acct_open(a, ta + b, b, cx);
                        a.pos = np;
                        XL = pl;
                        XHm1 = ph;
                    }
                    if (kind != 0) {  // exit at x
                        const bool hit = kind >= 2;
                        const int qi = hit ? x - 1 : x;
                        // (a later record's exit follows its entry bar a.sb: qi >= a.sb)
                        const Agg seg = dst_query_w(D, a.sb, FIRST ? max(qi, a.sb) : qi);
                        const int32_t cxx = cT[x];
                        const int64_t qx = ql[x], q2x = ql[kTile + x];
                        asm volatile("" ::"v"(cxx), "v"(qx), "v"(q2x));
                        const int32_t px = hit ? (kind == 2 ? XL : XHm1 + 1) : cxx;
                        close_trade(narrow_tag, first_tag, n32, ta, x, qi, px, seg, qx, q2x);
                    }
                };
                if (n > 0) {
                    record(std::true_type{}, 0);
#pragma unroll 1
                    for (int i = 1; i < n; ++i) record(std::false_type{}, i);
                }
                if (NARROW) {
                    a.gap = (uint32_t)n32.g;  // >= 0
                    a.mdd = (uint32_t)n32.m;
                }
            };
            // unsplit runs only (bar segments keep the wide max-plus forms)
            if (!SEG && __builtin_amdgcn_readfirstlane(nars[s]))
                records(std::true_type{});
            else
                records(std::false_type{});
            if (STAMPS) sa.mark(1);
            acct_tile_end(a, D, ql);
            __builtin_amdgcn_s_setprio(0);
        }
        if (k + 1 < T_end && !BT_ABL(g, 2)) flags(k + 1);
        if (STAMPS) sa.mark(2);
        __syncthreads();
        if (STAMPS) sa.barrier();
    }
    // roles: parameter waves 0-3 by wave (k-major lanes: wave 0 holds the busiest threshold), 4 the
    // helper, 5 the task-only waves, 6 the accountant
    if (STAMPS) sa.flush(out.dbg, wave < npw ? min(wave, 3) : (helper ? 4 : (accountant ? 6 : 5)), lane);
    // stamps: the raw HW_ID (SIMD in bits 4-5, CU in bits 8-11) of block 0's first 8 waves
    if (STAMPS && blockIdx.x == 0 && blockIdx.z == 0 && lane == 0 && hw_wave < 8 && out.dbg != nullptr)
        out.dbg[56 + hw_wave] = (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4) + 1;
    if (SEG) {
        if (keeps) {
            // a segment with no bars never reached its first accounted tile: the state passes
            // through (flat, or the fix pass's injected one)
            if (T_acct >= T_end) seg_write_start(seg_rec(), a.pos, a.e);
            seg_write_rest(a, seg_rec());
        }
        return;
    }
    if (keeps) acct_write(a, B, g.sqrt_ann, (size_t)blockIdx.x * P + pj_out, out);
    wave_add_trades(out, keeps ? a.ntr : 0);
}

// Folds the bar segments of every (symbol, param) in order: additive counts, pnl, hash and
// return sums; the drawdown forms composed from g = m = 0 (tile_common.h TradeAcct).
__global__ __launch_bounds__(256) void seg_combine(const SymDesc* __restrict__ syms,
                                                        int n_sym, int P, const SegRec* __restrict__ rec,
                                                        int G, double sqrt_ann, Out out) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t n = (size_t)n_sym * P;
    int ntr = 0;
    if (i < n) {
        const int s = (int)(i / P);
        int64_t expo = 0, R = 0, gap = 0, mdd = 0;
        uint64_t h = 0;
        i128 s1 = 0, s2 = 0;
        for (int q = 0; q < G; ++q) {
            const SegRec& r = rec[(size_t)q * n + i];
            ntr += r.ntr;
            expo += r.expo;
            R += r.R;
            h += r.h;
            s1 += (i128)(((unsigned __int128)(uint64_t)r.s1hi << 64) | r.s1lo);
            s2 += (i128)(((unsigned __int128)(uint64_t)r.s2hi << 64) | r.s2lo);
            mdd = max(mdd, max(gap + r.C, r.D));
            gap = max(gap + r.A, r.B);
        }
        const uint64_t s1lo = (uint64_t)s1, s2lo = (uint64_t)s2;
        const int64_t s1hi = (int64_t)(s1 >> 64), s2hi = (int64_t)(s2 >> 64);
        const double sh = sharpe_fx(s1lo, s1hi, s2lo, s2hi, syms[s].bars, sqrt_ann);
        bt_summary r;
        r.n_trades = ntr;
        r.status = 0;
        r.pnl = R;
        r.mdd = mdd;
        r.exposure = expo;
        r.sharpe = sh;
        r.hash = h;
        out.sum[i] = r;
        out.key[i] = order_key(sh);
        if (out.sums != nullptr) out.sums[i] = bt_sums{s1lo, s1hi, s2lo, s2hi};
    }
    wave_add_trades(out, ntr);
}

// ----------------------------------------------------------------------------- launchers
// Extra task-only waves per block (they take condition-word tasks only). The EMA kernel has one
// parameter wave per symbol on config 3 and is latency-bound at ~1.5 waves per SIMD: two extra
// waves take 4.96 -> 3.68 ms, four (with the parameter wave walking only, at raised priority)
// 3.32 ms, five 3.20 ms (8 waves: two blocks per CU still fit); six no longer fit two blocks per
// CU (5.0 ms). The Bollinger kernel runs 5 waves x 2 blocks per CU and its ~120 VGPRs cap a
// CU at 16 waves: two task-only waves, with the parameter waves then walking only, take config 4
// 12.3 -> 12.0 ms (250 symbols: 9.95 -> 9.76 ms); four no longer fit two blocks (19.4 ms).
static int tile_param_waves(int need, int cap) {
    int pw = std::min(need, cap);
#ifdef BT_PROFILING
    if (const char* v = getenv("BT_PW")) pw = std::max(1, std::min(atoi(v), pw));  // tuning aid
#endif
    return pw;
}

// Hardware wave -> role of a Bollinger block (k_tile boll_tile_kernel wave_map). Hardware wave w
// runs on SIMD w % 4, so waves w and w + 4 share one: each busy parameter wave (the walks, the
// busiest first) gets a task-only wave as its partner (task waves take fewer tasks when their
// SIMD is busy), the lightest parameter wave the helper, and the accountant of a split walk a
// light parameter wave. Identity for other block shapes.
static uint32_t boll_wave_map(int pw, int nsplit, int xw) {
    uint32_t m = 0;
    for (int w = 0; w < 8; ++w) m |= (uint32_t)w << (4 * w);
    const int nw = pw + 1 + nsplit + xw;
    if (nw == 8 && pw == 4) {
        // logical roles: 0-3 parameter groups, 4 helper, then the accountant, then tasks
        const int split_map[8] = {0, 1, 2, 3, 6, 7, 5, 4};
        const int plain_map[8] = {0, 1, 2, 3, 5, 6, 7, 4};
        const int* r = nsplit == 1 ? split_map : plain_map;
        m = 0;
        for (int w = 0; w < 8; ++w) m |= (uint32_t)r[w] << (4 * w);
    }
#ifdef BT_PROFILING
    if (const char* v = getenv("BT_WAVEMAP")) m = (uint32_t)strtoul(v, nullptr, 16);  // tuning aid
#endif
    return m;
}

// Split Bollinger walk (finder + accountant waves) on by default; BT_SPLIT=0 turns it off in the
// profiling build (A/B aid).
static bool tile_split_walk() {
    bool on = true;
#ifdef BT_PROFILING
    if (const char* v = getenv("BT_SPLIT")) on = atoi(v) != 0;
#endif
    return on;
}

static int tile_lanes_per_wave() {
    int l = 64;
#ifdef BT_PROFILING
    if (const char* v = getenv("BT_LPW")) l = std::max(1, std::min(atoi(v), 64));  // tuning aid
#endif
    return l;
}

// Compute units of the current device (one process per GPU).
int device_cus() {
    static int n = 0;
    if (n <= 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
    }
    return n;
}

static int tile_extra_waves(int used, int x) {
#ifdef BT_PROFILING
    if (const char* v = getenv("BT_XW")) x = atoi(v);  // tuning aid
#endif
    return std::max(0, std::min(x, 16 - used));
}

size_t ema_lds_bytes(const Grid& g, int ts) { return tile_lds_layout(0, g.ring, g.na, g.nb, 0, ts).total; }
size_t boll_lds_bytes(const Grid& g) {
    return tile_lds_layout(1, g.ring, g.na, g.nb, g.nc + g.nd).total;
}

int32_t ema_burn_tiles(int32_t max_span) {
    // fp64 EMA chains started from e = c met the true ones after 131-162 bars (span 10) to
    // 11,559-13,368 bars (span 780) over 18 starts each (round-2 measurement); started from the
    // weighted-sum estimate, after at most 2.6 (span 10) to 3.8 (span 780) spans (round 3,
    // 18 starts each): 6 spans, on top of the OLS lookback tiles the chain also runs through
    return std::max(kDefaultBurnTiles, (6 * max_span + kTile - 1) / kTile);
}

int32_t ema_auto_segments(int32_t n_sym, int32_t n_params, int32_t max_bars, int32_t burn_tiles) {
    if (n_sym <= 0) return 1;
    const int pw = std::min((n_params + 63) / 64, 1024 / 64 - 2);
    const long long blocks = (long long)n_sym * ((n_params + 64 * pw - 1) / (64 * pw));
    if (blocks > device_cus()) return 1;
    int G = (int)std::min<long long>(4, std::max<long long>(1, 2LL * device_cus() / blocks));
    const int ntiles = (max_bars + kTile - 1) / kTile;
    while (G > 1 && ntiles / G < 2 * burn_tiles) --G;
    return G;
}

// Tiles per stage of an EMA+OLS launch: 128-bar stages (TS = 2) when they keep as many blocks per
// CU as 64-bar ones (config 3: 80.2 KB vs 61.1 KB, two either way), else TS = 1.
int ema_stage_tiles(const Grid& g) {
    const size_t cu = 160 * 1024, l1 = ema_lds_bytes(g, 1), l2 = ema_lds_bytes(g, 2);
    return l2 <= cu && cu / l2 >= cu / l1 ? 2 : 1;
}

template <int TS>
static hipError_t launch_ema_ts(const SymDesc* syms, int32_t n_sym, const int32_t* close, const Grid& g,
                                const Out& out, bool parity, const SegArgs& seg, hipStream_t st) {
    const int lpw = tile_lanes_per_wave();
    const int pw = tile_param_waves((g.n_params + lpw - 1) / lpw, 1024 / 64 - 2);
    const int xw = tile_extra_waves(pw + 2, 5);
    const bool split = seg.G > 1 && !parity;
    const dim3 grid(n_sym, (g.n_params + lpw * pw - 1) / (lpw * pw), split ? seg.G : 1);
    const dim3 block(64 * (pw + 2 + xw));
    const size_t lds = ema_lds_bytes(g, TS);
#ifdef BT_PROFILING
    if (BT_ABL(g, 64) && !split) {
        hipLaunchKernelGGL((ema_tile_kernel<false, true, false, TS>), grid, block, lds, st, syms, close, g, out, xw, lpw, seg, 0);
        return hipGetLastError();
    }
#endif
    if (split) {
        // speculative segments (stamped in the profiling build), the fix pass of each boundary,
        // the fold
#ifdef BT_PROFILING
        if (BT_ABL(g, 64))
            hipLaunchKernelGGL((ema_tile_kernel<false, true, true, TS>), grid, block, lds, st, syms, close, g, out, xw, lpw, seg, 0);
        else
#endif
            hipLaunchKernelGGL((ema_tile_kernel<false, false, true, TS>), grid, block, lds, st, syms, close, g, out, xw, lpw, seg, 0);
        const dim3 fgrid(grid.x, grid.y, 1);
        for (int s = 1; s < seg.G; ++s)
            hipLaunchKernelGGL((ema_tile_kernel<false, false, true, TS>), fgrid, block, lds, st, syms, close, g, out, xw, lpw, seg, s);
        const size_t n = (size_t)n_sym * g.n_params;
        hipLaunchKernelGGL(seg_combine, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, syms, n_sym, g.n_params, seg.rec, seg.G, g.sqrt_ann, out);
    } else if (parity) {
        hipLaunchKernelGGL((ema_tile_kernel<true, false, false, TS>), grid, block, lds, st, syms, close, g, out, xw, lpw, seg, 0);
    } else {
        hipLaunchKernelGGL((ema_tile_kernel<false, false, false, TS>), grid, block, lds, st, syms, close, g, out, xw, lpw, seg, 0);
    }
    return hipGetLastError();
}

hipError_t launch_ema_ols(const SymDesc* syms, int32_t n_sym, const int32_t* close, const Grid& g,
                          const Out& out, bool parity, const SegArgs& seg, hipStream_t st) {
    if (n_sym <= 0) return hipSuccess;
    return ema_stage_tiles(g) == 2 ? launch_ema_ts<2>(syms, n_sym, close, g, out, parity, seg, st)
                                   : launch_ema_ts<1>(syms, n_sym, close, g, out, parity, seg, st);
}

// Bar segments per symbol for a shard of n_sym symbols: a shard with no more blocks than CUs
// leaves every CU one latency-bound block (config 4 on 8 GPUs: 250 symbols, 7.95 ms), so its
// series are cut into up to 4 segments, enough for two blocks per CU, each segment at least
// twice the burn-in long.
int32_t boll_auto_segments(int32_t n_sym, int32_t n_params, int32_t max_bars) {
    if (n_sym <= 0) return 1;
    const int pw = std::min((n_params + 63) / 64, 1024 / 64 - 1);
    const long long blocks = (long long)n_sym * ((n_params + 64 * pw - 1) / (64 * pw));
    if (blocks > device_cus()) return 1;
    int G = (int)std::min<long long>(4, std::max<long long>(1, 2LL * device_cus() / blocks));
    const int ntiles = (max_bars + kTile - 1) / kTile;
    while (G > 1 && ntiles / G < 2 * kDefaultBurnTiles) --G;
    return G;
}

hipError_t launch_boll(const SymDesc* syms, int32_t n_sym, const int32_t* high, const int32_t* low,
                       const int32_t* close, const Grid& g, const Out& out, bool parity,
                       const SegArgs& seg, hipStream_t st) {
    if (n_sym <= 0) return hipSuccess;
    const int lpw = tile_lanes_per_wave();
    const int pw = tile_param_waves((g.n_params + lpw - 1) / lpw, 1024 / 64 - 1);
    const bool split = seg.G > 1 && !parity;
    const dim3 grid(n_sym, (g.n_params + lpw * pw - 1) / (lpw * pw), split ? seg.G : 1);
    // Split walk: the parameter wave holding the smallest z threshold (lanes run k-major) trades
    // the most, and its lanes' serial trade chains set the tile time (config 4: 7.1 walk
    // iterations per tile against 1.0-4.3 for the other waves), so that wave only finds trades
    // and an accountant wave keeps their accounts a tile later.
    int split_grp = -1;
    if (tile_split_walk() && pw >= 2 && grid.y == 1) {
        const long long per_k = (long long)g.na * g.nc * g.nd;  // lanes per z threshold
        const int grp = (int)((g.kmin_idx * per_k) / lpw);
        if (grp < pw) split_grp = grp;
    }
    const int nsplit = split_grp < 0 ? 0 : 1;
    const int base = pw + 1 + nsplit;
    // at most one block per CU (config 4 on 8 GPUs: 250 symbols) leaves wave slots free: four
    // task-only waves (8.17 -> 7.90 ms vs two); otherwise as many as keep the block at 8 waves,
    // so two blocks share a CU at <= 128 VGPRs (config 4: three, 9.65 -> 9.51 ms; four 15.8 ms)
    const bool sparse = (long long)grid.x * grid.y * grid.z <= device_cus();
    const int xw = tile_extra_waves(base, sparse ? 4 : std::max(2, std::min(3, 8 - base)));
    const dim3 block(64 * (base + xw));
    const size_t lds = boll_lds_bytes(g);
    const uint32_t wmap = boll_wave_map(pw, nsplit, xw);
#ifdef BT_PROFILING
    if (BT_ABL(g, 64)) {
        hipLaunchKernelGGL((boll_tile_kernel<false, true, false>), grid, block, lds, st, syms, high, low, close, g, out, xw, lpw, seg, 0, split_grp, wmap);
        return hipGetLastError();
    }
#endif
    if (split) {
        // speculative segments, then the fix pass of each boundary in order (a block returns at
        // once when its lanes' starts were right), then the fold
        hipLaunchKernelGGL((boll_tile_kernel<false, false, true>), grid, block, lds, st, syms, high, low, close, g, out, xw, lpw, seg, 0, split_grp, wmap);
        const dim3 fgrid(grid.x, grid.y, 1);
        for (int s = 1; s < seg.G; ++s)
            hipLaunchKernelGGL((boll_tile_kernel<false, false, true>), fgrid, block, lds, st, syms, high, low, close, g, out, xw, lpw, seg, s, split_grp, wmap);
        const size_t n = (size_t)n_sym * g.n_params;
        hipLaunchKernelGGL(seg_combine, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, syms, n_sym, g.n_params, seg.rec, seg.G, g.sqrt_ann, out);
    } else if (parity) {
        hipLaunchKernelGGL((boll_tile_kernel<true, false, false>), grid, block, lds, st, syms, high, low, close, g, out, xw, lpw, seg, 0, split_grp, wmap);
    } else {
        hipLaunchKernelGGL((boll_tile_kernel<false, false, false>), grid, block, lds, st, syms, high, low, close, g, out, xw, lpw, seg, 0, split_grp, wmap);
    }
    return hipGetLastError();
}

}  // namespace bt
