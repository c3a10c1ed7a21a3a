// device_common.h — device helpers shared by the strategy kernels.
#pragma once
#include <type_traits>

#include "internal.h"

namespace bt {

// Trade hash (spec §4): h = sum over trades of mix(w) mod 2^64, w = entry | exit << 31 |
// (side > 0) << 62. A sum, so the hashes of consecutive bar segments add (k_tile.hip segments).
__host__ __device__ inline uint64_t trade_mix(uint64_t w) {
    const uint64_t z = (w ^ (w >> 29)) * 0xBF58476D1CE4E5B9ULL;
    return z ^ (z >> 32);
}
// trade_mix of the one-word trade term w = e | t << 31 | side << 62 (spec §4) for bar indices
// e, t < 2^22 (kMaxBars): w ^ (w >> 29) is formed in 32-bit halves with no 64-bit shift,
//   lo = e ^ (t << 2) ^ (t << 31),  hi = (t >> 1) ^ (side ? 2^30 + 2 : 0)
// (w >> 29 has lo = t << 2 and hi = side << 1 in that range; checked against trade_mix on 5e7
// random terms, and bit for bit by every GPU parity test through the hash).
__host__ __device__ inline uint64_t trade_mix_et(uint32_t e, uint32_t t, bool lg) {
    const uint32_t lo = e ^ (t << 2) ^ (t << 31);
    const uint32_t hi = (t >> 1) ^ (lg ? 0x40000002u : 0u);
    const uint64_t z = (((uint64_t)hi << 32) | lo) * 0xBF58476D1CE4E5B9ULL;
    return z ^ (z >> 32);
}
constexpr int kDstLevels = 6;      // log2(kTile)
constexpr int kKeyStride = kTile + 1;  // +1 double per key row: conflict-free ds_read_b64

typedef __int128 i128;
// explicit LDS (address space 3) element types, for pointers kept opaque in a VGPR so that
// accesses use small immediate offsets from it
typedef __attribute__((address_space(3))) double lds_f64;

// Price-path aggregate over a run of closes, in order: max, min, max drawdown (max over
// i<=j of c_i - c_j), max draw-up (max over i<=j of c_j - c_i). Prices < 2^31, so every
// field fits int32.
struct __attribute__((aligned(16))) Agg {
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

// Rows of the table are stored in reverse level order (row 5 - m holds level m): the row of a
// query (a, b) is then clz((a ^ b) | 1) - 26, one v_ffbh and no select, with a == b landing on
// level 0 (the single bar).
__device__ __forceinline__ int dst_row(int a, int b) {
    return __builtin_clz((unsigned)(a ^ b) | 1u) - (32 - kDstLevels);
}
// The row's base (the constant offset folds into the table's scalar base address).
__device__ __forceinline__ const Agg* dst_rowp(const Agg* D, int a, int b) {
    return D - (32 - kDstLevels) * kTile + __builtin_clz((unsigned)(a ^ b) | 1u) * kTile;
}

// Aggregate of closes cT[a..b], 0 <= a <= b < kTile.
__device__ __forceinline__ Agg dst_query(const Agg* D, const int32_t* cT, int a, int b) {
    if (a == b) return agg_one(cT[a]);
    const int r = dst_row(a, b);
    return agg_merge(D[r * kTile + a], D[r * kTile + b]);
}

// Branch-free form: for a == b level 0 holds the single bar (D[0][a] == one(c_a)), and
// merging it with itself leaves max/min unchanged and gives drawdown/draw-up 0.
__device__ __forceinline__ Agg dst_query_bf(const Agg* D, int a, int b) {
    const Agg* Dr = dst_rowp(D, a, b);
    return agg_merge(Dr[a], Dr[b]);
}

// dst_query_bf reading both 16-B entries whole (two ds_read_b128 in one round trip, kept live):
// callers that need drawdown or draw-up by side then wait once instead of a second time in a
// divergent branch.
__device__ __forceinline__ Agg dst_query_w(const Agg* D, int a, int b) {
    const Agg* Dr = dst_rowp(D, a, b);
    const int4 u = *reinterpret_cast<const int4*>(Dr + a);
    const int4 v = *reinterpret_cast<const int4*>(Dr + b);
    asm volatile("" ::"v"(u.x), "v"(u.y), "v"(u.z), "v"(u.w), "v"(v.x), "v"(v.y), "v"(v.z), "v"(v.w));
    return agg_merge(Agg{u.x, u.y, u.z, u.w}, Agg{v.x, v.y, v.z, v.w});
}

// Upward-biased reciprocal for exact floor keys (k_sma.hip floor_key): RN(RN(1/W) * (1 + 2^-47)).
__host__ __device__ inline double key_recip(int W) { return (1.0 / (double)W) * (1.0 + 0x1p-47); }

// Identity of agg_merge: merge(kAggId, x) == x for prices in [1, 2^31) (no int32 overflow:
// 0 - x.mn < 0 and x.mx - INT32_MAX <= 0).
constexpr Agg kAggId = {0, 0x7FFFFFFF, 0, 0};

// Wave64 inclusive scan of int64 with DPP (row_shr 1,2,4,8 inside 16-lane rows, then
// row_bcast15 / row_bcast31 across rows): no LDS round trip.
__device__ __forceinline__ int64_t wave_iscan_i64(int64_t x) {
    uint32_t lo = (uint32_t)x, hi = (uint32_t)((uint64_t)x >> 32);
#define BT_DPP_STEP(ctrl, rmask)                                                      \
    {                                                                                 \
        const uint32_t ylo = __builtin_amdgcn_update_dpp(0u, lo, ctrl, rmask, 0xf, false); \
        const uint32_t yhi = __builtin_amdgcn_update_dpp(0u, hi, ctrl, rmask, 0xf, false); \
        const uint64_t r = (((uint64_t)hi << 32) | lo) + (((uint64_t)yhi << 32) | ylo);   \
        lo = (uint32_t)r;                                                             \
        hi = (uint32_t)(r >> 32);                                                     \
    }
    BT_DPP_STEP(0x111, 0xf)  // row_shr:1
    BT_DPP_STEP(0x112, 0xf)  // row_shr:2
    BT_DPP_STEP(0x114, 0xf)  // row_shr:4
    BT_DPP_STEP(0x118, 0xf)  // row_shr:8
    BT_DPP_STEP(0x142, 0xa)  // row_bcast:15 into rows 1, 3
    BT_DPP_STEP(0x143, 0xc)  // row_bcast:31 into rows 2, 3
#undef BT_DPP_STEP
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

// The same scans with each step one add-with-carry pair whose first operand is the DPP-moved
// value (v_add_co_u32_dpp / v_addc_co_u32_dpp: lanes with no source add 0, rows outside the row
// mask keep x): the compiler's DPP combine does not reach a 64-bit add, so wave_iscan_i64 spends
// two DPP moves, their two `old` moves and a 64-bit add per step. gfx950 needs two wait states
// between a VALU write and a DPP read of the same VGPR: one scan pads each step with an s_nop,
// two interleaved scans need none; every block starts and ends with one, so the code around it
// needs no hazard tracking into the asm. Used by the EMA helper's tile scan only: there it
// measured -1.4 % (config 3, 500 symbols), in the Bollinger and SMA kernels +0.4 to +0.9 %
// (DESIGN.md §0.0 E11).
#define BT_S64_CTRLS(X)                                                                   \
    X("row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1")                                \
    X("row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1")                                \
    X("row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1")                                \
    X("row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1")                                \
    X("row_bcast:15 row_mask:0xa bank_mask:0xf")                                          \
    X("row_bcast:31 row_mask:0xc bank_mask:0xf")
__device__ __forceinline__ int64_t wave_iscan_i64_ac(int64_t x) {
    uint32_t lo = (uint32_t)x, hi = (uint32_t)((uint64_t)x >> 32);
#define BT_S64_ONE(ctrl)                                                                   \
    "s_nop 1\n"                                                                            \
    "v_add_co_u32_dpp %0, vcc, %0, %0 " ctrl "\n"                                          \
    "v_addc_co_u32_dpp %1, vcc, %1, %1, vcc " ctrl "\n"
    asm volatile(BT_S64_CTRLS(BT_S64_ONE) "s_nop 1" : "+v"(lo), "+v"(hi) : : "vcc");
#undef BT_S64_ONE
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
// two independent scans, interleaved (each DPP read three instructions after its write)
__device__ __forceinline__ void wave_iscan2_i64_ac(int64_t& x, int64_t& y) {
    uint32_t xl = (uint32_t)x, xh = (uint32_t)((uint64_t)x >> 32);
    uint32_t yl = (uint32_t)y, yh = (uint32_t)((uint64_t)y >> 32);
#define BT_S64_TWO(ctrl)                                                                   \
    "v_add_co_u32_dpp %0, vcc, %0, %0 " ctrl "\n"                                          \
    "v_addc_co_u32_dpp %1, vcc, %1, %1, vcc " ctrl "\n"                                    \
    "v_add_co_u32_dpp %2, vcc, %2, %2 " ctrl "\n"                                          \
    "v_addc_co_u32_dpp %3, vcc, %3, %3, vcc " ctrl "\n"
    asm volatile("s_nop 1\n" BT_S64_CTRLS(BT_S64_TWO) "s_nop 1"
                 : "+v"(xl), "+v"(xh), "+v"(yl), "+v"(yh) : : "vcc");
#undef BT_S64_TWO
    x = (int64_t)(((uint64_t)xh << 32) | xl);
    y = (int64_t)(((uint64_t)yh << 32) | yl);
}
#undef BT_S64_CTRLS

// Wave64 inclusive scan of uint32 (same DPP steps as wave_iscan_i64); lane 63 holds the total.
__device__ __forceinline__ uint32_t wave_iscan_u32(uint32_t x) {
    x += __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += __builtin_amdgcn_update_dpp(0u, x, 0x142, 0xa, 0xf, false);  // row_bcast:15
    x += __builtin_amdgcn_update_dpp(0u, x, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return x;
}

// ---- cross-lane moves without LDS (DPP / readlane; ds_bpermute costs an LDS round trip)
// DPP controls: quad_perm [p0 p1 p2 p3] = p0 | p1 << 2 | p2 << 4 | p3 << 6; row_shl:d = 0x100 + d;
// row_mirror 0x140; row_half_mirror 0x141 (lane i <-> 7 - i in each 8); row_newbcast:k = 0x150 + k
// (lane k of each 16-lane row to the whole row, gfx90a+). Lanes whose source falls outside the
// row keep `old`.
// The result is pinned where it is computed: a DPP move sunk into a divergent branch would read
// source lanes that EXEC has switched off there (and get `old`).
template <int CTRL>
__device__ __forceinline__ int32_t dpp(int32_t old, int32_t x) {
    int32_t r = (int32_t)__builtin_amdgcn_update_dpp((uint32_t)old, (uint32_t)x, CTRL, 0xf, 0xf, false);
    asm volatile("" : "+v"(r));
    return r;
}

// Partner value of the disjoint-sparse-table build at level m (group of 2^m lanes): a lane in
// the left half of its group reads the group's last lane, a lane in the right half its first.
template <int M>
__device__ __forceinline__ int32_t dst_partner(int32_t x, int lane) {
    if constexpr (M == 1) {
        return dpp<0xB1>(0, x);                                   // quad_perm [1 0 3 2]
    } else if constexpr (M == 2) {
        return dpp<0x0F>(0, x);                                   // quad_perm [3 3 0 0]
    } else if constexpr (M == 3) {
        const int32_t hm = dpp<0x141>(0, x);                      // i <-> 7 - i
        const int32_t q3 = dpp<0xFF>(0, hm), q0 = dpp<0x00>(0, hm);  // quad lane 3 / quad lane 0
        return (lane & 4) ? q3 : q0;
    } else if constexpr (M == 4) {
        const int32_t r0 = dpp<0x150>(0, x), r15 = dpp<0x15F>(0, x);  // row lane 0 / row lane 15
        return (lane & 8) ? r0 : r15;
    } else {
        static_assert(M == 5, "six levels for 64-lane tiles");
        const int32_t l0 = (int32_t)__builtin_amdgcn_readlane((uint32_t)x, 0);
        const int32_t l31 = (int32_t)__builtin_amdgcn_readlane((uint32_t)x, 31);
        const int32_t l32 = (int32_t)__builtin_amdgcn_readlane((uint32_t)x, 32);
        const int32_t l63 = (int32_t)__builtin_amdgcn_readlane((uint32_t)x, 63);
        return (lane & 16) ? ((lane & 32) ? l32 : l0) : ((lane & 32) ? l63 : l31);
    }
}

// The Agg of the level-M partner lane (dst_partner).
template <int M, bool LDSX = false>
__device__ __forceinline__ Agg dst_partner_agg(const Agg& a, int lane) {
    if constexpr (LDSX && M >= 3) {
        // one ds_bpermute per field instead of 3-7 DPP / readlane / select VALU: for a table
        // built as a task off the pipeline's critical path, issue slots count, not latency
        constexpr int half = 1 << (M - 1), grp = 1 << M;
        const int src = (lane & half) ? (lane & ~(grp - 1)) : (lane | (grp - 1));
        return Agg{__builtin_amdgcn_ds_bpermute(src << 2, a.mx), __builtin_amdgcn_ds_bpermute(src << 2, a.mn),
                   __builtin_amdgcn_ds_bpermute(src << 2, a.dd), __builtin_amdgcn_ds_bpermute(src << 2, a.du)};
    }
    return Agg{dst_partner<M>(a.mx, lane), dst_partner<M>(a.mn, lane), dst_partner<M>(a.dd, lane),
               dst_partner<M>(a.du, lane)};
}

// Disjoint sparse table of one 64-bar tile, one whole wave (lane = bar, c = its close): level 0
// the bar itself; level m = 1..5 the aggregate from the bar to the end of its half of the
// aligned 2^(m+1) block (left halves) or from the half's start to the bar (right halves).
// Doubling: at level m a lane in the left half of its 2^m group merges the right half (exposed
// as the group's last lane's prefix) into its suffix S, a right-half lane the left half (the
// first lane's suffix) into its prefix Pp; partners move by DPP / readlane, no LDS round trip.
template <bool LDSX = false>
__device__ __forceinline__ void dst_build(int32_t c, int lane, Agg* D) {
    if (LDSX) asm volatile("" : "+v"(lane));  // the partner addresses are not hoisted and kept live
    Agg S = agg_one(c), Pp = S;
    D[(kDstLevels - 1) * kTile + lane] = S;  // level 0: the last row (dst_row)
    auto level = [&](auto mtag) {
        constexpr int m = decltype(mtag)::value;
        const bool left = (lane & (1 << (m - 1))) == 0;
        const Agg part = dst_partner_agg<m, LDSX>(agg_sel(left, S, Pp), lane);
        S = agg_sel(left, agg_merge(S, part), S);
        Pp = agg_sel(left, Pp, agg_merge(part, Pp));
        D[(kDstLevels - 1 - m) * kTile + lane] = agg_sel(((lane >> m) & 1) != 0, Pp, S);
    };
    level(std::integral_constant<int, 1>{});
    level(std::integral_constant<int, 2>{});
    level(std::integral_constant<int, 3>{});
    level(std::integral_constant<int, 4>{});
    level(std::integral_constant<int, 5>{});
    static_assert(kDstLevels == 6, "levels 1..5 above");
}

// Value of lane 63 as a wave-uniform (SGPR) int64.
__device__ __forceinline__ int64_t lane63_i64(int64_t x) {
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)x, 63);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)((uint64_t)x >> 32), 63);
    return (int64_t)(((uint64_t)hi << 32) | lo);
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
