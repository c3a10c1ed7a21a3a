// internal.h — layouts shared by the host engine (engine.cpp) and the HIP kernels (k_*.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "../../include/bt.h"

// Profiling switches (phase ablation, s_memtime stamps, launch-shape overrides from the
// environment) exist only in the profiling build (`make PROFILING=1` -> libbt_prof.so). In the
// release libbt.so BT_ABL is the constant false: no environment variable can change a result.
#ifdef BT_PROFILING
#define BT_ABL(g, bit) (((g).ablate & (bit)) != 0)
// wave priority override (tuning aid): bit 20 set -> 2-bit field at `shift` replaces `dflt`
#define BT_PRIO(g, shift, dflt) (BT_ABL(g, 1 << 20) ? (((g).ablate >> (shift)) & 3) : (dflt))
#else
#define BT_ABL(g, bit) false
#define BT_PRIO(g, shift, dflt) (dflt)
#endif
// profiling stamps: slots [0, 80) role cycles, then where each of the first kDbgBlocks blocks'
// first 8 waves ran (HW_ID | XCC_ID << 32 | 1 << 40)
constexpr int kDbgSlots = 80, kDbgBlocks = 1024;

namespace bt {

constexpr int kTile = 64;          // bars per LDS tile (one bit per bar in a 64-bit word)
constexpr int kRowAlign = 64;      // symbol rows start on 64-element boundaries in HBM

// One symbol of the HBM-resident dataset: rows of int32 ticks at `off` in every column.
struct SymDesc {
    int64_t off;
    int32_t bars;
    int32_t id;                    // global symbol id (top-k tie-break, shard-independent)
};

// Device-side view of the parameter grid (copied once per engine).
struct Grid {
    int32_t strategy;
    int32_t n_params;
    int32_t na, nb, nc, nd;        // axis sizes (SMA: fast, slow; EMA: span, ols; BOLL: w,k,sl,tp)
    int32_t band_bps, k_den;
    int32_t wmax;                  // largest window of the grid (prefix ring sizing)
    int32_t ring;                  // prefix ring length >= wmax + 3 kTile (SMA: a power of two;
                                   // tile kernels: a multiple of kTile)
    double sqrt_ann;               // sqrt((double)annualization), computed on the host
    double kn2[8];                 // Bollinger: k_num^2 of the first 8 k values (kernel arguments,
                                   // so the z tests read them from scalar registers)
    int32_t kmin_idx;              // Bollinger: index of the smallest k_num (the busiest lanes)
    int32_t ablate;               // BT_PROFILING builds only (env BT_ABLATE): phases to skip;
                                   // always 0 in the release library (read through BT_ABL)
    const int32_t* a;              // device arrays
    const int32_t* b;
    const int32_t* c;
    const int32_t* d;
};

// Outputs of one run (device pointers).
struct Out {
    bt_summary* sum;               // [S * P]
    uint64_t* key;                 // [S * P] top-k order key (orderable sharpe)
    bt_sums* sums;                 // [S * P] parity mode, else nullptr
    bt_trade* trades;              // [S * P * trade_cap] parity mode, else nullptr
    int32_t trade_cap;
    unsigned long long* n_trades;  // total trades (one atomic per block)
    unsigned long long* dbg;       // profiling stamps (Grid::ablate & 64), else nullptr
};

// Bar-axis split of the tile kernels (k_tile.hip): each symbol's tiles are cut into G
// segments walked by separate workgroups. Segment s >= 1 starts flat `burn_tiles` tiles before
// its first bar (a walk whose accounting is discarded) and records the state it reached there;
// a fix pass per boundary re-walks a segment from the true state (the previous segment's end)
// if any lane's state differs, and a combine pass folds the segments' additive sums and
// max-plus drawdown forms into the summaries. One record per (segment, symbol, param), in
// result param order: rec[(s * n_sym + sym) * P + p].
struct SegRec {
    int32_t ntr, expo;
    int32_t start_pos, start_e;    // state at the segment's first accounted bar
    int32_t end_pos, end_e, end_ce, pad;
    int32_t end_agg[4];            // Agg of the open trade's path at the segment end
    int64_t R;                     // realized pnl of trades closed in the segment
    int64_t A, B, C, D;            // drawdown as functions of the entering gap g and mdd m:
                                   // gap' = max(g + A, B), mdd' = max(m, g + C, D)
    uint64_t h;                    // additive trade hash
    uint64_t s1lo;
    int64_t s1hi;
    uint64_t s2lo;
    int64_t s2hi;
};
static_assert(sizeof(SegRec) == 128, "SegRec layout");
// SMA bar segments (k_sma.hip): an SMA position is held from one crossover to the next, often
// for thousands of bars, so a segment cannot burn in to the entry of the trade open at its start.
// That trade is carried symbolically: the segment records where and at what price it closes
// and its path from the segment start, and the combine pass, which knows the entry from the
// earlier segments, closes it. One 128-B line per (segment, symbol, param), written whole by its
// lane (a full-line store; the combine reads it back once). The drawdown form A is -R (not
// stored) and the Sharpe sums' high words fit int32 (|S| < 2^78, spec §3).
struct SmaSegRec {
    int32_t ntr;                   // trades closed in the segment (the carried one included)
    int32_t e0;                    // first entry from flat in the segment (-1: none)
    int32_t start_pos, end_pos;    // position entering the first accounted bar / after the last
    int32_t end_e, end_ce;         // trade open at the end, opened in the segment (end_e = -1:
                                   // the carried trade is still open: entry unknown here)
    int32_t x1, px1;               // the carried trade's exit bar (-1: still open) and fill
    int32_t agg1[4];               // its path from the segment start to x1 (or to the end)
    int32_t end_agg[4];            // path of the trade open at the end, from its entry
    int64_t R;                     // pnl of the other trades closed in the segment (A = -R)
    int64_t B, C, D;               // their drawdown forms (SegRec)
    uint64_t h;                    // their additive hash
    uint64_t s1lo, s2lo;
    int32_t s1hi, s2hi;
};
static_assert(sizeof(SmaSegRec) == sizeof(SegRec), "SmaSegRec is one 128-B SegRec slot");
struct SegArgs {
    SegRec* rec;
    // SMA: the positions entering and leaving every (segment, symbol, param), int8 planes
    // [start | end] of G x S x P each: the fix pass compares them without touching the records
    int8_t* pos;
    unsigned long long* refixed;   // fix-pass blocks that re-walked their segment
    double* ema;                   // EMA+OLS: per (segment, symbol) the chains' values entering
                                   // the segment [0, 64) and leaving it [64, 128), lane = span
    int32_t G;                     // segments per symbol (1 = no split)
    int32_t burn_tiles;            // tiles walked before a speculative segment's first bar
};
constexpr int kDefaultBurnTiles = 64;
constexpr int kEmaSegStride = 128;  // doubles per (segment, symbol) in SegArgs::ema
// Launchers (k_*.hip). All enqueue on `st` and return hipError_t.
hipError_t launch_gen(const SymDesc* syms, int32_t n_sym, uint64_t seed, int32_t freq,
                      int32_t* o, int32_t* h, int32_t* l, int32_t* c, hipStream_t st);
size_t sma_lds_bytes(const Grid& g);  // dynamic LDS of the SMA kernel for this grid
struct SmaShape {                     // SMA launch shape for P parameters (k_sma.hip)
    int pw;                           // parameter waves per block
    int dedicated;                    // 1: an extra helper wave runs the tile scan
    int block, gy;                    // threads per block, y-blocks per symbol
};
SmaShape sma_shape(int P);
hipError_t launch_sma(const SymDesc* syms, int32_t n_sym, const int32_t* close, const Grid& g,
                      const Out& out, bool parity, const SegArgs& seg, hipStream_t st);
// SMA segments for this shard (auto mode) and the default burn-in (k_sma.hip)
int32_t sma_auto_segments(int32_t n_sym, int32_t n_params, int32_t max_bars, int32_t wmax,
                          int32_t burn_tiles);
constexpr int kSmaBurnTiles = 2;
int device_cus();  // compute units of the current device
// dynamic LDS of the EMA+OLS tile kernel with ts tiles per stage, and the ts an unsplit launch uses
size_t ema_lds_bytes(const Grid& g, int ts);
int ema_stage_tiles(const Grid& g);
size_t boll_lds_bytes(const Grid& g);  // dynamic LDS of the Bollinger tile kernel
hipError_t launch_ema_ols(const SymDesc* syms, int32_t n_sym, const int32_t* close, const Grid& g,
                          const Out& out, bool parity, const SegArgs& seg, hipStream_t st);
// EMA+OLS segments: count for this shard (auto mode) and the burn-in a speculative segment needs
// for every span's fp64 chain to meet the true one bit for bit (~16 spans of bars measured).
int32_t ema_auto_segments(int32_t n_sym, int32_t n_params, int32_t max_bars, int32_t burn_tiles);
int32_t ema_burn_tiles(int32_t max_span);
hipError_t launch_boll(const SymDesc* syms, int32_t n_sym, const int32_t* high, const int32_t* low,
                       const int32_t* close, const Grid& g, const Out& out, bool parity,
                       const SegArgs& seg, hipStream_t st);
// Segments per symbol the Bollinger launcher would choose for this shard (auto mode).
int32_t boll_auto_segments(int32_t n_sym, int32_t n_params, int32_t max_bars);

// Top-k by radix select over `key` (k_topk.hip): device-side finish into `out`.
constexpr int kTopkCap = 2048;      // candidates sorted in LDS by the finish kernel
constexpr int kTopkMax = 1024;      // largest k the engine accepts
struct TopkWork {
    unsigned int* hist;            // [4096]
    unsigned long long* state;     // [4]: prefix, decided-bit mask, remaining need
    unsigned int* counts;          // [2]: above, candidates
    unsigned long long* above;     // [cap]
    unsigned long long* cand;      // [cap]
    int cap;
    bt_topk_rec* out;              // [k]
    int32_t* out_n;                // [1]: records written, -1 = overflow (host finishes)
};
hipError_t launch_topk(const uint64_t* key, const bt_summary* sum, const SymDesc* syms,
                       int64_t n, int32_t P, int32_t k, const TopkWork& w, hipStream_t st, bool lds_free_hist = false);
hipError_t launch_topk_init(const TopkWork& w, hipStream_t st);  // once per buffer allocation

// Host-side pieces shared by engine.cpp and comm.cpp.
void set_last_error(const std::string& s);  // bt_last_error() of this thread
inline bool topk_less(const bt_topk_rec& a, const bt_topk_rec& b);  // "a ranks before b"
struct ExchangeView {
    hipStream_t tstream;
    int32_t device, topk;
    const bt_topk_rec* d_top;            // [0] = header (record count), then topk records
    const unsigned long long* d_ntr;     // trades of the last run
    int64_t bar_evals;
};
bool engine_exchange_view(bt_engine* e, ExchangeView& v, std::string& err);
void engine_exchange_enqueued(bt_engine* e);

// Shared host/device helpers.
__host__ __device__ inline uint64_t order_key(double x) {
    union { double d; uint64_t u; } v;
    v.d = x;
    return (v.u >> 63) ? ~v.u : (v.u | 0x8000000000000000ULL);
}

// int128 (lo, hi) -> double, round to nearest, ties to even (spec §4 conversion).
__host__ __device__ inline double i128_to_double(uint64_t lo, int64_t hi) {
    const bool neg = hi < 0;
    uint64_t mh = (uint64_t)hi, ml = lo;
    if (neg) {  // two's complement negate
        ml = ~ml + 1;
        mh = ~mh + (ml == 0 ? 1 : 0);
    }
    if (mh == 0 && ml == 0) return 0.0;
    int lz = mh ? __builtin_clzll(mh) : 64 + __builtin_clzll(ml);
    // normalise: leading one to bit 127
    uint64_t nh, nl;
    if (lz >= 64) {
        nh = ml << (lz - 64);
        nl = 0;
    } else if (lz == 0) {
        nh = mh;
        nl = ml;
    } else {
        nh = (mh << lz) | (ml >> (64 - lz));
        nl = ml << lz;
    }
    // top 53 bits = nh >> 11; remainder = low 11 bits of nh and all of nl
    uint64_t mant = nh >> 11;
    const uint64_t rem_hi = nh & 0x7FFULL;  // 11 bits
    const uint64_t half = 0x400ULL;
    bool up;
    if (rem_hi > half) up = true;
    else if (rem_hi < half) up = false;
    else up = (nl != 0) || (mant & 1);
    mant += up ? 1 : 0;
    // value = mant * 2^(127 - lz - 52)
    double r = (double)mant;  // exact: mant <= 2^53
#ifdef __HIP_DEVICE_COMPILE__
    r = ldexp(r, 75 - lz);
#else
    r = __builtin_ldexp(r, 75 - lz);
#endif
    return neg ? -r : r;
}

inline bool topk_less(const bt_topk_rec& a, const bt_topk_rec& b) {
    const uint64_t ka = order_key(a.sharpe), kb = order_key(b.sharpe);
    if (ka != kb) return ka > kb;
    if (a.sym != b.sym) return a.sym < b.sym;
    return a.param < b.param;
}

__host__ __device__ inline double sharpe_fx(uint64_t s1lo, int64_t s1hi, uint64_t s2lo,
                                            int64_t s2hi, int32_t bars, double sqrt_ann) {
    if (bars < 2) return 0.0;
    const double n = (double)(bars - 1);
    const double m = ldexp(i128_to_double(s1lo, s1hi), -56) / n;
    const double mm = m * m;
    const double v = ldexp(i128_to_double(s2lo, s2hi), -56) / n - mm;
    return v > 0 ? (m / sqrt(v)) * sqrt_ann : 0.0;
}

}  // namespace bt
