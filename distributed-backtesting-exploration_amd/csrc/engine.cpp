// engine.cpp — the C ABI of include/bt.h: engine lifecycle, HBM-resident datasets, the
// JobsReply batch entry point (drop-in for process_incoming_job,
// /root/reference/src/worker/process.rs:13-29) and result serialisation.
//
// Nothing here computes a backtest on the CPU: every result comes from the HIP kernels in
// k_*.hip. The host parses CSV bytes (ingest), moves bars to HBM, launches, and formats
// CompleteRequest.data strings (/root/reference/proto/backtesting.proto:29-32).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <charconv>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <string>
#include <thread>
#include <vector>

#include "csv.h"
#include "internal.h"

using namespace bt;

namespace {

thread_local std::string g_err;

void set_err(const std::string& s) { g_err = s; }

struct HipFail {
    std::string msg;
};

#define HIPCHK(x)                                                                              \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess)                                                                  \
            throw HipFail{std::string(#x) + ": " + hipGetErrorString(e_)};                     \
    } while (0)

template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    void ensure(size_t want) {
        if (want <= n && p) return;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        if (want == 0) return;
        HIPCHK(hipMalloc(&p, want * sizeof(T)));
        n = want;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
};

uint32_t next_pow2(uint32_t x) {
    uint32_t r = 1;
    while (r < x) r <<= 1;
    return r;
}

}  // namespace

void bt::set_last_error(const std::string& s) { set_err(s); }

constexpr int64_t kNtrRing = 64;  // per-run trade counter slots (bt_engine::d_ntr_ring)

struct bt_engine {
    bt_config cfg{};
    std::vector<int32_t> ax[4];  // owned copies of the grid axes
    Grid grid{};
    int32_t P = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    DevBuf<int32_t> d_axes[4];
    // dataset
    std::vector<SymDesc> syms;
    int64_t rows = 0;
    DevBuf<SymDesc> d_syms;
    DevBuf<int32_t> d_c, d_h, d_l;
    // outputs, double-buffered: run i writes buffer i % 2 while the top-k chain of run i-1
    // (on tstream) still reads the other one; `cur` is the buffer of the last run
    DevBuf<bt_summary> d_sum[2];
    DevBuf<uint64_t> d_key[2];
    // per-run trade counters: a ring of kNtrRing slots, run r accumulating into slot
    // r % kNtrRing; half the ring is zeroed every kNtrRing / 2 runs (slots last used >= 33 runs
    // earlier), so a run enqueues no memset of its own. ntr[b]: the slot of the last run that
    // wrote output buffer b
    DevBuf<unsigned long long> d_ntr_ring;
    unsigned long long* ntr[2] = {nullptr, nullptr};
    int cur = 0;
    int64_t nrun = 0;
    DevBuf<bt_sums> d_sums;
    DevBuf<bt_trade> d_trades;
    // Bollinger bar segments (k_tile.hip): requested count (0 = auto, 1 = off), burn-in tiles,
    // the records of a split run and the count the last run used
    int32_t seg_req = 0, seg_burn = kDefaultBurnTiles, seg_last = 1;
    bool seg_burn_set = false;
    DevBuf<SegRec> d_seg;
    DevBuf<double> d_segema;
    DevBuf<unsigned long long> d_refixed;
    DevBuf<unsigned long long> d_dbg;
    // top-k chain stream: the chain of run i overlaps the kernel of run i+1
    hipStream_t tstream = nullptr;
    hipEvent_t ev_kdone = nullptr;          // kernel of the last run finished (main stream)
    hipEvent_t ev_tdone[2] = {nullptr, nullptr};  // readers of buffer b finished (tstream)
    bool tdone_armed[2] = {false, false};
    // top-k work
    DevBuf<unsigned int> d_hist, d_counts;
    DevBuf<unsigned long long> d_state, d_above, d_cand;
    DevBuf<bt_topk_rec> d_top;
    bt_topk_rec* h_top = nullptr;     // pinned host copy of d_top
    // pipelined read-back slots: header + kTopkMax records + one record holding the trade count
    bt_topk_rec* h_slot[BT_PIPE_SLOTS] = {};
    hipEvent_t slot_ev[BT_PIPE_SLOTS] = {};
    bool slot_armed[BT_PIPE_SLOTS] = {};
    bool topk_ready = false;          // top-k buffers allocated and their state initialised
    bool ran = false;
    // timing of the dominant kernel
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pending, ev_pool;
    double kernel_ms = 0.0;
    int64_t launches = 0;
    // bt_run_batch: pinned host staging of the columns in device row layout (c, h, l), the
    // batch's summaries read back in one copy, phase events and the last batch's profile
    int32_t* h_stage[3] = {nullptr, nullptr, nullptr};
    size_t stage_rows[3] = {0, 0, 0};
    bt_summary* h_sum = nullptr;
    size_t h_sum_n = 0;
    hipEvent_t ev_batch[4] = {nullptr, nullptr, nullptr, nullptr};
    bt_batch_profile prof{};
    int64_t n_errors = 0;
};

namespace {

void activate(bt_engine* e) { HIPCHK(hipSetDevice(e->cfg.device)); }

bool has_hl(const bt_engine* e) { return e->cfg.strategy == BT_BOLL; }

const char* kernel_name(int32_t strategy) {
    switch (strategy) {
        case BT_SMA_CROSS: return "bt::sma_kernel";
        case BT_EMA_OLS: return "bt::ema_tile_kernel";
        default: return "bt::boll_tile_kernel";
    }
}

std::string validate_and_copy(bt_engine* e, const bt_config& c) {
    auto copy_axis = [&](int slot, const int32_t* src, int32_t n, const char* what, int32_t lo,
                         int32_t hi) -> std::string {
        if (n <= 0 || src == nullptr) return std::string("empty axis: ") + what;
        e->ax[slot].assign(src, src + n);
        for (int32_t v : e->ax[slot])
            if (v < lo || v > hi)
                return std::string("value out of range on axis ") + what + ": " + std::to_string(v);
        return "";
    };
    std::string err;
    e->grid.strategy = c.strategy;
    switch (c.strategy) {
        case BT_SMA_CROSS: {
            if (!(err = copy_axis(0, c.fast, c.n_fast, "fast", 1, kMaxBars)).empty()) return err;
            if (!(err = copy_axis(1, c.slow, c.n_slow, "slow", 1, kMaxBars)).empty()) return err;
            const int64_t mf = *std::max_element(e->ax[0].begin(), e->ax[0].end());
            const int64_t ms = *std::max_element(e->ax[1].begin(), e->ax[1].end());
            e->grid.na = c.n_fast;
            e->grid.nb = c.n_slow;
            e->grid.nc = e->grid.nd = 1;
            e->grid.wmax = (int32_t)std::max(mf, ms);
            // prefix ring: windows + three tiles in flight (k_sma.hip pipeline)
            e->grid.ring = (int32_t)next_pow2((uint32_t)e->grid.wmax + 3 * kTile);
            const size_t lds = sma_lds_bytes(e->grid);
            if (lds > 160 * 1024) return "SMA grid needs more LDS than a CU has (windows too long)";
            break;
        }
        case BT_EMA_OLS: {
            if (!(err = copy_axis(0, c.span, c.n_span, "span", 1, kMaxBars)).empty()) return err;
            if (!(err = copy_axis(1, c.ols, c.n_ols, "ols", 1, 1 << 16)).empty()) return err;
            if (c.band_bps < 0 || c.band_bps >= 10000) return "band_bps out of range";
            if (c.n_span > 64) return "EMA grid: at most 64 spans (one helper lane per span)";
            e->grid.na = c.n_span;
            e->grid.nb = c.n_ols;
            e->grid.nc = e->grid.nd = 1;
            e->grid.band_bps = c.band_bps;
            e->grid.wmax = *std::max_element(e->ax[1].begin(), e->ax[1].end());
            // prefix ring, a multiple of the tile (k_tile.hip): a window back from the stage
            // being flagged, which ends two 128-bar stages before the last scanned bar
            e->grid.ring = (e->grid.wmax + 5 * kTile - 1) / kTile * kTile;
            if (ema_lds_bytes(e->grid, 1) > 160 * 1024) return "EMA grid needs more LDS than a CU has (OLS windows too long)";
            break;
        }
        case BT_BOLL: {
            if (!(err = copy_axis(0, c.bwin, c.n_bwin, "bwin", 1, 1 << 16)).empty()) return err;
            if (!(err = copy_axis(1, c.k_num, c.n_k, "k_num", 0, 1 << 20)).empty()) return err;
            if (!(err = copy_axis(2, c.sl_bps, c.n_sl, "sl_bps", 0, 9999)).empty()) return err;
            if (!(err = copy_axis(3, c.tp_bps, c.n_tp, "tp_bps", 0, 9999)).empty()) return err;
            if (c.k_den < 1 || c.k_den > (1 << 20)) return "k_den out of range";
            e->grid.na = c.n_bwin;
            e->grid.nb = c.n_k;
            e->grid.nc = c.n_sl;
            e->grid.nd = c.n_tp;
            e->grid.k_den = c.k_den;
            e->grid.wmax = *std::max_element(e->ax[0].begin(), e->ax[0].end());
            // z tests D^2 kd^2 vs kn^2 Q with D^2, Q < w^2 2^62: exact in int128 while
            // w * max(k_num, k_den) < 2^32 (spec §4, oracle/oracle.c orc_boll)
            const int64_t kmax = std::max<int64_t>(c.k_den, *std::max_element(e->ax[1].begin(), e->ax[1].end()));
            if ((int64_t)e->grid.wmax * kmax >= (1LL << 32)) return "Bollinger grid outside the exact int128 range (window * k >= 2^32)";
            e->grid.ring = (e->grid.wmax + 4 * kTile - 1) / kTile * kTile;
            for (int q = 0; q < 8; ++q) {
                const int64_t kn = q < c.n_k ? e->ax[1][q] : 0;
                e->grid.kn2[q] = (double)(kn * kn);  // exact: kn <= 2^20
            }
            e->grid.kmin_idx = (int32_t)(std::min_element(e->ax[1].begin(), e->ax[1].end()) - e->ax[1].begin());
            if (boll_lds_bytes(e->grid) > 160 * 1024) return "Bollinger grid needs more LDS than a CU has (windows too long)";
            break;
        }
        default:
            return "unknown strategy";
    }
    const int64_t P = (int64_t)e->grid.na * e->grid.nb * e->grid.nc * e->grid.nd;
    if (P <= 0 || P > (1 << 20)) return "parameter grid too large";
    e->P = (int32_t)P;
    e->grid.n_params = e->P;
    if (c.annualization <= 0) return "annualization must be positive";
    e->grid.sqrt_ann = std::sqrt((double)c.annualization);
    if (c.topk < 0 || c.topk > kTopkMax) return "topk must be in [0, 1024]";
    if ((c.flags & BT_FLAG_PARITY) && c.trade_cap <= 0) return "parity mode needs trade_cap > 0";
    return "";
}

void upload_grid(bt_engine* e) {
    const int32_t** dst[4] = {&e->grid.a, &e->grid.b, &e->grid.c, &e->grid.d};
    for (int i = 0; i < 4; ++i) {
        *dst[i] = nullptr;
        if (e->ax[i].empty()) continue;
        e->d_axes[i].ensure(e->ax[i].size());
        HIPCHK(hipMemcpy(e->d_axes[i].p, e->ax[i].data(), e->ax[i].size() * 4, hipMemcpyHostToDevice));
        *dst[i] = e->d_axes[i].p;
    }
}

int64_t align_rows(int64_t bars) { return (bars + kRowAlign - 1) / kRowAlign * kRowAlign; }

void sync_all(bt_engine* e);

// Install a dataset: symbol descriptors (row offsets into the columns) and `rows` rows per
// column; allocates the columns the strategy needs.
void set_dataset(bt_engine* e, std::vector<SymDesc>&& syms, int64_t rows) {
    // the previous run's top-k chain (second stream) reads the symbol descriptors (ids of its
    // records), and a column may be reallocated below: both streams drain first (the upload on
    // the engine stream alone would be ordered after the kernel but not after that chain)
    sync_all(e);
    e->syms = std::move(syms);
    e->rows = rows;
    const size_t n_sym = e->syms.size();
    e->d_syms.ensure(std::max<size_t>(1, n_sym));
    if (n_sym)
        HIPCHK(hipMemcpyAsync(e->d_syms.p, e->syms.data(), n_sym * sizeof(SymDesc),
                              hipMemcpyHostToDevice, e->stream));
    const size_t r = std::max<int64_t>(1, rows);
    e->d_c.ensure(r);
    if (has_hl(e)) {
        e->d_h.ensure(r);
        e->d_l.ensure(r);
    }
    e->ran = false;
}

// Lay out rows (64-element aligned) and allocate the columns the strategy needs.
void layout(bt_engine* e, int32_t n_sym, const int32_t* bars, const int64_t* ids) {
    std::vector<SymDesc> syms((size_t)n_sym);
    int64_t off = 0;
    for (int32_t s = 0; s < n_sym; ++s) {
        syms[s].off = off;
        syms[s].bars = bars[s];
        syms[s].id = (int32_t)ids[s];
        off += align_rows(bars[s]);
    }
    set_dataset(e, std::move(syms), off);
}

template <class T>
void ensure_pinned(T*& p, size_t& have, size_t want) {
    if (want <= have && p) return;
    if (p) HIPCHK(hipHostFree(p));
    p = nullptr;
    have = 0;
    HIPCHK(hipHostMalloc(&p, std::max<size_t>(want, 1) * sizeof(T)));
    have = std::max<size_t>(want, 1);
}

TopkWork topk_work(bt_engine* e) {
    return TopkWork{e->d_hist.p, e->d_state.p, e->d_counts.p, e->d_above.p, e->d_cand.p,
                    kTopkCap, e->d_top.p + 1, reinterpret_cast<int32_t*>(e->d_top.p)};
}

void sync_all(bt_engine* e) {
    HIPCHK(hipStreamSynchronize(e->stream));
    if (e->tstream) HIPCHK(hipStreamSynchronize(e->tstream));
}

void ensure_outputs(bt_engine* e) {
    const size_t n = (size_t)e->syms.size() * e->P;
    for (int b = 0; b < 2; ++b) {
        e->d_sum[b].ensure(std::max<size_t>(1, n));
        e->d_key[b].ensure(std::max<size_t>(1, n));
    }
    e->d_ntr_ring.ensure(kNtrRing);
    if (e->cfg.flags & BT_FLAG_PARITY) {
        e->d_sums.ensure(std::max<size_t>(1, n));
        e->d_trades.ensure(std::max<size_t>(1, n * (size_t)e->cfg.trade_cap));
    }
    if (e->cfg.topk > 0 && !e->topk_ready) {
        e->d_hist.ensure(4096);
        e->d_counts.ensure(2);
        e->d_state.ensure(4);
        e->d_above.ensure(kTopkCap);
        e->d_cand.ensure(kTopkCap);
        e->d_top.ensure(kTopkMax + 1);  // [0] = header (record count), then the records
        if (!e->h_top) HIPCHK(hipHostMalloc(&e->h_top, (kTopkMax + 1) * sizeof(bt_topk_rec)));
        HIPCHK(launch_topk_init(topk_work(e), e->stream));
        e->topk_ready = true;
    }
}

void run_impl(bt_engine* e) {
    activate(e);
    ensure_outputs(e);
    const int32_t S = (int32_t)e->syms.size();
    const int64_t run = e->nrun++;
    const int b = (int)(run & 1);
    e->cur = b;
    // buffer b was last read by the top-k chain / read-back of run i-2: wait for them (no wait
    // packet when they have already finished, the steady state of a pipelined sweep)
    if (e->tdone_armed[b] && hipEventQuery(e->ev_tdone[b]) != hipSuccess)
        HIPCHK(hipStreamWaitEvent(e->stream, e->ev_tdone[b], 0));
    Out out{};
    out.sum = e->d_sum[b].p;
    out.key = e->d_key[b].p;
    const bool parity = (e->cfg.flags & BT_FLAG_PARITY) != 0;
    out.sums = parity ? e->d_sums.p : nullptr;
    out.trades = parity ? e->d_trades.p : nullptr;
    out.trade_cap = parity ? e->cfg.trade_cap : 0;
    const int slot = (int)(run % kNtrRing);
    if (slot % (kNtrRing / 2) == 0)
        HIPCHK(hipMemsetAsync(e->d_ntr_ring.p + slot, 0, (kNtrRing / 2) * sizeof(unsigned long long),
                              e->stream));
    e->ntr[b] = e->d_ntr_ring.p + slot;
    out.n_trades = e->ntr[b];
    out.dbg = nullptr;
    if (BT_ABL(e->grid, 64)) {  // profiling stamps (profiling build only)
        e->d_dbg.ensure(kDbgSlots + 8 * kDbgBlocks);
        HIPCHK(hipMemsetAsync(e->d_dbg.p, 0, (kDbgSlots + 8 * kDbgBlocks) * sizeof(unsigned long long),
                              e->stream));
        out.dbg = e->d_dbg.p;
    }
    const bool timing = (e->cfg.flags & BT_FLAG_TIMING) != 0;
    std::pair<hipEvent_t, hipEvent_t> ev{};
    if (timing) {
        if (!e->ev_pool.empty()) {
            ev = e->ev_pool.back();
            e->ev_pool.pop_back();
        } else {
            HIPCHK(hipEventCreate(&ev.first));
            HIPCHK(hipEventCreate(&ev.second));
        }
        HIPCHK(hipEventRecord(ev.first, e->stream));
    }
    hipError_t err = hipSuccess;
    switch (e->cfg.strategy) {
        case BT_SMA_CROSS: {
            // bar segments (k_sma.hip) for shards of few, long one-block-per-CU symbols
            SegArgs sg{nullptr, nullptr, nullptr, nullptr, 1, e->seg_burn_set ? e->seg_burn : kSmaBurnTiles};
            if (!parity) {
                int32_t maxb = 0;
                for (const SymDesc& sd : e->syms) maxb = std::max(maxb, sd.bars);
                sg.G = e->seg_req > 0 ? e->seg_req
                                      : sma_auto_segments(S, e->P, maxb, e->grid.wmax, sg.burn_tiles);
            }
            if (sg.G > 1) {
                // one SegRec slot per SmaSegRec, then the int8 start / end position planes
                const size_t nrec = (size_t)sg.G * S * e->P;
                e->d_seg.ensure(nrec + (2 * nrec + sizeof(SegRec) - 1) / sizeof(SegRec));
                sg.pos = reinterpret_cast<int8_t*>(e->d_seg.p + nrec);
                e->d_refixed.ensure(1);
                HIPCHK(hipMemsetAsync(e->d_refixed.p, 0, sizeof(unsigned long long), e->stream));
                sg.rec = e->d_seg.p;
                sg.refixed = e->d_refixed.p;
            }
            e->seg_last = sg.G;
            err = launch_sma(e->d_syms.p, S, e->d_c.p, e->grid, out, parity, sg, e->stream);
            break;
        }
        case BT_EMA_OLS: {
            int32_t maxspan = 1, maxb = 0;
            for (int32_t v : e->ax[0]) maxspan = std::max(maxspan, v);
            for (const SymDesc& sd : e->syms) maxb = std::max(maxb, sd.bars);
            // the default burn-in lets every span's chain meet the true one; an explicit one
            // (bt_set_segments) is honoured, the fix pass covering a short one
            const int32_t burn = e->seg_burn_set ? e->seg_burn : ema_burn_tiles(maxspan);
            SegArgs sg{nullptr, nullptr, nullptr, nullptr, 1, burn};
            if (!parity) sg.G = e->seg_req > 0 ? e->seg_req : ema_auto_segments(S, e->P, maxb, burn);
            if (sg.G > 1) {
                e->d_seg.ensure((size_t)sg.G * S * e->P);
                e->d_segema.ensure((size_t)sg.G * S * kEmaSegStride);
                e->d_refixed.ensure(1);
                HIPCHK(hipMemsetAsync(e->d_refixed.p, 0, sizeof(unsigned long long), e->stream));
                sg.rec = e->d_seg.p;
                sg.refixed = e->d_refixed.p;
                sg.ema = e->d_segema.p;
            }
            e->seg_last = sg.G;
            err = launch_ema_ols(e->d_syms.p, S, e->d_c.p, e->grid, out, parity, sg, e->stream);
            break;
        }
        case BT_BOLL: {
            SegArgs sg{nullptr, nullptr, nullptr, nullptr, 1, e->seg_burn};
            if (!parity) {
                int32_t maxb = 0;
                for (const SymDesc& sd : e->syms) maxb = std::max(maxb, sd.bars);
                sg.G = e->seg_req > 0 ? e->seg_req : boll_auto_segments(S, e->P, maxb);
            }
            if (sg.G > 1) {
                e->d_seg.ensure((size_t)sg.G * S * e->P);
                e->d_refixed.ensure(1);
                HIPCHK(hipMemsetAsync(e->d_refixed.p, 0, sizeof(unsigned long long), e->stream));
                sg.rec = e->d_seg.p;
                sg.refixed = e->d_refixed.p;
            }
            e->seg_last = sg.G;
            err = launch_boll(e->d_syms.p, S, e->d_h.p, e->d_l.p, e->d_c.p, e->grid, out, parity,
                              sg, e->stream);
            break;
        }
    }
    HIPCHK(err);
    if (timing) {
        HIPCHK(hipEventRecord(ev.second, e->stream));
        e->ev_pending.push_back(ev);
    }
    if (e->cfg.topk > 0) {
        // the chain waits for the kernel: on the timing end event when there is one (one
        // marker less between two runs' kernels)
        if (!timing) HIPCHK(hipEventRecord(e->ev_kdone, e->stream));
        HIPCHK(hipStreamWaitEvent(e->tstream, timing ? ev.second : e->ev_kdone, 0));
        // the chain's histograms take no LDS beside a strategy kernel whose blocks fill a CU's
        // (EMA+OLS in 128-bar stages: k_topk.hip topk_hist_global)
        const bool lds_free = e->grid.strategy == BT_EMA_OLS && ema_stage_tiles(e->grid) == 2;
        HIPCHK(launch_topk(e->d_key[b].p, e->d_sum[b].p, e->d_syms.p, (int64_t)S * e->P, e->P,
                           e->cfg.topk, topk_work(e), e->tstream, lds_free));
        HIPCHK(hipEventRecord(e->ev_tdone[b], e->tstream));
        e->tdone_armed[b] = true;
    }
    e->ran = true;
}

void drain_timing(bt_engine* e) {
    for (auto& ev : e->ev_pending) {
        HIPCHK(hipEventSynchronize(ev.second));
        float ms = 0.f;
        HIPCHK(hipEventElapsedTime(&ms, ev.first, ev.second));
        e->kernel_ms += ms;
        e->launches += 1;
        e->ev_pool.push_back(ev);
    }
    e->ev_pending.clear();
}


std::vector<bt_topk_rec> read_topk_impl(bt_engine* e, int32_t k) {
    if (!e->ran || e->cfg.topk <= 0) throw HipFail{"top-k not computed (topk == 0 or no run)"};
    // header + the configured k records in one copy into pinned memory
    const size_t nrec = (size_t)e->cfg.topk + 1;
    HIPCHK(hipMemcpyAsync(e->h_top, e->d_top.p, nrec * sizeof(bt_topk_rec), hipMemcpyDeviceToHost,
                          e->tstream));
    sync_all(e);
    int32_t n = 0;
    memcpy(&n, e->h_top, sizeof n);
    // the device selection is complete whatever the ties (k_topk.hip topk_finish_ties)
    if (n < 0 || n > e->cfg.topk) throw HipFail{"device top-k returned a bad record count"};
    std::vector<bt_topk_rec> res(e->h_top + 1, e->h_top + 1 + n);
    if ((int32_t)res.size() > k) res.resize(k);
    return res;
}

// One CompleteRequest.data line (spec §6). std::to_chars gives printf's "%.17g" (general
// format, precision 17) and plain decimal integers without the locale and format-string work of
// snprintf; tests/test_abi_cpu.py checks the bytes against Python's "%.17g" / "%016x".
char* put_lit(char* q, const char* s) {
    while (*s) *q++ = *s++;
    return q;
}

char* fmt_line(char* q, int32_t p, const bt_summary& x) {
    static const char kHex[] = "0123456789abcdef";
    q = put_lit(q, "{\"param\":");
    q = std::to_chars(q, q + 16, p).ptr;
    q = put_lit(q, ",\"n\":");
    q = std::to_chars(q, q + 16, x.n_trades).ptr;
    q = put_lit(q, ",\"pnl\":");
    q = std::to_chars(q, q + 24, (long long)x.pnl).ptr;
    q = put_lit(q, ",\"mdd\":");
    q = std::to_chars(q, q + 24, (long long)x.mdd).ptr;
    q = put_lit(q, ",\"exp\":");
    q = std::to_chars(q, q + 24, (long long)x.exposure).ptr;
    q = put_lit(q, ",\"sharpe\":\"");
    q = std::to_chars(q, q + 32, x.sharpe, std::chars_format::general, 17).ptr;
    q = put_lit(q, "\",\"h\":\"");
    for (int i = 15; i >= 0; --i) *q++ = kHex[(x.hash >> (4 * i)) & 15];
    return put_lit(q, "\"}\n");
}

constexpr size_t kLineMax = 192;  // longest line: 10 + 11 + 20 x 3 + 24 + 16 + fixed text < 192

size_t fmt_job_into(const bt_summary* r, int32_t P, char* out) {
    char* q = out;
    for (int32_t p = 0; p < P; ++p) q = fmt_line(q, p, r[p]);
    return (size_t)(q - out);
}

std::string json_escape(const std::string& in) {
    std::string o;
    for (char ch : in) {
        if (ch == '"' || ch == '\\') {
            o.push_back('\\');
            o.push_back(ch);
        } else if ((unsigned char)ch < 0x20) {
            o.push_back(' ');
        } else {
            o.push_back(ch);
        }
    }
    return o;
}

char* dup_string(const std::string& s) {
    char* p = (char*)malloc(s.size() + 1);
    if (!p) throw std::bad_alloc();
    memcpy(p, s.data(), s.size());
    p[s.size()] = 0;
    return p;
}


// Host threads of the batch ingest: host_threads, else the machine's, at most 16 (the worker's
// share of a GPU box; /root/reference/src/worker/handlers.rs:35 reports num_cpus/2 as cores).
int host_threads(const bt_engine* e, size_t n) {
    int nt = e->cfg.host_threads > 0
                 ? e->cfg.host_threads
                 : (int)std::min<unsigned>(16, std::max(1u, std::thread::hardware_concurrency()));
    return (int)std::min<size_t>((size_t)nt, std::max<size_t>(1, n));
}

// f(i) for i in [0, n) on nt threads (f must not throw).
template <class F>
void parallel_for(int nt, size_t n, const F& f) {
    std::atomic<size_t> next{0};
    auto work = [&]() {
        for (size_t i; (i = next.fetch_add(1)) < n;) f(i);
    };
    if (nt <= 1 || n <= 1) {
        work();
        return;
    }
    std::vector<std::thread> th;
    th.reserve((size_t)nt);
    for (int i = 0; i < nt; ++i) th.emplace_back(work);
    for (auto& t : th) t.join();
}

struct JobSlot {
    bool ok = false, binary = false;
    int32_t bars = 0;
    int64_t row = 0;
    size_t sym = 0;
    Bars parsed;  // CSV jobs only (binary payloads decode straight into the staging rows)
    std::string err;
};

double ms_between(std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
    return std::chrono::duration<double, std::milli>(b - a).count();
}

// The JobsReply as one GPU batch (drop-in for process_incoming_job's loop,
// /root/reference/src/worker/process.rs:21-25):
//   1. per job (host threads): binary payloads -> bar count from the header; CSV -> parsed;
//   2. rows of the good jobs laid out 64-aligned in pinned host staging;
//   3. per job (host threads): binary payloads validated and decoded straight into their rows
//      in one pass (decode_binary_into), CSV bars copied in;
//   4. one async H2D per column, the strategy kernel, one D2H of every summary, one wait;
//   5. per job (host threads): the CompleteRequest.data string.
void run_batch_impl(bt_engine* e, size_t n, const bt_job_in* jobs, bt_job_out* outs) {
    using clk = std::chrono::steady_clock;
    const auto t_start = clk::now();
    activate(e);
    sync_all(e);  // staging and h_sum may still be in use by an earlier call
    bt_batch_profile pr{};
    pr.n_jobs = (int64_t)n;
    const int nt = host_threads(e, n);
    const bool hl = has_hl(e);
    std::vector<JobSlot> js(n);
    for (size_t i = 0; i < n; ++i) pr.payload_bytes += (int64_t)jobs[i].len;
    parallel_for(nt, n, [&](size_t i) {
        JobSlot& j = js[i];
        try {
            const uint8_t* buf = jobs[i].file;
            const size_t len = jobs[i].len;
            if (!buf && len) {
                j.err = "null Job.File";
            } else if (buf && is_binary_payload(buf, len)) {
                j.binary = true;
                j.ok = binary_header(buf, len, j.bars, j.err);
            } else {
                j.ok = parse_csv(buf, len, j.parsed, j.err);
                j.bars = (int32_t)j.parsed.c.size();
            }
        } catch (...) {
            j.ok = false;
            j.err = "parse failure";
        }
    });
    int64_t rows = 0;
    for (size_t i = 0; i < n; ++i) {
        JobSlot& j = js[i];
        // what ingest touches: a CSV is parsed whole; a binary payload's header and its four price
        // columns are validated, its volume column is never read
        if (j.ok) pr.payload_bytes_read += j.binary ? (int64_t)binary_payload_size(j.bars, false)
                                                    : (int64_t)jobs[i].len;
        if (j.ok) {
            j.row = rows;
            rows += align_rows(j.bars);
        }
    }
    const int ncol = hl ? 3 : 1;
    for (int k = 0; k < ncol; ++k) ensure_pinned(e->h_stage[k], e->stage_rows[k], (size_t)std::max<int64_t>(rows, 1));
    parallel_for(nt, n, [&](size_t i) {
        JobSlot& j = js[i];
        if (!j.ok) return;
        try {
            int32_t* c = e->h_stage[0] + j.row;
            int32_t* h = hl ? e->h_stage[1] + j.row : nullptr;
            int32_t* l = hl ? e->h_stage[2] + j.row : nullptr;
            if (j.binary) {
                j.ok = decode_binary_into(jobs[i].file, jobs[i].len, h, l, c, j.err);
            } else {
                memcpy(c, j.parsed.c.data(), (size_t)j.bars * 4);
                if (hl) {
                    memcpy(h, j.parsed.h.data(), (size_t)j.bars * 4);
                    memcpy(l, j.parsed.l.data(), (size_t)j.bars * 4);
                }
                j.parsed = Bars();  // release early
            }
        } catch (...) {
            j.ok = false;
            j.err = "ingest failure";
        }
    });
    // a job that failed in step 3 leaves its rows unreferenced
    std::vector<SymDesc> syms;
    e->n_errors = 0;
    for (JobSlot& j : js) {
        if (!j.ok) {
            ++e->n_errors;
            continue;
        }
        j.sym = syms.size();
        syms.push_back(SymDesc{j.row, j.bars, (int32_t)syms.size()});
        pr.bars += j.bars;
    }
    const auto t_staged = clk::now();
    pr.host_ingest_ms = ms_between(t_start, t_staged);
    pr.n_failed = e->n_errors;
    const int32_t P = e->P;
    const size_t nres = syms.size() * (size_t)P;
    if (!syms.empty()) {
        for (hipEvent_t& ev : e->ev_batch)
            if (!ev) HIPCHK(hipEventCreate(&ev));
        ensure_pinned(e->h_sum, e->h_sum_n, nres);
        set_dataset(e, std::move(syms), rows);
        HIPCHK(hipEventRecord(e->ev_batch[0], e->stream));
        int32_t* dst[3] = {e->d_c.p, e->d_h.p, e->d_l.p};
        for (int k = 0; k < ncol; ++k)
            HIPCHK(hipMemcpyAsync(dst[k], e->h_stage[k], (size_t)rows * 4, hipMemcpyHostToDevice,
                                  e->stream));
        HIPCHK(hipEventRecord(e->ev_batch[1], e->stream));
        run_impl(e);
        HIPCHK(hipEventRecord(e->ev_batch[2], e->stream));
        HIPCHK(hipMemcpyAsync(e->h_sum, e->d_sum[e->cur].p, nres * sizeof(bt_summary),
                              hipMemcpyDeviceToHost, e->stream));
        HIPCHK(hipEventRecord(e->ev_batch[3], e->stream));
        sync_all(e);
        float ms = 0.f;
        HIPCHK(hipEventElapsedTime(&ms, e->ev_batch[0], e->ev_batch[1]));
        pr.upload_ms = ms;
        HIPCHK(hipEventElapsedTime(&ms, e->ev_batch[1], e->ev_batch[2]));
        pr.compute_ms = ms;
        HIPCHK(hipEventElapsedTime(&ms, e->ev_batch[2], e->ev_batch[3]));
        pr.readback_ms = ms;
    }
    const auto t_dev = clk::now();
    std::atomic<bool> alloc_fail{false};
    parallel_for(nt, n, [&](size_t i) {
        try {
            const JobSlot& j = js[i];
            if (j.ok) {
                char* buf = (char*)malloc((size_t)P * kLineMax + 1);
                if (!buf) throw std::bad_alloc();
                const size_t len = fmt_job_into(e->h_sum + j.sym * (size_t)P, P, buf);
                buf[len] = 0;
                char* fit = (char*)realloc(buf, len + 1);
                outs[i] = bt_job_out{fit ? fit : buf, len, 0, j.bars};
            } else {
                const std::string m = "{\"error\":\"" + json_escape(j.err) + "\"}\n";
                outs[i] = bt_job_out{dup_string(m), m.size(), -1, 0};
            }
        } catch (...) {
            alloc_fail = true;
        }
    });
    if (alloc_fail) throw std::bad_alloc();
    const auto t_end = clk::now();
    pr.format_ms = ms_between(t_dev, t_end);
    pr.total_ms = ms_between(t_start, t_end);
    e->prof = pr;
}

}  // namespace

// Device sources of the multi-GPU exchange (comm.cpp): the last run's top-k (header record +
// records) and trade counter, on the engine's top-k stream after the run's top-k chain.
bool bt::engine_exchange_view(bt_engine* e, ExchangeView& v, std::string& err) {
    if (!e || !e->ran || e->cfg.topk <= 0 || !e->d_top.p) {
        err = "exchange needs an engine with topk > 0 and a finished bt_run";
        return false;
    }
    v.tstream = e->tstream;
    v.device = e->cfg.device;
    v.topk = e->cfg.topk;
    v.d_top = e->d_top.p;
    v.d_ntr = e->ntr[e->cur];
    v.bar_evals = 0;
    for (const SymDesc& s : e->syms) v.bar_evals += (int64_t)s.bars * e->P;
    return true;
}

// The exchange's copies out of the run's buffers were enqueued on tstream: the next run that
// reuses those buffers waits for them (same bookkeeping as bt_topk_fetch_async).
void bt::engine_exchange_enqueued(bt_engine* e) {
    if (hipEventRecord(e->ev_tdone[e->cur], e->tstream) == hipSuccess) e->tdone_armed[e->cur] = true;
}

namespace {

#define ABI_GUARD(fail, ...)                                   \
    try {                                                      \
        __VA_ARGS__                                            \
    } catch (const HipFail& f) {                               \
        set_err(f.msg);                                        \
        return fail;                                           \
    } catch (const std::exception& x) {                        \
        set_err(std::string("exception: ") + x.what());        \
        return fail;                                           \
    } catch (...) {                                            \
        set_err("unknown exception");                          \
        return fail;                                           \
    }

}  // namespace

extern "C" {

int32_t bt_abi_version(void) { return BT_ABI_VERSION; }

const char* bt_last_error(void) { return g_err.c_str(); }

bt_engine* bt_engine_create(const bt_config* cfg, char* err, size_t errlen) {
    auto fail = [&](const std::string& m) -> bt_engine* {
        set_err(m);
        if (err && errlen) snprintf(err, errlen, "%s", m.c_str());
        return nullptr;
    };
    if (cfg == nullptr) return fail("null config");
    bt_engine* e = nullptr;
    try {
        e = new bt_engine();
        e->cfg = *cfg;
        std::string m = validate_and_copy(e, *cfg);
        if (!m.empty()) {
            delete e;
            return fail(m);
        }
        e->cfg.fast = e->cfg.slow = e->cfg.span = e->cfg.ols = nullptr;
        e->cfg.bwin = e->cfg.k_num = e->cfg.sl_bps = e->cfg.tp_bps = nullptr;
        int ndev = 0;
        HIPCHK(hipGetDeviceCount(&ndev));
        if (cfg->device < 0 || cfg->device >= ndev)
            throw HipFail{"HIP device " + std::to_string(cfg->device) + " not present (" +
                          std::to_string(ndev) + " visible)"};
        activate(e);
        if (cfg->stream) {
            e->stream = (hipStream_t)cfg->stream;
        } else {
            HIPCHK(hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
            e->own_stream = true;
        }
        HIPCHK(hipStreamCreateWithFlags(&e->tstream, hipStreamNonBlocking));
        HIPCHK(hipEventCreateWithFlags(&e->ev_kdone, hipEventDisableTiming));
        for (int b = 0; b < 2; ++b) HIPCHK(hipEventCreateWithFlags(&e->ev_tdone[b], hipEventDisableTiming));
        upload_grid(e);
#ifdef BT_PROFILING
        if (const char* ab = getenv("BT_ABLATE")) e->grid.ablate = atoi(ab);  // profiling build only
#endif
        return e;
    } catch (const HipFail& f) {
        delete e;
        return fail(f.msg);
    } catch (const std::exception& x) {
        delete e;
        return fail(std::string("exception: ") + x.what());
    }
}

void bt_engine_destroy(bt_engine* e) {
    if (!e) return;
    try {
        (void)hipSetDevice(e->cfg.device);
        if (e->stream) (void)hipStreamSynchronize(e->stream);
        if (e->tstream) (void)hipStreamSynchronize(e->tstream);
        for (auto& ev : e->ev_pending) {
            (void)hipEventDestroy(ev.first);
            (void)hipEventDestroy(ev.second);
        }
        for (auto& ev : e->ev_pool) {
            (void)hipEventDestroy(ev.first);
            (void)hipEventDestroy(ev.second);
        }
        for (auto& b : e->d_axes) b.release();
        e->d_syms.release();
        e->d_c.release();
        e->d_h.release();
        e->d_l.release();
        for (int b = 0; b < 2; ++b) {
            e->d_sum[b].release();
            e->d_key[b].release();
            if (e->ev_tdone[b]) (void)hipEventDestroy(e->ev_tdone[b]);
            e->ev_tdone[b] = nullptr;
            e->tdone_armed[b] = false;
        }
        if (e->ev_kdone) (void)hipEventDestroy(e->ev_kdone);
        e->ev_kdone = nullptr;
        e->d_ntr_ring.release();
        e->d_sums.release();
        e->d_trades.release();
        e->d_seg.release();
        e->d_segema.release();
        e->d_refixed.release();
        e->d_dbg.release();
        e->d_hist.release();
        e->d_counts.release();
        e->d_state.release();
        e->d_above.release();
        e->d_cand.release();
        e->d_top.release();
        if (e->h_top) (void)hipHostFree(e->h_top);
        e->h_top = nullptr;
        for (int i = 0; i < BT_PIPE_SLOTS; ++i) {
            if (e->h_slot[i]) (void)hipHostFree(e->h_slot[i]);
            if (e->slot_ev[i]) (void)hipEventDestroy(e->slot_ev[i]);
            e->h_slot[i] = nullptr;
            e->slot_ev[i] = nullptr;
            e->slot_armed[i] = false;
        }
        e->topk_ready = false;
        for (int i = 0; i < 3; ++i)
            if (e->h_stage[i]) (void)hipHostFree(e->h_stage[i]);
        if (e->h_sum) (void)hipHostFree(e->h_sum);
        for (hipEvent_t& ev : e->ev_batch)
            if (ev) (void)hipEventDestroy(ev);
        if (e->own_stream && e->stream) (void)hipStreamDestroy(e->stream);
        if (e->tstream) (void)hipStreamDestroy(e->tstream);
        e->tstream = nullptr;
    } catch (...) {
    }
    delete e;
}

int32_t bt_num_params(const bt_engine* e) { return e ? e->P : -1; }

int32_t bt_set_segments(bt_engine* e, int32_t segments, int32_t burn_tiles) {
    ABI_GUARD(-1, {
        if (!e || segments < 0 || segments > 64 || burn_tiles < 0) throw HipFail{"bad arguments"};
        e->seg_req = segments;
        e->seg_burn = burn_tiles > 0 ? burn_tiles : kDefaultBurnTiles;
        e->seg_burn_set = burn_tiles > 0;
        return 0;
    })
}

int32_t bt_last_segments(bt_engine* e, int64_t* refixed_blocks) {
    ABI_GUARD(-1, {
        if (!e) throw HipFail{"null engine"};
        if (refixed_blocks) {
            unsigned long long n = 0;
            if (e->seg_last > 1 && e->d_refixed.p) {
                activate(e);
                sync_all(e);
                HIPCHK(hipMemcpy(&n, e->d_refixed.p, sizeof n, hipMemcpyDeviceToHost));
            }
            *refixed_blocks = (int64_t)n;
        }
        return e->seg_last;
    })
}

int32_t bt_load_synthetic(bt_engine* e, uint64_t seed, int64_t sym_begin, int32_t n_sym,
                          int32_t n_bars, int32_t freq) {
    ABI_GUARD(-1, {
        if (!e) throw HipFail{"null engine"};
        if (n_sym < 0 || n_bars < 1 || n_bars > kMaxBars) throw HipFail{"bad synthetic shape"};
        if (sym_begin < 0 || sym_begin + n_sym > (1LL << 31)) throw HipFail{"bad symbol ids"};
        if (freq != BT_DAILY && freq != BT_MINUTE) throw HipFail{"bad freq"};
        activate(e);
        std::vector<int32_t> bars(n_sym, n_bars);
        std::vector<int64_t> ids(n_sym);
        for (int32_t s = 0; s < n_sym; ++s) ids[s] = sym_begin + s;
        layout(e, n_sym, bars.data(), ids.data());
        HIPCHK(launch_gen(e->d_syms.p, n_sym, seed, freq, nullptr, has_hl(e) ? e->d_h.p : nullptr,
                          has_hl(e) ? e->d_l.p : nullptr, e->d_c.p, e->stream));
        sync_all(e);
        return 0;
    })
}

int32_t bt_load_ohlc(bt_engine* e, int32_t n_sym, const int64_t* sym_ids, const int32_t* bars,
                     const int64_t* row_off, const int32_t* h, const int32_t* l, const int32_t* c) {
    ABI_GUARD(-1, {
        if (!e || n_sym < 0 || (n_sym > 0 && (!sym_ids || !bars || !row_off || !c)))
            throw HipFail{"bad arguments"};
        if (has_hl(e) && (!h || !l)) throw HipFail{"strategy needs high and low columns"};
        for (int32_t s = 0; s < n_sym; ++s)
            if (bars[s] < 1 || bars[s] > kMaxBars) throw HipFail{"bad bar count"};
        activate(e);
        sync_all(e);  // the pinned staging may still feed an earlier upload
        layout(e, n_sym, bars, sym_ids);
        // stage into pinned host rows with the device row layout, then one async copy per
        // column and a single wait
        const int ncol = has_hl(e) ? 3 : 1;
        const int32_t* src[3] = {c, h, l};
        int32_t* dst[3] = {e->d_c.p, e->d_h.p, e->d_l.p};
        if (e->rows > 0) {
            for (int k = 0; k < ncol; ++k) {
                ensure_pinned(e->h_stage[k], e->stage_rows[k], (size_t)e->rows);
                for (int32_t s = 0; s < n_sym; ++s)
                    memcpy(e->h_stage[k] + e->syms[s].off, src[k] + row_off[s], (size_t)bars[s] * 4);
                HIPCHK(hipMemcpyAsync(dst[k], e->h_stage[k], (size_t)e->rows * 4,
                                      hipMemcpyHostToDevice, e->stream));
            }
            sync_all(e);
        }
        return 0;
    })
}

int32_t bt_run(bt_engine* e) {
    ABI_GUARD(-1, {
        if (!e) throw HipFail{"null engine"};
        run_impl(e);
        return 0;
    })
}

int32_t bt_sync(bt_engine* e) {
    ABI_GUARD(-1, {
        if (!e) throw HipFail{"null engine"};
        activate(e);
        sync_all(e);
        return 0;
    })
}

int32_t bt_read_summaries(bt_engine* e, bt_summary* out, size_t n) {
    ABI_GUARD(-1, {
        if (!e || !e->ran) throw HipFail{"no results"};
        const size_t have = e->syms.size() * (size_t)e->P;
        if (n > have) throw HipFail{"n exceeds symbols x params"};
        activate(e);
        sync_all(e);
        HIPCHK(hipMemcpy(out, e->d_sum[e->cur].p, n * sizeof(bt_summary), hipMemcpyDeviceToHost));
        return 0;
    })
}

int32_t bt_read_sums(bt_engine* e, bt_sums* out, size_t n) {
    ABI_GUARD(-1, {
        if (!e || !e->ran || !(e->cfg.flags & BT_FLAG_PARITY)) throw HipFail{"no parity results"};
        if (n > e->syms.size() * (size_t)e->P) throw HipFail{"n too large"};
        activate(e);
        sync_all(e);
        HIPCHK(hipMemcpy(out, e->d_sums.p, n * sizeof(bt_sums), hipMemcpyDeviceToHost));
        return 0;
    })
}

int32_t bt_read_trades(bt_engine* e, bt_trade* out, size_t n) {
    ABI_GUARD(-1, {
        if (!e || !e->ran || !(e->cfg.flags & BT_FLAG_PARITY)) throw HipFail{"no parity results"};
        if (n > e->syms.size() * (size_t)e->P * e->cfg.trade_cap) throw HipFail{"n too large"};
        activate(e);
        sync_all(e);
        HIPCHK(hipMemcpy(out, e->d_trades.p, n * sizeof(bt_trade), hipMemcpyDeviceToHost));
        return 0;
    })
}

int32_t bt_read_topk(bt_engine* e, bt_topk_rec* out, int32_t k) {
    ABI_GUARD(-1, {
        if (!e || !out || k <= 0) throw HipFail{"bad arguments"};
        activate(e);
        std::vector<bt_topk_rec> r = read_topk_impl(e, std::min(k, e->cfg.topk));
        std::copy(r.begin(), r.end(), out);
        return (int32_t)r.size();
    })
}

int32_t bt_topk_fetch_async(bt_engine* e, int32_t slot) {
    ABI_GUARD(-1, {
        if (!e || slot < 0 || slot >= BT_PIPE_SLOTS) throw HipFail{"bad arguments"};
        if (!e->ran || e->cfg.topk <= 0) throw HipFail{"top-k not computed (topk == 0 or no run)"};
        activate(e);
        if (!e->h_slot[slot])
            HIPCHK(hipHostMalloc(&e->h_slot[slot], (kTopkMax + 2) * sizeof(bt_topk_rec)));
        if (!e->slot_ev[slot]) HIPCHK(hipEventCreateWithFlags(&e->slot_ev[slot], hipEventDisableTiming));
        bt_topk_rec* h = e->h_slot[slot];
        // behind the run's top-k chain on tstream; the trade counter of the run's buffer is
        // complete too (the chain waited for the kernel)
        HIPCHK(hipMemcpyAsync(h, e->d_top.p, ((size_t)e->cfg.topk + 1) * sizeof(bt_topk_rec),
                              hipMemcpyDeviceToHost, e->tstream));
        HIPCHK(hipMemcpyAsync(h + kTopkMax + 1, e->ntr[e->cur], sizeof(unsigned long long),
                              hipMemcpyDeviceToHost, e->tstream));
        HIPCHK(hipEventRecord(e->slot_ev[slot], e->tstream));
        HIPCHK(hipEventRecord(e->ev_tdone[e->cur], e->tstream));  // buffer readers now end here
        e->slot_armed[slot] = true;
        return 0;
    })
}

int32_t bt_topk_fetch_wait(bt_engine* e, int32_t slot, bt_topk_rec* out, int32_t k,
                           int64_t* n_trades) {
    ABI_GUARD(-1, {
        if (!e || slot < 0 || slot >= BT_PIPE_SLOTS || !out || k <= 0) throw HipFail{"bad arguments"};
        if (!e->slot_armed[slot]) throw HipFail{"no fetch pending on this slot"};
        activate(e);
        HIPCHK(hipEventSynchronize(e->slot_ev[slot]));
        const bt_topk_rec* h = e->h_slot[slot];
        int32_t n = 0;
        memcpy(&n, h, sizeof n);
        if (n < 0 || n > e->cfg.topk) throw HipFail{"device top-k returned a bad record count"};
        const int32_t m = std::min(n, std::min(k, e->cfg.topk));
        std::copy(h + 1, h + 1 + m, out);
        if (n_trades) {
            unsigned long long t = 0;
            memcpy(&t, h + kTopkMax + 1, sizeof t);
            *n_trades = (int64_t)t;
        }
        return m;
    })
}

int32_t bt_read_stats(bt_engine* e, bt_stats* out) {
    ABI_GUARD(-1, {
        if (!e || !out) throw HipFail{"bad arguments"};
        activate(e);
        sync_all(e);
        bt_stats st{};
        st.n_symbols = (int64_t)e->syms.size();
        st.n_params = e->P;
        for (const SymDesc& s : e->syms) st.bar_evals += (int64_t)s.bars * e->P;
        st.errors = e->n_errors;
        if (e->ran) {
            unsigned long long n = 0;
            HIPCHK(hipMemcpy(&n, e->ntr[e->cur], sizeof n, hipMemcpyDeviceToHost));
            st.trades = (int64_t)n;
        }
        *out = st;
        return 0;
    })
}

int32_t bt_read_close(bt_engine* e, int32_t sym_index, int32_t* out, int32_t n) {
    ABI_GUARD(-1, {
        if (!e || sym_index < 0 || sym_index >= (int32_t)e->syms.size()) throw HipFail{"bad symbol"};
        const SymDesc& sd = e->syms[sym_index];
        if (n > sd.bars) throw HipFail{"n exceeds bars"};
        activate(e);
        sync_all(e);
        HIPCHK(hipMemcpy(out, e->d_c.p + sd.off, (size_t)n * 4, hipMemcpyDeviceToHost));
        return 0;
    })
}

int32_t bt_read_debug(bt_engine* e, uint64_t* out, int32_t n) {
    ABI_GUARD(-1, {
        if (!e || !out || n < 0 || n > kDbgSlots + 8 * kDbgBlocks || !e->d_dbg.p) throw HipFail{"no debug stamps"};
        activate(e);
        sync_all(e);
        HIPCHK(hipMemcpy(out, e->d_dbg.p, (size_t)n * 8, hipMemcpyDeviceToHost));
        return 0;
    })
}

int32_t bt_kernel_timing(bt_engine* e, double* total_ms, int64_t* launches, const char** name) {
    ABI_GUARD(-1, {
        if (!e) throw HipFail{"null engine"};
        activate(e);
        drain_timing(e);
        if (total_ms) *total_ms = e->kernel_ms;
        if (launches) *launches = e->launches;
        if (name) *name = kernel_name(e->cfg.strategy);
        return 0;
    })
}

int32_t bt_reset_timing(bt_engine* e) {
    ABI_GUARD(-1, {
        if (!e) throw HipFail{"null engine"};
        activate(e);
        drain_timing(e);
        e->kernel_ms = 0.0;
        e->launches = 0;
        return 0;
    })
}

int32_t bt_run_batch(bt_engine* e, size_t n, const bt_job_in* jobs, bt_job_out* outs) {
    ABI_GUARD(-1, {
        if (!e || (n > 0 && (!jobs || !outs))) throw HipFail{"bad arguments"};
        for (size_t i = 0; i < n; ++i) outs[i] = bt_job_out{nullptr, 0, 0, 0};
        try {
            run_batch_impl(e, n, jobs, outs);
        } catch (...) {
            bt_job_out_free(outs, n);  // a failed call leaves no string allocated
            throw;
        }
        return 0;
    })
}

int32_t bt_last_batch_profile(bt_engine* e, bt_batch_profile* out) {
    ABI_GUARD(-1, {
        if (!e || !out) throw HipFail{"bad arguments"};
        *out = e->prof;
        return 0;
    })
}

int64_t bt_format_summaries(const bt_summary* r, int32_t P, char* out, size_t cap) {
    ABI_GUARD(-1, {
        if (P < 0) throw HipFail{"bad arguments"};
        if (!out) return (int64_t)((size_t)P * kLineMax);
        if (P > 0 && !r) throw HipFail{"bad arguments"};
        if (cap < (size_t)P * kLineMax) throw HipFail{"output buffer too small"};
        return (int64_t)fmt_job_into(r, P, out);
    })
}

void bt_job_out_free(bt_job_out* outs, size_t n) {
    if (!outs) return;
    for (size_t i = 0; i < n; ++i) {
        free(outs[i].data);
        outs[i].data = nullptr;
        outs[i].len = 0;
    }
}

int32_t bt_merge_topk(const bt_topk_rec* in, size_t n, int32_t k, bt_topk_rec* out) {
    ABI_GUARD(-1, {
        if ((n > 0 && !in) || !out || k < 0) throw HipFail{"bad arguments"};
        std::vector<bt_topk_rec> v(in, in + n);
        std::sort(v.begin(), v.end(), topk_less);
        const size_t m = std::min<size_t>(v.size(), (size_t)k);
        std::copy(v.begin(), v.begin() + m, out);
        return (int32_t)m;
    })
}

double bt_i128_to_double(uint64_t lo, int64_t hi) { return i128_to_double(lo, hi); }

int32_t bt_parse_csv(const uint8_t* buf, size_t len, int32_t cap, int32_t* h, int32_t* l,
                     int32_t* c, char* err, size_t errlen) {
    return bt_parse_job(buf, len, cap, h, l, c, err, errlen);
}

int64_t bt_encode_columns(const int32_t* o, const int32_t* h, const int32_t* l, const int32_t* c,
                          const int64_t* v, int32_t n, uint8_t* out, size_t cap) {
    ABI_GUARD(-1, {
        if (n < 1 || n > kMaxBars || !o || !h || !l || !c) throw HipFail{"bad arguments"};
        const size_t need = binary_payload_size(n, v != nullptr);
        if (!out) return (int64_t)need;
        if (cap < need) throw HipFail{"output buffer too small"};
        return (int64_t)encode_binary(o, h, l, c, v, n, out);
    })
}

int64_t bt_gen_payload(uint64_t seed, int64_t sym, int32_t bars, int32_t freq, uint8_t* out,
                       size_t cap) {
    ABI_GUARD(-1, {
        if (bars < 1 || bars > kMaxBars || (freq != BT_DAILY && freq != BT_MINUTE))
            throw HipFail{"bad arguments"};
        const size_t need = binary_payload_size(bars, true);
        if (!out) return (int64_t)need;
        if (cap < need) throw HipFail{"output buffer too small"};
        std::vector<int32_t> o((size_t)bars), h((size_t)bars), l((size_t)bars), c((size_t)bars);
        std::vector<int64_t> v((size_t)bars);
        gen_host(seed, sym, bars, freq, o.data(), h.data(), l.data(), c.data(), v.data());
        return (int64_t)encode_binary(o.data(), h.data(), l.data(), c.data(), v.data(), bars, out);
    })
}

int32_t bt_parse_job(const uint8_t* buf, size_t len, int32_t cap, int32_t* h, int32_t* l,
                     int32_t* c, char* err, size_t errlen) {
    ABI_GUARD(-1, {
        Bars b;
        std::string m;
        if (!parse_job(buf, len, b, m)) {
            if (err && errlen) snprintf(err, errlen, "%s", m.c_str());
            set_err(m);
            return -1;
        }
        if ((int64_t)b.c.size() > cap) throw HipFail{"cap too small"};
        if (h) memcpy(h, b.h.data(), b.h.size() * 4);
        if (l) memcpy(l, b.l.data(), b.l.size() * 4);
        if (c) memcpy(c, b.c.data(), b.c.size() * 4);
        return (int32_t)b.c.size();
    })
}

}  // extern "C"
