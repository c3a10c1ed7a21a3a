/*
 * oracle.h — scalar C restatement of the backtest hot path (TEST INFRASTRUCTURE ONLY).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this code,
 * and only as the checker / CPU baseline. The product never links or calls it.
 *
 * What it restates: the job function the reference worker runs on its compute OS thread,
 * `process_incoming_job` (/root/reference/src/worker/process.rs:13-29), which today only
 * sleeps 1000 ms per job (process.rs:23). The arithmetic that replaces the sleep is authored
 * in SURVEY.md Appendix A and frozen in docs/oracle_spec.md; this file follows that spec with
 * plain per-bar loops (the "scalar fp64 backtest" of BASELINE.json north_star, in C because
 * no Rust toolchain exists here: SURVEY.md §8(c)).
 *
 * PARITY STATUS: parity unpinned against the reference — the reference path has no
 * arithmetic (process.rs:23) and ships no tests or fixtures. The spec is
 * pinned by two independent restatements that must agree bit-for-bit: this file and
 * oracle/oracle_np.py (whose outputs are the committed tests/golden/ fixtures).
 */
#ifndef BT_ORACLE_H
#define BT_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORC_DAILY = 0, ORC_MINUTE = 1 };

typedef struct orc_summary {     /* first 48 B mirror bt_summary (include/bt.h) */
    int32_t n_trades;
    int32_t status;
    int64_t pnl;
    int64_t mdd;
    int64_t exposure;
    double sharpe;
    uint64_t hash;
    uint64_t s1_lo;              /* S1, S2 (int128, spec §4) as lo/hi words */
    int64_t s1_hi;
    uint64_t s2_lo;
    int64_t s2_hi;
    double sharpe_f64;           /* naive fp64 sequential-sum Sharpe (oracle only) */
    int64_t pad;
} orc_summary;

typedef struct orc_trade {
    int32_t entry_bar, exit_bar, side, pad;
    int64_t entry_px, exit_px;
} orc_trade;

/* Appendix A.1: one symbol, B bars, int32 ticks (v may be NULL etc.). */
void orc_gen(uint64_t seed, int64_t sym, int32_t B, int32_t freq,
             int32_t* o, int32_t* h, int32_t* l, int32_t* c, int32_t* v);

/* Appendix A.2: CSV bytes -> SoA ticks. Returns bar count, or -1 with err filled. */
int32_t orc_parse_csv(const char* buf, size_t len, int32_t cap,
                      int32_t* o, int32_t* h, int32_t* l, int32_t* c, int64_t* v,
                      char* err, size_t errlen);

/* Strategies (spec §5). trades may be NULL; at most cap trades are written. */
void orc_sma(const int32_t* c, int32_t B, int32_t f, int32_t s, int64_t ann,
             orc_summary* out, orc_trade* trades, int32_t cap);
void orc_ema_ols(const int32_t* c, int32_t B, int32_t n, int32_t w, int32_t band_bps,
                 int64_t ann, orc_summary* out, orc_trade* trades, int32_t cap);
void orc_boll(const int32_t* h, const int32_t* l, const int32_t* c, int32_t B,
              int32_t w, int32_t k_num, int32_t k_den, int32_t sl_bps, int32_t tp_bps,
              int64_t ann, orc_summary* out, orc_trade* trades, int32_t cap);

/* Multithreaded CPU baseline: SMA grid over S symbols of B bars each
 * (c is S x B row-major); one task per symbol on nthreads pthreads. out is S x (nf*ns). */
void orc_sma_grid_mt(const int32_t* c, int32_t S, int32_t B,
                     const int32_t* fast, int32_t nf, const int32_t* slow, int32_t ns,
                     int64_t ann, orc_summary* out, int32_t nthreads);
/* The same pool for EMA+OLS and Bollinger grids (S x B row-major columns, params in the
 * engine's order, include/bt.h). */
void orc_ema_grid_mt(const int32_t* c, int32_t S, int32_t B, const int32_t* span, int32_t nsp,
                     const int32_t* ols, int32_t nol, int32_t band_bps, int64_t ann,
                     orc_summary* out, int32_t nthreads);
void orc_boll_grid_mt(const int32_t* h, const int32_t* l, const int32_t* c, int32_t S, int32_t B,
                      const int32_t* win, int32_t nw, const int32_t* k_num, int32_t nk,
                      int32_t k_den, const int32_t* sl, int32_t nsl, const int32_t* tp,
                      int32_t ntp, int64_t ann, orc_summary* out, int32_t nthreads);

#ifdef __cplusplus
}
#endif
#endif
