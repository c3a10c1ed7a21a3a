/*
 * bt.h — C ABI of the MI355X-native backtest engine (libbt.so).
 *
 * This is the drop-in boundary for the reference worker's job function
 *     pub fn process_incoming_job(jobs_reply: JobsReply, complete_send: Sender<String>)
 *     (/root/reference/src/worker/process.rs:13-29)
 * which today sleeps 1000 ms per job (process.rs:23) and sends `job.id` per job (process.rs:24),
 * called from the worker's single compute OS thread (/root/reference/src/worker/main.rs:38-42).
 * The proto contract stays byte-identical (/root/reference/proto/backtesting.proto):
 * `Job{string id; bytes File}` in (proto:13-16), `CompleteRequest{string id; string data}` out
 * (proto:29-32). The Rust-side `extern "C"` block a maintainer would add is in INTEGRATION.md.
 *
 * Plain C types only. No C++ exception and no abort crosses this boundary: every entry point
 * catches and returns an int status (0 = OK, < 0 = error; message via bt_last_error()).
 * The engine is not thread-safe (the reference has exactly one caller thread, main.rs:38-42);
 * it sets its HIP device on every call, so it may be called from any one OS thread.
 * Semantics of every number produced: docs/oracle_spec.md.
 */
#ifndef BT_H
#define BT_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: bt_batch_profile.payload_bytes_read; the device top-k never overflows (bt_topk_fetch_wait
 *    and bt_exchange_wait return exact records on tie-heavy grids); bt_summary.hash is the
 *    additive trade hash of docs/oracle_spec.md §4 (version 1 hosts may hold FNV-1a hashes).
 * 3: bt_exchange_merge takes the gathered block's byte length and rejects a mismatch. */
#define BT_ABI_VERSION 3

typedef struct bt_engine bt_engine;

enum bt_strategy { BT_SMA_CROSS = 1, BT_EMA_OLS = 2, BT_BOLL = 3 };

enum bt_flags {
    BT_FLAG_PARITY = 1,  /* also record full trade lists and the int128 return sums */
    BT_FLAG_TIMING = 2,  /* time the dominant kernel with HIP events (bt_kernel_timing) */
};

enum bt_freq { BT_DAILY = 0, BT_MINUTE = 1 };

/* Engine configuration. The proto carries no strategy or params (proto:13-16), so the grid is
 * worker-side configuration (SURVEY.md §7 hard part 5). Arrays are copied at create time.
 * Accepted domain (docs/oracle_spec.md §7): windows up to 4,096 bars always, longer ones while the
 * prefix ring fits 160 KB of LDS; EMA at most 64 spans; Bollinger w * max(k_num, k_den) < 2^32;
 * at most 2^20 params. Anything else is refused by bt_engine_create, never approximated. */
typedef struct bt_config {
    int32_t strategy;                 /* enum bt_strategy */
    /* SMA crossover: params = n_fast x n_slow, param = i_fast * n_slow + i_slow */
    int32_t n_fast, n_slow;
    const int32_t* fast;
    const int32_t* slow;
    /* EMA + rolling OLS: params = n_span x n_ols, param = i_span * n_ols + i_ols */
    int32_t n_span, n_ols;
    const int32_t* span;
    const int32_t* ols;
    int32_t band_bps;
    /* Bollinger + SL/TP: param = ((i_w * n_k + i_k) * n_sl + i_sl) * n_tp + i_tp */
    int32_t n_bwin, n_k, n_sl, n_tp;
    const int32_t* bwin;
    const int32_t* k_num;
    int32_t k_den;
    const int32_t* sl_bps;
    const int32_t* tp_bps;
    int64_t annualization;            /* A in the Sharpe formula: 252 daily, 98280 1-min */
    int32_t device;                   /* HIP device ordinal */
    int32_t topk;                     /* k of bt_read_topk (0 = top-k disabled) */
    int32_t flags;                    /* enum bt_flags */
    int32_t host_threads;             /* CSV parse threads in bt_run_batch (0 = auto) */
    int32_t trade_cap;                /* parity mode: trades kept per (symbol, param) */
    void* stream;                     /* optional hipStream_t to launch on (NULL = own stream) */
} bt_config;

/* One Job of a JobsReply (proto:13-16). Borrowed for the duration of the call. */
typedef struct bt_job_in {
    const char* id;                   /* Job.id (UUIDv4 string from server/main.rs:169) */
    const uint8_t* file;              /* Job.File bytes (whole CSV, server/main.rs:170) */
    size_t len;
} bt_job_in;

/* One CompleteRequest.data (proto:31, UTF-8). Owned by the library: free with bt_job_out_free. */
typedef struct bt_job_out {
    char* data;
    size_t len;
    int32_t status;                   /* 0 = OK, < 0 = this job failed (data holds {"error":..}) */
    int32_t n_bars;
} bt_job_out;

/* Per (symbol, param) result, 48 bytes. */
typedef struct bt_summary {
    int32_t n_trades;
    int32_t status;
    int64_t pnl;                      /* ticks */
    int64_t mdd;                      /* ticks */
    int64_t exposure;                 /* bars held */
    double sharpe;
    uint64_t hash;                    /* additive trade-sequence hash (spec §4) */
} bt_summary;

typedef struct bt_trade {
    int32_t entry_bar, exit_bar, side, pad;
    int64_t entry_px, exit_px;
} bt_trade;

/* S1, S2 of spec §4 (int128 as lo/hi words); parity mode only. */
typedef struct bt_sums {
    uint64_t s1_lo;
    int64_t s1_hi;
    uint64_t s2_lo;
    int64_t s2_hi;
} bt_sums;

/* Global top-k record (24 B): ordered by sharpe desc, then sym asc, then param asc. */
typedef struct bt_topk_rec {
    double sharpe;
    int32_t sym;
    int32_t param;
    int64_t pnl;
} bt_topk_rec;

typedef struct bt_stats {
    int64_t n_symbols;
    int64_t n_params;
    int64_t bar_evals;                /* sum over symbols of bars x params */
    int64_t trades;                   /* sum of n_trades over every (symbol, param) */
    int64_t errors;                   /* symbols rejected */
} bt_stats;

/* ---- lifecycle */
bt_engine* bt_engine_create(const bt_config* cfg, char* err, size_t errlen);
void bt_engine_destroy(bt_engine* e);
const char* bt_last_error(void);      /* thread-local message of the last failed call */
int32_t bt_abi_version(void);
int32_t bt_num_params(const bt_engine* e);
/* Bar-axis split of every strategy's walk (k_tile.hip, k_sma.hip): segments per symbol (0 =
 * automatic: EMA+OLS and Bollinger split a shard with no more workgroups than the GPU has CUs, SMA
 * a shard of one-block-per-CU symbols that fills the GPU fewer than 16 times; 1 = never; n =
 * always n) and the burn-in tiles a speculative segment walks before its first bar (0 = the
 * default: 64 for Bollinger, 24 x the longest span for EMA+OLS, so every fp64 EMA chain meets the
 * true one, 2 for SMA, whose trade open at a boundary is carried symbolically into a combine
 * pass). Results are identical either way (a boundary whose speculative start differs from
 * the true one is re-walked); parity mode (trade lists) never splits. bt_last_segments: the count
 * the last bt_run used and, if refixed_blocks is not NULL, how many (symbol, boundary) blocks the
 * fix pass re-walked (waits for the run). */
int32_t bt_set_segments(bt_engine* e, int32_t segments, int32_t burn_tiles);
int32_t bt_last_segments(bt_engine* e, int64_t* refixed_blocks);

/* Phase times of the last bt_run_batch call (host clocks for host phases, HIP events for the
 * device ones). */
typedef struct bt_batch_profile {
    int64_t n_jobs, n_failed;
    int64_t payload_bytes;            /* sum of Job.File lengths */
    int64_t payload_bytes_read;       /* bytes ingest actually reads: a CSV whole, a DBXCOL1
                                         payload its header and price columns (never the
                                         volume column) */
    int64_t bars;                     /* bars of the good jobs */
    double host_ingest_ms;            /* parse / validate + copy into pinned staging */
    double upload_ms;                 /* H2D of the staged columns */
    double compute_ms;                /* strategy kernel (+ top-k when enabled) */
    double readback_ms;               /* one D2H of every summary of the batch */
    double format_ms;                 /* CompleteRequest.data strings */
    double total_ms;                  /* wall time of the call */
} bt_batch_profile;

/* ---- drop-in for process_incoming_job: a whole JobsReply in one GPU launch.
 * outs[i] answers jobs[i] (same order the reference sends completions, process.rs:21-25).
 * On a -1 return no output string is left allocated (outs are all NULL). */
int32_t bt_run_batch(bt_engine* e, size_t n, const bt_job_in* jobs, bt_job_out* outs);
void bt_job_out_free(bt_job_out* outs, size_t n);
int32_t bt_last_batch_profile(bt_engine* e, bt_batch_profile* out);

/* ---- HBM-resident path (configs 2-5, bench, multi-GPU shards) */
/* Generate n_sym synthetic symbols (spec §1) with ids sym_begin.. directly in HBM. */
int32_t bt_load_synthetic(bt_engine* e, uint64_t seed, int64_t sym_begin, int32_t n_sym,
                          int32_t n_bars, int32_t freq);
/* Upload host SoA bars: symbol s has bars[s] rows starting at row offset row_off[s] in h/l/c.
 * h and l may be NULL unless the strategy is BT_BOLL. */
int32_t bt_load_ohlc(bt_engine* e, int32_t n_sym, const int64_t* sym_ids, const int32_t* bars,
                     const int64_t* row_off, const int32_t* h, const int32_t* l,
                     const int32_t* c);
int32_t bt_run(bt_engine* e);         /* enqueue the whole hot path on the engine stream */
int32_t bt_sync(bt_engine* e);
int32_t bt_read_summaries(bt_engine* e, bt_summary* out, size_t n);     /* n = symbols x params */
int32_t bt_read_sums(bt_engine* e, bt_sums* out, size_t n);             /* parity mode */
int32_t bt_read_trades(bt_engine* e, bt_trade* out, size_t n);          /* n = sym x param x cap */
int32_t bt_read_topk(bt_engine* e, bt_topk_rec* out, int32_t k);        /* returns count */
int32_t bt_read_stats(bt_engine* e, bt_stats* out);
#define BT_PIPE_SLOTS 4 /* pinned read-back / exchange slots per engine / communicator */
/* Pipelined read-back of the last run's top-k and trade count: bt_topk_fetch_async enqueues
 * the device-to-host copy into pinned slot 0 .. BT_PIPE_SLOTS-1 behind the run (no host wait),
 * so the next bt_run (or the next BT_PIPE_SLOTS - 1) can be enqueued before this run's records
 * are consumed; bt_topk_fetch_wait waits for
 * that copy only and returns the record count. The device selection is exact on any grid (a
 * tie-heavy one takes a slower single-block finish, k_topk.hip). A slot stays valid until its
 * next fetch. */
int32_t bt_topk_fetch_async(bt_engine* e, int32_t slot);
int32_t bt_topk_fetch_wait(bt_engine* e, int32_t slot, bt_topk_rec* out, int32_t k,
                           int64_t* n_trades);
/* Read back the synthetic/uploaded close column of one symbol (tests). */
int32_t bt_read_close(bt_engine* e, int32_t sym_index, int32_t* out, int32_t n);
/* Average device time of the dominant kernel (BT_FLAG_TIMING), and how many launches. */
int32_t bt_kernel_timing(bt_engine* e, double* total_ms, int64_t* launches, const char** name);
int32_t bt_reset_timing(bt_engine* e);
/* Profiling aid of the developer build libbt_prof.so only (`make PROFILING=1`, env BT_ABLATE=64):
 * per-phase s_memtime sums of the last run (n <= 32). The release libbt.so reads no environment
 * variable and always returns -1 ("no debug stamps") here. */
int32_t bt_read_debug(bt_engine* e, uint64_t* out, int32_t n);

/* ---- top-k merge (host): merge sorted record lists from several shards (RCCL gather). */
int32_t bt_merge_topk(const bt_topk_rec* in, size_t n, int32_t k, bt_topk_rec* out);

/* ---- multi-GPU exchange (comm.cpp): one process per GPU, each running its own
 * symbol shard; per run ONE RCCL all-gather over xGMI of every rank's top-k records and
 * counters, straight from the engine's device buffers. Replaces nothing in the reference, whose
 * only parallelism is job farming over gRPC (/root/reference/src/server/main.rs:131-143).
 *   rank 0: bt_comm_unique_id(id); the launcher broadcasts the 128 bytes; every rank:
 *   bt_comm_create(id, rank, world, device, k) — a collective call, all ranks together.
 * bt_exchange_async enqueues the exchange of the engine's last run (which needs topk >= k) into
 * pinned slot 0 .. BT_PIPE_SLOTS-1 behind the run's top-k chain, without a host wait;
 * bt_exchange_wait returns the merged global top-k (count) and counters[2] = {bar-evals, trades}
 * summed over ranks.
 * Every rank must issue the same sequence of exchanges.
 * RCCL is loaded at run time (dlopen of librccl.so.1 on the first bt_comm_unique_id /
 * bt_comm_create): libbt.so does not link it, so a single-GPU host loads the engine without RCCL,
 * and these two calls fail with "RCCL is not loadable" there. */
#define BT_COMM_ID_BYTES 128
typedef struct bt_comm bt_comm;
int32_t bt_comm_unique_id(uint8_t* out);
bt_comm* bt_comm_create(const uint8_t* id, int32_t rank, int32_t world, int32_t device, int32_t k,
                        char* err, size_t errlen);
void bt_comm_destroy(bt_comm* c);
int32_t bt_exchange_async(bt_comm* c, bt_engine* e, int32_t slot);
int32_t bt_exchange_wait(bt_comm* c, int32_t slot, bt_topk_rec* out, int32_t k,
                         int64_t* counters);
/* The host half of bt_exchange_wait, callable without a GPU: `block` (block_bytes long, which
 * must equal world * bt_exchange_message_bytes(k_msg), else -1) holds `world` messages in rank
 * order, each [header record whose first int32 is
 * the record count n (clipped to k_msg; < 0 is an error) | k_msg records, the first n sorted |
 * int64 bar-evals | int64 trades], as the all-gather delivers them. Writes the min(k, k_msg,
 * sum n) best records in engine order and counters[2] = the summed counters; returns the count. */
int64_t bt_exchange_message_bytes(int32_t k_msg);
int32_t bt_exchange_merge(const uint8_t* block, size_t block_bytes, int32_t world, int32_t k_msg,
                          bt_topk_rec* out, int32_t k, int64_t* counters);

/* ---- self-test hooks (host-side helpers the tests call without a GPU) */
/* The CompleteRequest.data text of P summaries (spec §6, one JSON line per param), as
 * bt_run_batch writes it; returns its length, or the capacity needed when out is NULL. */
int64_t bt_format_summaries(const bt_summary* r, int32_t P, char* out, size_t cap);
double bt_i128_to_double(uint64_t lo, int64_t hi);
int32_t bt_parse_csv(const uint8_t* buf, size_t len, int32_t cap, int32_t* h, int32_t* l,
                     int32_t* c, char* err, size_t errlen);   /* same as bt_parse_job */
/* Host ingest of one Job.File (CSV or binary columns) into h/l/c ticks;
 * returns the bar count, or -1 with the message in err. */
int32_t bt_parse_job(const uint8_t* buf, size_t len, int32_t cap, int32_t* h, int32_t* l,
                     int32_t* c, char* err, size_t errlen);

/* ---- binary columnar Job.File payload (payload.cpp): "DBXCOL1\n", u32 n_bars, u32 flags
 * (bit 0: int64 volume follows), then int32 open/high/low/close columns. Both return the byte
 * size (the required size when out is NULL) or -1. */
int64_t bt_encode_columns(const int32_t* o, const int32_t* h, const int32_t* l, const int32_t* c,
                          const int64_t* v, int32_t n, uint8_t* out, size_t cap);
/* Spec §1 synthetic OHLCV of one symbol generated on the host as a binary payload (the
 * dispatcher-side producer for gRPC-fed runs; bit-identical to bt_load_synthetic). */
int64_t bt_gen_payload(uint64_t seed, int64_t sym, int32_t bars, int32_t freq, uint8_t* out,
                       size_t cap);

#ifdef __cplusplus
}
#endif
#endif
