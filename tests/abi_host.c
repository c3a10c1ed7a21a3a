/* abi_host.c — a compiled C99 host of the drop-in boundary (include/bt.h), the way the Rust
 * worker's process_incoming_job would drive it (the reference's job loop is
 * /root/reference/src/worker/process.rs:13-29): create an engine, one bt_run_batch per JobsReply,
 * free the library-owned strings, destroy. Test support only (tests/test_abi_cpu.py compiles it
 * with -std=c99 -pedantic -Werror and checks the struct layouts against the ctypes mirror;
 * tests/test_gpu_parity.py runs a batch through it and compares with the Python host).
 *
 *   abi_host layout                      struct sizes and field offsets as JSON (no GPU)
 *   abi_host run SEED N BARS              N synthetic daily jobs (DBXCOL1 payloads) as one batch;
 *                                        prints "== job i status s len n" and the data per job
 */
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "bt.h"

#define OFF(T, f) printf("\"%s.%s\": %zu, ", #T, #f, offsetof(T, f))
#define SZ(T) printf("\"%s\": %zu, ", #T, sizeof(T))

static int layout(void) {
    printf("{");
    SZ(bt_config);
    OFF(bt_config, strategy); OFF(bt_config, fast); OFF(bt_config, slow); OFF(bt_config, n_span);
    OFF(bt_config, span); OFF(bt_config, ols); OFF(bt_config, band_bps); OFF(bt_config, n_bwin);
    OFF(bt_config, bwin); OFF(bt_config, k_num); OFF(bt_config, k_den); OFF(bt_config, sl_bps);
    OFF(bt_config, tp_bps); OFF(bt_config, annualization); OFF(bt_config, device);
    OFF(bt_config, topk); OFF(bt_config, flags); OFF(bt_config, host_threads);
    OFF(bt_config, trade_cap); OFF(bt_config, stream);
    SZ(bt_job_in); OFF(bt_job_in, file); OFF(bt_job_in, len);
    SZ(bt_job_out); OFF(bt_job_out, len); OFF(bt_job_out, status); OFF(bt_job_out, n_bars);
    SZ(bt_summary); OFF(bt_summary, pnl); OFF(bt_summary, sharpe); OFF(bt_summary, hash);
    SZ(bt_trade); OFF(bt_trade, entry_px);
    SZ(bt_sums); SZ(bt_topk_rec); OFF(bt_topk_rec, sym); OFF(bt_topk_rec, pnl);
    SZ(bt_stats); SZ(bt_batch_profile); OFF(bt_batch_profile, payload_bytes_read);
    OFF(bt_batch_profile, bars); OFF(bt_batch_profile, host_ingest_ms);
    OFF(bt_batch_profile, total_ms);
    printf("\"abi_version\": %d}\n", (int)bt_abi_version());
    return 0;
}

static int run(uint64_t seed, int n, int bars) {
    static const int32_t fast[] = {4, 6, 10}, slow[] = {50, 60, 120};
    bt_config cfg;
    char err[256];
    bt_engine* e;
    bt_job_in* jobs = calloc((size_t)n, sizeof *jobs);
    bt_job_out* outs = calloc((size_t)n, sizeof *outs);
    uint8_t** bufs = calloc((size_t)n, sizeof *bufs);
    char (*ids)[32] = calloc((size_t)n, sizeof *ids);
    int i, rc = 0;
    if (!jobs || !outs || !bufs || !ids) return 2;
    memset(&cfg, 0, sizeof cfg);
    cfg.strategy = BT_SMA_CROSS;
    cfg.n_fast = 3;
    cfg.n_slow = 3;
    cfg.fast = fast;
    cfg.slow = slow;
    cfg.annualization = 252;
    e = bt_engine_create(&cfg, err, sizeof err);
    if (!e) {
        fprintf(stderr, "bt_engine_create: %s\n", err);
        return 1;
    }
    for (i = 0; i < n; ++i) {
        const int64_t need = bt_gen_payload(seed, i, bars, BT_DAILY, NULL, 0);
        bufs[i] = need > 0 ? malloc((size_t)need) : NULL;
        if (!bufs[i] || bt_gen_payload(seed, i, bars, BT_DAILY, bufs[i], (size_t)need) != need) {
            fprintf(stderr, "bt_gen_payload failed\n");
            return 1;
        }
        snprintf(ids[i], sizeof ids[i], "job-%d", i);
        jobs[i].id = ids[i];
        jobs[i].file = bufs[i];
        jobs[i].len = (size_t)need;
    }
    /* one JobsReply = one call; outs[i] answers jobs[i] */
    if (bt_run_batch(e, (size_t)n, jobs, outs) != 0) {
        fprintf(stderr, "bt_run_batch: %s\n", bt_last_error());
        rc = 1;
    } else {
        for (i = 0; i < n; ++i) {
            printf("== job %d status %d len %zu\n", i, (int)outs[i].status, outs[i].len);
            fwrite(outs[i].data, 1, outs[i].len, stdout);
        }
    }
    bt_job_out_free(outs, (size_t)n);
    bt_engine_destroy(e);
    for (i = 0; i < n; ++i) free(bufs[i]);
    free(bufs);
    free(ids);
    free(jobs);
    free(outs);
    return rc;
}

int main(int argc, char** argv) {
    if (argc >= 2 && strcmp(argv[1], "layout") == 0) return layout();
    if (argc >= 5 && strcmp(argv[1], "run") == 0)
        return run(strtoull(argv[2], NULL, 0), atoi(argv[3]), atoi(argv[4]));
    fprintf(stderr, "usage: abi_host layout | run SEED N BARS\n");
    return 2;
}
