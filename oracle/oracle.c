/*
 * oracle.c — scalar C restatement of the backtest hot path. TEST INFRASTRUCTURE ONLY
 * (see oracle.h for who may call it, what it restates and its parity status).
 *
 * Reference anchors:
 *   /root/reference/src/worker/process.rs:13-29  the job function this replaces (sleep stub)
 *   /root/reference/src/worker/main.rs:38-42     its caller: one compute OS thread, jobs in order
 *   /root/reference/src/server/main.rs:164-180   Job.File = whole file bytes (parsed here)
 *   /root/reference/proto/backtesting.proto:13-16,29-32  bytes in, string out
 * Spec: docs/oracle_spec.md (refined where marked [R]).
 *
 * Plain per-bar loops, running window sums, sequential state: the obvious scalar backtest.
 * Build with -ffp-contract=off (oracle/Makefile): the spec forbids FMA contraction.
 */
#include "oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <string.h>

#define GOLDEN 0x9E3779B97F4A7C15ULL
#define TWO56 72057594037927936.0
/* trade hash (spec §4): h = sum of mix(w) over trades, mod 2^64 */
#define MIX_K 0xBF58476D1CE4E5B9ULL
static uint64_t trade_mix(uint64_t w) {
    uint64_t z = (w ^ (w >> 29)) * MIX_K;
    return z ^ (z >> 32);
}

/* ---------------------------------------------------------------- A.1 generator */
static uint64_t draw(uint64_t s0, uint64_t k) {
    uint64_t z = s0 + (k + 1) * GOLDEN;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

void orc_gen(uint64_t seed, int64_t sym, int32_t B, int32_t freq, int32_t* o, int32_t* h,
             int32_t* l, int32_t* c, int32_t* v) {
    const uint64_t s0 = seed ^ ((uint64_t)sym * GOLDEN);
    const int64_t m = freq == ORC_DAILY ? 17320 : 866;
    const uint64_t r = (uint64_t)(m / 4 + 1);
    int64_t prev = 1000000 + (int64_t)(draw(s0, 0) % 9000001ULL);
    for (int32_t t = 0; t < B; ++t) {
        const uint64_t base = 1 + 7 * (uint64_t)t;
        int64_t op, cl;
        if (t == 0) {
            op = prev;
            cl = prev;
        } else {
            int64_t x = 0;
            for (int j = 0; j < 4; ++j) x += (int64_t)(draw(s0, base + j) % (uint64_t)(2 * m + 1));
            x -= 4 * m;
            const int64_t delta = (x * prev) / 1000000;  /* C division truncates toward zero */
            cl = prev + delta;
            if (cl < 10000) cl = 10000;
            if (cl > 2147483648LL - 1048576LL) cl = 2147483648LL - 1048576LL;
            op = prev;
        }
        const int64_t hi = op > cl ? op : cl, lo = op < cl ? op : cl;
        int64_t hh = hi + (int64_t)(draw(s0, base + 4) % r);
        int64_t ll = lo - (int64_t)(draw(s0, base + 5) % r);
        if (ll < 10000) ll = 10000;
        if (o) o[t] = (int32_t)op;
        if (h) h[t] = (int32_t)hh;
        if (l) l[t] = (int32_t)ll;
        if (c) c[t] = (int32_t)cl;
        if (v) v[t] = (int32_t)(1000 + (int64_t)(draw(s0, base + 6) % 100000ULL));
        prev = cl;
    }
}

/* ---------------------------------------------------------------- A.2 parser */
static int is_digit(char ch) { return ch >= '0' && ch <= '9'; }

static int parse_ts(const char* p, const char* e) {
    if (e - p < 10) return 0;
    for (int i = 0; i < 10; ++i) {
        if (i == 4 || i == 7) {
            if (p[i] != '-') return 0;
        } else if (!is_digit(p[i])) {
            return 0;
        }
    }
    p += 10;
    if (p == e) return 1;
    if (*p != ' ' && *p != 'T') return 0;
    ++p;
    if (p == e) return 0;
    for (; p < e; ++p)
        if (!(is_digit(*p) || *p == ':' || *p == '.' || *p == '+' || *p == '-' || *p == 'Z')) return 0;
    return 1;
}

/* digits[.digits] -> ticks (<=4 frac digits). Returns 0 on error. */
static int parse_px(const char* p, const char* e, int64_t* out) {
    int64_t ip = 0;
    int nd = 0;
    while (p < e && is_digit(*p)) {
        ip = ip * 10 + (*p - '0');
        if (ip > (1LL << 40)) return 0;
        ++p;
        ++nd;
    }
    if (nd == 0) return 0;
    int64_t fp = 0;
    int nf = 0;
    if (p < e && *p == '.') {
        ++p;
        while (p < e && is_digit(*p)) {
            if (nf == 4) return 0;
            fp = fp * 10 + (*p - '0');
            ++nf;
            ++p;
        }
    }
    if (p != e) return 0;
    while (nf < 4) {
        fp *= 10;
        ++nf;
    }
    *out = ip * 10000 + fp;
    return 1;
}

static int parse_vol(const char* p, const char* e, int64_t* out) {
    int64_t ip = 0;
    int nd = 0;
    while (p < e && is_digit(*p)) {
        if (ip < (1LL << 58)) ip = ip * 10 + (*p - '0');
        ++p;
        ++nd;
    }
    if (nd == 0) return 0;
    if (p < e && *p == '.') {
        ++p;
        while (p < e && is_digit(*p)) ++p;
    }
    if (p != e) return 0;
    *out = ip;
    return 1;
}

int32_t orc_parse_csv(const char* buf, size_t len, int32_t cap, int32_t* o, int32_t* h, int32_t* l,
                      int32_t* c, int64_t* v, char* err, size_t errlen) {
    const char* p = buf;
    const char* end = buf + len;
    int32_t n = 0;
    long line = 0;
    if (len > 0 && !is_digit(buf[0])) { /* header */
        while (p < end && *p != '\n') ++p;
        if (p < end) ++p;
        ++line;
    }
    while (p < end) {
        const char* ls = p;
        while (p < end && *p != '\n') ++p;
        const char* le = p;
        if (p < end) ++p;
        ++line;
        if (le > ls && le[-1] == '\r') --le;
        if (le == ls) continue;
        const char* f[7];
        const char* fe[7];
        int nfld = 0;
        const char* q = ls;
        while (1) {
            const char* s = q;
            while (q < le && *q != ',') ++q;
            if (nfld < 7) {
                f[nfld] = s;
                fe[nfld] = q;
            }
            ++nfld;
            if (q == le) break;
            ++q;
        }
        if (nfld != 5 && nfld != 6) {
            snprintf(err, errlen, "line %ld: expected 5 or 6 fields, got %d", line, nfld);
            return -1;
        }
        if (!parse_ts(f[0], fe[0])) {
            snprintf(err, errlen, "line %ld: bad timestamp", line);
            return -1;
        }
        int64_t px[4];
        for (int k = 0; k < 4; ++k) {
            if (!parse_px(f[1 + k], fe[1 + k], &px[k])) {
                snprintf(err, errlen, "line %ld: bad price field %d", line, k + 1);
                return -1;
            }
            if (px[k] < 1 || px[k] >= 2147483648LL) {
                snprintf(err, errlen, "line %ld: price out of range", line);
                return -1;
            }
        }
        int64_t vol = 0;
        if (nfld == 6 && !parse_vol(f[5], fe[5], &vol)) {
            snprintf(err, errlen, "line %ld: bad volume", line);
            return -1;
        }
        if (n >= cap) {
            snprintf(err, errlen, "too many bars (cap %d)", cap);
            return -1;
        }
        if (o) o[n] = (int32_t)px[0];
        if (h) h[n] = (int32_t)px[1];
        if (l) l[n] = (int32_t)px[2];
        if (c) c[n] = (int32_t)px[3];
        if (v) v[n] = vol;
        ++n;
    }
    if (n == 0) {
        snprintf(err, errlen, "no data rows");
        return -1;
    }
    if (n > (1 << 22)) {
        snprintf(err, errlen, "too many bars");
        return -1;
    }
    if (c) {
        for (int32_t t = 1; t < n; ++t) {
            int64_t d = (int64_t)c[t] - c[t - 1];
            if (d < 0) d = -d;
            if (d > c[t - 1]) {
                snprintf(err, errlen, "bar %d: close moves more than 100%% in one bar", t);
                return -1;
            }
        }
    }
    return n;
}

/* ---------------------------------------------------------------- accounting (spec §4) */
typedef struct acct {
    int32_t pos, entry_bar, ntr, cap;
    int64_t entry_px, R, peak, mdd, expo;
    __int128 s1, s2;
    double sr, sr2;
    uint64_t hash;
    orc_trade* tr;
} acct;

static void acct_init(acct* a, orc_trade* tr, int32_t cap) {
    memset(a, 0, sizeof(*a));
    a->hash = 0;
    a->tr = tr;
    a->cap = cap;
}

/* bar-t return with the position held since the previous close */
static void acct_returns(acct* a, const int32_t* c, int32_t t) {
    if (t < 1 || a->pos == 0) return;
    const double ret = (double)((int64_t)c[t] - c[t - 1]) / (double)c[t - 1];
    const int64_t q = (int64_t)rint(ret * TWO56);
    const double rr = ret * ret;
    const int64_t q2 = (int64_t)rint(rr * TWO56);
    a->s1 += (__int128)(a->pos * q);
    a->s2 += (__int128)q2;
    a->expo += 1;
    const double r = (double)a->pos * ret;
    a->sr += r;
    a->sr2 += r * r;
}

static void acct_close(acct* a, int32_t t, int64_t px) {
    a->R += a->pos * (px - a->entry_px);
    const uint64_t w = (uint64_t)(uint32_t)a->entry_bar | ((uint64_t)(uint32_t)t << 31) |
                       ((uint64_t)(a->pos > 0) << 62);
    a->hash += trade_mix(w);
    if (a->tr && a->ntr < a->cap) {
        orc_trade* r = &a->tr[a->ntr];
        r->entry_bar = a->entry_bar;
        r->exit_bar = t;
        r->side = a->pos;
        r->pad = 0;
        r->entry_px = a->entry_px;
        r->exit_px = px;
    }
    a->ntr++;
    a->pos = 0;
}

static void acct_open(acct* a, int32_t t, int32_t side, int64_t px) {
    a->pos = side;
    a->entry_bar = t;
    a->entry_px = px;
}

static void acct_equity(acct* a, int64_t close) {
    const int64_t E = a->pos ? a->R + a->pos * (close - a->entry_px) : a->R;
    if (E > a->peak) a->peak = E;
    if (a->peak - E > a->mdd) a->mdd = a->peak - E;
}

static double sharpe_fx(__int128 s1, __int128 s2, int32_t B, double sqrtA) {
    if (B < 2) return 0.0;
    const double n = (double)(B - 1);
    const double m = ldexp((double)s1, -56) / n;   /* __floattidf: round to nearest even */
    const double v = ldexp((double)s2, -56) / n - m * m;
    return v > 0 ? (m / sqrt(v)) * sqrtA : 0.0;
}

static void acct_finish(acct* a, int32_t B, int64_t ann, orc_summary* out) {
    const double sqrtA = sqrt((double)ann);
    out->n_trades = a->ntr;
    out->status = 0;
    out->pnl = a->R;
    out->mdd = a->mdd;
    out->exposure = a->expo;
    out->s1_lo = (uint64_t)a->s1;
    out->s1_hi = (int64_t)(a->s1 >> 64);
    out->s2_lo = (uint64_t)a->s2;
    out->s2_hi = (int64_t)(a->s2 >> 64);
    out->pad = 0;
    out->sharpe = sharpe_fx(a->s1, a->s2, B, sqrtA);
    out->hash = a->hash;
    if (B >= 2) {
        const double n = (double)(B - 1);
        const double m = a->sr / n;
        const double v = a->sr2 / n - m * m;
        out->sharpe_f64 = v > 0 ? (m / sqrt(v)) * sqrtA : 0.0;
    } else {
        out->sharpe_f64 = 0.0;
    }
}

/* ---------------------------------------------------------------- strategies (spec §5) */
void orc_sma(const int32_t* c, int32_t B, int32_t f, int32_t s, int64_t ann, orc_summary* out,
             orc_trade* trades, int32_t cap) {
    acct a;
    acct_init(&a, trades, cap);
    const int32_t warm = (f > s ? f : s) - 1;
    int64_t F = 0, L = 0;
    for (int32_t t = 0; t < B; ++t) {
        F += c[t];
        if (t >= f) F -= c[t - f];
        L += c[t];
        if (t >= s) L -= c[t - s];
        acct_returns(&a, c, t);
        int32_t np = a.pos;
        if (t == B - 1) {
            np = 0;
        } else if (t >= warm) {
            const __int128 lhs = (__int128)F * s, rhs = (__int128)L * f;
            if (lhs > rhs) np = 1;
            else if (lhs < rhs) np = -1;
        }
        if (np != a.pos) {
            if (a.pos) acct_close(&a, t, c[t]);
            if (np) acct_open(&a, t, np, c[t]);
        }
        acct_equity(&a, c[t]);
    }
    acct_finish(&a, B, ann, out);
}

void orc_ema_ols(const int32_t* c, int32_t B, int32_t n, int32_t w, int32_t band_bps, int64_t ann,
                 orc_summary* out, orc_trade* trades, int32_t cap) {
    acct a;
    acct_init(&a, trades, cap);
    const double alpha = 2.0 / ((double)n + 1.0);
    const double lo_mult = (double)(10000 - band_bps), hi_mult = (double)(10000 + band_bps);
    const int32_t warm = (n > w ? n : w) - 1;
    double e = 0.0;
    int64_t S = 0, T = 0; /* window sum and sum of k*c_k over the window ending at t */
    for (int32_t t = 0; t < B; ++t) {
        e = t == 0 ? (double)c[0] : e + alpha * ((double)c[t] - e);
        if (t < w) {
            S += c[t];
            T += (int64_t)t * c[t];
        } else {
            const int64_t old = c[t - w];
            T = T - (S - old) + (int64_t)(w - 1) * c[t];
            S = S - old + c[t];
        }
        const int64_t N = 2 * T - (int64_t)(w - 1) * S;
        acct_returns(&a, c, t);
        int32_t np = a.pos;
        if (t == B - 1) {
            np = 0;
        } else if (t >= warm) {
            const double cd = (double)c[t];
            if (a.pos == 1) {
                if (cd >= e) np = 0;
            } else if (a.pos == -1) {
                if (cd <= e) np = 0;
            } else {
                const double lhs = cd * 10000.0;
                if (lhs < e * lo_mult && N >= 0) np = 1;
                else if (lhs > e * hi_mult && N <= 0) np = -1;
            }
        }
        if (np != a.pos) {
            if (a.pos) acct_close(&a, t, c[t]);
            if (np) acct_open(&a, t, np, c[t]);
        }
        acct_equity(&a, c[t]);
    }
    acct_finish(&a, B, ann, out);
}

void orc_boll(const int32_t* h, const int32_t* l, const int32_t* c, int32_t B, int32_t w,
              int32_t k_num, int32_t k_den, int32_t sl_bps, int32_t tp_bps, int64_t ann,
              orc_summary* out, orc_trade* trades, int32_t cap) {
    acct a;
    acct_init(&a, trades, cap);
    int64_t Sc = 0;
    __int128 Sc2 = 0;
    int64_t sl_lvl = 0, tp_lvl = 0;
    const __int128 kd2 = (__int128)k_den * k_den, kn2 = (__int128)k_num * k_num;
    for (int32_t t = 0; t < B; ++t) {
        Sc += c[t];
        Sc2 += (__int128)c[t] * c[t];
        if (t >= w) {
            Sc -= c[t - w];
            Sc2 -= (__int128)c[t - w] * c[t - w];
        }
        acct_returns(&a, c, t);
        int exited = 0;
        if (a.pos != 0 && t >= a.entry_bar + 1) {
            if (a.pos == 1) {
                if (l[t] <= sl_lvl) { acct_close(&a, t, sl_lvl); exited = 1; }
                else if (h[t] >= tp_lvl) { acct_close(&a, t, tp_lvl); exited = 1; }
            } else {
                if (h[t] >= sl_lvl) { acct_close(&a, t, sl_lvl); exited = 1; }
                else if (l[t] <= tp_lvl) { acct_close(&a, t, tp_lvl); exited = 1; }
            }
        }
        if (t == B - 1) {
            if (a.pos) acct_close(&a, t, c[t]);
        } else if (t >= w - 1) {
            const int64_t D = (int64_t)w * c[t] - Sc;
            const __int128 Q = (__int128)w * Sc2 - (__int128)Sc * Sc;
            if (a.pos == 1 && D >= 0) {
                acct_close(&a, t, c[t]);
            } else if (a.pos == -1 && D <= 0) {
                acct_close(&a, t, c[t]);
            } else if (a.pos == 0 && !exited) {
                const __int128 lhs = (__int128)D * D * kd2, rhs = kn2 * Q;
                const int64_t ce = c[t];
                if (D < 0 && lhs > rhs) {
                    acct_open(&a, t, 1, ce);
                    sl_lvl = ce * (10000 - sl_bps) / 10000;
                    tp_lvl = ce * (10000 + tp_bps) / 10000;
                } else if (D > 0 && lhs > rhs) {
                    acct_open(&a, t, -1, ce);
                    sl_lvl = ce * (10000 + sl_bps) / 10000;
                    tp_lvl = ce * (10000 - tp_bps) / 10000;
                }
            }
        }
        acct_equity(&a, c[t]);
    }
    acct_finish(&a, B, ann, out);
}

/* ---------------------------------------------------------------- B4: multithreaded CPU path */
typedef struct mt_job {
    const int32_t* c;
    int32_t S, B, nf, ns;
    const int32_t *fast, *slow;
    int64_t ann;
    orc_summary* out;
    int32_t next;
    pthread_mutex_t mu;
} mt_job;

static void* mt_worker(void* arg) {
    mt_job* j = (mt_job*)arg;
    const int32_t P = j->nf * j->ns;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        const int32_t s = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (s >= j->S) break;
        const int32_t* cs = j->c + (size_t)s * j->B;
        for (int32_t i = 0; i < j->nf; ++i)
            for (int32_t k = 0; k < j->ns; ++k)
                orc_sma(cs, j->B, j->fast[i], j->slow[k], j->ann,
                        &j->out[(size_t)s * P + (size_t)i * j->ns + k], NULL, 0);
    }
    return NULL;
}

void orc_sma_grid_mt(const int32_t* c, int32_t S, int32_t B, const int32_t* fast, int32_t nf,
                     const int32_t* slow, int32_t ns, int64_t ann, orc_summary* out,
                     int32_t nthreads) {
    mt_job j = {c, S, B, nf, ns, fast, slow, ann, out, 0, PTHREAD_MUTEX_INITIALIZER};
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    for (int32_t i = 0; i < nthreads; ++i) pthread_create(&th[i], NULL, mt_worker, &j);
    for (int32_t i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
}

/* EMA+OLS and Bollinger grids on the same pool: one task per symbol, every param of it in the
 * engine's param order (include/bt.h). h and l may be NULL for EMA+OLS. */
typedef struct mt_grid {
    int32_t strategy; /* 2 = EMA+OLS, 3 = Bollinger */
    const int32_t *h, *l, *c;
    int32_t S, B;
    const int32_t* ax[4];
    int32_t n[4];
    int32_t band_bps, k_den;
    int64_t ann;
    orc_summary* out;
    int32_t next;
    pthread_mutex_t mu;
} mt_grid;

static void* mt_grid_worker(void* arg) {
    mt_grid* j = (mt_grid*)arg;
    const int32_t P = j->n[0] * j->n[1] * j->n[2] * j->n[3];
    for (;;) {
        pthread_mutex_lock(&j->mu);
        const int32_t s = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (s >= j->S) break;
        const size_t row = (size_t)s * j->B;
        orc_summary* o = j->out + (size_t)s * P;
        int32_t p = 0;
        for (int32_t a = 0; a < j->n[0]; ++a)
            for (int32_t b = 0; b < j->n[1]; ++b)
                for (int32_t c = 0; c < j->n[2]; ++c)
                    for (int32_t d = 0; d < j->n[3]; ++d, ++p) {
                        if (j->strategy == 2)
                            orc_ema_ols(j->c + row, j->B, j->ax[0][a], j->ax[1][b], j->band_bps,
                                        j->ann, &o[p], NULL, 0);
                        else
                            orc_boll(j->h + row, j->l + row, j->c + row, j->B, j->ax[0][a],
                                     j->ax[1][b], j->k_den, j->ax[2][c], j->ax[3][d], j->ann,
                                     &o[p], NULL, 0);
                    }
    }
    return NULL;
}

static void run_grid(mt_grid* j, int32_t nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    for (int32_t i = 0; i < nthreads; ++i) pthread_create(&th[i], NULL, mt_grid_worker, j);
    for (int32_t i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
}

void orc_ema_grid_mt(const int32_t* c, int32_t S, int32_t B, const int32_t* span, int32_t nsp,
                     const int32_t* ols, int32_t nol, int32_t band_bps, int64_t ann,
                     orc_summary* out, int32_t nthreads) {
    static const int32_t one = 0;
    mt_grid j = {2, NULL, NULL, c, S, B, {span, ols, &one, &one}, {nsp, nol, 1, 1}, band_bps, 1,
                 ann, out, 0, PTHREAD_MUTEX_INITIALIZER};
    run_grid(&j, nthreads);
}

void orc_boll_grid_mt(const int32_t* h, const int32_t* l, const int32_t* c, int32_t S, int32_t B,
                      const int32_t* win, int32_t nw, const int32_t* k_num, int32_t nk,
                      int32_t k_den, const int32_t* sl, int32_t nsl, const int32_t* tp,
                      int32_t ntp, int64_t ann, orc_summary* out, int32_t nthreads) {
    mt_grid j = {3, h, l, c, S, B, {win, k_num, sl, tp}, {nw, nk, nsl, ntp}, 0, k_den,
                 ann, out, 0, PTHREAD_MUTEX_INITIALIZER};
    run_grid(&j, nthreads);
}
