// csv.cpp — Job.File bytes -> columnar int32 ticks (spec §2).
//
// Job.File is the whole file as read by the dispatcher (/root/reference/src/server/main.rs:170)
// and arrives as proto bytes (/root/reference/proto/backtesting.proto:15). Prices are parsed by
// integer decimal arithmetic (never strtod) so that every bar is an exact tick count.
#include "csv.h"

#include <cstdio>
#include <cstring>

namespace bt {

namespace {

inline bool digit(uint8_t ch) { return ch >= '0' && ch <= '9'; }

// Cursor over one comma-separated field [p, e).
struct Field {
    const uint8_t* p;
    const uint8_t* e;
};

bool ts_ok(Field f) {
    const size_t n = (size_t)(f.e - f.p);
    if (n < 10) return false;
    static const char kShape[] = "dddd-dd-dd";
    for (int i = 0; i < 10; ++i) {
        const uint8_t ch = f.p[i];
        if (kShape[i] == 'd' ? !digit(ch) : ch != '-') return false;
    }
    if (n == 10) return true;
    if (f.p[10] != ' ' && f.p[10] != 'T') return false;
    if (n == 11) return false;
    for (const uint8_t* q = f.p + 11; q < f.e; ++q) {
        const uint8_t ch = *q;
        if (!(digit(ch) || ch == ':' || ch == '.' || ch == '+' || ch == '-' || ch == 'Z')) return false;
    }
    return true;
}

// digits[.digits] with <= 4 fraction digits -> ticks; false on malformed or >= 2^31 ticks.
bool ticks(Field f, int64_t& out) {
    const uint8_t* q = f.p;
    int64_t whole = 0;
    const uint8_t* ds = q;
    while (q < f.e && digit(*q)) {
        whole = whole * 10 + (*q - '0');
        if (whole >= 214749) return false;  // 214749 * 10^4 > 2^31: reject early, no overflow
        ++q;
    }
    if (q == ds) return false;
    int64_t frac = 0;
    int nfrac = 0;
    if (q < f.e && *q == '.') {
        ++q;
        while (q < f.e && digit(*q)) {
            if (++nfrac > 4) return false;
            frac = frac * 10 + (*q - '0');
            ++q;
        }
    }
    if (q != f.e) return false;
    static const int64_t kScale[5] = {10000, 1000, 100, 10, 1};
    out = whole * 10000 + frac * kScale[nfrac];
    return out < 2147483648LL;
}

bool volume_ok(Field f) {
    const uint8_t* q = f.p;
    const uint8_t* ds = q;
    while (q < f.e && digit(*q)) ++q;
    if (q == ds) return false;
    if (q < f.e && *q == '.') {
        ++q;
        while (q < f.e && digit(*q)) ++q;
    }
    return q == f.e;
}

}  // namespace

bool parse_csv(const uint8_t* buf, size_t len, Bars& out, std::string& err) {
    out.h.clear();
    out.l.clear();
    out.c.clear();
    const uint8_t* p = buf;
    const uint8_t* end = buf + len;
    long lineno = 0;
    char msg[128];
    if (len > 0 && !digit(buf[0])) {  // header line
        const uint8_t* nl = (const uint8_t*)memchr(p, '\n', len);
        p = nl ? nl + 1 : end;
        lineno = 1;
    }
    Field fld[6];
    while (p < end) {
        const uint8_t* nl = (const uint8_t*)memchr(p, '\n', (size_t)(end - p));
        const uint8_t* le = nl ? nl : end;
        const uint8_t* next = nl ? nl + 1 : end;
        ++lineno;
        if (le > p && le[-1] == '\r') --le;
        if (le == p) {
            p = next;
            continue;
        }
        int nf = 0;
        const uint8_t* s = p;
        for (const uint8_t* q = p;; ++q) {
            if (q == le || *q == ',') {
                if (nf < 6) fld[nf] = Field{s, q};
                ++nf;
                if (q == le) break;
                s = q + 1;
            }
        }
        if (nf < 5 || nf > 6) {
            snprintf(msg, sizeof msg, "line %ld: expected 5 or 6 fields, got %d", lineno, nf);
            err = msg;
            return false;
        }
        if (!ts_ok(fld[0])) {
            snprintf(msg, sizeof msg, "line %ld: bad timestamp", lineno);
            err = msg;
            return false;
        }
        int64_t px[4];
        for (int k = 0; k < 4; ++k) {
            if (!ticks(fld[1 + k], px[k]) || px[k] < 1) {
                snprintf(msg, sizeof msg, "line %ld: bad or out-of-range price in field %d", lineno,
                         k + 1);
                err = msg;
                return false;
            }
        }
        if (nf == 6 && !volume_ok(fld[5])) {
            snprintf(msg, sizeof msg, "line %ld: bad volume", lineno);
            err = msg;
            return false;
        }
        out.h.push_back((int32_t)px[1]);
        out.l.push_back((int32_t)px[2]);
        out.c.push_back((int32_t)px[3]);
        if (out.c.size() > (size_t)kMaxBars) {
            err = "too many bars";
            return false;
        }
        p = next;
    }
    if (out.c.empty()) {
        err = "no data rows";
        return false;
    }
    for (size_t t = 1; t < out.c.size(); ++t) {  // spec §3 validity: |dc| <= c_{t-1}
        const int64_t prev = out.c[t - 1];
        const int64_t d = (int64_t)out.c[t] - prev;
        if (d > prev || -d > prev) {
            snprintf(msg, sizeof msg, "bar %zu: close moves more than 100%% in one bar", t);
            err = msg;
            return false;
        }
    }
    return true;
}

}  // namespace bt
