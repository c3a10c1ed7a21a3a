// payload.cpp — the binary columnar Job.File payload and its host-side
// producer.
//
// The reference ships each symbol as the whole CSV file (Job.File bytes,
// /root/reference/proto/backtesting.proto:15, read at /root/reference/src/server/main.rs:170).
// One-minute files exceed grpc's default 4 MiB message and CSV parsing would
// dominate a gRPC-fed full-node sweep, so a worker also accepts pre-columnised bytes — still
// "bytes in", so the proto is unchanged:
//
//   offset 0   8 B   magic "DBXCOL1\n"
//          8   u32   n_bars (little endian), 1 <= n_bars <= kMaxBars
//         12   u32   flags: bit 0 = an int64 volume column follows the prices
//         16   i32   open[n], high[n], low[n], close[n]   (ticks, 1 tick = 1e-4)
//              i64   volume[n]                              (flag bit 0 only)
//
// Validation is the CSV path's (spec §2-§3): every price in [1, 2^31), |c_t - c_{t-1}| <=
// c_{t-1}, exact length. Decoding is a bounds-checked copy into the engine's columns.
#include <climits>
#include <cstring>

#include "csv.h"
#include "bt.h"

namespace bt {

namespace {

constexpr char kMagic[8] = {'D', 'B', 'X', 'C', 'O', 'L', '1', '\n'};

uint32_t rd32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

void wr32(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)v;
    p[1] = (uint8_t)(v >> 8);
    p[2] = (uint8_t)(v >> 16);
    p[3] = (uint8_t)(v >> 24);
}

// SplitMix64 in counter form (spec §1; same stream as k_gen.hip's device generator).
inline uint64_t sm64(uint64_t s0, uint64_t k) {
    uint64_t z = s0 + (k + 1) * 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

}  // namespace

bool is_binary_payload(const uint8_t* buf, size_t len) {
    return len >= 8 && memcmp(buf, kMagic, 8) == 0;
}

size_t binary_payload_size(int32_t n, bool volume) {
    return 16 + (size_t)n * 16 + (volume ? (size_t)n * 8 : 0);
}

bool parse_binary(const uint8_t* buf, size_t len, Bars& out, std::string& err) {
    if (len < 16 || !is_binary_payload(buf, len)) {
        err = "binary payload: bad header";
        return false;
    }
    const uint32_t n = rd32(buf + 8), flags = rd32(buf + 12);
    if (n < 1 || n > (uint32_t)kMaxBars) {
        err = "binary payload: bar count out of range";
        return false;
    }
    if ((flags & ~1u) != 0) {
        err = "binary payload: unknown flags";
        return false;
    }
    if (len != binary_payload_size((int32_t)n, flags & 1)) {
        err = "binary payload: length does not match the header";
        return false;
    }
    const uint8_t* col = buf + 16;
    out.h.resize(n);
    out.l.resize(n);
    out.c.resize(n);
    std::vector<int32_t> o(n);
    memcpy(o.data(), col, (size_t)n * 4);
    memcpy(out.h.data(), col + (size_t)n * 4, (size_t)n * 4);
    memcpy(out.l.data(), col + (size_t)n * 8, (size_t)n * 4);
    memcpy(out.c.data(), col + (size_t)n * 12, (size_t)n * 4);
    for (uint32_t t = 0; t < n; ++t) {
        if (o[t] < 1 || out.h[t] < 1 || out.l[t] < 1 || out.c[t] < 1) {
            err = "binary payload: bar " + std::to_string(t) + ": price out of range";
            return false;
        }
    }
    for (uint32_t t = 1; t < n; ++t) {  // spec §3 validity: |dc| <= c_{t-1}
        const int64_t prev = out.c[t - 1];
        const int64_t d = (int64_t)out.c[t] - prev;
        if (d > prev || -d > prev) {
            err = "bar " + std::to_string(t) + ": close moves more than 100% in one bar";
            return false;
        }
    }
    return true;
}

bool binary_header(const uint8_t* buf, size_t len, int32_t& n_bars, std::string& err) {
    if (len < 16 || !is_binary_payload(buf, len)) {
        err = "binary payload: bad header";
        return false;
    }
    const uint32_t n = rd32(buf + 8), flags = rd32(buf + 12);
    if (n < 1 || n > (uint32_t)kMaxBars) {
        err = "binary payload: bar count out of range";
        return false;
    }
    if ((flags & ~1u) != 0) {
        err = "binary payload: unknown flags";
        return false;
    }
    if (len != binary_payload_size((int32_t)n, flags & 1)) {
        err = "binary payload: length does not match the header";
        return false;
    }
    n_bars = (int32_t)n;
    return true;
}

// The batch ingest's decoder: validation (spec §2-§3) and the copy of the columns the strategy
// reads (h, l may be null) into the engine's staging rows in one pass over the payload, in
// L1-sized chunks (the payload may sit at any byte alignment; the chunks are aligned copies).
// On a failure the message comes from parse_binary, so both paths name the same first error.
bool decode_binary_into(const uint8_t* buf, size_t len, int32_t* h, int32_t* l, int32_t* c,
                        std::string& err) {
    int32_t nb = 0;
    if (!binary_header(buf, len, nb, err)) return false;
    const size_t n = (size_t)nb;
    const uint8_t* col = buf + 16;
    constexpr size_t kChunk = 2048;
    alignas(64) int32_t sc[3][kChunk];
    int64_t prev = 0;
    bool bad = false;
    for (size_t t0 = 0; t0 < n && !bad; t0 += kChunk) {
        const size_t m = n - t0 < kChunk ? n - t0 : kChunk;
        int32_t* po = sc[0];
        int32_t* ph = h ? h + t0 : sc[1];
        int32_t* pl = l ? l + t0 : sc[2];
        int32_t* pc = c + t0;
        memcpy(po, col + t0 * 4, m * 4);
        memcpy(ph, col + (n + t0) * 4, m * 4);
        memcpy(pl, col + (2 * n + t0) * 4, m * 4);
        memcpy(pc, col + (3 * n + t0) * 4, m * 4);
        int32_t mn = INT32_MAX;
        for (size_t t = 0; t < m; ++t) {
            const int32_t a = po[t] < ph[t] ? po[t] : ph[t], b = pl[t] < pc[t] ? pl[t] : pc[t];
            const int32_t x = a < b ? a : b;
            mn = x < mn ? x : mn;
        }
        // with every price >= 1, |c_t - c_{t-1}| <= c_{t-1} is c_t <= 2 c_{t-1}
        int64_t over = t0 > 0 ? (int64_t)pc[0] - 2 * prev : INT64_MIN;
        for (size_t t = 1; t < m; ++t) {
            const int64_t d = (int64_t)pc[t] - 2 * (int64_t)pc[t - 1];
            over = d > over ? d : over;
        }
        bad = mn < 1 || over > 0;
        prev = pc[m - 1];
    }
    if (bad) {
        Bars tmp;
        if (parse_binary(buf, len, tmp, err)) err = "binary payload: invalid";
        return false;
    }
    return true;
}

bool parse_job(const uint8_t* buf, size_t len, Bars& out, std::string& err) {
    return is_binary_payload(buf, len) ? parse_binary(buf, len, out, err)
                                       : parse_csv(buf, len, out, err);
}

size_t encode_binary(const int32_t* o, const int32_t* h, const int32_t* l, const int32_t* c,
                     const int64_t* v, int32_t n, uint8_t* out) {
    memcpy(out, kMagic, 8);
    wr32(out + 8, (uint32_t)n);
    wr32(out + 12, v ? 1u : 0u);
    uint8_t* col = out + 16;
    memcpy(col, o, (size_t)n * 4);
    memcpy(col + (size_t)n * 4, h, (size_t)n * 4);
    memcpy(col + (size_t)n * 8, l, (size_t)n * 4);
    memcpy(col + (size_t)n * 12, c, (size_t)n * 4);
    if (v) memcpy(col + (size_t)n * 16, v, (size_t)n * 8);
    return binary_payload_size(n, v != nullptr);
}

// Spec §1 synthetic OHLCV of one symbol on the host (the dispatcher-side payload producer for
// gRPC-fed runs; bit-identical to gen_kernel).
void gen_host(uint64_t seed, int64_t sym, int32_t bars, int32_t freq, int32_t* o, int32_t* h,
              int32_t* l, int32_t* c, int64_t* v) {
    const uint64_t s0 = seed ^ ((uint64_t)sym * 0x9E3779B97F4A7C15ULL);
    const int64_t m = freq == BT_DAILY ? 17320 : 866;
    const uint64_t span = (uint64_t)(2 * m + 1), r = (uint64_t)(m / 4 + 1);
    int64_t prev = 1000000 + (int64_t)(sm64(s0, 0) % 9000001ULL);
    for (int32_t t = 0; t < bars; ++t) {
        const uint64_t base = 1 + 7 * (uint64_t)t;
        int64_t op = prev, cl = prev;
        if (t > 0) {
            const int64_t x = (int64_t)(sm64(s0, base) % span) + (int64_t)(sm64(s0, base + 1) % span) +
                              (int64_t)(sm64(s0, base + 2) % span) +
                              (int64_t)(sm64(s0, base + 3) % span) - 4 * m;
            cl = prev + (x * prev) / 1000000;  // C truncation toward zero
            cl = cl < 10000 ? 10000 : cl;
            cl = cl > 2146435072LL ? 2146435072LL : cl;  // 2^31 - 2^20
        }
        const int64_t hi = op > cl ? op : cl, lo = op < cl ? op : cl;
        int64_t ll = lo - (int64_t)(sm64(s0, base + 5) % r);
        ll = ll < 10000 ? 10000 : ll;
        o[t] = (int32_t)op;
        c[t] = (int32_t)cl;
        h[t] = (int32_t)(hi + (int64_t)(sm64(s0, base + 4) % r));
        l[t] = (int32_t)ll;
        if (v) v[t] = 1000 + (int64_t)(sm64(s0, base + 6) % 100000ULL);
        prev = cl;
    }
}

}  // namespace bt
