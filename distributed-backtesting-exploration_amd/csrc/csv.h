// csv.h — host-side ingest of Job.File bytes (spec §2): CSV text or binary columns.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <string>
#include <vector>

namespace bt {

constexpr int32_t kMaxBars = 1 << 22;

struct Bars {
    std::vector<int32_t> h, l, c;  // ticks; open and volume are validated, not kept
};

bool parse_csv(const uint8_t* buf, size_t len, Bars& out, std::string& err);

// Binary columnar payload (payload.cpp): detection, decode, encode, host generator.
bool is_binary_payload(const uint8_t* buf, size_t len);
size_t binary_payload_size(int32_t n, bool volume);
bool parse_binary(const uint8_t* buf, size_t len, Bars& out, std::string& err);
// Header check only (magic, bar count, flags, exact length): the batch ingest sizes its rows
// from it before decoding.
bool binary_header(const uint8_t* buf, size_t len, int32_t& n_bars, std::string& err);
// Validate and copy the high/low/close columns (h, l may be null) in one pass.
bool decode_binary_into(const uint8_t* buf, size_t len, int32_t* h, int32_t* l, int32_t* c,
                        std::string& err);
// Job.File in either format (CSV or binary columns), dispatched on the magic.
bool parse_job(const uint8_t* buf, size_t len, Bars& out, std::string& err);
size_t encode_binary(const int32_t* o, const int32_t* h, const int32_t* l, const int32_t* c,
                     const int64_t* v, int32_t n, uint8_t* out);
void gen_host(uint64_t seed, int64_t sym, int32_t bars, int32_t freq, int32_t* o, int32_t* h,
              int32_t* l, int32_t* c, int64_t* v);

}  // namespace bt
