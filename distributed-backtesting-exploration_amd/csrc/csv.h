// csv.h — host-side ingest of Job.File bytes (spec §2).
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

}  // namespace bt
