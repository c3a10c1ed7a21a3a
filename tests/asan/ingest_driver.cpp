// ingest_driver.cpp — host-only harness of the Job.File ingest (csv.cpp, payload.cpp) for the
// AddressSanitizer / UBSan CPU test (tests/test_ingest_asan_cpu.py). For every input file: the
// standalone parser, and the batch path's header + in-place decode for binary payloads.
#include <cstdio>
#include <string>
#include <vector>

#include "csv.h"

int main(int argc, char** argv) {
    int accepted = 0;
    for (int i = 1; i < argc; ++i) {
        FILE* f = std::fopen(argv[i], "rb");
        if (!f) return 2;
        std::vector<uint8_t> buf;
        uint8_t chunk[65536];
        size_t n;
        while ((n = std::fread(chunk, 1, sizeof chunk, f)) > 0) buf.insert(buf.end(), chunk, chunk + n);
        std::fclose(f);
        // an exact-size heap copy, so any read past the end is an ASan error
        uint8_t* data = buf.empty() ? nullptr : new uint8_t[buf.size()];
        if (data) std::copy(buf.begin(), buf.end(), data);
        bt::Bars out;
        std::string err;
        const bool ok = bt::parse_job(data, buf.size(), out, err);
        accepted += ok ? 1 : 0;
        int32_t bars = 0;
        if (data && bt::is_binary_payload(data, buf.size()) && bt::binary_header(data, buf.size(), bars, err)) {
            std::vector<int32_t> h(bars), l(bars), c(bars);
            bt::decode_binary_into(data, buf.size(), h.data(), l.data(), c.data(), err);
        }
        delete[] data;
    }
    std::printf("accepted %d of %d\n", accepted, argc - 1);
    return 0;
}
