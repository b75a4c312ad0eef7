// Test harness (not product code): runs click_amd/host/ingest.cc's pcap
// reader over every file named on the command line, sizing pass then read
// pass, so that tests/test_ingest.py can build it with -fsanitize=address,
// undefined and feed it mutated files.  The library's error hook is the
// only symbol ingest.cc needs from the rest of the library.
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "click_amd_ingest.h"

extern "C" int clk_ctx_set_error_internal(clk_ctx *, const char *) { return 0; }

int main(int argc, char **argv)
{
    unsigned long records = 0;
    for (int a = 1; a < argc; a++) {
        clk_pcap_info info;
        for (int fip = 0; fip < 2; fip++) {
            if (clk_pcap_read(argv[a], fip, nullptr, 0, nullptr, nullptr, nullptr, nullptr, nullptr, 0, &info) < 0)
                continue;
            const size_t n = info.records ? info.records : 1;
            std::vector<uint8_t> arena(info.arena_bytes ? info.arena_bytes : 1);
            std::vector<uint64_t> off(n), ts(n);
            std::vector<uint32_t> cap(n), wl(n);
            std::vector<int32_t> nh(n);
            if (clk_pcap_read(argv[a], fip, arena.data(), info.arena_bytes, off.data(), cap.data(), wl.data(),
                              ts.data(), nh.data(), info.records, &info) < 0)
                return 3;
            for (size_t k = 0; k < info.records; k++)
                if (off[k] + cap[k] > info.arena_bytes || (nh[k] >= 0 && (uint32_t)nh[k] >= cap[k]))
                    return 4;
            records += info.records;
        }
    }
    printf("%lu\n", records);
    return 0;
}
