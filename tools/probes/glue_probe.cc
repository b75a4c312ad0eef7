// glue_probe.cc -- host cost of the element glue per packet, by phase
// (diagnostic, not product).  Config 1's 114 B frame, N copies in a host
// arena; for each element: push_burst of all N into one batch (BATCH >= N, so
// push() alone is timed), flush() (launch + wait + route), and popping the
// results; then with 64K batches (push_burst flushes as they fill).  FixIPSrc (no annotation) and IPGWOptions (no options) decide
// every frame on the host: their time is pure glue bookkeeping.
// Build: g++ -O2 -std=c++17 -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ tools/probes/glue_probe.cc
//        -Lclick_amd -lclick_amd_cksum -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,$PWD/click_amd -o tools/probes/glue_probe
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "click_amd_cksum.h"
#include "click_amd_elements.h"

static double now()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv)
{
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 600000;
    // the fake-iprouter frame: 14 B Ethernet + 20 B IP + 8 B UDP + 72 B
    uint8_t frame[114] = {0};
    frame[12] = 0x08;
    uint8_t *ip = frame + 14;
    ip[0] = 0x45; ip[2] = 0; ip[3] = 100; ip[8] = 64; ip[9] = 17;
    const uint8_t src[4] = {18, 26, 4, 24}, dst[4] = {1, 0, 0, 2};
    std::memcpy(ip + 12, src, 4);
    std::memcpy(ip + 16, dst, 4);
    uint32_t s = 0;
    for (int k = 0; k < 20; k += 2)
        s += (ip[k] << 8) | ip[k + 1];
    s = (s & 0xFFFF) + (s >> 16);
    s = ~s & 0xFFFF;
    ip[10] = s >> 8; ip[11] = s & 0xFF;
    std::vector<uint8_t> arena((size_t)n * 114 + 4096);
    uint8_t *base = (uint8_t *)(((uintptr_t)arena.data() + 4095) & ~uintptr_t(4095));
    std::vector<uint8_t *> ptrs(n);
    std::vector<uint32_t> lens(n, 114);
    std::vector<int32_t> nhs(n, 14);
    for (uint32_t i = 0; i < n; i++) {
        std::memcpy(base + (size_t)i * 114, frame, 114);
        ptrs[i] = base + (size_t)i * 114;
    }
    clk_ctx *ctx = nullptr;
    if (clk_ctx_create(0, &ctx) != CLK_SUCCESS)
        return 2;
    void *dev = nullptr;
    if (clk_host_register(ctx, base, (size_t)n * 114, &dev) != CLK_SUCCESS)
        return 3;
    const char *els[][2] = {{"FixIPSrc", "18.26.4.24"},
                            {"IPGWOptions", "18.26.4.24"},
                            {"CheckIPHeader", "INTERFACES 18.26.4.24/24"},
                            {"DecIPTTL", ""}};
    std::vector<uint64_t> tok(n + 1);
    std::vector<int32_t> port(n + 1);
    std::vector<uint32_t> len(n + 1);
    for (uint32_t batch : {n, 65536u})
    for (int zc = 0; zc < 2; zc++)
        for (auto &e : els) {
            char conf[256];
            snprintf(conf, sizeof conf, "%s%sBATCH %u%s", e[1], e[1][0] ? ", " : "", batch, zc ? ", ZEROCOPY true" : "");
            clk_element *el = nullptr;
            if (clk_element_create(ctx, e[0], conf, "x", 2, &el) != CLK_SUCCESS) {
                fprintf(stderr, "%s: %s\n", e[0], clk_last_error(ctx));
                return 4;
            }
            double best[3] = {1e9, 1e9, 1e9};
            for (int rep = 0; rep < 4; rep++) {
                const double t0 = now();
                if (clk_element_push_burst(el, ptrs.data(), lens.data(), nhs.data(), 0, n) != CLK_SUCCESS)
                    return 5;
                const double t1 = now();
                if (clk_element_flush(el) != CLK_SUCCESS)
                    return 6;
                const double t2 = now();
                const uint64_t got = clk_element_results(el, tok.data(), port.data(), len.data(), n + 1);
                const double t3 = now();
                if (got != n)
                    return 7;
                const double d[3] = {t1 - t0, t2 - t1, t3 - t2};
                for (int k = 0; k < 3; k++)
                    if (d[k] < best[k])
                        best[k] = d[k];
            }
            printf("{\"element\": \"%s\", \"zerocopy\": %d, \"n\": %u, \"batch\": %u, \"push_ns\": %.2f, "
                   "\"flush_ns\": %.2f, \"results_ns\": %.2f}\n",
                   e[0], zc, n, batch, best[0] / n * 1e9, best[1] / n * 1e9, best[2] / n * 1e9);
            clk_element_destroy(el);
        }
    clk_host_unregister(ctx, base);
    clk_ctx_destroy(ctx);
    return 0;
}
