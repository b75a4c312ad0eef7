// mt_glue.cc -- the element glue from T host threads on one GPU (a
// measurement program, not a test, not product code; bench.py --e2e runs it:
// click -j N's RouterThreads, each with its own glue element and context).
// C2's packets (64 B slots, a 46 B IP packet each) in one registered host
// arena; T threads, each with its own
// context (own stream) and element (ZEROCOPY true, BATCH 65536), each
// pinned to its own physical core, push a contiguous share of the packets
// packet by packet (clk_element_push_burst: push() per packet, flush_async
// per full batch), then flush.  Prints one JSON line per (element, T): the
// time from a common start to the last thread's end (the best of five runs
// after two warm-ups: the box's other tenants share its cores), Mpps, and
// each thread's own rate in that run.
// Built by click_amd.build.build_native_tests() into tests/native/bin/.
//   mt_glue [PACKETS [ELEMENT [staged|zerocopy [THREADS]]]]   (staged: without
//   ZEROCOPY, the packets gathered into pinned staging; the Set elements'
//   checksums then written by the host, not by the kernel over PCIe;
//   THREADS: one thread count instead of 1, 2 and 4)
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <set>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include <pthread.h>
#include <sched.h>

#include "click_amd_cksum.h"
#include "click_amd_elements.h"

static double now()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// allowed CPUs, one per physical core first (then the SMT siblings), the
// physical cores taken spread over the machine (every stride-th: other
// CCDs' L3s, and away from the low-numbered CPUs other processes favour)
static std::vector<int> core_order()
{
    cpu_set_t set;
    CPU_ZERO(&set);
    sched_getaffinity(0, sizeof set, &set);
    std::vector<int> first, rest;
    std::set<std::pair<int, int> > seen;
    for (int c = 0; c < CPU_SETSIZE; c++) {
        if (!CPU_ISSET(c, &set))
            continue;
        int pkg = 0, core = c;
        std::ifstream("/sys/devices/system/cpu/cpu" + std::to_string(c) + "/topology/physical_package_id") >> pkg;
        std::ifstream("/sys/devices/system/cpu/cpu" + std::to_string(c) + "/topology/core_id") >> core;
        (seen.insert({pkg, core}).second ? first : rest).push_back(c);
    }
    std::vector<int> spread;
    const size_t stride = std::max<size_t>(1, first.size() / 8);
    for (size_t o = 0; o < stride; o++)
        for (size_t k = o; k < first.size(); k += stride)
            spread.push_back(first[k]);
    spread.insert(spread.end(), rest.begin(), rest.end());
    return spread;
}

int main(int argc, char **argv)
{
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : (1u << 22);
    const char *only = argc > 2 && argv[2][0] ? argv[2] : nullptr;
    const bool staged = argc > 3 && std::strcmp(argv[3], "staged") == 0;
    const int only_t = argc > 4 ? atoi(argv[4]) : 0;
    const uint32_t SLOT = 64, L = 46;
    const size_t bytes = (size_t)n * SLOT;
    uint8_t *arena = (uint8_t *)std::aligned_alloc(4096, bytes);
    for (uint32_t i = 0; i < n; i++) {
        uint8_t *ip = arena + (size_t)i * SLOT;
        std::memset(ip, 0, SLOT);
        ip[0] = 0x45, ip[3] = L, ip[8] = 64, ip[9] = 17;
        ip[12] = 10, ip[15] = 1, ip[16] = 10, ip[19] = (uint8_t)(2 + (i & 0x7F));
        uint32_t s = 0;
        for (int k = 0; k < 20; k += 2)
            s += (uint32_t)(ip[k] << 8 | ip[k + 1]);
        while (s >> 16)
            s = (s & 0xFFFF) + (s >> 16);
        s = ~s & 0xFFFF;
        ip[10] = (uint8_t)(s >> 8), ip[11] = (uint8_t)s;
    }
    clk_ctx *rctx = nullptr;
    void *dev = nullptr;
    if (clk_ctx_create(0, &rctx) != CLK_SUCCESS || clk_host_register(rctx, arena, bytes, &dev) != CLK_SUCCESS) {
        std::fprintf(stderr, "register: %s\n", clk_last_error(rctx));
        return 2;
    }
    std::vector<uint8_t *> ptrs(n);
    std::vector<uint32_t> lens(n, L);
    std::vector<int32_t> nhs(n, 0);
    for (uint32_t i = 0; i < n; i++)
        ptrs[i] = arena + (size_t)i * SLOT;
    const std::vector<int> cpus = core_order();
    const char *els[] = {"CheckIPHeader", "SetIPChecksum", "IPOutputCombo"};
    for (const char *el : els) {
        if (only && std::strcmp(only, el) != 0)
            continue;
        for (int T : {1, 2, 4}) {
            if (only_t && T != only_t)
                continue;
            std::vector<clk_ctx *> ctx(T);
            std::vector<clk_element *> e(T);
            const std::string conf = std::string(std::strcmp(el, "IPOutputCombo") == 0 ? "1, 10.0.0.1, 1500, " : "") +
                                     (staged ? "BATCH 65536" : "BATCH 65536, ZEROCOPY true");
            for (int k = 0; k < T; k++)
                if (clk_ctx_create(0, &ctx[k]) != CLK_SUCCESS ||
                    clk_element_create(ctx[k], el, conf.c_str(), el, std::strcmp(el, "IPOutputCombo") == 0 ? 5 : 2,
                                       &e[k]) != CLK_SUCCESS) {
                    std::fprintf(stderr, "create %s: %s\n", el, clk_last_error(ctx[k]));
                    return 3;
                }
            std::vector<double> t_own(T), t_end(T), best_own(T, 1e30);
            double best = 1e30;
            std::atomic<int> ready{0};
            std::atomic<bool> go{false};
            const uint32_t share = n / (uint32_t)T;
            double t_start = 0;
            const int REPS = 7;                              // two warm-ups, then the best of five
            for (int rep = 0; rep < REPS; rep++) {
                ready = 0;
                go = false;
                std::vector<std::thread> th;
                for (int k = 0; k < T; k++)
                    th.emplace_back([&, k]() {
                        cpu_set_t s;
                        CPU_ZERO(&s);
                        CPU_SET(cpus[(size_t)k % cpus.size()], &s);
                        pthread_setaffinity_np(pthread_self(), sizeof s, &s);
                        ready++;
                        while (!go.load())
                            ;
                        const double t0 = now();
                        const uint32_t first = share * (uint32_t)k;
                        if (clk_element_push_burst(e[k], ptrs.data() + first, lens.data() + first, nhs.data() + first,
                                                   first, share) != CLK_SUCCESS ||
                            clk_element_flush(e[k]) != CLK_SUCCESS)
                            std::fprintf(stderr, "thread %d: %s\n", k, clk_element_last_error(e[k]));
                        t_end[(size_t)k] = now();
                        t_own[(size_t)k] = t_end[(size_t)k] - t0;
                    });
                while (ready.load() < T)
                    ;
                t_start = now();
                go = true;
                for (auto &x : th)
                    x.join();
                std::vector<uint64_t> tok(share + 1);
                std::vector<int32_t> port(share + 1);
                for (int k = 0; k < T; k++)                  // results outside the timed region
                    clk_element_results(e[k], tok.data(), port.data(), nullptr, share + 1);
                double last = 0;
                for (double x : t_end)
                    last = std::max(last, x - t_start);
                if (rep >= 2 && last < best) {
                    best = last;
                    best_own = t_own;
                }
            }
            const double last = best;
            t_own = best_own;
            double gpu_ms = 0;                           // the element kernels' time (HIP events), all threads
            for (int k = 0; k < T; k++) {
                char buf[64];
                clk_element_read_handler(e[(size_t)k], "gpu_ns", buf, sizeof buf);
                gpu_ms += std::strtod(buf, nullptr) / 1e6 / REPS;   // REPS runs each
            }
            std::printf("{\"element\": \"%s\", \"mode\": \"%s\", \"threads\": %d, \"packets\": %u, \"seconds\": %.4f, "
                        "\"mpps\": %.1f, \"kernel_ms_per_run\": %.2f, \"per_thread_mpps\": [",
                        el, staged ? "staged" : "zerocopy", T, share * (uint32_t)T, last, share * (double)T / last / 1e6,
                        gpu_ms);
            for (int k = 0; k < T; k++)
                std::printf("%s%.1f", k ? ", " : "", share / t_own[(size_t)k] / 1e6);
            std::printf("], \"cpus\": [");
            for (int k = 0; k < T; k++)
                std::printf("%s%d", k ? ", " : "", cpus[(size_t)k % cpus.size()]);
            std::printf("]}\n");
            std::fflush(stdout);
            for (int k = 0; k < T; k++) {
                clk_element_destroy(e[(size_t)k]);
                clk_ctx_destroy(ctx[(size_t)k]);
            }
        }
    }
    clk_host_unregister(rctx, arena);
    clk_ctx_destroy(rctx);
    std::free(arena);
    return 0;
}
