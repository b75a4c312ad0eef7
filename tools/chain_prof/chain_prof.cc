// chain_prof.cc -- tools only (never shipped, not a test): config 1's
// five-element chain (bench.py C1_CHAINS["elements"]) through the chain C
// ABI from C++, as bench.py's elements_chain leg runs it, so the host glue
// can be profiled (tools/chain_prof/run.sh builds the glue's host files into
// this executable).  Prints the median Mpps of the timed runs and
// clk_chain_stats.  With SAMPLES=file it samples the program counter every
// 50 us of CPU time inside the timed region (SIGPROF) and writes one line per
// sample: the offset from the executable's start, or the shared object's
// name; tools/chain_prof/resolve.py turns that into lines and functions.
//   chain_prof FRAME_HEX [RUNS] [BATCH] [combos|elements] [staged|zerocopy] [separate]
// (separate: the members as separate elements, as bench.py's separate legs:
// each takes all frames -- push_burst, flush, results -- then the next)
#include <algorithm>
#include <dlfcn.h>
#include <signal.h>
#include <sys/syscall.h>
#include <sys/time.h>
#include <time.h>
#include <unistd.h>
#include <ucontext.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>
#include "click_amd_cksum.h"
#include "click_amd_elements.h"

extern "C" char __executable_start;
static uintptr_t g_pc[1 << 22];
static volatile size_t g_npc = 0;
static volatile int g_on = 0;

static void on_prof(int, siginfo_t *, void *uc)
{
    if (g_on && g_npc < (1u << 22))
        g_pc[g_npc++] = (uintptr_t)((ucontext_t *)uc)->uc_mcontext.gregs[REG_RIP];
}

static void write_samples(const char *path)
{
    FILE *f = std::fopen(path, "w");
    if (!f)
        return;
    for (size_t k = 0; k < g_npc; k++) {
        Dl_info di;
        if (dladdr((void *)g_pc[k], &di) && di.dli_fbase == (void *)&__executable_start)
            std::fprintf(f, "0x%lx\n", (unsigned long)(g_pc[k] - (uintptr_t)&__executable_start));
        else
            std::fprintf(f, "@%s\n", dladdr((void *)g_pc[k], &di) && di.dli_fname ? di.dli_fname : "?");
    }
    std::fclose(f);
}

int main(int argc, char **argv)
{
    const char *samples = std::getenv("SAMPLES");
    if (argc < 2)
        return 2;
    std::vector<uint8_t> frame;
    for (const char *h = argv[1]; h[0] && h[1]; h += 2)
        frame.push_back((uint8_t)std::strtoul(std::string(h, 2).c_str(), nullptr, 16));
    const int runs = argc > 2 ? std::atoi(argv[2]) : 5;
    const bool zc = argc > 5 && std::string(argv[5]) == "zerocopy";
    const std::string B = ", BATCH " + std::string(argc > 3 ? argv[3] : "65536") + (zc ? ", ZEROCOPY true" : "");
    const uint32_t n = 600000, L = (uint32_t)frame.size();
    clk_ctx *ctx = nullptr;
    if (clk_ctx_create(0, &ctx) != CLK_SUCCESS) {
        std::printf("{\"skip\": \"no GPU\"}\n");
        return 0;
    }
    struct Spec { const char *cls, *conf; int nout; };
    const bool combos = argc > 4 && std::string(argv[4]) == "combos";
    const std::vector<Spec> spec = combos
        ? std::vector<Spec>{{"IPInputCombo", "2, INTERFACES 18.26.4.1/24 18.26.7.1/24", 1},
                            {"IPOutputCombo", "1, 18.26.4.24, 300", 5}}
        : std::vector<Spec>{{"CheckIPHeader", "INTERFACES 18.26.4.1/24 18.26.7.1/24, OFFSET 14", 2},
                            {"IPGWOptions", "18.26.4.24", 2}, {"FixIPSrc", "18.26.4.24", 1},
                            {"DecIPTTL", "", 2}, {"IPFragmenter", "300", 2}};
    const int last = (int)spec.size() - 1;
    std::vector<clk_element *> els;
    for (const Spec &s : spec) {
        clk_element *e = nullptr;
        std::string conf = std::string(s.conf) + (s.conf[0] ? B : B.substr(2));
        if (clk_element_create(ctx, s.cls, conf.c_str(), s.cls, s.nout, &e) != CLK_SUCCESS) {
            std::fprintf(stderr, "%s: %s\n", s.cls, clk_last_error(ctx));
            return 3;
        }
        els.push_back(e);
    }
    const bool sep = argc > 6 && std::string(argv[6]) == "separate";
    clk_chain *c = nullptr;
    if (!sep && clk_chain_create(els.data(), (int)els.size(), &c) != CLK_SUCCESS)
        return 3;
    std::vector<int32_t> nhs(n, 14);
    if (samples) {                                   // armed once the GPU is set up (a signal interrupts its ioctls)
        struct sigaction sa = {};
        sa.sa_sigaction = on_prof;
        sa.sa_flags = SA_SIGINFO | SA_RESTART;
        sigaction(SIGPROF, &sa, nullptr);
        sigevent ev = {};                            // a high-resolution timer aimed at this thread
        ev.sigev_notify = SIGEV_THREAD_ID;
        ev.sigev_signo = SIGPROF;
        ev._sigev_un._tid = (pid_t)syscall(SYS_gettid);
        timer_t tm;
        if (timer_create(CLOCK_MONOTONIC, &ev, &tm) == 0) {
            itimerspec its = {{0, 20000}, {0, 20000}};
            timer_settime(tm, 0, &its, nullptr);
        }
    }
    std::vector<uint64_t> tok(n + 1);
    std::vector<int32_t> mem(n + 1), port(n + 1);
    std::vector<uint32_t> len(n + 1), aux(n + 1), lens(n, L);
    std::vector<uint8_t *> ptrs(n);
    std::vector<double> mpps;
    uint64_t fwd = 0;
    for (int r = 0; r <= runs; r++) {               // run 0 warms up
        std::vector<uint8_t> arena((size_t)n * L);
        for (uint32_t i = 0; i < n; i++) {
            std::copy(frame.begin(), frame.end(), arena.begin() + (size_t)i * L);
            ptrs[i] = arena.data() + (size_t)i * L;
        }
        void *dev = nullptr;
        if (zc && clk_host_register(ctx, arena.data(), arena.size(), &dev) != CLK_SUCCESS) {
            std::fprintf(stderr, "register: %s\n", clk_last_error(ctx));
            return 4;
        }
        const auto t0 = std::chrono::steady_clock::now();
        g_on = r > 0;
        uint64_t k = 0;
        if (sep) {
            for (size_t m = 0; m < els.size(); m++) {
                if (clk_element_push_burst(els[m], ptrs.data(), lens.data(), nhs.data(), 0, n) != CLK_SUCCESS ||
                    clk_element_flush(els[m]) != CLK_SUCCESS) {
                    std::fprintf(stderr, "element: %s\n", clk_element_last_error(els[m]));
                    return 4;
                }
                k = clk_element_results(els[m], tok.data(), port.data(), len.data(), n + 1);
                std::fill(mem.begin(), mem.begin() + (ptrdiff_t)k, (int32_t)m);
            }
        } else {
            if (clk_chain_push_burst(c, ptrs.data(), lens.data(), nullptr, 0, n) != CLK_SUCCESS ||
                clk_chain_flush(c) != CLK_SUCCESS) {
                std::fprintf(stderr, "chain: %s\n", clk_chain_last_error(c));
                return 4;
            }
            k = clk_chain_results(c, tok.data(), mem.data(), port.data(), len.data(), aux.data(), n + 1);
        }
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        g_on = 0;
        if (zc)
            clk_host_unregister(ctx, arena.data());
        fwd = 0;
        for (uint64_t j = 0; j < k; j++)
            fwd += mem[j] == last && port[j] == 0;
        if (r)
            mpps.push_back(n / s / 1e6);
    }
    std::vector<double> sorted = mpps;
    std::sort(sorted.begin(), sorted.end());
    double st[8] = {0};
    if (c)
        clk_chain_stats(c, st, 8);
    std::printf("{\"leg\": \"%s%s_%s\", \"forwarded\": %llu, \"mpps\": %.2f, \"runs_mpps\": [",
                combos ? "combos" : "elements", zc ? "_zerocopy" : "", sep ? "separate" : "chain",
                (unsigned long long)fwd, sorted[sorted.size() / 2]);
    for (size_t k = 0; k < mpps.size(); k++)
        std::printf("%s%.2f", k ? ", " : "", mpps[k]);
    const double per = 1e9 / ((runs + 1) * (double)n);
    std::printf("], \"ns_per_packet\": {\"push\": %.1f, \"gpu\": %.1f, \"h2d\": %.1f, \"route\": %.1f, \"copy_back\": %.1f}}\n",
                st[0] * per, st[2] * per, st[4] * per, st[6] * per, st[7] * per);
    if (samples)
        write_samples(samples);
    if (c)
        clk_chain_destroy(c);
    for (clk_element *e : els)
        clk_element_destroy(e);
    clk_ctx_destroy(ctx);
    return 0;
}
