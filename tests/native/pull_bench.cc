// Adapter-core measurement (not a test, not product code; bench.py --e2e
// runs it): config 1 pushed through five elements or one chain, and the
// Click adapter's core in pull context on one thread, through the
// native harness (harness.hh), Queue -> X -> Y -> pulled downstream (as
// ToDevice pulls), with the packets already in the queue.  Prints one JSON
// line per leg (after an untimed warm-up drain of n/4 packets): Mpps over
// the whole drain and the per-pull() latency
// distribution (most pulls hand out a ready packet; a refill launches the
// next batch and routes the one before, hipcore.hh).
//   pull_bench [SCALE]     packet counts divided by SCALE
//   pull_bench SCALE chain REPS   the push_c1 chain leg only, REPS times
//                                 (BATCH 2048, the Click adapter's default)
//   pull_bench SCALE pull         the pull legs only
#include <algorithm>
#include <x86intrin.h>
#include "harness.hh"

namespace {

const uint32_t ADAPTER_BATCH = 2048;                    // hipbatch.hh HIPBatchElement::ADAPTER_BATCH

uint16_t fold_sum(const uint8_t *b, uint32_t n, uint32_t acc)   // RFC 1071 over n bytes
{
    for (uint32_t k = 0; k + 1 < n; k += 2)
        acc += (uint32_t)(b[k] << 8 | b[k + 1]);
    if (n & 1)
        acc += (uint32_t)b[n - 1] << 8;
    while (acc >> 16)
        acc = (acc & 0xFFFF) + (acc >> 16);
    return (uint16_t)~acc;
}

// One IPv4/UDP packet of L bytes with both checksums set.
std::vector<uint8_t> udp_packet(uint32_t L)
{
    std::vector<uint8_t> b(L, 0);
    for (uint32_t k = 28; k < L; k++)
        b[k] = (uint8_t)(k * 131 + 7);
    b[0] = 0x45;
    b[2] = (uint8_t)(L >> 8), b[3] = (uint8_t)L;
    b[8] = 64, b[9] = 17;
    const uint8_t src[4] = {10, 0, 0, 1}, dst[4] = {10, 0, 0, 2};
    std::memcpy(b.data() + 12, src, 4);
    std::memcpy(b.data() + 16, dst, 4);
    b[20] = 0x30, b[21] = 0x39, b[22] = 0x00, b[23] = 0x35;
    const uint32_t ul = L - 20;
    b[24] = (uint8_t)(ul >> 8), b[25] = (uint8_t)ul;
    const uint16_t ip = fold_sum(b.data(), 20, 0);
    b[10] = (uint8_t)(ip >> 8), b[11] = (uint8_t)ip;
    uint32_t pseudo = (10 << 8) + 1 + (10 << 8) + 2 + 17 + ul;   // src, dst, proto, UDP length
    uint16_t u = fold_sum(b.data() + 20, ul, pseudo);
    if (u == 0)
        u = 0xFFFF;
    b[26] = (uint8_t)(u >> 8), b[27] = (uint8_t)u;
    return b;
}

// zerocopy: both elements ZEROCOPY true, the packets in a registered
// receive ring (up to 384 MiB of 64 B-aligned slots, the bytes written once;
// the kernels read them, and the Set element's kernel writes its checksum,
// where they lie) instead of packets of their own
template <class CA, class CB>
void leg(const char *name, const char *ga, const char *gb, uint32_t L, int n, uint32_t batch, bool zerocopy = false)
{
    const std::string conf = "BATCH " + std::to_string(batch) + (zerocopy ? ", ZEROCOPY true" : "");
    const std::vector<uint8_t> x = udp_packet(L);
    const size_t SLOT = (L + 63) & ~size_t(63);
    const size_t RING = std::min<size_t>((size_t)n, (size_t(384) << 20) / SLOT);
    uint8_t *arena = nullptr;
    clk_ctx *rctx = nullptr;
    std::vector<TPacket> pk;
    if (zerocopy) {
        arena = (uint8_t *)std::aligned_alloc(4096, RING * SLOT);
        for (size_t k = 0; k < RING; k++)
            std::memcpy(arena + k * SLOT, x.data(), L);
        void *dbase = nullptr;
        if (clk_ctx_create(0, &rctx) != CLK_SUCCESS || clk_host_register(rctx, arena, RING * SLOT, &dbase) != CLK_SUCCESS) {
            std::printf("{\"leg\": \"%s_zerocopy\", \"error\": \"clk_host_register failed\"}\n", name);
            std::free(arena);
            return;
        }
        pk.resize((size_t)n);
    }
    Host<CA> a(ga, conf, 2);
    Host<CB> b(gb, conf, 2);
    b.upstream = [&a]() { return a.pull(); };
    auto fill = [&](int k) {
        for (int i = 0; i < k; i++) {
            TPacket *p;
            if (zerocopy) {                            // the ring's slot, metadata reset
                p = &pk[(size_t)i];
                p->raw = arena + (size_t)i % RING * SLOT;
                p->ring = true;
                p->off = 0, p->len = L;
                p->a = TAnno();
                p->a.id = i;
            } else {
                p = make(x.data(), L, i);
            }
            p->nh = 0;
            a.input.push_back(p);
        }
    };
    // warm-up (untimed): the first refills allocate the staging and device
    // buffers and load the kernels
    fill(n / 4);
    for (TPacket *p; (p = b.pull()) != nullptr;)
        TOps::kill(p);
    const std::string b0 = a.handler("batches"), b1 = b.handler("batches");
    fill(n);
    std::vector<TPacket *> got;
    std::vector<uint32_t> lat;
    got.reserve((size_t)n);
    lat.reserve((size_t)n + 1);
    // each pull timed with the TSC (a few ns, where a clock_gettime call per
    // pull would add ~20 ns to every packet), scaled by the steady clock
    typedef std::chrono::steady_clock clock;
    const auto t0 = clock::now();
    const uint64_t c0 = __rdtsc();
    uint64_t s = c0;
    for (;;) {
        TPacket *p = b.pull();
        const uint64_t e = __rdtsc();
        lat.push_back((uint32_t)std::min<uint64_t>(e - s, 0xFFFFFFFFu));
        s = e;
        if (!p)
            break;
        got.push_back(p);
    }
    const double sec = std::chrono::duration<double>(clock::now() - t0).count();
    const double ns_per_tick = s > c0 ? sec * 1e9 / (double)(s - c0) : 1.0;
    for (uint32_t &t : lat)
        t = (uint32_t)std::min(4.0e9, t * ns_per_tick);
    std::vector<uint32_t> v(lat.begin(), lat.end() - 1);     // the pulls that returned a packet
    std::sort(v.begin(), v.end());
    auto pct = [&](double f) { return v.empty() ? 0u : v[(size_t)(f * (double)(v.size() - 1))]; };
    size_t slow = 0;
    for (uint32_t t : v)
        slow += t > 10000;
    std::printf("{\"leg\": \"%s%s\", \"graph\": \"Queue -> %s -> %s -> pull\", \"batch\": %u, \"bytes\": %u, \"packets\": %d, "
                "\"delivered\": %zu, \"dropped\": %zu, \"seconds\": %.4f, \"mpps\": %.2f, "
                "\"pull_ns\": {\"p50\": %u, \"p99\": %u, \"p999\": %u, \"max\": %u}, \"pulls_over_10us\": %zu, "
                "\"batches\": [%llu, %llu]}\n",
                name, zerocopy ? "_zerocopy" : "", ga, gb, batch, L, n, got.size(), a.out[1].size() + b.out[1].size(), sec,
                (double)got.size() / sec / 1e6, pct(0.5), pct(0.99), pct(0.999), v.empty() ? 0u : v.back(), slow,
                std::stoull(a.handler("batches")) - std::stoull(b0), std::stoull(b.handler("batches")) - std::stoull(b1));
    std::fflush(stdout);
    for (TPacket *p : got)
        TOps::kill(p);
    if (zerocopy) {
        clk_host_unregister(rctx, arena);
        clk_ctx_destroy(rctx);
        std::free(arena);
    }
}

// Push context, config 1 (fake-iprouter's forwarding path: 114 B frames,
// CheckIPHeader OFFSET 14 -> IPGWOptions -> FixIPSrc -> DecIPTTL ->
// IPFragmenter), through the adapter core: five elements, each output 0
// pushing into the next, or one chain (hipcore chains, as the Click adapter
// forms it).  Two sources: the frames all made before the clock starts (each
// push then meets a packet out of the host caches), or -- as fake-iprouter's
// InfiniteSource does, pushing a clone of its packet that the first writer
// uniqueifies (infinitesource.cc:125-153) -- each frame made from a packet
// pool (Click's, packet.cc) as it is pushed, Discard after the last element;
// all are pushed, then the latency timer's flush runs.
std::vector<uint8_t> c1_frame()
{
    std::vector<uint8_t> f(14, 0);
    f[12] = 0x08;
    const std::vector<uint8_t> ip = udp_packet(100);
    f.insert(f.end(), ip.begin(), ip.end());
    return f;
}

void push_c1(int n, bool chained, uint32_t batch, bool source = false)
{
    g_pool.on = source;
    const std::string B = "BATCH " + std::to_string(batch);
    const std::vector<uint8_t> f = c1_frame();
    std::vector<TPacket *> in((size_t)n);
    auto fill = [&]() {
        for (int i = 0; i < n; i++)
            in[(size_t)i] = make(f.data(), f.size(), i);
    };
    double sec = 0;
    size_t out0 = 0;
    if (chained) {
        Member<CheckIPC> c0("CheckIPHeader", "OFFSET 14, " + B, 2);
        c0.cls.offset = 14;
        Member<GWOptC> c1("IPGWOptions", "10.0.0.2, " + B, 2);
        Member<FixSrcC> c2("FixIPSrc", "10.0.0.2, " + B, 1);
        Member<DecTTLC> c3("DecIPTTL", B, 2);
        Member<FragC> c4("IPFragmenter", "1500, " + B, 2);
        c4.cls.mtu = 1500;
        ChainHost ch({&c0, &c1, &c2, &c3, &c4});
        size_t fwd = 0;
        if (source)                                     // Discard after the chain
            ch.sink = [&fwd](int k, int port, TPacket *p) {
                fwd += k == 4 && port == 0;
                TOps::kill(p);
            };
        for (int run = 0; run < 2; run++) {            // the first run warms up
            if (!source)
                fill();
            const auto t0 = std::chrono::steady_clock::now();
            if (source)                                 // packets made as they are pushed
                for (int i = 0; i < n; i++)
                    ch.push(make(f.data(), f.size(), i));
            else
                for (TPacket *p : in)
                    ch.push(p);
            ch.timer();
            sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            out0 = source ? fwd : c4.out[0].size();
            fwd = 0;
            for (auto *m : ch.m)
                for (auto &v : m->out) {
                    for (TPacket *p : v)
                        TOps::kill(p);
                    v.clear();
                }
        }
    } else {
        Host<CheckIPC> h0("CheckIPHeader", "OFFSET 14, " + B, 2);
        h0.cls.offset = 14;
        Host<GWOptC> h1("IPGWOptions", "10.0.0.2, " + B, 2);
        Host<FixSrcC> h2("FixIPSrc", "10.0.0.2, " + B, 1);
        Host<DecTTLC> h3("DecIPTTL", B, 2);
        Host<FragC> h4("IPFragmenter", "1500, " + B, 2);
        h4.cls.mtu = 1500;
        h0.downstream = [&](TPacket *p) { h1.push(p); };
        h1.downstream = [&](TPacket *p) { h2.push(p); };
        h2.downstream = [&](TPacket *p) { h3.push(p); };
        h3.downstream = [&](TPacket *p) { h4.push(p); };
        size_t fwd = 0;
        if (source)                                     // Discard after the last element
            h4.downstream = [&fwd](TPacket *p) {
                fwd++;
                TOps::kill(p);
            };
        for (int run = 0; run < 2; run++) {
            if (!source)
                fill();
            const auto t0 = std::chrono::steady_clock::now();
            if (source)                                 // packets made as they are pushed
                for (int i = 0; i < n; i++)
                    h0.push(make(f.data(), f.size(), i));
            else
                for (TPacket *p : in)
                    h0.push(p);
            h0.timer();
            h1.timer();
            h2.timer();
            h3.timer();
            h4.timer();
            sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            out0 = source ? fwd : h4.out[0].size();
            fwd = 0;
            for (auto *h : std::initializer_list<std::vector<std::vector<TPacket *> > *>{&h0.out, &h1.out, &h2.out,
                                                                                         &h3.out, &h4.out})
                for (auto &v : *h) {
                    for (TPacket *p : v)
                        TOps::kill(p);
                    v.clear();
                }
        }
    }
    g_pool.on = false;
    std::printf("{\"leg\": \"push_c1_%s%s\", \"graph\": \"CheckIPHeader(14) -> IPGWOptions -> FixIPSrc -> DecIPTTL -> "
                "IPFragmenter(1500), %s\", \"batch\": %u, \"bytes\": %zu, \"packets\": %d, \"forwarded\": %zu, "
                "\"seconds\": %.4f, \"mpps\": %.2f}\n",
                chained ? "chain" : "elements", source ? "_source" : "", chained ? "one chain" : "five elements", batch, f.size(), n, out0, sec,
                (double)n / sec / 1e6);
    std::fflush(stdout);
}

// Push context, C3: CheckUDPHeader alone (1500 B packets), each packet
// pushed through the core as Click pushes it (one push per packet from the
// source, Discard after the element), staged (the glue gathers every packet
// into pinned staging) or ZEROCOPY (the kernel reads the packet where it
// lies, in host memory registered with clk_host_register).  The packets
// come from a receive ring of RING 1536 B buffers (384 MiB: past the host's
// last-level cache, so a packet is not cache-resident when it is pushed,
// as NIC-written memory is not), the bytes written once; the source hands
// out the next one with its metadata reset, as FromDPDKDevice wraps the
// mbufs of its ring (fromdpdkdevice.cc:98-115).
void push_c3(int n, bool zerocopy, uint32_t batch)
{
    enum { RING = 262144, SLOT = 1536, L = 1500 };
    uint8_t *arena = (uint8_t *)std::aligned_alloc(4096, (size_t)RING * SLOT);
    const std::vector<uint8_t> x = udp_packet(L);
    for (size_t k = 0; k < RING; k++)
        std::memcpy(arena + k * SLOT, x.data(), L);
    std::vector<TPacket> ring(RING);
    for (size_t k = 0; k < RING; k++) {
        ring[k].raw = arena + k * SLOT;
        ring[k].ring = true;
    }
    clk_ctx *rctx = nullptr;
    void *dbase = nullptr;
    if (zerocopy && (clk_ctx_create(0, &rctx) != CLK_SUCCESS ||
                     clk_host_register(rctx, arena, (size_t)RING * SLOT, &dbase) != CLK_SUCCESS)) {
        std::printf("{\"leg\": \"push_c3_zerocopy\", \"error\": \"clk_host_register failed\"}\n");
        std::free(arena);
        return;
    }
    const std::string conf = "BATCH " + std::to_string(batch) + (zerocopy ? ", ZEROCOPY true" : "");
    double sec = 0;
    size_t fwd = 0;
    {
        Host<PlainC> h("CheckUDPHeader", conf, 2);
        h.downstream = [&fwd](TPacket *p) {           // Discard
            fwd++;
            TOps::kill(p);
        };
        size_t next = 0;
        for (int run = 0; run < 2; run++) {            // the first run warms up
            fwd = 0;
            const auto t0 = std::chrono::steady_clock::now();
            for (int i = 0; i < n; i++) {
                TPacket *p = &ring[next];
                next = next + 1 == RING ? 0 : next + 1;
                p->off = 0, p->len = L, p->nh = 0;     // as received: the IP header at data()
                p->a.id = i;
                h.push(p);
            }
            h.timer();
            sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        }
    }
    if (rctx) {
        clk_host_unregister(rctx, arena);
        clk_ctx_destroy(rctx);
    }
    std::free(arena);
    std::printf("{\"leg\": \"push_c3_%s\", \"graph\": \"source -> CheckUDPHeader -> Discard\", \"batch\": %u, "
                "\"bytes\": %d, \"packets\": %d, \"forwarded\": %zu, \"seconds\": %.4f, \"mpps\": %.2f, "
                "\"gib_s\": %.2f}\n",
                zerocopy ? "zerocopy" : "staged", batch, (int)L, n, fwd, sec, (double)n / sec / 1e6,
                (double)n * L / sec / (1u << 30));
    std::fflush(stdout);
}

}   // namespace

int main(int argc, char **argv)
{
    if (clk_device_count() < 1) {
        std::printf("{\"skip\": \"no gfx950 GPU\"}\n");
        return 0;
    }
    const int scale = argc > 1 ? std::max(1, std::atoi(argv[1])) : 1;
    if (argc > 3 && (std::string(argv[2]) == "chain" || std::string(argv[2]) == "chain_source")) {
        // profiling (tools/core_profile): the chain leg only
        for (int r = std::atoi(argv[3]); r > 0; r--)
            push_c1(600000 / scale, true, ADAPTER_BATCH, std::string(argv[2]) == "chain_source");
        return 0;
    }
    if (argc > 2 && std::string(argv[2]) == "pull") {   // the pull legs only
        for (uint32_t batch : {65536u, 4096u})
            for (bool zc : {false, true}) {
                leg<CheckIPC, SetC>("pull_c2", "CheckIPHeader", "SetIPChecksum", 64, 2000000 / scale, batch, zc);
                leg<PlainC, SetC>("pull_c3", "CheckUDPHeader", "SetUDPChecksum", 1500, 1000000 / scale, batch, zc);
            }
        return 0;
    }
    if (argc > 2 && std::string(argv[2]) == "c3") {     // the C3 push legs only
        for (bool zc : {false, true})
            push_c3(2000000 / scale, zc, ADAPTER_BATCH);
        return 0;
    }
    for (bool zc : {false, true})
        push_c3(2000000 / scale, zc, ADAPTER_BATCH);
    // BATCH bounds the longest pull (one refill stages a batch and routes
    // the one before): the default and a small one
    for (uint32_t batch : {65536u, 8192u})
        for (bool source : {false, true}) {
            push_c1(600000 / scale, false, batch, source);
            push_c1(600000 / scale, true, batch, source);
        }
    for (uint32_t batch : {65536u, 4096u})
        for (bool zc : {false, true}) {
            leg<CheckIPC, SetC>("pull_c2", "CheckIPHeader", "SetIPChecksum", 64, 2000000 / scale, batch, zc);
            leg<PlainC, SetC>("pull_c3", "CheckUDPHeader", "SetUDPChecksum", 1500, 1000000 / scale, batch, zc);
        }
    return 0;
}
