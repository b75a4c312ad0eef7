// Pull-mode measurement (not a test, not product code; bench.py --e2e runs
// it): the Click adapter's core in pull context on one thread, through the
// native harness (harness.hh), Queue -> X -> Y -> pulled downstream (as
// ToDevice pulls), with the packets already in the queue.  Prints one JSON
// line per leg (after an untimed warm-up drain of n/4 packets): Mpps over
// the whole drain and the per-pull() latency
// distribution (most pulls hand out a ready packet; a refill launches the
// next batch and routes the one before, hipcore.hh).
//   pull_bench [SCALE]     packet counts divided by SCALE
#include <algorithm>
#include "harness.hh"

namespace {

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

template <class CA, class CB>
void leg(const char *name, const char *ga, const char *gb, uint32_t L, int n, uint32_t batch)
{
    const std::string conf = "BATCH " + std::to_string(batch);
    Host<CA> a(ga, conf, 2);
    Host<CB> b(gb, conf, 2);
    b.upstream = [&a]() { return a.pull(); };
    const std::vector<uint8_t> x = udp_packet(L);
    auto fill = [&](int k) {
        for (int i = 0; i < k; i++) {
            TPacket *p = make(x.data(), L, i);
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
    typedef std::chrono::steady_clock clock;
    const auto t0 = clock::now();
    auto s = t0;
    for (;;) {
        TPacket *p = b.pull();
        const auto e = clock::now();
        lat.push_back((uint32_t)std::chrono::duration_cast<std::chrono::nanoseconds>(e - s).count());
        s = e;
        if (!p)
            break;
        got.push_back(p);
    }
    const double sec = std::chrono::duration<double>(s - t0).count();
    std::vector<uint32_t> v(lat.begin(), lat.end() - 1);     // the pulls that returned a packet
    std::sort(v.begin(), v.end());
    auto pct = [&](double f) { return v.empty() ? 0u : v[(size_t)(f * (double)(v.size() - 1))]; };
    size_t slow = 0;
    for (uint32_t t : v)
        slow += t > 10000;
    std::printf("{\"leg\": \"%s\", \"graph\": \"Queue -> %s -> %s -> pull\", \"batch\": %u, \"bytes\": %u, \"packets\": %d, "
                "\"delivered\": %zu, \"dropped\": %zu, \"seconds\": %.4f, \"mpps\": %.2f, "
                "\"pull_ns\": {\"p50\": %u, \"p99\": %u, \"p999\": %u, \"max\": %u}, \"pulls_over_10us\": %zu, "
                "\"batches\": [%llu, %llu]}\n",
                name, ga, gb, batch, L, n, got.size(), a.out[1].size() + b.out[1].size(), sec,
                (double)got.size() / sec / 1e6, pct(0.5), pct(0.99), pct(0.999), v.empty() ? 0u : v.back(), slow,
                std::stoull(a.handler("batches")) - std::stoull(b0), std::stoull(b.handler("batches")) - std::stoull(b1));
    std::fflush(stdout);
    for (TPacket *p : got)
        TOps::kill(p);
}

}   // namespace

int main(int argc, char **argv)
{
    if (clk_device_count() < 1) {
        std::printf("{\"skip\": \"no gfx950 GPU\"}\n");
        return 0;
    }
    const int scale = argc > 1 ? std::max(1, std::atoi(argv[1])) : 1;
    // BATCH bounds the longest pull (one refill stages a batch and routes
    // the one before): the default and a small one
    for (uint32_t batch : {65536u, 4096u}) {
        leg<CheckIPC, SetC>("pull_c2", "CheckIPHeader", "SetIPChecksum", 64, 2000000 / scale, batch);
        leg<PlainC, SetC>("pull_c3", "CheckUDPHeader", "SetUDPChecksum", 1500, 1000000 / scale, batch);
    }
    return 0;
}
