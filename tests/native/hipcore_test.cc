// Test harness (not product code): drives the Click adapter's core
// (click_integration/elements/hip/hipcore.hh) with a packet type, lock and
// host of its own -- no Click headers -- on the GPU through the element glue
// (include/click_amd_elements.h), and checks every output against the CPU
// oracle (oracle/cksum_oracle.h).  tests/test_gpu_adapter_core.py runs it.
//
// Scenarios: push context with double-buffered batches and the latency
// timer; pull context (one batch per refill, output 1 pushed); IPFragmenter
// extras with annotations copied from their parent; a failed flush, then
// the retry; the retry limit (abandon, runcount released); a downstream
// element that pushes back into the element while it delivers; four
// threads with a state each while a "home" thread fires their timers;
// cleanup of a held partial batch.  Prints one line per scenario and exits
// nonzero if any fails.
#include <atomic>
#include <cstdio>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "click_amd_elements.h"
#include "../../oracle/cksum_oracle.h"
#include "../../click_integration/elements/hip/hipcore.hh"

extern "C" void clk_glue_inject_fault_internal(int nth);

namespace {

struct TPacket {
    std::vector<uint8_t> mem;
    size_t off = 0, len = 0;
    int nh = -1;
    long id = 0;
    uint32_t paint = 0, dst = 0, prob = 0;
    bool fix_src = false, bcast = false;
    uint8_t *data() { return mem.data() + off; }
};

std::atomic<long> g_live{0};

TPacket *make(const uint8_t *bytes, size_t len, long id)
{
    TPacket *p = new TPacket;
    p->mem.assign(bytes, bytes + len);
    p->len = len;
    p->id = id;
    g_live++;
    return p;
}

TPacket *clone(const TPacket *q)
{
    TPacket *p = new TPacket(*q);
    g_live++;
    return p;
}

struct TLock {
    std::mutex m;
    void acquire() { m.lock(); }
    void release() { m.unlock(); }
};

class Host;
typedef hipcore::Core<TPacket, Host, TLock> Core;
typedef hipcore::State<TPacket, TLock> St;

// The test's "element": what HIPBatchElement and its subclasses do in Click,
// with the outputs recorded.
class Host {
  public:
    std::string cls;
    Core core;
    std::vector<St> st;
    std::mutex out_mu;
    std::vector<std::vector<TPacket *> > out;   // per output port, in push order
    std::atomic<int> runcount{0};
    std::vector<int> sched;                     // per state: scheduled flag
    std::deque<TPacket *> input;                // pull context source
    std::vector<std::string> chat, msgs;
    std::atomic<long> kills{0};
    uint32_t color = 0;
    // re-entrancy probe: called on every output-0 packet (may push back in)
    void (*on_out0)(Host &, TPacket *) = nullptr;

    Host(const std::string &c, const std::string &conf, int noutputs, int nstates = 1)
        : cls(c), st(nstates), out(5), sched(nstates, 0)
    {
        for (int k = 0; k < nstates; k++) {
            st[k].id = k;
            if (clk_ctx_create(0, &st[k].ctx) != CLK_SUCCESS ||
                clk_element_create(st[k].ctx, c.c_str(), conf.c_str(), c.c_str(), noutputs, &st[k].e) != CLK_SUCCESS) {
                std::fprintf(stderr, "create %s(%s): %s\n", c.c_str(), conf.c_str(), clk_last_error(st[k].ctx));
                std::exit(3);
            }
        }
        char buf[64];
        clk_element_read_handler(st[0].e, "batch", buf, sizeof buf);
        core.set_batch((uint32_t)std::strtoul(buf, nullptr, 10));
    }
    ~Host()
    {
        for (St &t : st)
            core.cleanup(*this, t);
        for (auto &v : out)
            for (TPacket *p : v)
                kill(p);
    }

    // ---- the core's host interface --------------------------------------------
    TPacket *prepare(TPacket *p, uint32_t *anno, TPacket **extra)
    {
        if (cls == "IPOutputCombo") {
            if (p->bcast) {
                *anno = CLK_ANNO_BCAST;
                return p;
            }
            *anno = CLK_ANNO_PAINT(p->paint) | (p->fix_src ? CLK_ANNO_FIX_IP_SRC : 0);
            if (p->paint == color)
                *extra = clone(p);
        }
        return p;
    }
    uint8_t *data(TPacket *p) { return p->data(); }
    uint32_t length(TPacket *p) { return (uint32_t)p->len; }
    int32_t nh_offset(TPacket *p) { return p->nh; }
    bool primary(int32_t port, uint32_t aux)
    {
        if (cls == "IPOutputCombo")
            return aux != CLK_AUX_CLONE;
        if (cls == "IPFragmenter")
            return aux == 0;
        (void)port;
        return true;
    }
    TPacket *make_packet(clk_element *e, uint32_t key)
    {
        int64_t n = clk_element_take_packet(e, key, nullptr, 0);
        if (n < 0)
            return nullptr;
        std::vector<uint8_t> b((size_t)n);
        clk_element_take_packet(e, key, b.data(), b.size());
        TPacket *p = make(b.data(), b.size(), -1);
        p->nh = 0;
        return p;
    }
    int finish(St &t, hipcore::Routed<TPacket> &r, TPacket **outp)
    {
        if (cls == "IPOutputCombo") {
            if (r.extra && !r.p) {               // the PaintTee clone
                *outp = r.extra;
                return 1;
            }
            if (r.port == CLK_PORT_KILL) {
                if (r.p) kill(r.p);
                if (r.extra) kill(r.extra);
                return -1;
            }
            if (r.port == CLK_PORT_OUT2)
                r.p->prob = r.aux;
            if (r.anno & CLK_ANNO_FIX_IP_SRC)
                r.p->fix_src = false;
            *outp = r.p;
            return r.port;
        }
        if (cls == "IPFragmenter") {
            if (r.made) {                        // a fragment after the first
                if (r.parent)
                    r.made->paint = r.parent->paint, r.made->id = r.parent->id;
                *outp = r.made;
                return 0;
            }
            TPacket *p = r.p;
            if (!p)
                return -1;
            if (r.port == CLK_PORT_OUT0 && r.len < p->len) {   // the first fragment: a clone cut to len
                TPacket *first = clone(p);
                first->len = r.len;
                if (t.frag_parent)
                    kill(t.frag_parent);
                t.frag_parent = p;
                *outp = first;
                return 0;
            }
            if (r.port == CLK_PORT_KILL) {
                kill(p);
                return -1;
            }
            *outp = p;
            return r.port;
        }
        TPacket *p = r.p;
        if (!p)
            return -1;
        if (r.port == CLK_PORT_KILL) {
            kill(p);
            return -1;
        }
        if (cls == "CheckIPHeader" && r.port == CLK_PORT_OUT0) {   // checkipheader.cc:213-223
            if (p->len > r.len)
                p->len = r.len;
            std::memcpy(&p->dst, p->data() + 16, 4);
        }
        *outp = p;
        return r.port;
    }
    void end_of_batch(St &t)
    {
        if (t.frag_parent) {
            kill(t.frag_parent);
            t.frag_parent = nullptr;
        }
    }
    void output_push(int port, TPacket *p)
    {
        {
            std::lock_guard<std::mutex> g(out_mu);
            out[(size_t)port].push_back(p);
        }
        if (port == 0 && on_out0)
            on_out0(*this, p);
    }
    TPacket *input_pull()
    {
        if (input.empty())
            return nullptr;
        TPacket *p = input.front();
        input.pop_front();
        return p;
    }
    void kill(TPacket *p)
    {
        kills++;
        g_live--;
        delete p;
    }
    void adjust_runcount(int d) { runcount += d; }
    void schedule(St &t, unsigned) { sched[(size_t)t.id] = 1; }
    void unschedule(St &t) { sched[(size_t)t.id] = 0; }
    bool scheduled(St &t) { return sched[(size_t)t.id] != 0; }
    void chatter(const char *s) { chat.push_back(s); }
    void message(const char *s) { msgs.push_back(s); }

    void push(TPacket *p, int state = 0) { core.push(*this, st[(size_t)state], p); }
    TPacket *pull(int state = 0) { return core.pull(*this, st[(size_t)state]); }
    void timer(int state = 0) { core.timer(*this, st[(size_t)state]); }
    std::string handler(const char *h, int state = 0)
    {
        char buf[256];
        clk_element_read_handler(st[(size_t)state].e, h, buf, sizeof buf);
        return buf;
    }
};

int g_fail = 0;
#define CHECK(c)                                                                    \
    do {                                                                            \
        if (!(c)) {                                                                 \
            std::printf("  FAILED %s:%d: %s\n", __FILE__, __LINE__, #c);            \
            ok = false;                                                             \
        }                                                                           \
    } while (0)

void report(const char *name, bool ok)
{
    std::printf("%s %s\n", ok ? "PASS" : "FAIL", name);
    if (!ok)
        g_fail++;
}

// An IPv4/UDP packet of L bytes (synthetic, checksums set by the oracle).
std::vector<uint8_t> udp_bytes(uint32_t L, long id, int proto = 17)
{
    std::vector<uint8_t> b(L);
    oracle_gen_packet(b.data(), L, proto, 0x5EED, (uint64_t)id);
    oracle_set_ip_checksum(b.data(), L);
    if (proto == 17 && L >= 28)
        oracle_set_udp_checksum(b.data(), L);
    return b;
}

// 1. push context: CheckIPHeader, double-buffered full batches, the timer
void push_check_ip()
{
    bool ok = true;
    Host h("CheckIPHeader", "BATCH 1000", 2);
    const int n = 2500;
    std::vector<int> expect_code(n);
    std::vector<uint32_t> expect_len(n);
    for (int i = 0; i < n; i++) {
        std::vector<uint8_t> b = udp_bytes(100, i);
        if (i % 7 == 3) b[13] ^= 0x10;                 // bad checksum
        if (i % 13 == 5) b[0] = 0x65;                  // version 6
        if (i % 11 == 2) b.resize(108, 0xAB);          // trailing bytes: trimmed to ip_len
        if (i % 29 == 7) b.resize(10);                 // tiny
        expect_code[i] = oracle_check_ip_header(b.data(), (uint32_t)b.size(), 0, 1, nullptr, 0, nullptr, 0);
        expect_len[i] = expect_code[i] == 0 ? 100 : (uint32_t)b.size();
        h.push(make(b.data(), b.size(), i));
        if (i == 1999) {
            // batch 1 launched at push 1000 and routed when batch 2 launched
            CHECK(h.out[0].size() + h.out[1].size() == 1000);
            CHECK(h.runcount == 1);
        }
    }
    CHECK(h.runcount == 1 && h.scheduled(h.st[0]));
    h.timer();                                         // the partial batch
    CHECK(h.runcount == 0 && !h.scheduled(h.st[0]));
    CHECK(h.out[0].size() + h.out[1].size() == (size_t)n);
    long last0 = -1, last1 = -1;
    for (TPacket *p : h.out[0]) {
        CHECK(p->id > last0 && expect_code[p->id] == 0 && p->len == expect_len[p->id]);
        last0 = p->id;
    }
    for (TPacket *p : h.out[1]) {
        CHECK(p->id > last1 && expect_code[p->id] != 0);
        last1 = p->id;
    }
    CHECK(h.handler("drops") == std::to_string(h.out[1].size()));
    CHECK(h.msgs.size() == 1 && h.msgs[0].find("CheckIPHeader") != std::string::npos);   // the first drop only
    report("push_check_ip_header_double_buffered_and_timer", ok);
}

// 2. pull context: SetUDPChecksum (a/ah): output 0 pulled, output 1 pushed
void pull_set_udp()
{
    bool ok = true;
    Host h("SetUDPChecksum", "BATCH 700", 2);
    const int n = 3000;
    std::vector<std::vector<uint8_t> > ref(n);
    std::vector<int> code(n);
    for (int i = 0; i < n; i++) {
        std::vector<uint8_t> b = udp_bytes(200 + (i % 5) * 300, i);
        b[26] = b[27] = 0;                             // uh_sum zero: the Set fills it
        if (i % 17 == 4) b[6] |= 0x20;                 // IP_MF: a fragment -> output 1
        ref[i] = b;
        code[i] = oracle_set_udp_checksum(ref[i].data(), (uint32_t)b.size());
        TPacket *p = make(b.data(), b.size(), i);
        p->nh = 0;
        h.input.push_back(p);
    }
    std::vector<TPacket *> got;
    TPacket *p;
    int refills = 0;
    while ((p = h.pull()) != nullptr) {
        got.push_back(p);
        if (h.input.empty() && refills == 0)
            refills = 1;
        CHECK(h.runcount == 0);
    }
    CHECK(h.pull() == nullptr);                        // the input is dry
    size_t n0 = 0;
    long last = -1;
    for (TPacket *q : got) {
        CHECK(q->id > last && code[q->id] == 0);
        CHECK(q->len == ref[q->id].size() && std::memcmp(q->data(), ref[q->id].data(), q->len) == 0);
        last = q->id;
        n0++;
    }
    for (TPacket *q : h.out[1])
        CHECK(code[q->id] == 1);
    CHECK(n0 + h.out[1].size() == (size_t)n && h.out[0].empty());
    CHECK(h.handler("batches") == std::to_string((n + 699) / 700));
    for (TPacket *q : got)
        h.kill(q);
    report("pull_set_udp_checksum", ok);
}

// 3. IPFragmenter (push): fragments after their first, annotations copied
void fragmenter()
{
    bool ok = true;
    Host h("IPFragmenter", "MTU 576, BATCH 64", 2);
    const int n = 150;
    std::vector<std::vector<uint8_t> > expect0;
    std::vector<long> expect0_id, expect1_id;
    for (int i = 0; i < n; i++) {
        const uint32_t L = i % 5 == 0 ? 400 : 1500;
        std::vector<uint8_t> b = udp_bytes(L, 1000 + i);
        if (i % 9 == 1) b[6] |= 0x40;                  // DF with HONOR_DF: output 1
        if (i % 9 == 1) oracle_set_ip_checksum(b.data(), L);
        // oracle: first fragment then the rest, in order
        std::vector<uint8_t> c = b, arena(4 * 1600);
        uint64_t pos = 0, nfrag = 0, foff[8];
        uint32_t flen[8], first = 0;
        int port = oracle_ip_fragment(c.data(), L, 576, 1, -1, arena.data(), &pos, foff, flen, &nfrag, &first);
        if (port == 1) {
            expect1_id.push_back(i);
        } else {
            expect0.push_back(std::vector<uint8_t>(c.begin(), c.begin() + first));
            expect0_id.push_back(i);
            for (uint64_t k = 0; k < nfrag; k++) {
                expect0.push_back(std::vector<uint8_t>(arena.begin() + (long)foff[k],
                                                       arena.begin() + (long)(foff[k] + flen[k])));
                expect0_id.push_back(i);
            }
        }
        TPacket *p = make(b.data(), b.size(), i);
        p->nh = 0;
        p->paint = (uint32_t)(i % 200);
        h.push(p);
    }
    h.timer();
    CHECK(h.runcount == 0);
    CHECK(h.out[0].size() == expect0.size());
    for (size_t k = 0; k < h.out[0].size() && k < expect0.size(); k++) {
        TPacket *q = h.out[0][k];
        CHECK(q->len == expect0[k].size() && std::memcmp(q->data(), expect0[k].data(), q->len) == 0);
        CHECK(q->id == expect0_id[k] && q->paint == (uint32_t)(expect0_id[k] % 200));
    }
    CHECK(h.out[1].size() == expect1_id.size());
    for (size_t k = 0; k < h.out[1].size() && k < expect1_id.size(); k++)
        CHECK(h.out[1][k]->id == expect1_id[k]);
    report("ip_fragmenter_extras_and_annotations", ok);
}

// 4. a failed flush, then the retry (SetUDPChecksum and the rewriting
//    IPOutputCombo, staged -- retried from the bytes as staged)
void failed_flush_retry(const char *cls, const char *conf, int nth)
{
    bool ok = true;
    Host h(cls, conf, std::string(cls) == "IPOutputCombo" ? 5 : 2);
    h.color = 1;                                       // IPOutputCombo's COLOR: no packet is painted 1
    const int n = 300;
    std::vector<std::vector<uint8_t> > ref(n);
    std::vector<int> code(n);
    for (int i = 0; i < n; i++) {
        std::vector<uint8_t> b = udp_bytes(600, 5000 + i);
        ref[i] = b;
        int prob = 0;
        code[i] = std::string(cls) == "IPOutputCombo"
                      ? oracle_ip_output_combo(ref[i].data(), 600, 600, 0, 0x18041A12, 1500, 0, &prob)
                      : oracle_set_udp_checksum(ref[i].data(), 600);
        TPacket *p = make(b.data(), b.size(), i);
        p->nh = 0;
        h.push(p);
    }
    clk_glue_inject_fault_internal(nth);
    h.timer();                                         // fails: nothing routed, still held
    clk_glue_inject_fault_internal(0);
    CHECK(h.out[0].empty() && h.runcount == 1 && h.scheduled(h.st[0]));
    CHECK(!h.chat.empty() && h.chat.back().find("retry") != std::string::npos);
    h.timer();                                         // the retry
    CHECK(h.runcount == 0 && h.out[0].size() == (size_t)n);
    for (TPacket *q : h.out[0])
        CHECK(code[q->id] == 0 && std::memcmp(q->data(), ref[q->id].data(), 600) == 0);
    char name[128];
    if (nth < 0)
        std::snprintf(name, sizeof name, "failed_flush_then_retry_%s_completion", cls);
    else
        std::snprintf(name, sizeof name, "failed_flush_then_retry_%s_fault%d", cls, nth);
    report(name, ok);
}

// 5. the retry limit: abandon, every held packet killed, runcount released
void retry_limit()
{
    bool ok = true;
    Host h("SetUDPChecksum", "", 2);
    h.core.set_max_retries(3);
    const int n = 200;
    for (int i = 0; i < n; i++) {
        std::vector<uint8_t> b = udp_bytes(300, i);
        TPacket *p = make(b.data(), b.size(), i);
        p->nh = 0;
        h.push(p);
    }
    const long k0 = h.kills;
    for (int k = 0; k < 3; k++) {
        CHECK(h.runcount == 1);
        clk_glue_inject_fault_internal(1);
        h.timer();
    }
    clk_glue_inject_fault_internal(0);
    CHECK(h.runcount == 0 && !h.scheduled(h.st[0]));
    CHECK(h.kills - k0 == n && h.out[0].empty() && h.out[1].empty());
    CHECK(h.handler("lost") == std::to_string(n));
    CHECK(!h.chat.empty() && h.chat.back().find("packets killed") != std::string::npos);
    // the element works again afterwards
    std::vector<uint8_t> b = udp_bytes(300, 7);
    TPacket *p = make(b.data(), b.size(), 7);
    p->nh = 0;
    h.push(p);
    h.timer();
    CHECK(h.out[0].size() == 1 && h.runcount == 0);
    report("retry_limit_abandons_and_releases_runcount", ok);
}

// 6. a downstream element pushing back into this one while it delivers
void reentrant_push()
{
    bool ok = true;
    Host h("CheckIPHeader", "BATCH 64", 2);
    h.on_out0 = [](Host &hh, TPacket *p) {
        if (p->id < 40) {                              // a copy of it, pushed back in on the same thread
            TPacket *q = clone(p);
            q->id = p->id + 100000;
            hh.push(q);
        }
    };
    const int n = 300;
    for (int i = 0; i < n; i++) {
        std::vector<uint8_t> b = udp_bytes(80, i);
        h.push(make(b.data(), b.size(), i));
    }
    h.timer();
    h.timer();                                         // the copies staged by the last delivery
    CHECK(h.runcount == 0);
    CHECK(h.out[0].size() == (size_t)n + 40);
    std::vector<long> pos(n + 100000 + 40, -1);
    for (size_t k = 0; k < h.out[0].size(); k++)
        pos[(size_t)h.out[0][k]->id] = (long)k;
    long last = -1;
    for (int i = 0; i < n; i++) {
        CHECK(pos[(size_t)i] > last);                 // originals in order
        last = pos[(size_t)i];
    }
    for (int i = 0; i < 40; i++)
        CHECK(pos[(size_t)(i + 100000)] > pos[(size_t)i]);
    report("reentrant_push_from_downstream", ok);
}

// 7. four pushing threads (a state each) while the home thread fires timers
void threads()
{
    bool ok = true;
    const int T = 4, n = 20000;
    Host h("CheckIPHeader", "BATCH 4096", 2, T);
    std::atomic<int> done{0};
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++)
        th.emplace_back([&h, &done, t]() {
            for (int i = 0; i < n; i++) {
                std::vector<uint8_t> b = udp_bytes(64, (long)t * n + i);
                if (i % 97 == 0) b[12] ^= 1;
                h.push(make(b.data(), b.size(), (long)t * n + i), t);
            }
            done++;
        });
    while (done < T)
        for (int t = 0; t < T; t++)
            h.timer(t);                                // the home thread's latency timers
    for (std::thread &x : th)
        x.join();
    for (int t = 0; t < T; t++)
        h.timer(t);
    CHECK(h.runcount == 0);
    std::vector<long> last(T, -1);
    size_t bad = 0;
    for (TPacket *p : h.out[0]) {
        const int t = (int)(p->id / n);
        CHECK(p->id > last[(size_t)t] && (p->id % n) % 97 != 0);
        last[(size_t)t] = p->id;
    }
    for (TPacket *p : h.out[1])
        bad += (p->id % n) % 97 == 0;
    CHECK(h.out[0].size() + h.out[1].size() == (size_t)T * n && bad == h.out[1].size());
    report("four_threads_with_home_thread_timers", ok);
}

// 8. cleanup of a held partial batch: everything killed, nothing pushed
void cleanup_partial()
{
    bool ok = true;
    const long live0 = g_live;
    {
        Host h("SetUDPChecksum", "", 2);
        for (int i = 0; i < 500; i++) {
            std::vector<uint8_t> b = udp_bytes(300, i);
            TPacket *p = make(b.data(), b.size(), i);
            p->nh = 0;
            h.push(p);
        }
        CHECK(h.runcount == 1);
        h.core.cleanup(h, h.st[0]);
        CHECK(h.runcount == 0 && h.out[0].empty() && h.out[1].empty() && h.kills == 500);
    }
    CHECK(g_live == live0);
    report("cleanup_kills_held_packets_pushes_nothing", ok);
}

}   // namespace

int main()
{
    if (clk_device_count() < 1) {
        std::printf("SKIP no gfx950 GPU\n");
        return 0;
    }
    push_check_ip();
    pull_set_udp();
    fragmenter();
    // the n-th checked HIP call of the first flush fails: the packets H2D
    // (4), a verdict D2H (SetUDPChecksum 9, IPOutputCombo 10), the packets
    // back D2H (IPOutputCombo 11); -1: the completion wait
    for (int nth : {4, 9, -1})
        failed_flush_retry("SetUDPChecksum", "", nth);
    for (int nth : {4, 10, 11, -1})
        failed_flush_retry("IPOutputCombo", "1, 18.26.4.24, 1500", nth);
    retry_limit();
    reentrant_push();
    threads();
    cleanup_partial();
    std::printf("live packets at exit: %ld\n", (long)g_live);
    return g_fail ? 1 : 0;
}
