// Test harness (not product code): drives the Click adapter's core
// (click_integration/elements/hip/hipcore.hh) AND the element classes' shipped
// logic (hipclasses.hh) with a packet type, packet-operations trait, lock and
// host of its own -- no Click headers -- on the GPU through the element glue
// (include/click_amd_elements.h), and checks every output against the CPU
// oracle (oracle/cksum_oracle.h).  tests/test_gpu_adapter_core.py runs it.
// The packet type, trait and host are tests/native/harness.hh.
//
// Scenarios: every element class over fuzzed packets (outputs, bytes, trims,
// Strip, annotations, clones, uniqueify against a clone the test holds);
// push context with double-buffered batches and the latency deadline; pull
// context, double-buffered, and through two GPU-backed elements in a row;
// IPFragmenter extras; IPOutputCombo when the copy fails; a failed flush
// and its retry; the retry limit; a downstream element that pushes back into
// the element while it delivers; four threads each polling its own state
// (packets delivered on their own thread only); cleanup of a held batch;
// chains of five elements and of the combos (IPOutputCombo a member after
// the head: its clones from the bytes the glue kept) against the elements.
// Prints one line per scenario and exits nonzero if any fails.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "click_amd_elements.h"
#include "../../oracle/cksum_oracle.h"
#include "../../click_integration/elements/hip/hipcore.hh"
#include "../../click_integration/elements/hip/hipclasses.hh"
#include "harness.hh"

extern "C" void clk_glue_inject_fault_internal(int nth);

namespace {

const uint32_t MY_IP = 0x18041A12;   // as the glue reads "18.26.4.24" (network order in memory)
const char *MY_IP_TXT = "18.26.4.24";

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
    std::fflush(stdout);
    if (!ok)
        g_fail++;
}

uint64_t g_rng = 0x9E3779B97F4A7C15ull;
uint32_t rnd(uint32_t n)
{
    g_rng = oracle_splitmix64(g_rng);
    return (uint32_t)(g_rng % n);
}

// An IPv4 packet of L bytes (synthetic, checksums set by the oracle).
std::vector<uint8_t> ip_bytes(uint32_t L, long id, int proto = 17)
{
    std::vector<uint8_t> b(L);
    oracle_gen_packet(b.data(), L, proto, 0x5EED, (uint64_t)id);
    oracle_set_ip_checksum(b.data(), L);
    if (proto == 17 && L >= 28)
        oracle_set_udp_checksum(b.data(), L);
    if (proto == 6 && L >= 40)
        oracle_set_tcp_checksum(b.data(), L, 0);
    return b;
}

// `words` 32-bit words of Record Route / NOP / EOL options inserted after the
// 20-byte header (ip_hl, ip_len and the IP checksum fixed): the option walk
// of IPGWOptions / IPOutputCombo, with pointers before, at and past the end.
std::vector<uint8_t> with_options(const std::vector<uint8_t> &b, int words)
{
    std::vector<uint8_t> o(4 * words, 1);            // NOPs
    const int ln = 4 * words - 1;
    if (ln >= 7) {
        o[0] = 7;                                    // RR
        o[1] = (uint8_t)ln;
        const uint8_t ptrs[] = {4, 8, (uint8_t)(ln + 1), 3, (uint8_t)(ln - 2)};
        o[2] = ptrs[rnd(5)];
        for (int k = 3; k < ln; k++)
            o[k] = (uint8_t)rnd(256);
        o[ln] = 0;                                   // EOL
    }
    std::vector<uint8_t> r(b.begin(), b.begin() + 20);
    r.insert(r.end(), o.begin(), o.end());
    r.insert(r.end(), b.begin() + 20, b.end());
    r[0] = (uint8_t)(0x40 | (5 + words));
    const uint16_t ipl = (uint16_t)r.size();
    r[2] = (uint8_t)(ipl >> 8), r[3] = (uint8_t)ipl;
    r[10] = r[11] = 0;
    oracle_set_ip_checksum(r.data(), (uint32_t)r.size());
    return r;
}

// ---------------------------------------------------------------------------
// 1. Every element class: the shipped class logic over fuzzed packets.
//    What the test expects per packet is the reference's behaviour: the
//    oracle's verdict / rewritten bytes, the port the reference pushes to,
//    and what its simple_action does to the Packet (trim, Strip, annotations,
//    clone order).  The test holds a clone of every pushed packet: an element
//    that writes must have uniqueified first, so the clone keeps its bytes.
// ---------------------------------------------------------------------------
struct Expect {
    long id;
    std::vector<uint8_t> bytes;      // data() .. data() + length()
    int nh;                          // network_header_offset(), -2: not checked
    TAnno a;
};

struct Case {
    std::vector<uint8_t> frame;      // what is pushed
    int nh;                          // its network header offset (-1 none)
    TAnno a;
};

template <class C>
bool run_class(const char *name, Host<C> &h, std::vector<Case> &cases,
               std::vector<std::vector<Expect> > &want, long *killed = nullptr)
{
    bool ok = true;
    const long k0 = g_kills;
    std::vector<TPacket *> held;                     // the test's clones
    for (size_t i = 0; i < cases.size(); i++) {
        TPacket *p = make(cases[i].frame.data(), cases[i].frame.size(), (long)i);
        p->nh = cases[i].nh >= 0 ? cases[i].nh : -1;
        long id = p->a.id;
        p->a = cases[i].a;
        p->a.id = id;
        held.push_back(TOps::clone(p));
        h.push(p);
    }
    h.timer();
    CHECK(h.runcount == 0 && !h.armed());
    if (killed)
        *killed = g_kills - k0;
    for (int port = 0; port < 5; port++) {
        const auto &got = h.out[(size_t)port];
        const auto &exp = want[(size_t)port];
        CHECK(got.size() == exp.size());
        if (got.size() != exp.size())
            std::printf("  %s port %d: %zu results, want %zu\n", name, port, got.size(), exp.size());
        for (size_t k = 0; k < got.size() && k < exp.size(); k++) {
            TPacket *q = got[k];
            const Expect &e = exp[k];
            const bool same = q->a.id == e.id && q->len == e.bytes.size() &&
                              std::memcmp(TOps::data(q), e.bytes.data(), q->len) == 0 &&
                              (e.nh == -2 || TOps::network_header_offset(q) == e.nh) &&
                              q->a.paint == e.a.paint && q->a.dst == e.a.dst && q->a.prob == e.a.prob &&
                              q->a.fix_src == e.a.fix_src;
            if (!same && ok)
                std::printf("  %s port %d #%zu: id %ld/%ld len %zu/%zu nh %d/%d paint %u/%u dst %08x/%08x "
                            "prob %u/%u fix %d/%d bytes %s\n",
                            name, port, k, q->a.id, e.id, q->len, e.bytes.size(),
                            TOps::network_header_offset(q), e.nh, q->a.paint, e.a.paint, q->a.dst, e.a.dst,
                            q->a.prob, e.a.prob, q->a.fix_src, e.a.fix_src,
                            q->len == e.bytes.size() && !std::memcmp(TOps::data(q), e.bytes.data(), q->len)
                                ? "same" : "differ");
            CHECK(same);
        }
    }
    for (size_t i = 0; i < cases.size(); i++)        // nothing written through a shared buffer
            CHECK(held[i]->len == cases[i].frame.size() &&
                  std::memcmp(TOps::data(held[i]), cases[i].frame.data(), held[i]->len) == 0);
    for (TPacket *q : held)
        TOps::kill(q);
    return ok;
}

Expect expect_of(long id, const std::vector<uint8_t> &bytes, int nh, TAnno a)
{
    a.id = id;
    return Expect{id, bytes, nh, a};
}

uint32_t ld32(const uint8_t *p)
{
    uint32_t v;
    std::memcpy(&v, p, 4);
    return v;
}

// IP packets with every verdict the checks distinguish
std::vector<Case> fuzz_cases(int n, int proto, int eth, bool for_check)
{
    std::vector<Case> cs;
    for (int i = 0; i < n; i++) {
        uint32_t L = proto == 1 ? 28 + rnd(600) : 40 + rnd(1400);
        std::vector<uint8_t> b = ip_bytes(L, i, proto);
        if (for_check) {
            switch (rnd(12)) {
            case 0: b[13] ^= 0x10; break;                          // IP checksum (and pseudo-header)
            case 1: b[L - 1] ^= 0x04; break;                       // payload: L4 checksum
            case 2: b[0] = 0x65; break;                            // version
            case 3: b.resize(L + 1 + rnd(20), 0xAB); break;        // link padding: trimmed to ip_len
            case 4: b.resize(10); break;                           // tiny
            case 5: b[2] ^= 0x40; oracle_set_ip_checksum(b.data(), (uint32_t)b.size()); break;   // ip_len
            default: break;
            }
        }
        Case c;
        c.frame.assign((size_t)eth, 0xEE);
        c.frame.insert(c.frame.end(), b.begin(), b.end());
        c.nh = eth ? -1 : 0;
        cs.push_back(c);
    }
    return cs;
}

void every_class()
{
    // CheckIPHeader(OFFSET 14): output 0 trimmed to ip_len, network header at
    // 14, dst annotation; output 1 untouched (checkipheader.cc:143-159,213-223)
    {
        bool ok = true;
        Host<CheckIPC> h("CheckIPHeader", "OFFSET 14, BATCH 300", 2);
        h.cls.offset = 14;
        std::vector<Case> cs = fuzz_cases(1000, 17, 14, true);
        std::vector<std::vector<Expect> > w(5);
        for (size_t i = 0; i < cs.size(); i++) {
            const auto &f = cs[i].frame;
            int code = oracle_check_ip_header(f.data(), (uint32_t)f.size(), 14, 1, nullptr, 0, nullptr, 0);
            if (code == 0) {
                const uint32_t ipl = (uint32_t)f[16] << 8 | f[17];
                std::vector<uint8_t> t(f.begin(), f.begin() + 14 + ipl);
                TAnno a;
                a.dst = ld32(f.data() + 14 + 16);
                w[0].push_back(expect_of((long)i, t, 14, a));
            } else
                w[1].push_back(expect_of((long)i, f, -2, TAnno()));
        }
        ok = run_class("CheckIPHeader", h, cs, w) && ok;
        report("class_CheckIPHeader", ok);
    }
    // CheckIPHeader2: no checksum test (checkipheader2.cc)
    {
        bool ok = true;
        Host<CheckIPC> h("CheckIPHeader2", "BATCH 256", 2);
        std::vector<Case> cs = fuzz_cases(700, 6, 0, true);
        std::vector<std::vector<Expect> > w(5);
        for (size_t i = 0; i < cs.size(); i++) {
            const auto &f = cs[i].frame;
            int code = oracle_check_ip_header(f.data(), (uint32_t)f.size(), 0, 0, nullptr, 0, nullptr, 0);
            if (code == 0) {
                const uint32_t ipl = (uint32_t)f[2] << 8 | f[3];
                TAnno a;
                a.dst = ld32(f.data() + 16);
                w[0].push_back(expect_of((long)i, std::vector<uint8_t>(f.begin(), f.begin() + ipl), 0, a));
            } else
                w[1].push_back(expect_of((long)i, f, -2, TAnno()));
        }
        ok = run_class("CheckIPHeader2", h, cs, w) && ok;
        report("class_CheckIPHeader2", ok);
    }
    // IPInputCombo(COLOR 2): Paint, Strip(14), the checks; bad packets killed
    // (ipinputcombo.cc:66-140)
    {
        bool ok = true;
        Host<InputComboC> h("IPInputCombo", "2, BATCH 400", 1);
        h.cls.color = 2;
        std::vector<Case> cs = fuzz_cases(1000, 17, 14, true);
        std::vector<std::vector<Expect> > w(5);
        size_t bad = 0;
        for (size_t i = 0; i < cs.size(); i++) {
            const auto &f = cs[i].frame;
            cs[i].a.paint = 7;
            int code = oracle_check_ip_header(f.data(), (uint32_t)f.size(), 14, 1, nullptr, 0, nullptr, 0);
            if (code == 0) {
                const uint32_t ipl = (uint32_t)f[16] << 8 | f[17];
                TAnno a;
                a.paint = 2;
                a.dst = ld32(f.data() + 14 + 16);
                w[0].push_back(expect_of((long)i, std::vector<uint8_t>(f.begin() + 14, f.begin() + 14 + ipl), 0, a));
            } else
                bad++;
        }
        long killed = 0;
        ok = run_class("IPInputCombo", h, cs, w, &killed) && ok;
        CHECK(killed == (long)bad && bad > 0);
        report("class_IPInputCombo", ok);
    }
    // CheckUDPHeader / CheckTCPHeader / CheckICMPHeader: untouched, 0 or 1
    {
        const struct { const char *cls; int proto; } ls[] = {{"CheckUDPHeader", 17}, {"CheckTCPHeader", 6},
                                                             {"CheckICMPHeader", 1}};
        for (const auto &l : ls) {
            bool ok = true;
            Host<PlainC> h(l.cls, "BATCH 333", 2);
            std::vector<Case> cs = fuzz_cases(900, l.proto, 0, true);
            std::vector<std::vector<Expect> > w(5);
            for (size_t i = 0; i < cs.size(); i++) {
                const auto &f = cs[i].frame;
                const uint32_t c = (uint32_t)f.size();
                int code = l.proto == 17 ? oracle_check_udp_header(f.data(), c)
                           : l.proto == 6 ? oracle_check_tcp_header(f.data(), c) : oracle_check_icmp_header(f.data(), c);
                w[code ? 1 : 0].push_back(expect_of((long)i, f, 0, TAnno()));
            }
            ok = run_class(l.cls, h, cs, w) && ok;
            report((std::string("class_") + l.cls).c_str(), ok);
        }
    }
    // SetIPChecksum / SetUDPChecksum / SetTCPChecksum: uniqueify, the field
    // written; SetUDPChecksum's fragments to output 1; bad lengths killed
    {
        const struct { const char *cls; int proto; } ls[] = {{"SetIPChecksum", 17}, {"SetUDPChecksum", 17},
                                                             {"SetTCPChecksum", 6}};
        for (const auto &l : ls) {
            bool ok = true;
            Host<SetC> h(l.cls, "BATCH 500", std::string(l.cls) == "SetUDPChecksum" ? 2 : 1);
            std::vector<Case> cs = fuzz_cases(900, l.proto, 0, false);
            std::vector<std::vector<Expect> > w(5);
            for (size_t i = 0; i < cs.size(); i++) {
                auto &f = cs[i].frame;
                if (rnd(10) == 0)
                    f[6] |= 0x20;                                  // IP_MF: SetUDPChecksum's output 1
                if (rnd(15) == 0)
                    f.resize(f.size() > 30 ? 30 : f.size());       // short
                std::vector<uint8_t> r = f;
                const uint32_t c = (uint32_t)r.size();
                int code = std::string(l.cls) == "SetIPChecksum" ? oracle_set_ip_checksum(r.data(), c)
                           : l.proto == 17 ? oracle_set_udp_checksum(r.data(), c) : oracle_set_tcp_checksum(r.data(), c, 0);
                if (code == CLK_SET_OK)
                    w[0].push_back(expect_of((long)i, r, 0, TAnno()));
                else if (code == CLK_SET_OUTPUT1)
                    w[1].push_back(expect_of((long)i, r, 0, TAnno()));
            }
            ok = run_class(l.cls, h, cs, w) && ok;
            report((std::string("class_") + l.cls).c_str(), ok);
        }
    }
    // DecIPTTL: writable only when decremented; expired to output 1
    {
        bool ok = true;
        Host<DecTTLC> h("DecIPTTL", "BATCH 300", 2);
        std::vector<Case> cs = fuzz_cases(800, 17, 0, false);
        std::vector<std::vector<Expect> > w(5);
        for (size_t i = 0; i < cs.size(); i++) {
            auto &f = cs[i].frame;
            f[8] = (uint8_t)(rnd(4) == 0 ? rnd(3) : 2 + rnd(250));
            oracle_set_ip_checksum(f.data(), (uint32_t)f.size());
            std::vector<uint8_t> r = f;
            int code = oracle_dec_ip_ttl(r.data(), (uint32_t)r.size(), 1);
            w[code == CLK_TTL_EXPIRED ? 1 : 0].push_back(expect_of((long)i, r, 0, TAnno()));
        }
        ok = run_class("DecIPTTL", h, cs, w) && ok;
        report("class_DecIPTTL", ok);
    }
    // IPGWOptions(MYADDR): Record Route rewrites, parameter problems to 1
    // with ICMP_PARAMPROB_ANNO (ipgwoptions.cc:53-172)
    {
        bool ok = true;
        Host<GWOptC> h("IPGWOptions", std::string(MY_IP_TXT) + ", BATCH 250", 2);
        std::vector<Case> cs = fuzz_cases(700, 17, 0, false);
        std::vector<std::vector<Expect> > w(5);
        size_t nprob = 0;
        for (size_t i = 0; i < cs.size(); i++) {
            auto &f = cs[i].frame;
            if (rnd(2))
                f = with_options(f, 1 + (int)rnd(9));
            std::vector<uint8_t> r = f;
            int prob = 0;
            int code = oracle_ip_gw_options_element(r.data(), (uint32_t)r.size(), MY_IP, &MY_IP, 1, 0, &prob);
            TAnno a;
            if (code == CLK_GWOPT_ERROR) {
                a.prob = (uint32_t)prob;
                nprob++;
                w[1].push_back(expect_of((long)i, r, 0, a));
            } else
                w[0].push_back(expect_of((long)i, r, 0, a));
        }
        ok = run_class("IPGWOptions", h, cs, w) && ok;
        CHECK(nprob > 0);
        report("class_IPGWOptions", ok);
    }
    // FixIPSrc(IPADDR): annotated packets rewritten, annotation cleared
    {
        bool ok = true;
        Host<FixSrcC> h("FixIPSrc", std::string("IPADDR ") + MY_IP_TXT + ", BATCH 200", 1);
        std::vector<Case> cs = fuzz_cases(600, 17, 0, false);
        std::vector<std::vector<Expect> > w(5);
        for (size_t i = 0; i < cs.size(); i++) {
            cs[i].a.fix_src = rnd(3) == 0;
            std::vector<uint8_t> r = cs[i].frame;
            oracle_fix_ip_src(r.data(), (uint32_t)r.size(), cs[i].a.fix_src, MY_IP);
            w[0].push_back(expect_of((long)i, r, 0, TAnno()));
        }
        ok = run_class("FixIPSrc", h, cs, w) && ok;
        report("class_FixIPSrc", ok);
    }
    // IPOutputCombo(COLOR 1, IPADDR, MTU 700): broadcast killed (no clone),
    // the painted clone to 1 before its packet with the bytes as pushed,
    // parameter problem 2, TTL 3, MTU 4 (ipoutputcombo.cc:44-205)
    {
        bool ok = true;
        Host<OutComboC> h("IPOutputCombo", std::string("1, ") + MY_IP_TXT + ", 700, BATCH 300", 5);
        h.cls.color = 1;
        std::vector<Case> cs = fuzz_cases(900, 17, 0, false);
        std::vector<std::vector<Expect> > w(5);
        size_t nb = 0;
        for (size_t i = 0; i < cs.size(); i++) {
            auto &f = cs[i].frame;
            if (rnd(3) == 0)
                f = with_options(f, 1 + (int)rnd(9));
            if (rnd(6) == 0) {
                f[8] = (uint8_t)rnd(2);                   // TTL 0/1: expired
                oracle_set_ip_checksum(f.data(), (uint32_t)f.size());
            }
            cs[i].a.paint = rnd(3);
            cs[i].a.fix_src = rnd(4) == 0;
            cs[i].a.bcast = rnd(20) == 0;
            if (cs[i].a.bcast) {
                nb++;
                continue;
            }
            if (cs[i].a.paint == 1)
                w[1].push_back(expect_of((long)i, f, 0, cs[i].a));
            std::vector<uint8_t> r = f;
            int prob = 0;
            int port = oracle_ip_output_combo(r.data(), (uint32_t)r.size(), (uint32_t)r.size(),
                                              cs[i].a.fix_src ? 1 : 0, MY_IP, 700, 0, &prob);
            TAnno a = cs[i].a;
            if (port == 2)
                a.prob = (uint32_t)prob;
            else if (a.fix_src)
                a.fix_src = false;
            w[(size_t)port].push_back(expect_of((long)i, r, 0, a));
        }
        long killed = 0;
        // the clones on output 1 come out in packet order, with the bytes
        // as pushed (w[1])
        ok = run_class("IPOutputCombo", h, cs, w, &killed) && ok;
        CHECK(killed == (long)nb && nb > 0);
        report("class_IPOutputCombo", ok);
    }
}

// 2. IPOutputCombo when uniqueify fails: the reference has already pushed the
//    PaintTee clone (ipoutputcombo.cc:56-60); the clone leaves on output 1,
//    the packet is gone, nothing is staged
void output_combo_copy_fails()
{
    bool ok = true;
    Host<OutComboC> h("IPOutputCombo", std::string("1, ") + MY_IP_TXT + ", 1500", 5);
    h.cls.color = 1;
    std::vector<uint8_t> b = ip_bytes(200, 1);
    TPacket *p = make(b.data(), b.size(), 1);
    p->nh = 0;
    p->a.paint = 1;
    TPacket *keep = TOps::clone(p);                  // shared: uniqueify must copy
    g_uniq_fail = 1;                                 // ... and that copy fails
    h.push(p);
    g_uniq_fail = 0;
    CHECK(h.out[1].size() == 1 && h.out[0].empty() && h.runcount == 0);
    if (h.out[1].size() == 1)
        CHECK(h.out[1][0]->a.id == 1 && std::memcmp(TOps::data(h.out[1][0]), b.data(), b.size()) == 0);
    CHECK(h.handler("packets") == "0");
    TOps::kill(keep);
    report("output_combo_clone_survives_failed_copy", ok);
}

// 3. push context: CheckIPHeader, double-buffered full batches, the deadline
void push_check_ip()
{
    bool ok = true;
    Host<CheckIPC> h("CheckIPHeader", "BATCH 1000", 2);
    h.core.set_latency(200);                           // LATENCY 200 ms: the pushes below take less
    const int n = 2500;
    std::vector<int> expect_code(n);
    std::vector<uint32_t> expect_len(n);
    for (int i = 0; i < n; i++) {
        std::vector<uint8_t> b = ip_bytes(100, i);
        if (i % 7 == 3) b[13] ^= 0x10;
        if (i % 13 == 5) b[0] = 0x65;
        if (i % 11 == 2) b.resize(108, 0xAB);
        if (i % 29 == 7) b.resize(10);
        expect_code[i] = oracle_check_ip_header(b.data(), (uint32_t)b.size(), 0, 1, nullptr, 0, nullptr, 0);
        expect_len[i] = expect_code[i] == 0 ? 100 : (uint32_t)b.size();
        h.push(make(b.data(), b.size(), i));
        if (i == 1999) {
            CHECK(h.out[0].size() + h.out[1].size() == 1000);
            CHECK(h.runcount == 1);
        }
    }
    CHECK(h.runcount == 1 && h.armed() && h.wakes >= 1);
    CHECK(h.poll());                                   // before the deadline: nothing flushed
    CHECK(h.out[0].size() + h.out[1].size() == 1000);  // (batch 2 in flight, 500 staged)
    std::this_thread::sleep_for(std::chrono::milliseconds(210));
    CHECK(h.poll());                                   // past it: the 500 staged launched, batch 2 routed
    CHECK(h.out[0].size() + h.out[1].size() == 2000 && h.runcount == 1);
    std::this_thread::sleep_for(std::chrono::milliseconds(210));
    CHECK(!h.poll());                                  // past the next, nothing new: the rest waited for
    CHECK(h.runcount == 0 && !h.armed());
    CHECK(h.out[0].size() + h.out[1].size() == (size_t)n);
    long last0 = -1, last1 = -1;
    for (TPacket *p : h.out[0]) {
        CHECK(p->a.id > last0 && expect_code[p->a.id] == 0 && p->len == expect_len[p->a.id]);
        last0 = p->a.id;
    }
    for (TPacket *p : h.out[1]) {
        CHECK(p->a.id > last1 && expect_code[p->a.id] != 0);
        last1 = p->a.id;
    }
    CHECK(h.handler("drops") == std::to_string(h.out[1].size()));
    CHECK(h.msgs.size() == 1 && h.msgs[0].find("CheckIPHeader") != std::string::npos);
    report("push_check_ip_header_double_buffered_and_deadline", ok);
}

// 4. pull context, double-buffered: SetUDPChecksum (a/ah): output 0 pulled,
//    output 1 pushed; each refill launches a batch and hands out the one before
void pull_set_udp()
{
    bool ok = true;
    Host<SetC> h("SetUDPChecksum", "BATCH 700", 2);
    const int n = 3000;
    std::vector<std::vector<uint8_t> > ref(n);
    std::vector<int> code(n);
    for (int i = 0; i < n; i++) {
        std::vector<uint8_t> b = ip_bytes(200 + (i % 5) * 300, i);
        b[26] = b[27] = 0;
        if (i % 17 == 4) b[6] |= 0x20;
        ref[i] = b;
        code[i] = oracle_set_udp_checksum(ref[i].data(), (uint32_t)b.size());
        TPacket *p = make(b.data(), b.size(), i);
        p->nh = 0;
        h.input.push_back(p);
    }
    std::vector<TPacket *> got;
    TPacket *p;
    size_t max_inflight = 0;
    while ((p = h.pull()) != nullptr) {
        got.push_back(p);
        CHECK(h.runcount == 0);
        // the packets taken from the input and not yet handed out or pushed
        const size_t taken = (size_t)n - h.input.size();
        const size_t done = got.size() + h.out[1].size();
        max_inflight = std::max(max_inflight, taken - done);
    }
    CHECK(h.pull() == nullptr);
    // double-buffered: a refill launches batch k+1 while batch k is handed out
    CHECK(max_inflight > 700);
    size_t n0 = 0;
    long last = -1;
    for (TPacket *q : got) {
        CHECK(q->a.id > last && code[q->a.id] == 0);
        CHECK(q->len == ref[q->a.id].size() && std::memcmp(TOps::data(q), ref[q->a.id].data(), q->len) == 0);
        last = q->a.id;
        n0++;
    }
    for (TPacket *q : h.out[1])
        CHECK(code[q->a.id] == 1);
    CHECK(n0 + h.out[1].size() == (size_t)n && h.out[0].empty());
    CHECK(h.handler("batches") == std::to_string((n + 699) / 700));
    for (TPacket *q : got)
        TOps::kill(q);
    report("pull_set_udp_checksum_double_buffered", ok);
}

// 5. pull through two GPU-backed elements in a row: CheckIPHeader's pull()
//    is SetUDPChecksum's input (a Queue -> CheckIPHeader -> SetUDPChecksum ->
//    ToDevice graph in pull mode)
void pull_two_elements()
{
    bool ok = true;
    Host<CheckIPC> a("CheckIPHeader", "BATCH 512", 2);
    Host<SetC> b("SetUDPChecksum", "BATCH 300", 2);
    b.upstream = [&a]() { return a.pull(); };
    const int n = 2000;
    std::vector<std::vector<uint8_t> > ref(n);
    std::vector<int> ipc(n), sc(n);
    for (int i = 0; i < n; i++) {
        std::vector<uint8_t> x = ip_bytes(60 + (i * 37) % 1400, i);
        if (i % 9 == 2) x[13] ^= 1;                   // bad IP checksum: CheckIPHeader's output 1
        x[26] = x[27] = 0;
        if (i % 23 == 5) { x[6] |= 0x20; oracle_set_ip_checksum(x.data(), (uint32_t)x.size()); }
        ref[i] = x;
        ipc[i] = oracle_check_ip_header(x.data(), (uint32_t)x.size(), 0, 1, nullptr, 0, nullptr, 0);
        sc[i] = ipc[i] ? -1 : oracle_set_udp_checksum(ref[i].data(), (uint32_t)x.size());
        TPacket *p = make(x.data(), x.size(), i);
        a.input.push_back(p);
    }
    std::vector<TPacket *> got;
    TPacket *p;
    while ((p = b.pull()) != nullptr)
        got.push_back(p);
    size_t want0 = 0, want_a1 = 0, want_b1 = 0;
    for (int i = 0; i < n; i++) {
        want_a1 += ipc[i] != 0;
        want0 += sc[i] == 0;
        want_b1 += sc[i] == 1;
    }
    CHECK(got.size() == want0 && a.out[1].size() == want_a1 && b.out[1].size() == want_b1);
    long last = -1;
    for (TPacket *q : got) {
        CHECK(q->a.id > last && sc[q->a.id] == 0);
        CHECK(q->len == ref[q->a.id].size() && std::memcmp(TOps::data(q), ref[q->a.id].data(), q->len) == 0);
        CHECK(q->a.dst == ld32(ref[q->a.id].data() + 16));    // CheckIPHeader's annotation came along
        last = q->a.id;
    }
    for (TPacket *q : got)
        TOps::kill(q);
    report("pull_through_two_gpu_elements", ok);
}

// 6. IPFragmenter (push): fragments after their first, annotations copied
void fragmenter()
{
    bool ok = true;
    Host<FragC> h("IPFragmenter", "MTU 576, BATCH 64", 2);
    h.cls.mtu = 576;
    const int n = 150;
    std::vector<std::vector<uint8_t> > expect0;
    std::vector<long> expect0_id, expect1_id;
    for (int i = 0; i < n; i++) {
        const uint32_t L = i % 5 == 0 ? 400 : 1500;
        std::vector<uint8_t> b = ip_bytes(L, 1000 + i);
        if (i % 9 == 1) b[6] |= 0x40;
        if (i % 9 == 1) oracle_set_ip_checksum(b.data(), L);
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
        p->a.paint = (uint32_t)(i % 200);
        TPacket *keep = TOps::clone(p);              // the pushed packet is shared: uniqueify copies
        h.push(p);
        TOps::kill(keep);
    }
    h.timer();
    CHECK(h.runcount == 0);
    CHECK(h.out[0].size() == expect0.size());
    for (size_t k = 0; k < h.out[0].size() && k < expect0.size(); k++) {
        TPacket *q = h.out[0][k];
        CHECK(q->len == expect0[k].size() && std::memcmp(TOps::data(q), expect0[k].data(), q->len) == 0);
        CHECK(q->a.id == expect0_id[k] && q->a.paint == (uint32_t)(expect0_id[k] % 200));
        CHECK(TOps::network_header_offset(q) == 0);
    }
    CHECK(h.out[1].size() == expect1_id.size());
    for (size_t k = 0; k < h.out[1].size() && k < expect1_id.size(); k++)
        CHECK(h.out[1][k]->a.id == expect1_id[k]);
    report("ip_fragmenter_extras_and_annotations", ok);
}

// 7. a failed flush, then the retry (SetUDPChecksum and the rewriting
//    IPOutputCombo, staged -- retried from the bytes as staged)
void set_color(OutComboC &c, uint32_t color) { c.color = color; }
void set_color(SetC &, uint32_t) { }

template <class C>
void failed_flush_retry(const char *cls, const char *conf, int nth)
{
    bool ok = true;
    const bool combo = std::string(cls) == "IPOutputCombo";
    Host<C> h(cls, conf, combo ? 5 : 2);
    set_color(h.cls, 1);                               // COLOR 1: no packet is painted 1
    const int n = 300;
    std::vector<std::vector<uint8_t> > ref(n);
    std::vector<int> code(n);
    for (int i = 0; i < n; i++) {
        std::vector<uint8_t> b = ip_bytes(600, 5000 + i);
        ref[i] = b;
        int prob = 0;
        code[i] = combo ? oracle_ip_output_combo(ref[i].data(), 600, 600, 0, MY_IP, 1500, 0, &prob)
                        : oracle_set_udp_checksum(ref[i].data(), 600);
        TPacket *p = make(b.data(), b.size(), i);
        p->nh = 0;
        h.push(p);
    }
    clk_glue_inject_fault_internal(nth);
    h.timer();                                         // fails: nothing routed, still held
    clk_glue_inject_fault_internal(0);
    CHECK(h.out[0].empty() && h.runcount == 1 && h.armed());
    CHECK(!h.chat.empty() && h.chat.back().find("retry") != std::string::npos);
    h.timer();                                         // the retry
    CHECK(h.runcount == 0 && h.out[0].size() == (size_t)n);
    for (TPacket *q : h.out[0])
        CHECK(code[q->a.id] == 0 && std::memcmp(TOps::data(q), ref[q->a.id].data(), 600) == 0);
    char name[128];
    if (nth < 0)
        std::snprintf(name, sizeof name, "failed_flush_then_retry_%s_completion", cls);
    else
        std::snprintf(name, sizeof name, "failed_flush_then_retry_%s_fault%d", cls, nth);
    report(name, ok);
}

// 8. the retry limit: abandon, every held packet killed, runcount released
void retry_limit()
{
    bool ok = true;
    Host<SetC> h("SetUDPChecksum", "", 2);
    h.core.set_max_retries(3);
    const int n = 200;
    for (int i = 0; i < n; i++) {
        std::vector<uint8_t> b = ip_bytes(300, i);
        TPacket *p = make(b.data(), b.size(), i);
        p->nh = 0;
        h.push(p);
    }
    const long k0 = g_kills;
    for (int k = 0; k < 3; k++) {
        CHECK(h.runcount == 1);
        clk_glue_inject_fault_internal(1);
        h.timer();
    }
    clk_glue_inject_fault_internal(0);
    CHECK(h.runcount == 0 && !h.armed());
    CHECK(g_kills - k0 == n && h.out[0].empty() && h.out[1].empty());
    CHECK(h.handler("lost") == std::to_string(n));
    CHECK(!h.chat.empty() && h.chat.back().find("packets killed") != std::string::npos);
    std::vector<uint8_t> b = ip_bytes(300, 7);
    TPacket *p = make(b.data(), b.size(), 7);
    p->nh = 0;
    h.push(p);
    h.timer();
    CHECK(h.out[0].size() == 1 && h.runcount == 0);
    report("retry_limit_abandons_and_releases_runcount", ok);
}

// 9. a downstream element pushing back into this one while it delivers
void reentrant_push()
{
    bool ok = true;
    Host<CheckIPC> h("CheckIPHeader", "BATCH 64", 2);
    h.on_out0 = [](Host<CheckIPC> &hh, TPacket *p) {
        if (p->a.id < 40) {
            TPacket *q = TOps::clone(p);
            q->buf = std::make_shared<std::vector<uint8_t> >(*p->buf);
            q->raw = q->buf->data();
            q->a.id = p->a.id + 100000;
            hh.push(q);
        }
    };
    const int n = 300;
    for (int i = 0; i < n; i++) {
        std::vector<uint8_t> b = ip_bytes(80, i);
        h.push(make(b.data(), b.size(), i));
    }
    h.timer();
    h.timer();
    CHECK(h.runcount == 0);
    CHECK(h.out[0].size() == (size_t)n + 40);
    std::vector<long> pos(n + 100000 + 40, -1);
    for (size_t k = 0; k < h.out[0].size(); k++)
        pos[(size_t)h.out[0][k]->a.id] = (long)k;
    long last = -1;
    for (int i = 0; i < n; i++) {
        CHECK(pos[(size_t)i] > last);
        last = pos[(size_t)i];
    }
    for (int i = 0; i < 40; i++)
        CHECK(pos[(size_t)(i + 100000)] > pos[(size_t)i]);
    report("reentrant_push_from_downstream", ok);
}

// 10. four pushing threads, each with its own state whose deadline it polls
//     itself (the Click adapter's per-RouterThread Task): every packet is
//     delivered on the thread that pushed it, in push order
void threads()
{
    bool ok = true;
    const int T = 4, n = 20000;
    Host<CheckIPC> h("CheckIPHeader", "BATCH 4096", 2, T);
    std::vector<std::thread> th;
    std::vector<std::thread::id> tid(T);
    for (int t = 0; t < T; t++)
        th.emplace_back([&h, &tid, t]() {
            tid[(size_t)t] = std::this_thread::get_id();
            for (int i = 0; i < n; i++) {
                std::vector<uint8_t> b = ip_bytes(64, (long)t * n + i);
                if (i % 97 == 0) b[12] ^= 1;
                h.push(make(b.data(), b.size(), (long)t * n + i), t);
                if (i % 512 == 0)
                    h.poll(t);                         // the thread's Task between pushes
            }
            while (h.poll(t))                          // the Task until the deadline flushes the rest
                std::this_thread::sleep_for(std::chrono::microseconds(200));
        });
    for (std::thread &x : th)
        x.join();
    CHECK(h.runcount == 0);
    std::vector<long> last(T, -1);
    size_t bad = 0, wrong_thread = 0;
    for (int port = 0; port < 2; port++)
        for (size_t k = 0; k < h.out[(size_t)port].size(); k++) {
            TPacket *p = h.out[(size_t)port][k];
            const int t = (int)(p->a.id / n);
            wrong_thread += h.out_thread[(size_t)port][k] != tid[(size_t)t];
            if (port == 0) {
                CHECK(p->a.id > last[(size_t)t] && (p->a.id % n) % 97 != 0);
                last[(size_t)t] = p->a.id;
            } else
                bad += (p->a.id % n) % 97 == 0;
        }
    CHECK(wrong_thread == 0);
    CHECK(h.out[0].size() + h.out[1].size() == (size_t)T * n && bad == h.out[1].size());
    report("four_threads_each_delivered_on_its_own_thread", ok);
}

// 10b. a catch-all state (State::shared: the Click adapter's state for a
//      thread id past the RouterThreads) that two threads push into at once
//      takes its lock: every packet is routed exactly once, each thread's in
//      its push order
void shared_state_two_threads()
{
    bool ok = true;
    const int T = 2, n = 30000;
    Host<CheckIPC> h("CheckIPHeader", "BATCH 2048", 2, 1);
    h.st[0].shared = true;
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++)
        th.emplace_back([&h, t]() {
            for (int i = 0; i < n; i++) {
                std::vector<uint8_t> b = ip_bytes(64, (long)t * n + i);
                if (i % 89 == 0) b[12] ^= 1;
                h.push(make(b.data(), b.size(), (long)t * n + i), 0);
            }
        });
    for (std::thread &x : th)
        x.join();
    h.timer();
    CHECK(h.runcount == 0);
    std::vector<long> last(T, -1);
    size_t bad = 0;
    std::vector<uint8_t> seen((size_t)T * n, 0);
    for (int port = 0; port < 2; port++)
        for (TPacket *p : h.out[(size_t)port]) {
            const int t = (int)(p->a.id / n);
            CHECK(!seen[(size_t)p->a.id]);
            seen[(size_t)p->a.id] = 1;
            if (port == 0) {
                CHECK(p->a.id > last[(size_t)t] && (p->a.id % n) % 89 != 0);
                last[(size_t)t] = p->a.id;
            } else
                bad += (p->a.id % n) % 89 == 0;
        }
    CHECK(h.out[0].size() + h.out[1].size() == (size_t)T * n && bad == h.out[1].size());
    report("shared_state_two_threads_locked", ok);
}

// 11. cleanup of a held partial batch: everything killed, nothing pushed
void cleanup_partial()
{
    bool ok = true;
    const long live0 = g_live, k0 = g_kills;
    {
        Host<SetC> h("SetUDPChecksum", "", 2);
        for (int i = 0; i < 500; i++) {
            std::vector<uint8_t> b = ip_bytes(300, i);
            TPacket *p = make(b.data(), b.size(), i);
            p->nh = 0;
            h.push(p);
        }
        CHECK(h.runcount == 1);
        h.core.cleanup(h, h.st[0]);
        CHECK(h.runcount == 0 && h.out[0].empty() && h.out[1].empty() && g_kills - k0 == 500 && !h.armed());
    }
    CHECK(g_live == live0);
    report("cleanup_kills_held_packets_pushes_nothing", ok);
}

// 12. a chain (hipcore chains): CheckIPHeader -> IPGWOptions -> FixIPSrc ->
//     DecIPTTL -> IPFragmenter run by one state as a clk_chain, against the
//     same classes as five separate elements, each pushed what the one before
//     put out on output 0.  Every member's every output: the same packets in
//     the same order, byte for byte, with the same length, network header and
//     annotations; the members' handlers agree.
bool same_packet(const TPacket *a, const TPacket *b)
{
    return a->a.id == b->a.id && a->len == b->len && (a->nh - (long)a->off) == (b->nh - (long)b->off) &&
           a->a.dst == b->a.dst && a->a.fix_src == b->a.fix_src && a->a.prob == b->a.prob &&
           a->a.paint == b->a.paint && std::memcmp(a->buf->data() + a->off, b->buf->data() + b->off, a->len) == 0;
}

void chain_vs_elements(uint32_t batch, uint32_t flush_every)
{
    bool ok = true;
    const int n = 2500;
    const std::string B = "BATCH " + std::to_string(batch);
    Member<CheckIPC> c0("CheckIPHeader", "DETAILS true, " + B, 2);
    Member<GWOptC> c1("IPGWOptions", std::string(MY_IP_TXT) + ", " + B, 2);
    Member<FixSrcC> c2("FixIPSrc", std::string(MY_IP_TXT) + ", " + B, 1);
    Member<DecTTLC> c3("DecIPTTL", B, 2);
    Member<FragC> c4("IPFragmenter", "576, " + B, 2);
    c4.cls.mtu = 576;
    ChainHost ch({&c0, &c1, &c2, &c3, &c4});
    Host<CheckIPC> h0("CheckIPHeader", "DETAILS true, " + B, 2);
    Host<GWOptC> h1("IPGWOptions", std::string(MY_IP_TXT) + ", " + B, 2);
    Host<FixSrcC> h2("FixIPSrc", std::string(MY_IP_TXT) + ", " + B, 1);
    Host<DecTTLC> h3("DecIPTTL", B, 2);
    Host<FragC> h4("IPFragmenter", "576, " + B, 2);
    h4.cls.mtu = 576;
    for (int i = 0; i < n; i++) {
        std::vector<uint8_t> b = ip_bytes(40 + (uint32_t)(i * 53) % 1400, i);
        if (i % 7 == 3)
            b = with_options(b, 1 + i % 4);
        if (i % 11 == 5) {                           // TTL 0-2: DecIPTTL's output 1
            b[8] = (uint8_t)(i % 3);
            oracle_set_ip_checksum(b.data(), (uint32_t)b.size());
        }
        if (i % 9 == 1) {                            // DF: IPFragmenter's output 1 when too long
            b[6] |= 0x40;
            oracle_set_ip_checksum(b.data(), (uint32_t)b.size());
        }
        if (i % 13 == 6)
            b[12] ^= 1;                              // a bad checksum: CheckIPHeader's output 1
        for (int run = 0; run < 2; run++) {
            TPacket *p = make(b.data(), b.size(), i);
            p->a.fix_src = i % 4 == 0;
            p->a.paint = (uint32_t)(i % 3);
            if (run == 0) {
                ch.push(p);
                if (flush_every && (i + 1) % flush_every == 0)
                    ch.timer();
            } else
                h0.push(p);
        }
    }
    ch.timer();
    h0.timer();
    // the separate elements: each takes what the one before put out on output 0
    auto feed = [](std::vector<TPacket *> &from, auto &to) {
        for (TPacket *p : from)
            to.push(p);
        from.clear();
        to.timer();
    };
    feed(h0.out[0], h1);
    feed(h1.out[0], h2);
    feed(h2.out[0], h3);
    feed(h3.out[0], h4);
    std::vector<std::vector<std::vector<TPacket *> > *> sep = {&h0.out, &h1.out, &h2.out, &h3.out, &h4.out};
    size_t total = 0;
    for (size_t k = 0; k < 5; k++)
        for (size_t q = 0; q < 5; q++) {
            const std::vector<TPacket *> &x = ch.m[k]->out[q], &y = (*sep[k])[q];
            CHECK(x.size() == y.size());
            for (size_t j = 0; j < x.size() && j < y.size(); j++)
                if (!same_packet(x[j], y[j])) {
                    std::printf("  member %zu port %zu #%zu: id %ld / %ld\n", k, q, j, x[j]->a.id, y[j]->a.id);
                    CHECK(same_packet(x[j], y[j]));
                    break;
                }
            total += x.size();
        }
    CHECK(!ch.m[0]->out[1].empty() && !ch.m[3]->out[1].empty() && !ch.m[4]->out[1].empty());
    CHECK(ch.m[4]->out[0].size() > (size_t)n / 2);
    const char *hs[] = {"drops", "drop_details", "packets", "fragments"};
    CHECK(ch.handler(0, "drops") == h0.handler("drops") && ch.handler(0, "drop_details") == h0.handler("drop_details"));
    CHECK(ch.handler(1, "drops") == h1.handler("drops") && ch.handler(3, "drops") == h3.handler("drops"));
    CHECK(ch.handler(4, "fragments") == h4.handler("fragments") && ch.handler(4, "drops") == h4.handler("drops"));
    for (const char *h : hs)
        CHECK(ch.handler(2, h) == h2.handler(h));
    CHECK(ch.runcount == 0 && h0.runcount == 0);
    CHECK(total > (size_t)n);
    std::string label = "chain_of_five_matches_separate_elements_batch_" + std::to_string(batch) +
                        (flush_every ? "_flush_" + std::to_string(flush_every) : std::string());
    report(label.c_str(), ok);
}

// 13. the combos as one chain: IPInputCombo(1) -> IPOutputCombo(1, ..., 600)
//     run by the core, against the two classes as separate elements.
//     IPOutputCombo is a member after the head, so its PaintTee clone (most
//     packets: IPInputCombo paints COLOR 1) is the bytes the glue kept as the
//     packet reached it, with the packet's annotations at that point; every
//     output (the clones on output 1 included) byte for byte, with lengths,
//     network header and annotations; the handlers agree.
void combos_chain_vs_elements(uint32_t batch)
{
    bool ok = true;
    const int n = 2000;
    const std::string B = "BATCH " + std::to_string(batch);
    const std::string OC = std::string("1, ") + MY_IP_TXT + ", 600, " + B;
    Member<InputComboC> c0("IPInputCombo", "1, " + B, 1);
    Member<OutComboC> c1("IPOutputCombo", OC, 5);
    c0.cls.color = c1.cls.color = 1;
    ChainHost ch({&c0, &c1});
    Host<InputComboC> h0("IPInputCombo", "1, " + B, 1);
    Host<OutComboC> h1("IPOutputCombo", OC, 5);
    h0.cls.color = h1.cls.color = 1;
    for (int i = 0; i < n; i++) {
        std::vector<uint8_t> b = ip_bytes(40 + (uint32_t)(i * 37) % 1300, i);
        if (i % 7 == 3)
            b = with_options(b, 1 + i % 4);
        if (i % 11 == 5) {                           // TTL 0-2: IPOutputCombo's output 3
            b[8] = (uint8_t)(i % 3);
            oracle_set_ip_checksum(b.data(), (uint32_t)b.size());
        }
        if (i % 13 == 6)
            b[12] ^= 1;                              // a bad checksum: IPInputCombo kills it
        std::vector<uint8_t> f(14, 0);
        f[0] = (uint8_t)i, f[12] = 0x08;
        f.insert(f.end(), b.begin(), b.end());
        for (int run = 0; run < 2; run++) {
            TPacket *p = make(f.data(), f.size(), i);
            p->a.fix_src = i % 5 == 0;
            p->a.bcast = i % 17 == 2;                // DropBroadcasts: killed, no clone
            p->a.paint = (uint32_t)(i % 3);
            if (run == 0)
                ch.push(p);
            else
                h0.push(p);
        }
    }
    ch.timer();
    h0.timer();
    for (TPacket *p : h0.out[0])
        h1.push(p);
    h0.out[0].clear();
    h1.timer();
    std::vector<std::vector<std::vector<TPacket *> > *> sep = {&h0.out, &h1.out};
    for (size_t k = 0; k < 2; k++)
        for (size_t q = 0; q < 5; q++) {
            const std::vector<TPacket *> &x = ch.m[k]->out[q], &y = (*sep[k])[q];
            CHECK(x.size() == y.size());
            for (size_t j = 0; j < x.size() && j < y.size(); j++)
                if (!same_packet(x[j], y[j])) {
                    std::printf("  member %zu port %zu #%zu: id %ld / %ld\n", k, q, j, x[j]->a.id, y[j]->a.id);
                    CHECK(same_packet(x[j], y[j]));
                    break;
                }
        }
    CHECK(ch.m[1]->out[1].size() > (size_t)n / 2);   // the clones
    CHECK(!ch.m[1]->out[0].empty() && !ch.m[1]->out[3].empty());
    for (const char *h : {"drops", "packets", "lost"}) {
        CHECK(ch.handler(0, h) == h0.handler(h));
        CHECK(ch.handler(1, h) == h1.handler(h));
    }
    CHECK(ch.runcount == 0 && h0.runcount == 0 && h1.runcount == 0);
    report(("combos_chain_matches_separate_elements_batch_" + std::to_string(batch)).c_str(), ok);
}

// 14. converging outputs (fake-iprouter.click: several members' error
//     outputs reach one element, ICMPError -> rt): CheckIPHeader's output 1
//     (bad checksums) and DecIPTTL's output 1 (expired TTLs) of one chain
//     push into one recording sink.  The reference pushes depth first, so
//     the sink would see the drops in push (token) order
//     (element.cc:2891-2896).  A chain hands its results out a batch at a
//     time, each member's in push order, member after member: the contract
//     (INTEGRATION.md "Ordering") is that the sink sees, batch by batch,
//     CheckIPHeader's drops of the batch in push order, then DecIPTTL's.
//     Asserted exactly, for the batches the flushes formed; the same drops,
//     each member's in push order, as the reference's.
void converging_outputs(uint32_t batch)
{
    bool ok = true;
    const int n = 3000;
    const std::string B = "BATCH " + std::to_string(batch);
    Member<CheckIPC> c0("CheckIPHeader", B, 2);
    Member<GWOptC> c1("IPGWOptions", std::string(MY_IP_TXT) + ", " + B, 2);
    Member<FixSrcC> c2("FixIPSrc", std::string(MY_IP_TXT) + ", " + B, 1);
    Member<DecTTLC> c3("DecIPTTL", B, 2);
    Member<FragC> c4("IPFragmenter", "1500, " + B, 2);
    c4.cls.mtu = 1500;
    ChainHost ch({&c0, &c1, &c2, &c3, &c4});
    std::vector<std::pair<int, long> > sink;         // (member, packet id) as they arrive
    size_t other = 0;
    ch.sink = [&](int k, int port, TPacket *p) {
        if (port == 1 && (k == 0 || k == 3))
            sink.emplace_back(k, p->a.id);
        else
            other++;
        TOps::kill(p);
    };
    std::vector<int> drop_at(n, -1);                 // the member that drops packet i (-1: none)
    for (int i = 0; i < n; i++) {
        std::vector<uint8_t> b = ip_bytes(60 + (uint32_t)(i * 29) % 900, i);
        if (i % 11 == 5) {                           // TTL 0-1: DecIPTTL's output 1
            b[8] = (uint8_t)(i % 2);
            oracle_set_ip_checksum(b.data(), (uint32_t)b.size());
            drop_at[i] = 3;
        }
        if (i % 13 == 6) {                           // a bad checksum: CheckIPHeader's output 1
            b[12] ^= 1;
            drop_at[i] = 0;
        }
        TPacket *p = make(b.data(), b.size(), i);
        p->nh = 0;
        ch.push(p);
    }
    ch.timer();
    // the contract: batch by batch (the flushes' batches: BATCH packets in
    // push order, at most the core's in-flight cap), member 0's drops in
    // push order, then member 3's
    const uint32_t eb = std::min<uint32_t>(batch, (uint32_t)ChainHost::Core::INFLIGHT);
    std::vector<std::pair<int, long> > want, ref;
    for (int b0 = 0; b0 < n; b0 += (int)eb)
        for (int k : {0, 3})
            for (int i = b0; i < n && i < b0 + (int)eb; i++)
                if (drop_at[i] == k)
                    want.emplace_back(k, i);
    for (int i = 0; i < n; i++)                      // the reference's depth-first order
        if (drop_at[i] >= 0)
            ref.emplace_back(drop_at[i], i);
    CHECK(sink == want);
    std::vector<std::pair<int, long> > a = sink, r = ref;
    std::sort(a.begin(), a.end());
    std::sort(r.begin(), r.end());
    CHECK(a == r);                                   // the same drops at the same members
    for (int k : {0, 3}) {                           // each member's in push order
        long last = -1;
        for (auto &x : sink)
            if (x.first == k) {
                CHECK(x.second > last);
                last = x.second;
            }
    }
    CHECK(other + sink.size() == (size_t)n);
    std::printf("  converging sink: %zu drops, %s the reference's order\n", sink.size(),
                sink == ref ? "equal to" : "batch-major, not");
    report(("converging_outputs_batch_order_" + std::to_string(batch)).c_str(), ok);
}

}   // namespace

int main()
{
    if (clk_device_count() < 1) {
        std::printf("SKIP no gfx950 GPU\n");
        return 0;
    }

    every_class();
    output_combo_copy_fails();
    push_check_ip();
    pull_set_udp();
    pull_two_elements();
    fragmenter();
    // the n-th checked HIP call of the first flush fails: the packets H2D
    // (4), a verdict D2H (SetUDPChecksum 9, IPOutputCombo 10), IPOutputCombo's
    // checksums D2H (11), the packets back D2H (IPOutputCombo 12); -1: the
    // completion wait
    for (int nth : {4, 9, -1})
        failed_flush_retry<SetC>("SetUDPChecksum", "", nth);
    for (int nth : {4, 10, 11, 12, -1})
        failed_flush_retry<OutComboC>("IPOutputCombo", "1, 18.26.4.24, 1500", nth);
    retry_limit();
    reentrant_push();
    threads();
    shared_state_two_threads();
    cleanup_partial();
    chain_vs_elements(65536, 0);
    chain_vs_elements(300, 0);
    chain_vs_elements(1000, 777);
    combos_chain_vs_elements(65536);
    combos_chain_vs_elements(300);
    converging_outputs(300);
    converging_outputs(65536);
    std::printf("live packets at exit: %ld\n", (long)g_live);
    return g_fail ? 1 : 0;
}
