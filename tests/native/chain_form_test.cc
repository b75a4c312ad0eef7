// chain_form_test.cc -- the Click adapter's chain rules (click_integration/
// elements/hip/hipchain.hh), as hipbatch.cc applies them at initialize(),
// over router graphs built here: which GPU-backed elements join the chain
// of the one before them and which run alone.  The class traits are the
// shipped ones (hipclasses.hh).  CPU only: no GPU, no glue library calls.
// Prints one line per case and "ALL OK" at the end (tests/test_chain_form.py).
#include <cstdio>
#include <cstdint>
#include <map>
#include <string>
#include <vector>

#include "click_amd_elements.h"
#include "../../click_integration/elements/hip/hipcore.hh"
#include "../../click_integration/elements/hip/hipclasses.hh"
#include "../../click_integration/elements/hip/hipchain.hh"

namespace {

struct NoPacket {};
struct NoOps {};
template <template <class, class> class C> struct Traits {
    typedef C<NoPacket, NoOps> K;
    enum { may_write = K::may_write, chain_last = K::chain_last, chain_head_only = K::chain_head_only,
           pass_effects = K::pass_effects };
};

// One element of a router graph.  gpu: a HIPBatchElement (its class traits
// below); push: its ports are push (a pull element's are not).
struct Elt {
    std::string name;
    bool gpu = false;
    bool push = true;
    bool chain = true;          // CHAIN
    int device = -1;            // DEVICE
    bool may_write = false, chain_last = false, chain_head_only = false, pass_effects = false;
};

struct Conn {
    Elt *from;
    int fport;
    Elt *to;
    int tport;
};

struct Graph {
    std::vector<Elt *> nodes;
    std::vector<Conn> conns;
    std::map<std::string, Elt *> by;

    ~Graph()
    {
        for (Elt *n : nodes)
            delete n;
    }
    template <class T> Elt *gpu(const std::string &name, int device = -1, bool chain = true)
    {
        Elt *n = add(name);
        n->gpu = true;
        n->device = device;
        n->chain = chain;
        n->may_write = T::may_write;
        n->chain_last = T::chain_last;
        n->chain_head_only = T::chain_head_only;
        n->pass_effects = T::pass_effects;
        return n;
    }
    Elt *add(const std::string &name, bool push = true)
    {
        Elt *n = new Elt;
        n->name = name;
        n->push = push;
        nodes.push_back(n);
        by[name] = n;
        return n;
    }
    void connect(const std::string &a, int ap, const std::string &b, int bp) { conns.push_back({by[a], ap, by[b], bp}); }
    // a -> b -> c ... on output 0 / input 0
    void line(const std::vector<std::string> &v)
    {
        for (size_t i = 0; i + 1 < v.size(); i++)
            connect(v[i], 0, v[i + 1], 0);
    }
};

// The trait, as hipbatch.cc's HIPChainGraph answers it over Click's Router
struct G {
    typedef Elt *Node;
    Graph &g;
    Node push_next(Node x) const
    {
        if (!x->push)
            return nullptr;
        for (const Conn &c : g.conns)
            if (c.from == x && c.fport == 0)
                return c.tport == 0 && c.to->gpu ? c.to : nullptr;
        return nullptr;
    }
    Node sole_upstream(Node y) const
    {
        if (!y->push)
            return nullptr;
        Node first = nullptr;
        int n = 0;
        for (const Conn &c : g.conns)
            if (c.to == y && c.tport == 0 && n++ == 0)
                first = c.from;
        return n == 1 && first->gpu ? first : nullptr;
    }
    bool chain_conf(Node x) const { return x->chain; }
    int device(Node x) const { return x->device; }
    bool may_write(Node x) const { return x->may_write; }
    bool chain_last(Node x) const { return x->chain_last; }
    bool chain_head_only(Node x) const { return x->chain_head_only; }
    bool pass_effects(Node x) const { return x->pass_effects; }
};

typedef Traits<hipcore::Plain> Check;                    // CheckUDPHeader, CheckTCPHeader, CheckIPHeader2 ...
typedef Traits<hipcore::CheckIPHeaderClass> CheckIP;
typedef Traits<hipcore::IPInputComboClass> InCombo;
typedef Traits<hipcore::SetChecksumClass> Set;
typedef Traits<hipcore::DecIPTTLClass> DecTTL;
typedef Traits<hipcore::IPGWOptionsClass> GWOpt;
typedef Traits<hipcore::FixIPSrcClass> FixSrc;
typedef Traits<hipcore::IPOutputComboClass> OutCombo;
typedef Traits<hipcore::IPFragmenterClass> Frag;

int failures = 0;

// every GPU-backed element's chain, "A[A,B,C]" joined by spaces, in node
// order; a member is marked "*" (its own chain is [itself]: it runs alone
// only when something pushes to it directly)
std::string chains(Graph &g)
{
    G t{g};
    std::string s;
    for (Elt *n : g.nodes) {
        if (!n->gpu)
            continue;
        std::vector<Elt *> c;
        hipcore::form_chain(t, n, c);
        if (!s.empty())
            s += " ";
        s += n->name + "[";
        for (size_t i = 0; i < c.size(); i++)
            s += (i ? "," : "") + c[i]->name;
        s += "]";
        if (hipcore::chain_member(t, n))
            s += "*";                                   // runs in the chain of the one before it
    }
    return s;
}

void expect(const char *label, const std::string &got, const std::string &want)
{
    bool ok = got == want;
    std::printf("%s %s\n", ok ? "PASS" : "FAIL", label);
    if (!ok) {
        std::printf("  got:  %s\n  want: %s\n", got.c_str(), want.c_str());
        failures++;
    }
}

void expect_u64(const char *label, uint64_t got, uint64_t want)
{
    bool ok = got == want;
    std::printf("%s %s\n", ok ? "PASS" : "FAIL", label);
    if (!ok) {
        std::printf("  got:  %llx\n  want: %llx\n", (unsigned long long)got, (unsigned long long)want);
        failures++;
    }
}

// conf/fake-iprouter.click:38-50, one interface's path: the elements between
// CheckIPHeader and IPGWOptions are not GPU-backed
void fake_iprouter()
{
    Graph g;
    g.add("c0");                                        // Classifier
    g.add("strip");                                     // Strip(14)
    g.gpu<CheckIP>("chk");
    g.add("gip");                                       // GetIPAddress(16)
    g.add("rt");                                        // StaticIPLookup
    g.add("db");                                        // DropBroadcasts
    g.add("pt");                                        // PaintTee
    g.gpu<GWOpt>("gio");
    g.gpu<FixSrc>("fix");
    g.gpu<DecTTL>("dt");
    g.gpu<Frag>("fr");
    g.add("arpq");                                      // ARPQuerier
    g.add("icmp");                                      // ICMPError
    g.line({"c0", "strip", "chk", "gip", "rt", "db", "pt", "gio", "fix", "dt", "fr", "arpq"});
    g.connect("gio", 1, "icmp", 0);
    g.connect("dt", 1, "icmp", 0);
    g.connect("fr", 1, "icmp", 0);
    expect("fake_iprouter", chains(g), "chk[chk] gio[gio,fix,dt,fr] fix[fix]* dt[dt]* fr[fr]*");
    G t{g};
    std::vector<Elt *> c;
    hipcore::form_chain(t, g.by["gio"], c);
    expect("fake_iprouter_writes", hipcore::chain_writes(t, c) ? "writes" : "reads", "writes");
    // FixIPSrc clears its annotation on the packets it passes (member 1)
    expect_u64("fake_iprouter_report", hipcore::chain_report(t, c), 0x2);
}

// the five elements back to back: one chain; the fragmenter ends it, so the
// SetIPChecksum after it runs alone
void five_then_set()
{
    Graph g;
    g.add("src");
    g.gpu<CheckIP>("chk");
    g.gpu<GWOpt>("gio");
    g.gpu<FixSrc>("fix");
    g.gpu<DecTTL>("dt");
    g.gpu<Frag>("fr");
    g.gpu<Set>("set");
    g.line({"src", "chk", "gio", "fix", "dt", "fr", "set"});
    expect("five_then_set", chains(g), "chk[chk,gio,fix,dt,fr] gio[gio]* fix[fix]* dt[dt]* fr[fr]* set[set]");
    G t{g};
    std::vector<Elt *> c;
    hipcore::form_chain(t, g.by["chk"], c);
    expect_u64("five_report", hipcore::chain_report(t, c), 0x5);   // CheckIPHeader (0), FixIPSrc (2)
}

// the combos: IPOutputCombo joins the chain of IPInputCombo (its PaintTee
// clone, as a member after the head, comes from the bytes the glue keeps as
// the packet reaches it), and the chain writes
void combos()
{
    Graph g;
    g.add("src");
    g.gpu<InCombo>("in");
    g.gpu<OutCombo>("out");
    g.gpu<Check>("cu");
    g.gpu<Set>("su");
    g.line({"src", "in", "out", "cu", "su"});
    expect("combos", chains(g), "in[in,out,cu,su] out[out]* cu[cu]* su[su]*");
    G t{g};
    std::vector<Elt *> c;
    hipcore::form_chain(t, g.by["in"], c);
    expect("combos_in_writes", hipcore::chain_writes(t, c) ? "writes" : "reads", "writes");
    expect_u64("combos_report", hipcore::chain_report(t, c), 0x3);   // IPInputCombo (0), IPOutputCombo (1)
}

// a class that may only head a chain (chain_head_only: none of the shipped
// classes, the rule stays) never joins one: it heads its own
struct HeadOnly {
    enum { may_write = 1, chain_last = 0, chain_head_only = 1, pass_effects = 0 };
};
void head_only()
{
    Graph g;
    g.add("src");
    g.gpu<InCombo>("in");
    g.gpu<HeadOnly>("h");
    g.gpu<Check>("cu");
    g.line({"src", "in", "h", "cu"});
    expect("head_only", chains(g), "in[in] h[h,cu] cu[cu]*");
}

// a member pushed into by two outputs cannot join: it heads its own chain
void two_upstreams()
{
    Graph g;
    g.add("s1");
    g.add("s2");
    g.gpu<CheckIP>("a");
    g.gpu<Check>("b");
    g.gpu<Set>("c");
    g.gpu<Set>("d");
    g.line({"s1", "a", "c", "d"});
    g.line({"s2", "b"});
    g.connect("b", 0, "c", 0);
    expect("two_upstreams", chains(g), "a[a] b[b] c[c,d] d[d]*");
}

// DEVICE differs: the chain breaks there
void devices()
{
    Graph g;
    g.add("s");
    g.gpu<Check>("a", 0);
    g.gpu<Set>("b", 1);
    g.gpu<Set>("c", 1);
    g.gpu<Set>("d", -1);
    g.line({"s", "a", "b", "c", "d"});
    expect("devices", chains(g), "a[a] b[b,c] c[c]* d[d]");
}

// CHAIN false: on a middle element (it runs alone, the next heads), on a head
void chain_false()
{
    Graph g;
    g.add("s");
    g.gpu<Check>("a");
    g.gpu<Set>("b", -1, false);
    g.gpu<Set>("c");
    g.gpu<Set>("d");
    g.line({"s", "a", "b", "c", "d"});
    expect("chain_false_middle", chains(g), "a[a] b[b] c[c,d] d[d]*");
    Graph h;
    h.add("s");
    h.gpu<Check>("a", -1, false);
    h.gpu<Set>("b");
    h.gpu<Set>("c");
    h.line({"s", "a", "b", "c"});
    expect("chain_false_head", chains(h), "a[a] b[b,c] c[c]*");
}

// only output 0 into input 0 joins; pull elements never
void ports_and_pull()
{
    Graph g;
    g.add("s");
    g.gpu<Check>("a");
    g.gpu<Set>("b");
    g.gpu<Set>("c");
    g.gpu<Set>("d");
    g.line({"s", "a"});
    g.connect("a", 0, "b", 1);                          // into input 1
    g.connect("a", 1, "c", 0);                          // from output 1
    g.connect("c", 0, "d", 0);
    expect("ports", chains(g), "a[a] b[b] c[c,d] d[d]*");
    Graph h;
    h.add("q", false);                                  // a Queue: pull output
    h.gpu<Check>("a");
    h.gpu<Set>("b");
    h.add("u", false);                                  // ToDevice: pull input
    h.by["a"]->push = false;                            // agnostic in pull context
    h.by["b"]->push = false;
    h.line({"q", "a", "b", "u"});
    expect("pull", chains(h), "a[a] b[b]");
}

// a ring of GPU-backed elements: every one is the sole upstream of the next,
// so none heads a chain and each runs alone (no endless walk)
void cycle()
{
    Graph g;
    g.gpu<Check>("a");
    g.gpu<Set>("b");
    g.gpu<Set>("c");
    g.line({"a", "b", "c", "a"});
    expect("cycle", chains(g), "a[a]* b[b]* c[c]*");
}

// more members than the pass report's 64 bits: the chain stops at 64; the
// rest run as separate elements, pushed to by the last member's output 0
void long_line()
{
    Graph g;
    g.add("s");
    std::vector<std::string> v{"s"};
    for (int i = 0; i < 70; i++) {
        std::string n = "e" + std::to_string(i);
        g.gpu<Check>(n);
        v.push_back(n);
    }
    g.line(v);
    G t{g};
    std::vector<Elt *> c;
    hipcore::form_chain(t, g.by["e0"], c);
    expect("long_line_64", std::to_string(c.size()), std::to_string((int)hipcore::CHAIN_MAX));
    hipcore::form_chain(t, g.by["e64"], c);
    expect("long_line_rest_alone", std::to_string(c.size()), "1");
}

// the head's readying of a packet: writable when a member writes, the
// members' annotations staged (hipchain.hh chain_ready)
struct Pk {
    bool shared;
    bool fix;
    bool bcast;
    uint32_t paint;
};
struct PkOps {
    static bool fail;
    static Pk *uniqueify(Pk *p)
    {
        if (fail) {
            delete p;
            return nullptr;
        }
        p->shared = false;
        return p;
    }
    static bool fix_ip_src(Pk *p) { return p->fix; }
    static bool broadcast_or_multicast(Pk *p) { return p->bcast; }
    static uint32_t paint(Pk *p) { return p->paint; }
};
bool PkOps::fail = false;

void ready()
{
    uint32_t anno = 0;
    Pk *p = new Pk{true, true, false, 7};
    p = hipcore::chain_ready<Pk, PkOps>(p, false, &anno);
    bool ok = p && p->shared && anno == (CLK_ANNO_FIX_IP_SRC | CLK_ANNO_PAINT(7));
    p = hipcore::chain_ready<Pk, PkOps>(p, true, &(anno = 0));
    ok = ok && p && !p->shared;
    p->fix = false, p->bcast = true, p->paint = 300;
    p = hipcore::chain_ready<Pk, PkOps>(p, true, &(anno = 0));
    ok = ok && p && anno == (CLK_ANNO_BCAST | CLK_ANNO_PAINT(300));
    PkOps::fail = true;
    ok = ok && !hipcore::chain_ready<Pk, PkOps>(p, true, &(anno = 0));
    expect("chain_ready", ok ? "ok" : "wrong", "ok");
}

}   // namespace

int main()
{
    fake_iprouter();
    five_then_set();
    combos();
    head_only();
    two_upstreams();
    devices();
    chain_false();
    ports_and_pull();
    cycle();
    long_line();
    ready();
    if (failures) {
        std::printf("%d FAILED\n", failures);
        return 1;
    }
    std::printf("ALL OK\n");
    return 0;
}
