// elements.hh -- host-side C++ element glue for the GPU checksum path.
//
// Each class keeps the reference element's configuration keywords, routing
// (output 0 / output 1 / kill), counters, handlers and click_chatter text,
// and runs the checksum work as one GPU batch per flush() through the C ABI
// (include/click_amd_cksum.h).  See include/click_amd_elements.h.
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <string>
#include <memory>
#include <atomic>
#include <vector>

#include <hip/hip_runtime.h>

#include "../../include/click_amd_cksum.h"
#include "../../include/click_amd_elements.h"

struct clk_element;          // include/click_amd_elements.h

namespace clk {
namespace host {

struct Result {
    uint64_t token;
    int32_t port;        // 0..4, or -1 (kill)
    uint32_t length;     // packet length after the element
    uint32_t aux;        // clk_element_results_aux (problem offset, clone flag, new-packet key)
};

// Routed results in push order: appended by flush(), popped by the caller.
// Struct of arrays over raw buffers with a read index: appends are plain
// stores after one capacity check per batch (reserve_more), pops are bulk
// copies, storage is reused once everything has been popped.
class ResultQueue {
  public:
    ResultQueue() = default;
    ResultQueue(const ResultQueue &) = delete;
    ResultQueue &operator=(const ResultQueue &) = delete;
    ~ResultQueue()
    {
        std::free(tok_);
        std::free(port_);
        std::free(len_);
        std::free(aux_);
    }
    void reserve_more(size_t k)
    {
        if (head_ > 4096 && head_ * 2 > n_)          // a caller that never drains: drop the popped prefix
            compact();
        if (n_ + k > cap_)
            grow(n_ + k);
    }
    void push_back(const Result &r)
    {
        if (n_ == cap_)
            grow(n_ + 1);
        push_unchecked(r);
    }
    void push_unchecked(const Result &r)             // after reserve_more
    {
        tok_[n_] = r.token;
        port_[n_] = r.port;
        len_[n_] = r.length;
        aux_[n_] = r.aux;
        n_++;
    }
    bool empty() const { return head_ == n_; }
    size_t size() const { return n_ - head_; }
    uint64_t pop(uint64_t *tokens, int32_t *ports, uint32_t *lengths, uint32_t *aux, uint64_t cap)
    {
        const size_t k = (size_t)std::min<uint64_t>(cap, size());
        if (tokens) std::memcpy(tokens, tok_ + head_, k * sizeof(uint64_t));
        if (ports) std::memcpy(ports, port_ + head_, k * sizeof(int32_t));
        if (lengths) std::memcpy(lengths, len_ + head_, k * sizeof(uint32_t));
        if (aux) std::memcpy(aux, aux_ + head_, k * sizeof(uint32_t));
        head_ += k;
        if (head_ == n_)
            head_ = n_ = 0;
        return k;
    }

  private:
    void grow(size_t need)
    {
        const size_t c = std::max<size_t>(need, std::max<size_t>(cap_ * 2, 1024));
        tok_ = (uint64_t *)realloc_or_die(tok_, c * sizeof(uint64_t));
        port_ = (int32_t *)realloc_or_die(port_, c * sizeof(int32_t));
        len_ = (uint32_t *)realloc_or_die(len_, c * sizeof(uint32_t));
        aux_ = (uint32_t *)realloc_or_die(aux_, c * sizeof(uint32_t));
        cap_ = c;
    }
    static void *realloc_or_die(void *p, size_t bytes)
    {
        void *q = std::realloc(p, bytes);
        if (!q)
            std::abort();                             // as std::vector's bad_alloc, without exceptions
        return q;
    }
    void compact()
    {
        const size_t k = n_ - head_;
        std::memmove(tok_, tok_ + head_, k * sizeof(uint64_t));
        std::memmove(port_, port_ + head_, k * sizeof(int32_t));
        std::memmove(len_, len_ + head_, k * sizeof(uint32_t));
        std::memmove(aux_, aux_ + head_, k * sizeof(uint32_t));
        n_ = k;
        head_ = 0;
    }
    uint64_t *tok_ = nullptr;
    int32_t *port_ = nullptr;
    uint32_t *len_ = nullptr, *aux_ = nullptr;
    size_t cap_ = 0, n_ = 0, head_ = 0;
};

// Click-style configuration: comma-separated arguments, "KEYWORD value".
struct ConfArgs {
    std::vector<std::pair<std::string, std::string>> kw;   // keyword arguments
    std::vector<std::string> pos;                          // positional arguments
    static bool split(const std::string &conf, ConfArgs *out, std::string *err);
    bool take(const char *key, std::string *value);        // removes it
};
bool parse_bool(const std::string &s, bool *v);
bool parse_int(const std::string &s, long *v);
bool parse_ip(const std::string &s, uint32_t *saddr);       // raw network-order s_addr
bool parse_prefix(const std::string &s, uint32_t *saddr, uint32_t *mask);

// Copy n staged bytes.  Spans up to 128 B move as whole 16 B pieces when
// the packet has them (avail: bytes readable from src): fixed-size moves
// instead of a variable-length memcpy call.  The bytes copied past n stay
// inside the 64 B of slack every staging slot is grown with and are
// overwritten by the next packet's slot.
// how many packets ahead a chain loop prefetches the header it reads
#ifndef CLK_CHAIN_PF
#define CLK_CHAIN_PF 24
#endif
// a push burst prefetches each staged packet's span this many packets ahead
#ifndef CLK_BURST_PF
#define CLK_BURST_PF 3
#endif
// a packet pushed alone (not in a burst) whose staged span is at least this
// long is gathered at launch, in one loop over the batch with its next
// packets' lines prefetched (0: at push)
#ifndef CLK_STAGE_DEFER
#define CLK_STAGE_DEFER 256
#endif
inline const uint8_t *chain_hdr(const uint8_t *data, int32_t nh) { return data + (nh > 0 ? nh : 0); }

inline void stage_copy(uint8_t *dst, const uint8_t *src, uint32_t n, uint32_t avail)
{
    if (n == 0)
        return;
    const uint64_t q = ((uint64_t)n + 15) >> 4;
    if (q <= 8 && 16 * q <= avail) {
        for (uint64_t k = 0; k < q; k++)
            std::memcpy(dst + 16 * k, src + 16 * k, 16);
    } else {
        std::memcpy(dst, src, n);
    }
}

class BatchElement;

// One member's share of a chain flush (class Chain, chain.cc).
struct ChainView {           // a packet as a chain member sees it
    uint8_t *data;
    uint64_t token, slot;    // slot: the staging offset of data
    uint32_t length;
    int32_t nh;
    uint16_t anno;
    uint16_t done;           // it has left the chain (a 16-bit store: a byte store would alias
                             // every field the loops keep in registers)
};
struct ChainExit {           // a result leaving the chain at `member` (24 B)
    uint64_t token;
    uint32_t length, aux;
    uint32_t idx;            // the packet's place in the batch (~0u: a clone / new packet)
    int16_t member, port;    // (a chain has at most 64 members; ports are small, CLK_PORT_* negative)
    ChainExit() = default;
    ChainExit(uint64_t t, int32_t m, int32_t p, uint32_t l, uint32_t a, uint32_t i)
        : token(t), length(l), aux(a), idx(i), member((int16_t)m), port((int16_t)p) { }
};
// A member's decision a chain can take without asking it: the packets its
// span() decides on the host and its route() then passes on unchanged
// (no write, no annotation, no result of its own but the count).
// How a staged chain member's rewrite reaches the packet.
enum ChainHostRewrite {
    CHAIN_HOST_NONE = 0,     // copied back (write extent past nh)
    CHAIN_HOST_ALL,          // route() writes it from the verdict (DecIPTTL, the Set elements)
    CHAIN_HOST_SIMPLE,       // route() writes it for simple packets, the rest copied back (IPOutputCombo)
};
enum ChainPass {
    CHAIN_PASS_NONE = 0,
    CHAIN_PASS_NO_OPTIONS,   // IPGWOptions: no header, or ip_hl <= 5
    CHAIN_PASS_NO_FIX,       // FixIPSrc: no FIX_IP_SRC annotation, or no header
    CHAIN_PASS_WITHIN,       // IPFragmenter: network length <= param (MTU), or no header
    CHAIN_PASS_TTL,          // DecIPTTL: param == 0 (ACTIVE false), or no header
};
// A reached packet's code at a member: its GPU index (>= 0), its host
// decision (-1 - code), a pass rule's pass (CHAIN_CODE_PASS), or not looked
// at yet (the member's prep loop has not run over it)
enum : int32_t { CHAIN_CODE_PASS = INT32_MIN };
struct ChainWork {
    ChainView *views = nullptr;               // per chain packet, updated as it passes members
    uint32_t *reached = nullptr;              // the packets that reached this member, in push order
    int32_t *code = nullptr;                  // per reached packet (CHAIN_CODE_PASS, GPU index, -1 - host code)
    uint32_t *span_off = nullptr;             // per reached packet with a descriptor: its span
    uint32_t *span_len = nullptr;
    size_t nreached = 0;
    size_t nprep = 0;                         // reached packets the prep loop has looked at
    size_t routed = 0;                        // reached packets routed so far
    uint64_t *h_off = nullptr;                // the member's batch (pinned)
    uint32_t *h_len = nullptr;
    uint8_t *h_anno = nullptr;
    const uint8_t *h_codes = nullptr;
    const uint16_t *h_sums = nullptr;
    size_t n = 0;                             // packets in the member's GPU batch
    uint32_t maxlen = 0;
    std::vector<ChainExit> *out = nullptr;
    // staged batches: per packet, the bytes to copy back (grown by each
    // member that rewrites it: shift + its write extent), its first slot
    uint32_t *back = nullptr;
    const uint32_t *staged = nullptr;
    const uint64_t *slot0 = nullptr;          // per chain packet: its staging offset as pushed
    uint32_t wext = 0;                        // the member's write extent past nh (~0u: all; 0: none)
    bool wext_unless_simple = false;          // CHAIN_HOST_SIMPLE: only packets that are not simple
    int member = 0;
    uint32_t strip = 0;                       // the member's strip() / nh_after()
    int32_t nh_after = -2;
    uint8_t pass = CHAIN_PASS_NONE;           // ChainPass, with pass_param
    uint32_t pass_param = 0;
    bool clones = false;                      // the prep loop met a packet to clone (clone_key)
    uint32_t *clone_key = nullptr;            // a member after the head with pre results (IPOutputCombo's
                                              // PaintTee clone): per chain packet, the key of the bytes
                                              // as they reached the member (Chain::run_member), 0: none
    bool last = false;
    bool report_passes = false;               // a CLK_PORT_NEXT record for each packet passed on
    ChainWork *next = nullptr;                // member k+1's (0 for the last)
    BatchElement *elem = nullptr;             // member k
    uint64_t counted = 0;                     // packets member k took in a loop (its packets_, added at the end)
    void reset()
    {
        nreached = 0;
        nprep = 0;
        clones = false;
        routed = 0;
        n = 0;
        maxlen = 0;
    }
    // the packet passes this member unchanged, decided without the member
    bool passes(const ChainView &v) const
    {
        const bool nohdr = v.nh < 0 || (uint32_t)v.nh >= v.length;
        switch (pass) {
        case CHAIN_PASS_NO_OPTIONS:
            return nohdr || v.length - (uint32_t)v.nh < 20 || (v.data[v.nh] & 0xF) <= 5;
        case CHAIN_PASS_NO_FIX:
            return nohdr || !(v.anno & CLK_ANNO_FIX_IP_SRC);
        case CHAIN_PASS_WITHIN: {
            const uint32_t nh = v.nh >= 0 ? (uint32_t)v.nh : 0u;
            return nh > v.length || (int)(v.length - nh) <= (int)pass_param;
        }
        case CHAIN_PASS_TTL:
            return pass_param == 0 || v.nh < 0 || (uint32_t)v.nh > v.length;
        default:
            return false;
        }
    }
};

// The final classes' fast loops: push_burst() and route_stage() over the
// class's own span() / route(), called qualified so they inline (no
// virtual call per packet).
#define CLK_INL __attribute__((always_inline))
#define CLK_GLUE_LOOPS(C)                                                                                       \
    int push(uint8_t *d_, uint32_t l_, int32_t nh_, uint64_t t_, uint32_t a_ = 0, int32_t th_ = -1) override    \
    {                                                                                                           \
        return push_one([this](const Pending &p, uint32_t *o, uint32_t *l, int32_t *c) CLK_INL {                 \
            bool r_; [[clang::always_inline]] r_ = this->C::span(p, o, l, c);                                   \
            return r_;                                                                                          \
        }, d_, l_, nh_, t_, a_, hold_, th_);                                                                    \
    }                                                                                                           \
    int push_burst(uint8_t *const *d_, const uint32_t *l_, const int32_t *nh_, uint64_t t0_, uint32_t n_) override \
    {                                                                                                           \
        return burst_loop([this](const Pending &p, uint32_t *o, uint32_t *l, int32_t *c) CLK_INL {               \
            bool r_; [[clang::always_inline]] r_ = this->C::span(p, o, l, c);                                   \
            return r_;                                                                                          \
        }, d_, l_, nh_, t0_, n_);                                                                               \
    }                                                                                                           \
    void route_stage(Stage &g_) override                                                                        \
    {                                                                                                           \
        route_loop(g_, [this](Pending &p, int code, uint16_t sum, Result *r) CLK_INL {                          \
            [[clang::always_inline]] this->C::route(p, code, sum, r);                                           \
        }, [this](Pending &p, Result *r) CLK_INL {                                                              \
            bool r_; [[clang::always_inline]] r_ = this->C::pre_route(p, r);                                    \
            return r_;                                                                                          \
        });                                                                                                     \
    }                                                                                                           \
    void chain_prep(ChainWork &w_) override                                                                    \
    {                                                                                                           \
        chain_prep_loop(w_, [this](const Pending &p, uint32_t *o, uint32_t *l, int32_t *c) CLK_INL {             \
            bool r_; [[clang::always_inline]] r_ = this->C::span(p, o, l, c);                                   \
            return r_;                                                                                          \
        }, [this](const ChainView &v) CLK_INL {                                                                 \
            bool r_; [[clang::always_inline]] r_ = this->C::pre_clone(v);                                       \
            return r_;                                                                                          \
        });                                                                                                     \
    }                                                                                                           \
    void chain_route_all(ChainWork &w_) override                                                               \
    {                                                                                                           \
        chain_route_loop(w_, [this](Pending &p, int code, uint16_t sum, Result *r) CLK_INL {                    \
            [[clang::always_inline]] this->C::route(p, code, sum, r);                                           \
        }, [this](Pending &p, Result *r) CLK_INL {                                                              \
            bool r_; [[clang::always_inline]] r_ = this->C::pre_route(p, r);                                    \
            return r_;                                                                                          \
        });                                                                                                     \
    }

class Chain;

// Each element on cache lines of its own (alignas: no line shared with
// another thread's element, whose per-packet fields would bounce it)
class alignas(128) BatchElement {
  public:
    BatchElement(clk_ctx *ctx, const std::string &name, int noutputs);
    virtual ~BatchElement();
    virtual const char *class_name() const = 0;
    virtual int configure(ConfArgs &args, std::string *err);
    // one packet (the final classes run it with their span() inlined,
    // CLK_GLUE_LOOPS); th_offset: the transport header annotation
    // (clk_element_push_th), -1 unknown
    virtual int push(uint8_t *data, uint32_t length, int32_t nh_offset, uint64_t token, uint32_t anno = 0,
                     int32_t th_offset = -1);
    // a burst of packets (tokens first_token + k), flushing double-buffered
    // whenever the batch fills; the final classes run it with their span()
    // inlined (CLK_GLUE_LOOPS)
    virtual int push_burst(uint8_t *const *datas, const uint32_t *lengths, const int32_t *nh_offsets,
                           uint64_t first_token, uint32_t n);
    int flush();          // run the staged batch, wait for every batch in flight, route
    int flush_async();    // route the batch in flight (if any), launch the staged one, return
    uint64_t abandon();   // route every staged / in-flight packet as killed (a GPU that keeps failing)
    uint64_t pop_results(uint64_t *tokens, int32_t *ports, uint32_t *lengths, uint32_t *aux, uint64_t cap);
    int64_t take_packet(uint32_t key, uint8_t *buf, size_t cap);
    virtual std::string read_handler(const std::string &h) const;
    std::string take_messages();
    void hold_packets(bool on) { hold_ = on; }   // deferred gather allowed (clk_element_hold_packets)
    void share_messages(const BatchElement &with) { gate_ = with.gate_; }
    const std::string &name() const { return name_; }
    std::string declaration() const { return name_ + " :: " + class_name(); }
    const std::string &last_error() const { return err_; }
    size_t pending() const { return st_[cur_].pend.size(); }

  protected:
    struct Pending {         // 48 bytes: staged per packet, read by launch() and flush()
        uint8_t *data;
        uint64_t token;
        uint64_t slot;       // staging offset of the span
        uint32_t length;
        int32_t nh_off;
        uint32_t span_off;   // span start relative to data
        uint32_t span_len;
        uint32_t index;      // position in the GPU batch (staged packets)
        int16_t host_code;   // >= 0: decided on the host (not staged)
        uint16_t anno;       // CLK_ANNO_* bits (and ANNO_CANON)
    };
    // Pending::anno: staged as a canonical copy (push_irregular); span_off
    // is then the transport header's offset from data
    static constexpr uint16_t ANNO_CANON = 0x4;
    // Bytes the kernel needs, relative to data; return false to decide on the
    // host with *code (routed like a kernel result).
    virtual bool span(const Pending &p, uint32_t *off, uint32_t *len, int32_t *code) const = 0;
    virtual int run(const clk_batch *b, uint8_t *d_codes, uint16_t *d_sums) = 0;
    virtual void route(Pending &p, int code, uint16_t sum, Result *r) = 0;
    virtual bool wants_sums() const { return false; }
    // copy the device batch back into the staging arena after run() (the
    // kernel rewrote bytes route() writes back into the packet)
    virtual bool wants_arena_back() const { return false; }
    // false when running the element twice on the same packet bytes changes
    // them again (DecIPTTL, IPGWOptions, IPOutputCombo, IPFragmenter): a
    // ZEROCOPY batch of such an element whose kernel may have run is not
    // retried after a failed completion but abandoned (its packets killed)
    virtual bool idempotent() const { return true; }
    // upload anno & 0xFF of the staged packets; run() finds it in d_anno_
    virtual bool wants_anno() const { return false; }
    // called by flush() before route(): results() of the packet that precede
    // its own (IPOutputCombo's clone); only when has_pre_route_
    // (returns whether it made one, in *r)
    virtual bool pre_route(Pending &, Result *) { return false; }
    // called after route(): results that follow the packet's own (fragments);
    // only when has_post_route_
    virtual void post_route(Pending &, int, ResultQueue &) {}
    bool has_pre_route_ = false, has_post_route_ = false;
    // ---- chain mode (class Chain: consecutive elements on one staged batch)
    // A packet route() sends to output 0 goes on to the next element of a
    // chain with the result's length; the element may pull bytes off its
    // front (IPInputCombo's Strip(14)) and set its network header offset
    // (-2: unchanged).
    virtual uint32_t strip() const { return 0; }
    virtual int32_t nh_after() const { return -2; }
    // the bytes from data() the element's kernel can read / write of a packet
    // of `length` bytes whose network header is at nh (~0u: all of it)
    virtual uint32_t chain_extent(int32_t nh, uint32_t length) const { (void)nh, (void)length; return 0xFFFFFFFFu; }
    // the element's kernel writes packet bytes (a chain copies them back)
    virtual bool writes() const { return wants_sums() || wants_arena_back() || !idempotent(); }
    // a chain's loops over the packets that reached a member (CLK_GLUE_LOOPS
    // inlines the class's span / route into them: one call per member and
    // batch).  chain_prep(): each reached packet not looked at yet -- a pass
    // rule's pass, its descriptor (it waits for the GPU) or its host decision.
    // chain_route_all(): after the member's kernel, every reached packet not
    // routed yet, in push order; each one passed on reaches member k+1.
    virtual void chain_prep(ChainWork &w);
    virtual void chain_route_all(ChainWork &w);
    // the decision the chain may take for the member (ChainPass)
    virtual void chain_pass(uint8_t *kind, uint32_t *param) const { *kind = CHAIN_PASS_NONE, *param = 0; }
    // the bytes past the network header the kernel may write (~0u: any)
    virtual uint32_t chain_write_past_nh() const { return writes() ? 0xFFFFFFFFu : 0u; }
    // a chain member after the head: pre_route() will make a clone of this
    // packet as it reaches the member (the chain keeps its bytes first)
    virtual bool pre_clone(const ChainView &v) const { (void)v; return false; }
    void drop_packet(uint32_t key) { packets_kept_.erase(key); }
    // in a staged chain, route() writes the member's rewrite into the packet
    // from its verdict (ChainHostRewrite) instead of the chain copying it back
    virtual uint8_t chain_host_rewrite() const
    {
        return wants_sums() && !wants_arena_back() ? CHAIN_HOST_ALL : CHAIN_HOST_NONE;
    }
    bool chain_ = false;             // a chain runs the element (it copies the rewritten bytes back)
    std::vector<Chain *> chains_;    // the chains the element is a member of (detached when it goes)
    template <class SpanF, class CloneF>
    void chain_prep_loop(ChainWork &w, SpanF &&span_f, CloneF &&clone_f);
    // a pass rule's pass: counted, on to member k+1 (the last member: a
    // result on output 0)
    CLK_INL void chain_pass_on(ChainWork &w, uint32_t i)
    {
        w.counted++;
        if (w.last) {
            const ChainView &v = w.views[i];
            w.out->push_back(ChainExit{v.token, w.member, 0, v.length, 0, i});
            w.views[i].done = 1;
        } else {
            chain_forward(w, i);
        }
    }
    // packet i, passed on by member k, reaches member k+1 -- and goes on at
    // once through each member after it whose pass rule lets it through
    // while no packet before it waits there (that member's list is empty),
    // counted by each (the member would route it to output 0 unchanged); it
    // joins the list of the first member that must look at it, or leaves
    // the last on output 0
    CLK_INL static void chain_forward(ChainWork &w, uint32_t i)
    {
        ChainWork *n = w.next;
        const ChainView &v = w.views[i];
        while (n->pass && n->routed == n->nreached && n->passes(v)) {
            n->elem->packets_++;
            if (n->last) {
                n->out->push_back(ChainExit{v.token, n->member, 0, v.length, 0, i});
                n->views[i].done = 1;
                return;
            }
            n = n->next;
        }
        n->reached[n->nreached++] = i;
    }
    template <class RouteF, class PreF>
    CLK_INL bool chain_route_at(ChainWork &w, size_t q, RouteF &&route_f, PreF &&pre_f);
    template <class RouteF, class PreF>
    void chain_route_loop(ChainWork &w, RouteF &&route_f, PreF &&pre_f);
    template <class RouteF, class PreF>
    CLK_INL bool chain_route_pending(ChainWork &w, uint32_t i, Pending &p, int code, uint16_t sum, RouteF &&route_f,
                                     PreF &&pre_f);
    ResultQueue chain_side_;          // a member's pre/post results while a chain routes
    friend class Chain;
    // after the batch completed, before any packet is routed: nonzero fails
    // the flush (a kernel's internal fault report in the codes)
    virtual int verify(const uint8_t *, size_t) { return 0; }
    // Double buffering: push() stages into st_[cur_]; flush_async() launches
    // it and flips cur_, so the host stages batch k+1 while batch k is on
    // the GPU.  At most one stage is in flight; its results are routed
    // before the next launch (element state such as IPFragmenter's
    // fragment buffers serves one batch at a time).
    struct Stage {
        std::vector<Pending> pend;
        // long spans are gathered at launch, not at push: one loop over the
        // batch that fetches the next packets' lines while it copies
        struct Gather {
            const uint8_t *src;
            uint64_t slot;
            uint32_t n, avail;
        };
        std::vector<Gather> gather;
        uint8_t *h_arena = nullptr;
        size_t h_arena_cap = 0, h_used = 0;
        uint8_t *h_back = nullptr;          // the rewritten arena (wants_arena_back): h_arena stays as
        size_t h_back_cap = 0;              // staged, so a failed batch is retried from its original bytes
        uint64_t *h_off = nullptr;
        uint32_t *h_len = nullptr;
        uint8_t *h_codes = nullptr, *h_anno = nullptr, *h_aux8 = nullptr;
        uint16_t *h_sums = nullptr;
        size_t h_n_cap = 0;
        uint8_t *d_arena = nullptr;
        size_t d_arena_cap = 0;
        uint64_t *d_off = nullptr;
        uint32_t *d_len = nullptr;
        uint8_t *d_codes = nullptr, *d_anno = nullptr, *d_aux8 = nullptr;
        uint16_t *d_sums = nullptr;
        size_t d_n_cap = 0;
        const uint8_t *zc_host = nullptr;   // the batch's registered region (zero-copy)
        uint8_t *zc_dev = nullptr;
        void *ev[3] = {nullptr, nullptr, nullptr};   // kernel start, kernel end, batch done
        size_t n = 0;                       // packets on the GPU
        size_t ngpu = 0;                    // staged packets for the GPU (h_off / h_len / h_anno filled at push)
        uint32_t maxlen = 0;
        bool inflight = false, zc = false;
    };
    // The per-packet loops, with the class's span() / route() given as
    // callables: the generic push() and route pass virtual calls; the final
    // classes pass qualified (inlined) ones through CLK_GLUE_LOOPS.
    template <class SpanF>
    // one packet; `held`: pushed alone by a caller that holds its packets
    // (its long span is gathered at launch), not from a burst (which
    // prefetches the spans ahead itself)
    int push_one(SpanF &&span_f, uint8_t *data, uint32_t length, int32_t nh_offset, uint64_t token, uint32_t anno,
                 bool held, int32_t th_offset = -1);
    // The L4 elements read the transport header where its annotation says,
    // as udp_header() / tcp_header() / icmp_header() do (checkudpheader.cc:87,
    // checktcpheader.cc:88, checkicmpheader.cc:85, setudpchecksum.cc:45,
    // settcpchecksum.cc:49); the kernels find it at ip_hl.  A packet whose
    // annotation is elsewhere (ip_hl rewritten after the header was marked)
    // comes here (reads_th_): the host decides what the reference decides
    // from the header and lengths, and the checksum runs on the GPU over a
    // canonical copy -- the IP header with ip_hl 5 and the pseudo-header's
    // destination (in_cksum.c:86-108) followed by the segment at the
    // annotation (stage_canonical).  NOT_IRREGULAR: handle it as any packet.
    static constexpr int NOT_IRREGULAR = -1000;
    virtual int push_irregular(Pending &p, int32_t th_offset);
    int stage_canonical(Pending &p, const uint8_t *ip20, const uint8_t *seg, uint32_t seglen);
    int host_decided(Pending &p, int32_t code);
    bool reads_th_ = false;
    template <class SpanF>
    int burst_loop(SpanF &&span_f, uint8_t *const *datas, const uint32_t *lengths, const int32_t *nh_offsets,
                   uint64_t first_token, uint32_t n);
    template <class RouteF, class PreF>
    void route_loop(Stage &g, RouteF &&route_f, PreF &&pre_f);
    // route every packet of a completed stage, in push order (results_)
    virtual void route_stage(Stage &g);

    void write_back(const Pending &p, uint32_t nbytes) const;   // staged span -> packet
    uint32_t keep_packet(const uint8_t *bytes, uint32_t len);   // new packet, returns its key
    void chatter(const std::string &s) { msgs_.push_back(s); }
    static uint32_t be16(const uint8_t *p) { return (uint32_t(p[0]) << 8) | p[1]; }

    clk_ctx *ctx_;
    std::string name_;
    int noutputs_;
    uint32_t batch_cap_ = 65536;
    // staged (gather) batches copy at most this many bytes of a packet's span
    // while its full length is what the kernel is told: for kernels that read
    // only the header but check lengths against the packet (CheckIPHeader:
    // OFFSET + 60, DecIPTTL: 20)
    uint32_t stage_cap_ = 0xFFFFFFFFu;
    // ... and at most stage_hl_off_ + the IP header's length (ip_hl * 4, at
    // least 20) for elements that read no byte past the header there
    // (CheckIPHeader, IPInputCombo; disabled: ~0u)
    uint32_t stage_hl_off_ = 0xFFFFFFFFu;
    std::string err_;
    uint64_t batches_ = 0, packets_ = 0, gpu_ns_ = 0, lost_ = 0;
    // counts the events that gate once-only chatter (the first drop's
    // reason, SetUDPChecksum's fragment warning, IPFragmenter's first five
    // DF lines); shared by the elements that stand for one reference
    // element (clk_element_share_messages)
    std::shared_ptr<std::atomic<uint64_t>> gate_ = std::make_shared<std::atomic<uint64_t>>(0);
    uint64_t gate_bump() { return gate_->fetch_add(1, std::memory_order_relaxed); }
    bool zerocopy_ = false;          // ZEROCOPY: packets read/written in registered host memory
    bool hold_ = false;              // the caller holds its packets until popped (clk_element_hold_packets)
    bool in_place_ = false;          // routing a zero-copy batch: the kernel already wrote the packets
    // the launching stage's buffers (valid in run()) and the routing
    // stage's host results (valid in route())
    uint8_t *d_anno_ = nullptr;      // per staged packet (wants_anno)
    uint8_t *d_aux8_ = nullptr;      // per staged packet, element use (problem offsets)
    uint8_t *h_aux8_ = nullptr;

  private:
    int grow_host(Stage &g, size_t bytes, size_t n);
    int grow_dev(Stage &g, size_t bytes, size_t n);
    int launch(Stage &g);
    int launch_failed(Stage &g, hipError_t e, const char *what);
    int failed_after_run(Stage &g, hipError_t e, const char *what, const std::string &why = std::string(),
                         int rc = CLK_EHIP);
    int complete(Stage &g);
    int abandon_stage(Stage &g);
    void free_stage(Stage &g);
    Stage st_[2];
    int cur_ = 0;
    const Stage *rt_ = &st_[0];          // the stage being routed
    ResultQueue results_;
    std::vector<std::string> msgs_;
    std::map<uint32_t, std::vector<uint8_t>> packets_kept_;
    uint32_t next_key_ = 1;
    const uint8_t *zc_last_ = nullptr;   // last region found (lookup cache)
    size_t zc_last_bytes_ = 0;
    uint8_t *zc_last_dev_ = nullptr;
    uint64_t zc_gen_ = 0;                // clk_host_generation_internal() of the cache
};

// Check elements share drop(): elements/ip/checkipheader.cc:143-159 and the
// CheckUDPHeader/CheckTCPHeader copies of it.
class CheckElement : public BatchElement {
  public:
    using BatchElement::BatchElement;
    std::string read_handler(const std::string &h) const override;

  protected:
    virtual const char *const *reason_texts() const = 0;
    virtual int nreasons() const = 0;
    virtual std::string drop_message(const char *reason) const = 0;
    int drop(int reason);   // returns the port
    int conf_verbose_details(ConfArgs &args, std::string *err);
    bool verbose_ = false;
    bool details_ = false;
    uint32_t drops_ = 0;
    std::vector<uint32_t> reason_drops_;
};

class CheckIPHeader : public CheckElement {
  public:
    CheckIPHeader(clk_ctx *ctx, const std::string &name, int noutputs, bool checksum_default = true);
    ~CheckIPHeader() override;
    const char *class_name() const override { return checksum_default_ ? "CheckIPHeader" : "CheckIPHeader2"; }
    int configure(ConfArgs &args, std::string *err) override;
    std::string read_handler(const std::string &h) const override;   // + "offset" (OFFSET)

    CLK_GLUE_LOOPS(CheckIPHeader)

  protected:
    bool span(const Pending &p, uint32_t *off, uint32_t *len, int32_t *code) const override;
    int run(const clk_batch *b, uint8_t *d_codes, uint16_t *d_sums) override;
    void route(Pending &p, int code, uint16_t sum, Result *r) override;
    int32_t nh_after() const override { return (int32_t)offset_; }
    uint32_t chain_extent(int32_t, uint32_t) const override { return offset_ + 60; }
    const char *const *reason_texts() const override;
    int nreasons() const override { return 6; }
    std::string drop_message(const char *reason) const override;

  protected:
    int conf_addresses(ConfArgs &args, std::string *err);   // INTERFACES, BADSRC, GOODDST
    int upload_addresses(std::string *err);
    bool checksum_default_;
    bool checksum_ = true;
    uint32_t offset_ = 0;
    std::vector<uint32_t> bad_src_, good_dst_;
    uint32_t *d_lists_ = nullptr;
};

// IPInputCombo (elements/ip/ipinputcombo.cc:66-140): Paint(COLOR) +
// Strip(14) + CheckIPHeader in one element.  The GPU work is CheckIPHeader's
// kernel at OFFSET 14; every bad packet is killed and the first one chatters
// "IP checksum failed".  The result length is the length after Strip(14)
// and the ip_len trim; painting and pulling the 14 bytes are Packet
// operations the Click-side adapter performs.
class IPInputCombo : public CheckIPHeader {
  public:
    IPInputCombo(clk_ctx *ctx, const std::string &name, int noutputs);
    const char *class_name() const override { return "IPInputCombo"; }
    int configure(ConfArgs &args, std::string *err) override;
    std::string read_handler(const std::string &h) const override;

    CLK_GLUE_LOOPS(IPInputCombo)

  protected:
    void route(Pending &p, int code, uint16_t sum, Result *r) override;
    uint32_t strip() const override { return 14; }
    int32_t nh_after() const override { return 0; }

  private:
    long color_ = 0;
};

class SetIPChecksum : public BatchElement {
  public:
    using BatchElement::BatchElement;
    const char *class_name() const override { return "SetIPChecksum"; }
    std::string read_handler(const std::string &h) const override;

    CLK_GLUE_LOOPS(SetIPChecksum)

  protected:
    bool span(const Pending &p, uint32_t *off, uint32_t *len, int32_t *code) const override;
    int run(const clk_batch *b, uint8_t *d_codes, uint16_t *d_sums) override;
    void route(Pending &p, int code, uint16_t sum, Result *r) override;
    uint32_t chain_extent(int32_t nh, uint32_t) const override { return (nh > 0 ? (uint32_t)nh : 0u) + 60; }
    uint32_t chain_write_past_nh() const override { return 60; }
    bool wants_sums() const override { return true; }

  private:
    uint32_t drops_ = 0;
};

// CheckUDPHeader / CheckTCPHeader / CheckICMPHeader (proto 17 / 6 / 1).
class CheckL4Header : public CheckElement {
  public:
    CheckL4Header(clk_ctx *ctx, const std::string &name, int noutputs, int proto);
    const char *class_name() const override
    {
        return proto_ == 17 ? "CheckUDPHeader" : proto_ == 6 ? "CheckTCPHeader" : "CheckICMPHeader";
    }
    int configure(ConfArgs &args, std::string *err) override;

    CLK_GLUE_LOOPS(CheckL4Header)

  protected:
    bool span(const Pending &p, uint32_t *off, uint32_t *len, int32_t *code) const override;
    int run(const clk_batch *b, uint8_t *d_codes, uint16_t *d_sums) override;
    void route(Pending &p, int code, uint16_t sum, Result *r) override;
    const char *const *reason_texts() const override;
    int nreasons() const override { return 3; }
    std::string drop_message(const char *reason) const override;
    int push_irregular(Pending &p, int32_t th_offset) override;

  private:
    int proto_;
};

class SetL4Checksum : public BatchElement {
  public:
    SetL4Checksum(clk_ctx *ctx, const std::string &name, int noutputs, int proto);
    const char *class_name() const override { return proto_ == 17 ? "SetUDPChecksum" : "SetTCPChecksum"; }
    int configure(ConfArgs &args, std::string *err) override;

    CLK_GLUE_LOOPS(SetL4Checksum)

  protected:
    bool span(const Pending &p, uint32_t *off, uint32_t *len, int32_t *code) const override;
    int run(const clk_batch *b, uint8_t *d_codes, uint16_t *d_sums) override;
    void route(Pending &p, int code, uint16_t sum, Result *r) override;
    bool wants_sums() const override { return true; }
    int push_irregular(Pending &p, int32_t th_offset) override;

  private:
    int proto_;
    bool fixoff_ = false;
};

// DecIPTTL (elements/ip/decipttl.cc): ACTIVE, MULTICAST; handlers drops,
// active.  Expired packets (ip_ttl <= 1) go to output 1 or are killed.
class DecIPTTL : public BatchElement {
  public:
    using BatchElement::BatchElement;
    const char *class_name() const override { return "DecIPTTL"; }
    int configure(ConfArgs &args, std::string *err) override;
    std::string read_handler(const std::string &h) const override;

    CLK_GLUE_LOOPS(DecIPTTL)

  protected:
    bool idempotent() const override { return false; }
    bool span(const Pending &p, uint32_t *off, uint32_t *len, int32_t *code) const override;
    int run(const clk_batch *b, uint8_t *d_codes, uint16_t *d_sums) override;
    void route(Pending &p, int code, uint16_t sum, Result *r) override;
    uint32_t chain_extent(int32_t nh, uint32_t) const override { return (nh > 0 ? (uint32_t)nh : 0u) + 20; }
    uint32_t chain_write_past_nh() const override { return 20; }
    void chain_pass(uint8_t *k, uint32_t *a) const override { *k = CHAIN_PASS_TTL, *a = active_ ? 1u : 0u; }
    bool wants_sums() const override { return true; }

  private:
    bool active_ = true, multicast_ = true;
    uint32_t drops_ = 0;
};

// IPGWOptions (elements/ip/ipgwoptions.cc): MYADDR, [OTHERADDRS]; parameter
// problems to output 1 (or killed) with the offset as aux; handler drops.
class IPGWOptions : public BatchElement {
  public:
    using BatchElement::BatchElement;
    ~IPGWOptions() override;
    const char *class_name() const override { return "IPGWOptions"; }
    int configure(ConfArgs &args, std::string *err) override;
    std::string read_handler(const std::string &h) const override;

    CLK_GLUE_LOOPS(IPGWOptions)

  protected:
    bool idempotent() const override { return false; }
    bool span(const Pending &p, uint32_t *off, uint32_t *len, int32_t *code) const override;
    int run(const clk_batch *b, uint8_t *d_codes, uint16_t *d_sums) override;
    void route(Pending &p, int code, uint16_t sum, Result *r) override;
    uint32_t chain_extent(int32_t nh, uint32_t) const override { return (nh > 0 ? (uint32_t)nh : 0u) + 64; }
    uint32_t chain_write_past_nh() const override { return 64; }
    void chain_pass(uint8_t *k, uint32_t *a) const override { *k = CHAIN_PASS_NO_OPTIONS, *a = 0; }
    bool wants_arena_back() const override { return true; }

  private:
    uint32_t my_ip_ = 0;
    std::vector<uint32_t> addrs_;        // OTHERADDRS + MYADDR (ipgwoptions.cc:46)
    uint32_t *d_addrs_ = nullptr;
    uint32_t drops_ = 0;
};

// FixIPSrc (elements/ip/fixipsrc.cc): IPADDR; rewrites ip_src and ip_sum of
// packets pushed with CLK_ANNO_FIX_IP_SRC.
class FixIPSrc : public BatchElement {
  public:
    using BatchElement::BatchElement;
    const char *class_name() const override { return "FixIPSrc"; }
    int configure(ConfArgs &args, std::string *err) override;

    CLK_GLUE_LOOPS(FixIPSrc)

  protected:
    bool span(const Pending &p, uint32_t *off, uint32_t *len, int32_t *code) const override;
    int run(const clk_batch *b, uint8_t *d_codes, uint16_t *d_sums) override;
    void route(Pending &p, int code, uint16_t sum, Result *r) override;
    uint32_t chain_extent(int32_t nh, uint32_t) const override { return (nh > 0 ? (uint32_t)nh : 0u) + 64; }
    uint32_t chain_write_past_nh() const override { return 64; }
    void chain_pass(uint8_t *k, uint32_t *a) const override { *k = CHAIN_PASS_NO_FIX, *a = 0; }
    bool wants_arena_back() const override { return true; }

  private:
    uint32_t my_ip_ = 0;
};

// IPOutputCombo (elements/ip/ipoutputcombo.cc): COLOR, IPADDR, MTU; five
// outputs.
class IPOutputCombo : public BatchElement {
  public:
    IPOutputCombo(clk_ctx *ctx, const std::string &name, int noutputs) : BatchElement(ctx, name, noutputs)
    {
        has_pre_route_ = true;
    }
    const char *class_name() const override { return "IPOutputCombo"; }
    int configure(ConfArgs &args, std::string *err) override;
    std::string read_handler(const std::string &h) const override;

    CLK_GLUE_LOOPS(IPOutputCombo)

  protected:
    bool idempotent() const override { return false; }
    bool span(const Pending &p, uint32_t *off, uint32_t *len, int32_t *code) const override;
    int run(const clk_batch *b, uint8_t *d_codes, uint16_t *d_sums) override;
    bool pre_route(Pending &p, Result *r) override;
    bool pre_clone(const ChainView &v) const override
    {
        return !(v.anno & CLK_ANNO_BCAST) && (long)((v.anno >> 8) & 0xFF) == color_ && noutputs_ >= 2;
    }
    void route(Pending &p, int code, uint16_t sum, Result *r) override;
    uint32_t chain_extent(int32_t nh, uint32_t) const override { return (nh > 0 ? (uint32_t)nh : 0u) + 64; }
    uint32_t chain_write_past_nh() const override { return 64; }
    bool wants_arena_back() const override { return true; }
    bool wants_anno() const override { return true; }
    bool wants_sums() const override { return !zerocopy_; }   // the checksum route() writes (staged)
    uint8_t chain_host_rewrite() const override { return CHAIN_HOST_SIMPLE; }
  public:
    // a packet whose combo rewrite is the TTL and the checksum alone: no
    // FIX_IP_SRC annotation, no options walked (ip_out_kernel's condition)
    static bool simple_rewrite(const uint8_t *iph, uint32_t span_len, uint32_t anno)
    {
        const uint32_t hl = (uint32_t)(iph[0] & 0xF) << 2;
        return !(anno & CLK_ANNO_FIX_IP_SRC) && !(hl > 20 && hl <= span_len);
    }
  protected:

  private:
    long color_ = 0;
    uint32_t my_ip_ = 0, mtu_ = 0;
};

// IPFragmenter (elements/ip/ipfragmenter.cc): MTU, [HONOR_DF], [VERBOSE],
// HEADROOM; handlers drops, fragments.
class IPFragmenter : public BatchElement {
  public:
    IPFragmenter(clk_ctx *ctx, const std::string &name, int noutputs) : BatchElement(ctx, name, noutputs)
    {
        has_post_route_ = true;
    }
    ~IPFragmenter() override;
    const char *class_name() const override { return "IPFragmenter"; }
    int configure(ConfArgs &args, std::string *err) override;
    std::string read_handler(const std::string &h) const override;

    CLK_GLUE_LOOPS(IPFragmenter)

  protected:
    bool idempotent() const override { return false; }
    bool span(const Pending &p, uint32_t *off, uint32_t *len, int32_t *code) const override;
    int run(const clk_batch *b, uint8_t *d_codes, uint16_t *d_sums) override;
    void route(Pending &p, int code, uint16_t sum, Result *r) override;
    uint32_t chain_extent(int32_t nh, uint32_t length) const override   // within the MTU: untouched (165-171)
    {
        const uint32_t h = nh > 0 ? (uint32_t)nh : 0u;
        return h <= length && length - h <= mtu_ ? 0u : 0xFFFFFFFFu;
    }
    void chain_pass(uint8_t *k, uint32_t *a) const override { *k = CHAIN_PASS_WITHIN, *a = mtu_; }
    int verify(const uint8_t *codes, size_t n) override;
    void post_route(Pending &p, int code, ResultQueue &out) override;
    bool wants_arena_back() const override { return true; }

  private:
    uint32_t mtu_ = 0;
    long headroom_ = 28;   // Packet::default_headroom (packet.hh:45; 48 on MiniOS)
    bool honor_df_ = true, verbose_ = false;
    uint32_t drops_ = 0;
    uint64_t fragments_ = 0;
    // device / host fragment buffers of the last flush
    uint8_t *d_frag_ = nullptr;
    uint64_t d_frag_cap_ = 0;
    uint64_t *d_foff_ = nullptr;
    uint32_t *d_flen_ = nullptr, *d_fsrc_ = nullptr, *d_first_ = nullptr;
    uint64_t *d_ffirst_ = nullptr, *d_totals_ = nullptr;
    uint16_t *d_newid_ = nullptr;
    uint64_t d_nfrag_cap_ = 0, d_npkt_cap_ = 0;
    std::vector<uint8_t> h_frag_;
    std::vector<uint64_t> h_foff_, h_ffirst_;
    std::vector<uint32_t> h_flen_, h_first_;
    std::vector<uint16_t> h_newid_;
    uint64_t nfrag_ = 0;
};

// The packets that reached the member and were not looked at yet: a pass
// rule's pass, or the class's span() -- a descriptor of the member's batch
// (the bytes to copy back grown for a writing member) or a host decision.
template <class SpanF, class CloneF>
inline void BatchElement::chain_prep_loop(ChainWork &w0, SpanF &&span_f, CloneF &&clone_f)
{
    // a private copy of the member's work: its fields stay in registers
    // across the loop's byte stores (which may alias anything in memory)
    ChainWork w = w0;
    w.counted = 0;
    for (size_t q = w.nprep; q < w.nreached; q++) {
        const uint32_t i = w.reached[q];
        if (CLK_CHAIN_PF && q + CLK_CHAIN_PF < w.nreached) {   // the header a pass rule / span reads
            const ChainView &a = w.views[w.reached[q + CLK_CHAIN_PF]];
            __builtin_prefetch(chain_hdr(a.data, a.nh));
            __builtin_prefetch(chain_hdr(a.data, a.nh) + 16);
        }
        const ChainView &v = w.views[i];
        if (w.pass && w.passes(v)) {
            w.code[q] = CHAIN_CODE_PASS;
            if (w.routed == q) {                 // nothing before it waits: it goes on now
                w.routed = q + 1;
                chain_pass_on(w, i);
            }
            continue;
        }
        if (w.clone_key && !w.clones && clone_f(v))   // a clone to keep before the kernel runs
            w.clones = true;
        Pending p{v.data, v.token, v.slot, v.length, v.nh, 0, 0, 0, -1, v.anno};
        uint32_t off = 0, len = 0;
        int32_t hc = 0;
        if (!span_f(p, &off, &len, &hc)) {
            w.code[q] = -1 - hc;
            w.span_off[q] = 0;
            w.span_len[q] = 0;
            continue;
        }
        w.h_off[w.n] = v.slot + off;
        w.h_len[w.n] = len;
        w.h_anno[w.n] = (uint8_t)v.anno;
        w.maxlen = std::max(w.maxlen, len);
        w.span_off[q] = off;
        w.span_len[q] = len;
        w.code[q] = (int32_t)w.n++;
        if (w.wext && w.back &&                  // the bytes this member's kernel may rewrite, to copy back
            !(w.wext_unless_simple && IPOutputCombo::simple_rewrite(v.data + off, len, v.anno))) {
            const uint64_t shift = v.slot - w.slot0[i];
            const uint64_t e = w.wext == 0xFFFFFFFFu ? (uint64_t)0xFFFFFFFFu
                                                     : shift + (v.nh > 0 ? (uint32_t)v.nh : 0u) + w.wext;
            w.back[i] = (uint32_t)std::max<uint64_t>(w.back[i], std::min<uint64_t>(e, w.staged[i]));
        }
    }
    w0.nprep = w.nreached;
    w0.routed = w.routed;
    w0.n = w.n;
    w0.maxlen = w.maxlen;
    w0.clones = w.clones;
    packets_ += w.counted;
}

template <class RouteF, class PreF>
inline bool BatchElement::chain_route_pending(ChainWork &w, uint32_t i, Pending &p, int code, uint16_t sum,
                                              RouteF &&route_f, PreF &&pre_f)
{
    ChainView &v = w.views[i];
    Result pr;
    if (has_pre_route_ && pre_f(p, &pr)) {
        uint32_t aux = pr.aux;
        if (w.clone_key && w.clone_key[i]) {  // the clone's bytes, kept as it reached this member
            aux = CLK_AUX_CLONE | w.clone_key[i];
            w.clone_key[i] = 0;
        }
        w.out->push_back(ChainExit{pr.token, w.member, pr.port, pr.length, aux, ~0u});
    }
    Result r{p.token, 0, p.length, 0};
    w.counted++;
    route_f(p, code, sum, &r);
    const bool pass = r.port == 0 && !w.last;
    if (pass) {
        v.data += w.strip;
        v.slot += w.strip;
        v.length = r.length;
        if (w.nh_after != -2)
            v.nh = w.nh_after;
        v.anno = p.anno;                      // the annotations the member set / cleared
        if (w.report_passes)
            w.out->push_back(ChainExit{r.token, w.member, CLK_PORT_NEXT, r.length, r.aux, i});
    } else {
        w.out->push_back(ChainExit{r.token, w.member, r.port, r.length, r.aux, i});
        v.done = 1;
    }
    if (has_post_route_) {                    // results that follow the packet's own (fragments)
        post_route(p, code, chain_side_);
        uint64_t tok[64];
        int32_t port[64];
        uint32_t len[64], aux[64];
        uint64_t got;
        while ((got = chain_side_.pop(tok, port, len, aux, 64)) > 0)
            for (uint64_t k = 0; k < got; k++)
                w.out->push_back(ChainExit{tok[k], w.member, port[k], len[k], aux[k], ~0u});
    }
    return pass;
}

template <class RouteF, class PreF>
inline bool BatchElement::chain_route_at(ChainWork &w, size_t q, RouteF &&route_f, PreF &&pre_f)
{
    const uint32_t i = w.reached[q];
    const int32_t c = w.code[q];
    const int code = c >= 0 ? w.h_codes[c] : -1 - c;
    const ChainView &v = w.views[i];
    Pending p{v.data, v.token, v.slot, v.length, v.nh, w.span_off[q], w.span_len[q], c >= 0 ? (uint32_t)c : 0u,
              (int16_t)(c >= 0 ? -1 : code), v.anno};
    return chain_route_pending(w, i, p, code, c >= 0 && w.h_sums ? w.h_sums[c] : 0, route_f, pre_f);
}

BatchElement *make_element(clk_ctx *ctx, const std::string &cls, const std::string &name, int noutputs);
BatchElement *element_impl(::clk_element *w);
hipError_t glue_checked(hipError_t e);                        // the glue's test fault hook       // the C ABI handle's element

// A chain of elements in one thread, member k+1 connected to member k's
// output 0 (chain.cc): each packet is staged once and enters member 0 at
// push (going on at once through members that decide it on the host); a
// flush copies the batch to HBM once, runs every member's kernel in order --
// member k over the packets members 0..k-1 passed on output 0 -- routing each
// member's verdicts through its own route() (counters, handlers, chatter as
// if it had run alone) before the next member's kernel, and copies the
// rewritten bytes back once (a member whose verdict carries its rewrite
// writes it from route() instead).  The GPU analogue of click-xform's combos
// (ipinputcombo.cc:66-140, ipoutputcombo.cc:44-205).
class alignas(128) Chain {
  public:
    explicit Chain(const std::vector<BatchElement *> &members) : m_(members) {}
    ~Chain();
    void attach();                            // registered with its members
    void member_gone(BatchElement *e);        // a member is being destroyed: the chain is dead
    int check(std::string *err) const;
    int push(uint8_t *data, uint32_t length, int32_t nh_offset, uint64_t token, uint32_t anno);
    int push_burst(uint8_t *const *datas, const uint32_t *lengths, const int32_t *nh_offsets, uint64_t first_token,
                   uint32_t n);
    int flush();                              // everything pushed routed (both batches)
    int flush_async();                        // double-buffered (the batch before finished, this one launched)
    uint64_t abandon();
    uint64_t pop(uint64_t *tokens, int32_t *members, int32_t *ports, uint32_t *lengths, uint32_t *aux, uint64_t cap);
    const std::string &last_error() const { return err_; }
    size_t pending() const { return b_[0].np + b_[1].np; }
    void report_passes(uint64_t members) { report_passes_ = members; }
    // host seconds spent so far, by phase (include/click_amd_elements.h,
    // clk_chain_stats)
    int stats(double *sec, int n) const
    {
        for (int k = 0; k < n && k < 8; k++)
            sec[k] = stats_[k];
        return 8;
    }

  private:
    struct Member {          // one member's batch buffers (per chain batch)
        uint64_t *h_off = nullptr, *d_off = nullptr;
        uint32_t *h_len = nullptr, *d_len = nullptr;
        uint8_t *h_codes = nullptr, *d_codes = nullptr, *h_anno = nullptr, *d_anno = nullptr;
        uint8_t *h_aux8 = nullptr, *d_aux8 = nullptr;
        uint16_t *h_sums = nullptr, *d_sums = nullptr;
        size_t cap = 0;
        void *ev[3] = {nullptr, nullptr, nullptr};   // kernel start, kernel end, step done
        float ms = 0;
        bool rebuild = false;                 // resumed: rebuild the batch of the packets not routed
        std::vector<uint32_t> reached, span_off, span_len;
        std::vector<int32_t> code;
        ChainWork w;
    };
    // One batch of the chain: its packets, staging, device copy, members'
    // work, and its routed results until they are handed out.  Two: one is
    // pushed into while the other is in flight.
    struct Batch {
        std::vector<Member> mm;
        std::vector<ChainView> views;             // as they move through the members
        std::vector<uint64_t> slot0;              // staging offset as pushed (data moves with slot)
        std::vector<uint32_t> staged, back, clone_key;   // bytes staged / to copy back, a kept clone's key
        std::vector<uint8_t> copied;              // bytes copied back
        size_t np = 0, mcap = 0;                  // packets in the batch; the arrays' size
        uint8_t *h_arena = nullptr, *h_back = nullptr, *h_snap = nullptr, *d_arena = nullptr;
        size_t h_cap = 0, back_cap = 0, snap_cap = 0, d_cap = 0, used = 0;
        size_t sent = 0;                          // staged bytes already copied to the device
        bool sent_ok = true, h2d_done = false;
        const uint8_t *zc_host = nullptr;         // ZEROCOPY: the batch's registered region
        uint8_t *zc_dev = nullptr;
        uint64_t seq = 0;                         // batches in push order
        bool zc_zeroed = false;                   // staged / back / copied all 0 (ZEROCOPY batches)
        bool started = false;                     // flushed: in flight until its last member is routed
        size_t at = 0;                            // the member its routing has reached
        bool waiting = false;                     // member at's GPU step is queued, not awaited
        bool launched = false;                    // ... and its kernels were queued
        int kill_rc = CLK_SUCCESS;                // a rewriting member's packets were killed (kill_member)
        std::string kill_why;
        std::vector<ChainExit> out;               // routed results not handed out yet (publish)
    };
    hipStream_t stream() const;
    int begin_batch(Batch &B);
    int grow_batch(Batch &B);
    void size_packets(Batch &B, size_t c);
    static bool host_writes(const BatchElement *e);
    int device_arena(Batch &B, size_t bytes);
    void send_chunk(Batch &B);
    static constexpr size_t H2D_CHUNK = size_t(1) << 20;
    int grow_members(Batch &B, size_t c, int keep);
    void setup(Batch &B, size_t k);
    int start(Batch &B);
    int step(Batch &B);
    int finish(Batch &B);
    int fail(Batch &B, int r);
    int launch_member(Batch &B, size_t k);
    int await_member(Batch &B);
    bool kill_member(Batch &B, size_t k, int r);
    int keep_clones(Batch &B, size_t k);
    void drop_clones(Batch &B, size_t k, size_t q0, size_t q1);
    int copy_back(Batch &B, bool all);
    void publish(Batch &B);
    void release();
    void end_batch(Batch &B);
    void free_batch(Batch &B);
    uint32_t extent(int32_t nh, uint32_t length)
    {
        return nh == ext_nh_ && length == ext_len_ ? ext_ : extent_slow(nh, length);
    }
    uint32_t extent_slow(int32_t nh, uint32_t length);
    int push_slow(uint8_t *data, uint32_t length, int32_t nh_offset, uint64_t token, uint32_t anno);
    void record(Batch &B, uint8_t *data, uint32_t length, int32_t nh_offset, uint64_t token, uint32_t anno,
                uint64_t slot, uint32_t need);
    size_t cap0_ = 0;                         // member 0's BATCH, ZEROCOPY (begin_batch)
    bool zerocopy_ = false;
    std::vector<BatchElement *> m_;
    Batch b_[2];
    int cur_ = 0;                             // the batch pushes go to
    uint64_t seq_ = 0;
    bool failed_ = false;                     // a flush failed: the chain must be flushed (or abandoned)
    bool dead_ = false;                       // a member was destroyed first: nothing runs any more
    const uint8_t *zc_last_ = nullptr;        // last region found (lookup cache)
    size_t zc_last_bytes_ = 0;
    uint8_t *zc_last_dev_ = nullptr;
    uint64_t zc_gen_ = 0;
    std::deque<std::pair<uint64_t, std::vector<ChainExit>>> held_;   // published, behind an older batch (seq)
    std::deque<std::vector<ChainExit>> ready_;   // results handed out (pop), one vector per publish
    std::vector<std::vector<ChainExit>> spare_;  // drained vectors' storage, for the batches
    size_t head_ = 0;                         // into ready_.front()
    double stats_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int32_t ext_nh_ = -3;                     // extent() cache: the nh and length it was computed for
    uint32_t ext_len_ = 0, ext_ = 0;
    bool init_ = false;
    uint64_t report_passes_ = 0;              // bit k: member k reports its passes
    std::string err_;
};

template <class RouteF, class PreF>
void BatchElement::chain_route_loop(ChainWork &w0, RouteF &&route_f, PreF &&pre_f)
{
    ChainWork w = w0;                         // a private copy, as in chain_prep_loop
    w.counted = 0;
    if (w.out->capacity() < w.out->size() + 2 * (w.nreached - w.routed))   // a result and a clone per packet
        w.out->reserve(std::max(w.out->size() + 2 * (w.nreached - w.routed), 2 * w.out->capacity()));
    for (size_t q = w.routed; q < w.nreached; q++) {
        w.routed = q + 1;
        if (CLK_CHAIN_PF && q + CLK_CHAIN_PF < w.nreached) {   // the header route() reads (and a member may write)
            const ChainView &a = w.views[w.reached[q + CLK_CHAIN_PF]];
            __builtin_prefetch(chain_hdr(a.data, a.nh), 1);
            __builtin_prefetch(chain_hdr(a.data, a.nh) + 16, 1);
        }
        const uint32_t i = w.reached[q];
        if (w.code[q] == CHAIN_CODE_PASS)
            chain_pass_on(w, i);
        else if (chain_route_at(w, q, route_f, pre_f) && !w.last)
            chain_forward(w, i);
    }
    w0.routed = w.routed;
    packets_ += w.counted;
}

} // namespace host
} // namespace clk
