// -*- c-basic-offset: 4 -*-
#ifndef CLICK_HIPCORE_HH
#define CLICK_HIPCORE_HH
/*
 * hipcore.hh -- the Click-independent core of the GPU-backed elements'
 * adapter (HIPBatchElement, hipbatch.hh): holding packets while their batch
 * is on the GPU, tokens, routing results, the runcount, the latency flush,
 * failed-flush retries and pull-mode batching.
 *
 * It is a template over the packet type P, the per-thread lock type L and
 * the Host -- the adapter -- so the same code runs inside Click (P = Packet,
 * L = Spinlock, Host = HIPBatchElement) and in tests/native/hipcore_test.cc
 * (P = the test's packet, L = a std::mutex wrapper, Host = a test element
 * that records its outputs), where it is driven on the GPU against the
 * oracle.  Only include/click_amd_elements.h and the C++ library are used.
 *
 * Click's Element API hands over one packet at a time (element.cc:2891-2972);
 * the GPU wants batches.  The reference classes on this path are agnostic
 * (CheckIPHeader, CheckUDPHeader, CheckTCPHeader, CheckICMPHeader, DecIPTTL,
 * SetUDPChecksum, IPGWOptions: PROCESSING_A_AH, checkipheader.hh:114;
 * SetIPChecksum, SetTCPChecksum, FixIPSrc, IPInputCombo: AGNOSTIC, the
 * default of element.cc:1127) or push (IPOutputCombo, IPFragmenter), so:
 *   push context: push() stages the packet and holds it; a full batch is
 *     launched double-buffered (the previous one is routed), a partial one
 *     once its latency deadline passes (poll(), run by the state's Task on
 *     its own thread; timer() flushes at once).  While a thread state holds packets it
 *     holds one runcount reference (Router::adjust_runcount,
 *     router.cc:832-846), so the router cannot stop before they are routed.
 *   pull context: pull() on output 0 hands out one packet per call from a
 *     ready queue; when it is empty, a refill pulls up to BATCH packets from
 *     input 0 (until the input returns null), launches them and routes the
 *     batch the previous refill launched, queueing its output-0 packets
 *     (it waits for the GPU only when nothing is ready); other results
 *     leave on their push outputs as checked_output_push does (output 1 of
 *     a/ah).
 * Results are taken from the glue under the thread state's lock (a state
 * one thread owns needs none: State::shared) but DELIVERED (annotations,
 * output pushes) after it is released, in push order: a downstream element that re-enters this element on the same
 * thread stages its packet and returns (the running delivery loop delivers
 * the new results after the current ones), so there is no deadlock and no
 * reordering.  cleanup() kills whatever is held; it pushes nothing
 * downstream (router teardown may already have cleaned those elements up).
 * A flush that fails leaves its batch staged (include/click_amd_elements.h);
 * after `max_retries` consecutive failures the batch is abandoned
 * (clk_element_abandon: every held packet killed, counted by the glue's
 * "lost" handler) and the runcount released, so the router can stop.
 *
 * Chains: a state whose `chain` is set runs its element and the GPU-backed
 * elements after it on output 0 as one clk_chain (include/
 * click_amd_elements.h): one staged batch, one flush, results tagged with
 * the member they leave (mem[k] is member k's glue element on the state's
 * context).  A packet passed from member k to k+1 comes as a pass record
 * (CLK_PORT_NEXT): member k's finish() applies its side effects (network
 * header, trim, Strip, annotations) and nothing is pushed; a result leaving
 * at member k is finished by member k and pushed on member k's output.  The
 * host's prepare() readies a packet for the whole chain (writable if any
 * member writes, the annotations every member reads).
 *
 * Results are taken from the glue a chunk at a time into per-state arrays
 * (Chunk: the held packets they belong to, ports, lengths, aux words) and
 * delivered in runs of one member: the host's deliver(m, ..) finishes a
 * whole run through member m's class logic -- one call per run, the class's
 * finish() inlined in its loop (deliver_run) -- and pushes each packet on
 * member m's output.  A packet's results stay in push order per member.
 *
 * Host interface (all called on the thread that drives the core; m is the
 * chain member, 0 without a chain):
 *   the class hooks of hipclasses.hh -- prepare(), nh_offset(), primary(m,..),
 *        make_packet(m,..), end_of_batch(m,..) -- which the host forwards to
 *        the element class's shipped logic (the Click adapter and the native
 *        test instantiate the same classes)
 *   bool extra_results(m)       member m's class has results besides its
 *        packets' own (clones, fragments): primary() is asked only then
 *   void deliver(int m, S &t, const Chunk<P> &c, uint32_t i, uint32_t j,
 *        std::vector<P *> *ready)   results [i, j) of c, all member m's:
 *        deliver_run() over member m's class, pushing on member m's outputs
 *        (checked_output_push); with `ready` (pull context, last member) the
 *        output-0 packets go there instead
 *   int32_t th_offset(P *p)      the transport header annotation's offset
 *        from data() (-2: none, -1: unknown), for clk_element_push_th
 *   uint8_t *data(P *p); uint32_t length(P *p)
 *   P *input_pull()                              input(0).pull(0)
 *   void kill(P *p)
 *   void adjust_runcount(int delta)
 *   uint64_t now_ns()                            a steady clock
 *   void wake(S &t)                              make sure poll(t) runs on t's
 *        thread soon (Click: the state's Task, moved to that RouterThread)
 *   void chatter(const char *text)               the adapter's own messages
 *   void message(int m, const char *line)        member m's chatter lines from the glue
 *
 * Latency flush on the state's own thread: a state that holds packets has a
 * deadline (LATENCY after its last flush); poll(t), run by the thread's
 * Task, launches what was staged since (double-buffered) and delivers the
 * batch before once it has passed, and at the next deadline with nothing
 * new staged waits for the rest.  So every packet of thread
 * k is staged, flushed and pushed downstream on thread k (the reference's
 * per-thread model; a Timer would run on the element's home thread,
 * timer.cc:245-246).
 *
 * Pull context, double-buffered: when the ready queue is empty, pull() takes
 * up to BATCH packets from input 0 (until it returns null), launches them
 * (clk_element_flush_async) and so routes the batch launched by the previous
 * refill: those packets are handed out while the new batch is on the GPU.
 * Only when nothing is ready after that (the first refill, or a batch that
 * kept no packet) does pull() wait for the batch in flight.
  */
#include <stddef.h>
#include <stdint.h>
#include <string.h>
#include <deque>
#include <string>
#include <vector>
#include "click_amd_elements.h"

namespace hipcore {

template <class P> struct Held {
    P *p;           // the packet staged (writable if the element writes it)
    P *extra;       // a second packet held with it (IPOutputCombo's PaintTee clone)
    uint32_t anno;  // the CLK_ANNO_* bits it was staged with
};

// The packets a state holds, by token: a ring over a power-of-two vector
// (held[k] is token base + k), grown by doubling.
template <class T> class HeldRing {
  public:
    size_t size() const { return n_; }
    bool empty() const { return n_ == 0; }
    T &operator[](size_t k) { return v_[(h_ + k) & mask_]; }
    T &front() { return v_[h_]; }
    void push_back(const T &x)
    {
        if (n_ == cap_)
            grow();
        v_[(h_ + n_) & mask_] = x;
        n_++;
    }
    void pop_back() { n_--; }
    void pop_front()
    {
        h_ = (h_ + 1) & mask_;
        n_--;
    }
    void clear() { h_ = n_ = 0; }

  private:
    void grow()
    {
        std::vector<T> w(v_.empty() ? 1024 : v_.size() * 2);
        for (size_t k = 0; k < n_; k++)
            w[k] = (*this)[k];
        v_.swap(w);
        h_ = 0;
        cap_ = v_.size();
        mask_ = cap_ - 1;
    }
    std::vector<T> v_;
    size_t h_ = 0, n_ = 0;
    size_t cap_ = 0, mask_ = 0;     // v_.size() and v_.size() - 1, kept (no division per access)
};

// One result as a class's finish() sees it (built in registers from a Chunk
// entry by deliver_run, or for the rare result a stage leaves behind).
template <class P> struct Routed {
    P *p;           // the held packet (its primary result), 0 otherwise
    P *extra;       // the held second packet (IPOutputCombo's clone result)
    P *made;        // a new packet from the glue (IPFragmenter's fragment)
    P *parent;      // for a fragment: the packet it was cut from (annotations)
    uint32_t anno;
    int32_t port;
    uint32_t len, aux;
    int member;     // chains: the member whose result it is (0: the state's own element)
    bool pass;      // chains: p went on to the next member (its finish() applies, no push)
};

// A chunk of results taken from the glue, struct of arrays, in the glue's
// order.  `end`: the glue had no more (the end of a batch follows them).
template <class P> struct Chunk {
    enum { CAP = 256 };
    uint32_t n = 0;
    bool end = false;
    P *p[CAP];
    P *extra[CAP];
    P *made[CAP];
    P *parent[CAP];
    uint32_t anno[CAP], len[CAP], aux[CAP];
    int32_t port[CAP], mem[CAP];
    uint8_t pass[CAP];
    void put(uint32_t k, const Routed<P> &r)
    {
        p[k] = r.p, extra[k] = r.extra, made[k] = r.made, parent[k] = r.parent;
        anno[k] = r.anno, port[k] = r.port, len[k] = r.len, aux[k] = r.aux, mem[k] = r.member;
        pass[k] = r.pass;
    }
    Routed<P> at(uint32_t k) const
    {
        Routed<P> r = {p[k], extra[k], made[k], parent[k], anno[k], port[k], len[k], aux[k], mem[k], pass[k] != 0};
        return r;
    }
};

// Deliver results [i, j) of chunk c -- all of one member -- through class
// `cls` (its finish() inlined here), pushing each result's packet with
// push(port, p); with `ready` (pull context) output-0 packets go there.
template <class P, class C, class S, class O, class Push>
inline void deliver_run(C &cls, S &t, const Chunk<P> &c, uint32_t i, uint32_t j, std::vector<P *> *ready, Push &&push)
{
    for (uint32_t k = i; k < j; k++) {
        if (k + 4 < j && c.p[k + 4])              // its bytes, 4 results ahead (route()
            __builtin_prefetch(O::data(c.p[k + 4]));  // prefetched the packet itself)
        Routed<P> r = c.at(k);
        P *out = 0;
        const int port = cls.finish(t, r, &out);
        if (r.pass || port < 0 || !out)           // a pass: the member's side effects only
            continue;
        if (ready && port == 0)
            ready->push_back(out);
        else
            push(port, out);
    }
}

template <class P, class L> struct State {
    clk_ctx *ctx;
    clk_element *e;
    clk_chain *chain;             // set: e heads a chain -- mem[k] is member k's glue element
    std::vector<clk_element *> mem;   // on ctx (mem[0] == e; the others are the state's own)
    int id;                       // the thread (Click: the RouterThread id)
    HeldRing<Held<P> > held;      // held[k] has token base + k
    uint64_t base, next;
    bool counted;                 // holds a runcount reference
    unsigned fails;               // consecutive failed flushes
    bool draining;                // a delivery loop is running on this state
    bool unrouted;                // the glue may hold results route() has not taken
    bool routed_any;              // results taken since the last end-of-batch mark
    uint32_t fresh;               // packets staged since the last flush
    bool armed;                   // the latency deadline is set
    uint64_t deadline;            // now_ns() at which poll() flushes
    uint64_t push_errors;         // packets push() could not stage (chatter is rate-limited)
    Chunk<P> *chunk;              // the results being delivered (route() fills it)
    Chunk<P> *side_chunk;         // the same for `side`
    std::vector<Routed<P> > side; // results a stage leaves behind (IPOutputCombo's clone when the copy fails)
    uint64_t xmask;               // bit m: member m's class has extra results (host extra_results)
    std::deque<P *> ready;        // pull context: output-0 packets ready to hand out
    P *last_primary;              // route(): the packet of the last primary result
    P *frag_parent;               // host use (IPFragmenter's first-fragment parent)
    L lock;
    // several threads may drive the state (a host's catch-all state): its
    // lock is taken.  A state one thread owns -- the Click adapter's state
    // k is RouterThread k's, its Task moved there; teardown runs after the
    // threads stopped -- is driven without it: the lock's atomic exchange
    // was the largest single cost of a push (a full barrier per packet,
    // profiles/r05/core_gprof_r05r.txt)
    bool shared;
    void enter() { if (shared) lock.acquire(); }
    void leave() { if (shared) lock.release(); }
    State() : ctx(0), e(0), chain(0), id(0), base(0), next(0), counted(false), fails(0), draining(false),
              unrouted(false), routed_any(false), fresh(0), armed(false),
              deadline(0), push_errors(0), chunk(0), side_chunk(0), xmask(~uint64_t(0)), last_primary(0), frag_parent(0),
              shared(true) { }
    ~State() { delete chunk; delete side_chunk; }
    State(const State &) = delete;
    State &operator=(const State &) = delete;
};

template <class P, class Host, class L> class Core {
  public:
    typedef State<P, L> S;
    typedef Routed<P> R;

    // push context launches a batch once INFLIGHT packets are staged, whatever
    // BATCH: with two batches in flight and the one being staged, a state
    // then holds at most 3 x INFLIGHT packets, whose Packet structures, data
    // and the glue's per-packet records stay in the host caches between
    // staging and delivery.  In Click (profiles/r06/click_batch_tcache_r06l.json,
    // Mpps at 512 / 1024 / 2048 / 4096 / 8192): C3 SetUDPChecksum 5.4 / 6.3 /
    // 6.4 / 4.6 / 3.6 (its uniqueified copies), CheckUDPHeader 5.9 / 7.6 /
    // 8.4 / 8.8 / 7.3, config 1 3.8 / 4.7 / 5.1 / 5.6 / 5.0
    enum { INFLIGHT = 2048 };

    Core() : _batch(65536), _latency_ms(1), _max_retries(3) { }

    void set_batch(uint32_t b)       { _batch = b ? b : 1; }
    void set_latency(unsigned ms)    { _latency_ms = ms; }
    void set_max_retries(unsigned k) { _max_retries = k ? k : 1; }
    uint32_t batch() const           { return _batch; }

    // ---- push context --------------------------------------------------------
    void push(Host &h, S &t, P *p)
    {
        t.enter();
        stage(h, t, p, true);
        // most pushes only stage: deliver when there is something to
        const bool deliver = (!t.side.empty() || t.unrouted) && !t.draining;
        t.leave();
        if (deliver)
            drain(h, t, false);
    }

    // run state t's partial batch now and route everything (the deadline
    // passed, or the router asks)
    void timer(Host &h, S &t)
    {
        t.enter();
        flush(h, t, true);
        t.leave();
        drain(h, t, false);
    }

    // the state's Task: flush once its deadline has passed.  Returns true
    // while the state still holds a deadline (the Task runs again).
    bool poll(Host &h, S &t)
    {
        t.enter();
        if (!t.armed) {
            t.leave();
            return false;
        }
        if (h.now_ns() < t.deadline) {
            t.leave();
            return true;
        }
        // packets staged since the last flush: launch them and route the
        // batch before (double-buffered, as a full batch); only what is
        // already in flight: wait for it.  At rates under INFLIGHT packets
        // per LATENCY the deadline, not a full batch, launches every batch,
        // and a waiting flush each time stalled the thread on the GPU
        // (Click, C3 CheckUDPHeader: a quarter of the samples in HIP's
        // event wait, profiles/r06/click_samples_c3chk_r06h.txt)
        flush(h, t, t.fresh == 0);
        t.leave();
        drain(h, t, false);
        t.enter();
        const bool again = t.armed;
        t.leave();
        return again;
    }

    bool armed(S &t)
    {
        t.enter();
        const bool a = t.armed;
        t.leave();
        return a;
    }

    // ---- pull context (output 0) --------------------------------------------
    P *pull(Host &h, S &t)
    {
        t.enter();
        if (t.ready.empty()) {
            t.leave();
            refill_and_launch(h, t);     // launches a batch, routes the one in flight
            t.enter();
            // nothing ready (the first refill, or a batch that kept no packet
            // for output 0): wait for what is in flight -- retried at once,
            // abandoned after max_retries -- and launch the next batch before
            // handing these out
            while (t.ready.empty() && !t.held.empty() && t.e) {
                flush(h, t, true);
                const bool failed = t.fails != 0;
                t.leave();
                drain(h, t, true);
                if (!failed)
                    refill_and_launch(h, t);
                t.enter();
            }
        }
        P *p = 0;
        if (!t.ready.empty()) {
            p = t.ready.front();
            t.ready.pop_front();
        }
        t.leave();
        return p;
    }

    // ---- teardown: kill everything held; no downstream pushes ----------------
    void cleanup(Host &h, S &t)
    {
        t.enter();
        for (size_t i = 0; i < t.held.size(); i++) {
            if (t.held[i].p)
                h.kill(t.held[i].p);
            if (t.held[i].extra)
                h.kill(t.held[i].extra);
        }
        t.held.clear();
        for (size_t i = 0; i < t.side.size(); i++)
            if (t.side[i].extra)
                h.kill(t.side[i].extra);
        t.side.clear();
        while (!t.ready.empty()) {
            h.kill(t.ready.front());
            t.ready.pop_front();
        }
        if (t.frag_parent) {
            h.kill(t.frag_parent);
            t.frag_parent = 0;
        }
        t.armed = false;
        if (t.counted) {
            t.counted = false;
            h.adjust_runcount(-1);
        }
        if (t.chain) {
            clk_chain_destroy(t.chain);
            t.chain = 0;
        }
        for (size_t m = 1; m < t.mem.size(); m++)
            clk_element_destroy(t.mem[m]);
        t.mem.clear();
        if (t.e) {
            clk_element_destroy(t.e);
            t.e = 0;
        }
        if (t.ctx) {
            clk_ctx_destroy(t.ctx);
            t.ctx = 0;
        }
        t.leave();
    }

  private:
    // Pull context (unlocked): up to one batch from input 0, until it runs
    // dry, staged and launched; the batch in flight before is routed and
    // delivered (its output-0 packets to the ready queue).
    void refill_and_launch(Host &h, S &t)
    {
        // pulled in groups without the lock (input 0 is another element),
        // each group staged under one lock
        enum { GROUP = 64 };
        P *grp[GROUP];
        uint32_t k = 0;
        bool dry = false;
        while (k < _batch && !dry) {
            uint32_t g = 0;
            const uint32_t want = _batch - k < (uint32_t) GROUP ? _batch - k : (uint32_t) GROUP;
            while (g < want && (grp[g] = h.input_pull()) != 0)
                g++;
            dry = g < want;
            t.enter();
            for (uint32_t j = 0; j < g; j++) {
                if (j + 4 < g)           // the bytes staging reads, 4 packets ahead
                    __builtin_prefetch(h.data(grp[j + 4]));
                if (stage(h, t, grp[j], false))
                    k++;
            }
            t.leave();
        }
        t.enter();
        if (!t.held.empty())
            flush(h, t, false);
        t.leave();
        drain(h, t, true);
    }

    // Stage one packet (locked).  Returns true if it is held.
    bool stage(Host &h, S &t, P *p, bool push_ctx)
    {
        uint32_t anno = 0;
        P *extra = 0;
        if (!t.e) {                      // no GPU for this thread: as a failed uniqueify
            h.kill(p);
            return false;
        }
        if (!(p = h.prepare(p, &anno, &extra))) {
            if (extra) {                 // consumed, with a result of its own (IPOutputCombo's
                R r;                     // clone when the copy failed): delivered as it stands
                memset(&r, 0, sizeof(r));
                r.extra = extra;
                r.port = CLK_PORT_OUT1;
                t.side.push_back(r);
            }
            return false;
        }
        Held<P> e = {p, extra, anno};
        t.held.push_back(e);
        if (push_ctx && !t.counted) {    // keep the router running until this batch is routed
            h.adjust_runcount(1);
            t.counted = true;
            arm(h, t);
        }
        // (the L4 classes read the transport header annotation: clk_element_push_th)
        int r = t.chain ? clk_chain_push_anno(t.chain, h.data(p), h.length(p), h.nh_offset(p), anno, t.next)
                        : clk_element_push_th(t.e, h.data(p), h.length(p), h.nh_offset(p), h.th_offset(p), anno,
                                              t.next);
        if (r < 0) {                     // not staged
            t.held.pop_back();
            h.kill(p);
            if (extra)
                h.kill(extra);
            if (r == CLK_EHIP) {
                // a flush inside the push failed (a ZEROCOPY batch ends where
                // the next packet's memory region starts): the staged batch
                // counts a failed flush, as a timer flush would
                failed_flush(h, t);
                t.unrouted = true;
            } else if (t.push_errors++ == 0 || (t.push_errors & 0xFFFF) == 0) {
                char buf[640];           // per-packet errors, once per 65536
                snprintf(buf, sizeof(buf), "%llu packet(s) not staged: %s", (unsigned long long) t.push_errors,
                         last_error(t).c_str());
                h.chatter(buf);
            }
            release_if_idle(h, t);
            return false;
        }
        t.next++;
        t.fresh++;
        if (t.fails && t.chain) {        // the chain retried its failed flush first and it went through
            t.fails = 0;                 // (clk_chain_push_anno): its results wait to be routed
            t.unrouted = true;
        }
        if ((r == 1 || t.fresh >= (uint32_t) INFLIGHT) && push_ctx)   // batch full: launch it, route the one before
            flush(h, t, false);
        return true;
    }

    void arm(Host &h, S &t)
    {
        t.deadline = h.now_ns() + (uint64_t) _latency_ms * 1000000u;
        if (!t.armed) {
            t.armed = true;
            h.wake(t);
        }
    }

    // one failed flush of the staged batch (locked): counted, the batch
    // abandoned after max_retries in a row
    void failed_flush(Host &h, S &t)
    {
        t.fails++;
        char buf[640];
        if (t.fails >= _max_retries) {
            const std::string why = last_error(t);
            uint64_t k = t.chain ? clk_chain_abandon(t.chain) : clk_element_abandon(t.e);
            snprintf(buf, sizeof(buf), "GPU batch failed %u times, %llu packets killed: %s", t.fails,
                     (unsigned long long) k, why.c_str());
            t.fails = 0;
        } else
            snprintf(buf, sizeof(buf), "GPU batch failed (retry %u of %u): %s", t.fails, _max_retries - 1,
                     last_error(t).c_str());
        h.chatter(buf);
    }

    // wait: route everything staged (timer, pull); otherwise double-buffered
    // (launch the staged batch, route the previous one, return).  Locked.
    void flush(Host &h, S &t, bool wait)
    {
        if (!t.e)
            return;
        int r = t.chain ? (wait ? clk_chain_flush(t.chain) : clk_chain_flush_async(t.chain))
                        : wait ? clk_element_flush(t.e) : clk_element_flush_async(t.e);
        t.fresh = 0;
        if (r != CLK_SUCCESS)            // nothing of the failed batch was routed; it stays staged
            failed_flush(h, t);
        else
            t.fails = 0;
        t.unrouted = true;               // drain() takes the results, a chunk at a time
        if (t.counted)                   // a new deadline for what is still held
            arm(h, t);
    }

    void release_if_idle(Host &h, S &t)
    {
        if (t.held.empty()) {
            t.armed = false;
            if (t.counted) {
                t.counted = false;
                h.adjust_runcount(-1);   // stop may now proceed
            }
        }
    }

    static std::string last_error(S &t)
    {
        return t.chain ? clk_chain_last_error(t.chain) : clk_element_last_error(t.e);
    }

    // Take up to one chunk of the glue's results into t.chunk (locked): each
    // result with the held packet it belongs to (moved out of the held ring
    // unless it is a pass record: the packet goes on in the chain).  drain()
    // delivers them before it takes the next, so the results stay in cache
    // between here and their delivery.  Once the glue has none left: the end
    // of the batch, the elements' chatter, and the runcount released if
    // nothing is held.
    void route(Host &h, S &t)
    {
        enum { CAP = Chunk<P>::CAP };
        if (!t.chunk)
            t.chunk = new Chunk<P>;
        Chunk<P> &c = *t.chunk;
        uint64_t tok[CAP];
        uint64_t n;
        if (t.chain)
            n = clk_chain_results(t.chain, tok, c.mem, c.port, c.len, c.aux, CAP);
        else if ((n = clk_element_results_aux(t.e, tok, c.port, c.len, c.aux, CAP)) > 0)
            memset(c.mem, 0, sizeof(int32_t) * (size_t) n);
        c.n = (uint32_t) n;
        c.end = false;
        if (n)
            t.routed_any = true;
        const uint64_t base = t.base, nheld = t.held.size();
        for (uint64_t i = 0; i < n; i++) {
            const uint64_t k = tok[i] - base;
            Held<P> *e = tok[i] >= base && k < nheld ? &t.held[(size_t) k] : 0;
            const int32_t port = c.port[i], m = c.mem[i];
            P *p = 0, *extra = 0, *made = 0, *parent = 0;
            uint8_t pass = 0;
            if (port == CLK_PORT_NEXT) {         // chains: on to the next member, still held
                pass = 1;
                c.port[i] = CLK_PORT_OUT0;
                p = e ? e->p : 0;
                t.last_primary = p;
            } else if (!(t.xmask >> (m & 63) & 1) || h.primary(m, port, c.aux[i])) {
                if (e) {
                    p = e->p;
                    e->p = 0;
                    if (port == CLK_PORT_KILL && e->extra) {   // e.g. a broadcast: no clone either
                        extra = e->extra;
                        e->extra = 0;
                    }
                }
                t.last_primary = p;
            } else if (c.aux[i] == CLK_AUX_CLONE) {
                if (e) {
                    extra = e->extra;
                    e->extra = 0;
                }
            } else {                             // a new packet made by the element
                made = h.make_packet(m, t.chain ? t.mem[(size_t) m] : t.e, c.aux[i]);
                // a clone kept by a chain (CLK_AUX_CLONE | key: IPOutputCombo
                // after the head) comes before its packet's own result: the
                // packet is still held; a fragment follows its packet's
                parent = (c.aux[i] & CLK_AUX_CLONE) && e ? e->p : t.last_primary;
            }
            c.p[i] = p;
            c.extra[i] = extra;
            c.made[i] = made;
            c.parent[i] = parent;
            c.anno[i] = e ? e->anno : 0;
            c.pass[i] = pass;
            if (p)                               // finish() reads it soon: the packet staged long ago is
                __builtin_prefetch(p);           // out of the cache by now
        }
        while (!t.held.empty() && !t.held.front().p && !t.held.front().extra) {
            t.held.pop_front();
            t.base++;
        }
        if (n == CAP)
            return;                              // more to come
        t.unrouted = false;
        c.end = t.routed_any;
        t.routed_any = false;
        release_if_idle(h, t);
        // the elements' click_chatter lines (e.g. the first drop's reason)
        char buf[8192];
        const size_t nm = t.chain ? t.mem.size() : 1;
        for (size_t m = 0; m < nm; m++)
            if (clk_element_take_messages(t.chain ? t.mem[m] : t.e, buf, sizeof(buf)) > 0)
                for (char *s = buf, *e; *s; s = e) {
                    if (!(e = strchr(s, '\n')))
                        e = s + strlen(s);
                    else
                        *e++ = 0;
                    h.message((int) m, s);
                }
    }

    // Deliver the results in order, without the lock: each chunk in runs of
    // one member (one host call per run).  Re-entrant calls on the same state
    // (a downstream element pushing back into this one) only stage: the
    // running loop delivers their results after these.
    void drain(Host &h, S &t, bool pull_ctx)
    {
        std::vector<P *> ready;                 // pull context: output-0 packets, queued under one lock
        t.enter();
        if (t.draining) {
            t.leave();
            return;
        }
        t.draining = true;
        const int last = (int) (t.chain ? t.mem.size() : 1) - 1;
        for (;;) {
            if (!t.side.empty()) {               // results a stage left behind, as they stand
                if (!t.side_chunk)
                    t.side_chunk = new Chunk<P>;
                Chunk<P> &c = *t.side_chunk;
                c.n = 0;
                for (size_t i = 0; i < t.side.size() && c.n < (uint32_t) Chunk<P>::CAP; i++)
                    c.put(c.n++, t.side[i]);
                t.side.erase(t.side.begin(), t.side.begin() + c.n);
                t.leave();
                deliver_chunk(h, t, c, 0, pull_ctx, last, ready);
                t.enter();
                if (!ready.empty()) {            // (pull context: queued now, whatever ends the loop)
                    t.ready.insert(t.ready.end(), ready.begin(), ready.end());
                    ready.clear();
                }
                continue;
            }
            if (!t.unrouted || !t.e)
                break;
            route(h, t);
            Chunk<P> &c = *t.chunk;
            t.leave();
            deliver_chunk(h, t, c, c.end, pull_ctx, last, ready);
            t.enter();
            if (!ready.empty()) {
                t.ready.insert(t.ready.end(), ready.begin(), ready.end());
                ready.clear();
            }
        }
        t.draining = false;
        t.leave();
    }

    // (unlocked) chunk c in runs of one member, then the end of the batch
    void deliver_chunk(Host &h, S &t, Chunk<P> &c, bool end, bool pull_ctx, int last, std::vector<P *> &ready)
    {
        for (uint32_t i = 0, j; i < c.n; i = j) {
            const int32_t m = c.mem[i];
            for (j = i + 1; j < c.n && c.mem[j] == m; j++)
                ;
            h.deliver(m, t, c, i, j, pull_ctx && m == last ? &ready : 0);
        }
        c.n = 0;
        c.end = false;
        if (end)
            for (int m = 0; m <= last; m++)
                h.end_of_batch(m, t);
    }

    uint32_t _batch;
    unsigned _latency_ms;
    unsigned _max_retries;
};

} // namespace hipcore
#endif
