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
 * Results are taken from the glue under the thread state's lock but
 * DELIVERED (annotations, output pushes) after it is released, in push
 * order: a downstream element that re-enters this element on the same
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
 * Host interface (all called on the thread that drives the core; m is the
 * chain member, 0 without a chain):
 *   the class hooks of hipclasses.hh -- prepare(), nh_offset(), primary(m,..),
 *        make_packet(m,..), finish(m,..), end_of_batch(m,..) -- which the
 *        host forwards to the element class's shipped logic (the Click
 *        adapter and the native test instantiate the same classes)
 *   uint8_t *data(P *p); uint32_t length(P *p)
 *   void output_push(int m, int port, P *p)      member m's checked_output_push
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
 * deadline (LATENCY after its batch started); poll(t), run by the thread's
 * Task, flushes and delivers once it has passed.  So every packet of thread
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
    T &operator[](size_t k) { return v_[(h_ + k) & (v_.size() - 1)]; }
    T &front() { return v_[h_]; }
    void push_back(const T &x)
    {
        if (n_ == v_.size())
            grow();
        v_[(h_ + n_++) & (v_.size() - 1)] = x;
    }
    void pop_back() { n_--; }
    void pop_front()
    {
        h_ = (h_ + 1) & (v_.size() - 1);
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
    }
    std::vector<T> v_;
    size_t h_ = 0, n_ = 0;
};

// One result, handed to the host's finish() after the lock is released.
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
    bool end;       // not a result: the end of a batch (host end_of_batch)
};

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
    bool armed;                   // the latency deadline is set
    uint64_t deadline;            // now_ns() at which poll() flushes
    uint64_t push_errors;         // packets push() could not stage (chatter is rate-limited)
    std::vector<Routed<P> > outbox;
    std::vector<Routed<P> > spare;    // delivery storage kept between batches
    std::deque<P *> ready;        // pull context: output-0 packets ready to hand out
    P *last_primary;              // route(): the packet of the last primary result
    P *frag_parent;               // host use (IPFragmenter's first-fragment parent)
    L lock;
    State() : ctx(0), e(0), chain(0), id(0), base(0), next(0), counted(false), fails(0), draining(false),
              unrouted(false), routed_any(false), armed(false),
              deadline(0), push_errors(0), last_primary(0), frag_parent(0) { }
};

template <class P, class Host, class L> class Core {
  public:
    typedef State<P, L> S;
    typedef Routed<P> R;

    Core() : _batch(65536), _latency_ms(1), _max_retries(3) { }

    void set_batch(uint32_t b)       { _batch = b ? b : 1; }
    void set_latency(unsigned ms)    { _latency_ms = ms; }
    void set_max_retries(unsigned k) { _max_retries = k ? k : 1; }
    uint32_t batch() const           { return _batch; }

    // ---- push context --------------------------------------------------------
    void push(Host &h, S &t, P *p)
    {
        t.lock.acquire();
        stage(h, t, p, true);
        // most pushes only stage: deliver when there is something to
        const bool deliver = (!t.outbox.empty() || t.unrouted) && !t.draining;
        t.lock.release();
        if (deliver)
            drain(h, t, false);
    }

    // run state t's partial batch now and route everything (the deadline
    // passed, or the router asks)
    void timer(Host &h, S &t)
    {
        t.lock.acquire();
        flush(h, t, true);
        t.lock.release();
        drain(h, t, false);
    }

    // the state's Task: flush once its deadline has passed.  Returns true
    // while the state still holds a deadline (the Task runs again).
    bool poll(Host &h, S &t)
    {
        t.lock.acquire();
        if (!t.armed) {
            t.lock.release();
            return false;
        }
        if (h.now_ns() < t.deadline) {
            t.lock.release();
            return true;
        }
        flush(h, t, true);
        t.lock.release();
        drain(h, t, false);
        t.lock.acquire();
        const bool again = t.armed;
        t.lock.release();
        return again;
    }

    bool armed(S &t)
    {
        t.lock.acquire();
        const bool a = t.armed;
        t.lock.release();
        return a;
    }

    // ---- pull context (output 0) --------------------------------------------
    P *pull(Host &h, S &t)
    {
        t.lock.acquire();
        if (t.ready.empty()) {
            t.lock.release();
            refill_and_launch(h, t);     // launches a batch, routes the one in flight
            t.lock.acquire();
            // nothing ready (the first refill, or a batch that kept no packet
            // for output 0): wait for what is in flight -- retried at once,
            // abandoned after max_retries -- and launch the next batch before
            // handing these out
            while (t.ready.empty() && !t.held.empty() && t.e) {
                flush(h, t, true);
                const bool failed = t.fails != 0;
                t.lock.release();
                drain(h, t, true);
                if (!failed)
                    refill_and_launch(h, t);
                t.lock.acquire();
            }
        }
        P *p = 0;
        if (!t.ready.empty()) {
            p = t.ready.front();
            t.ready.pop_front();
        }
        t.lock.release();
        return p;
    }

    // ---- teardown: kill everything held; no downstream pushes ----------------
    void cleanup(Host &h, S &t)
    {
        t.lock.acquire();
        for (size_t i = 0; i < t.held.size(); i++) {
            if (t.held[i].p)
                h.kill(t.held[i].p);
            if (t.held[i].extra)
                h.kill(t.held[i].extra);
        }
        t.held.clear();
        for (size_t i = 0; i < t.outbox.size(); i++) {
            R &r = t.outbox[i];
            if (r.pass)                  // the packet is still held (killed above)
                continue;
            if (r.p) h.kill(r.p);
            if (r.extra) h.kill(r.extra);
            if (r.made) h.kill(r.made);
        }
        t.outbox.clear();
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
        t.lock.release();
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
            t.lock.acquire();
            for (uint32_t j = 0; j < g; j++) {
                if (j + 4 < g)           // the bytes staging reads, 4 packets ahead
                    __builtin_prefetch(h.data(grp[j + 4]));
                if (stage(h, t, grp[j], false))
                    k++;
            }
            t.lock.release();
        }
        t.lock.acquire();
        if (!t.held.empty())
            flush(h, t, false);
        t.lock.release();
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
                t.outbox.push_back(r);
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
        int r = t.chain ? clk_chain_push_anno(t.chain, h.data(p), h.length(p), h.nh_offset(p), anno, t.next)
                        : clk_element_push_anno(t.e, h.data(p), h.length(p), h.nh_offset(p), anno, t.next);
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
        if (r == 1 && push_ctx)          // batch full: launch it, route the one before
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
        // a chain runs its members one after another on the batch: synchronous
        int r = t.chain ? clk_chain_flush(t.chain) : wait ? clk_element_flush(t.e) : clk_element_flush_async(t.e);
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

    // Move up to one chunk of the glue's results into the outbox (locked):
    // drain() delivers them before it takes the next, so the results stay in
    // cache between here and their delivery.  Once the glue has none left:
    // the end of the batch, the elements' chatter, and the runcount released
    // if nothing is held.
    void route(Host &h, S &t)
    {
        enum { CAP = 256 };
        uint64_t tok[CAP];
        int32_t mem[CAP], port[CAP];
        uint32_t len[CAP], aux[CAP];
        uint64_t n;
        {
            if (t.chain)
                n = clk_chain_results(t.chain, tok, mem, port, len, aux, CAP);
            else if ((n = clk_element_results_aux(t.e, tok, port, len, aux, CAP)) > 0)
                memset(mem, 0, sizeof(int32_t) * (size_t) n);
            if (n)
                t.routed_any = true;
            for (uint64_t i = 0; i < n; i++) {
                t.outbox.emplace_back(); // built in place, zeroed (value-initialized)
                R &r = t.outbox.back();
                r.member = mem[i];
                r.port = port[i];
                r.len = len[i];
                r.aux = aux[i];
                const bool have = tok[i] >= t.base && tok[i] - t.base < t.held.size();
                Held<P> *e = have ? &t.held[(size_t) (tok[i] - t.base)] : 0;
                if (e)
                    r.anno = e->anno;
                if (port[i] == CLK_PORT_NEXT) {  // chains: on to the next member, still held
                    r.pass = true;
                    r.port = CLK_PORT_OUT0;
                    r.p = e ? e->p : 0;
                    t.last_primary = r.p;
                } else if (h.primary(r.member, port[i], aux[i])) {
                    if (e) {
                        r.p = e->p;
                        e->p = 0;
                        if (port[i] == CLK_PORT_KILL && e->extra) {   // e.g. a broadcast: no clone either
                            r.extra = e->extra;
                            e->extra = 0;
                        }
                    }
                    t.last_primary = r.p;
                } else if (aux[i] == CLK_AUX_CLONE) {
                    if (e) {
                        r.extra = e->extra;
                        e->extra = 0;
                    }
                } else {                 // a new packet made by the element
                    r.made = h.make_packet(r.member, t.chain ? t.mem[(size_t) r.member] : t.e, aux[i]);
                    r.parent = t.last_primary;
                }
                if (r.p)                 // finish() reads it soon: the packet staged long ago is
                    __builtin_prefetch(r.p);     // out of the cache by now
            }
            while (!t.held.empty() && !t.held.front().p && !t.held.front().extra) {
                t.held.pop_front();
                t.base++;
            }
        }
        if (n == CAP)
            return;                      // more to come
        t.unrouted = false;
        if (t.routed_any) {
            t.routed_any = false;
            R end;
            memset(&end, 0, sizeof(end));
            end.end = true;
            t.outbox.push_back(end);
        }
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

    // Deliver the outbox in order, without the lock.  Re-entrant calls on
    // the same state (a downstream element pushing back into this one) only
    // append: the running loop delivers their results after these.
    void drain(Host &h, S &t, bool pull_ctx)
    {
        std::vector<P *> ready;                 // pull context: output-0 packets, queued under one lock
        t.lock.acquire();
        if (t.draining) {
            t.lock.release();
            return;
        }
        t.draining = true;
        std::vector<R> work;
        work.swap(t.spare);                     // a delivered outbox's storage, reused
        for (;;) {
            if (t.outbox.empty() && t.unrouted && t.e)
                route(h, t);
            if (t.outbox.empty())
                break;
            work.swap(t.outbox);
            t.lock.release();
            for (size_t i = 0; i < work.size(); i++) {
                R &r = work[i];
                if (i + 8 < work.size() && work[i + 8].p)   // its bytes, 8 results ahead
                    __builtin_prefetch(h.data(work[i + 8].p));
                if (r.end) {
                    const size_t nm = t.chain ? t.mem.size() : 1;
                    for (size_t m = 0; m < nm; m++)
                        h.end_of_batch((int) m, t);
                    continue;
                }
                P *out = 0;
                int port = h.finish(r.member, t, r, &out);
                if (r.pass || port < 0 || !out)  // a pass: the member's side effects only
                    continue;
                if (pull_ctx && port == 0 && r.member + 1 == (int) (t.chain ? t.mem.size() : 1))
                    ready.push_back(out);
                else
                    h.output_push(r.member, port, out);
            }
            work.clear();
            t.lock.acquire();
            if (t.outbox.empty())
                t.outbox.swap(work);             // the next chunk goes into this storage
            t.ready.insert(t.ready.end(), ready.begin(), ready.end());
            ready.clear();
        }
        t.spare.swap(work);
        t.draining = false;
        t.lock.release();
    }

    uint32_t _batch;
    unsigned _latency_ms;
    unsigned _max_retries;
};

} // namespace hipcore
#endif
