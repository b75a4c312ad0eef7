#ifndef CLICK_HIPBATCH_HH
#define CLICK_HIPBATCH_HH
#include <click/element.hh>
#include <click/task.hh>
#include <click/timestamp.hh>
#include <click/sync.hh>
#include <click/packet_anno.hh>
#include <clicknet/ip.h>
#include "click_amd_elements.h"
#include "hipcore.hh"
#include "hipclasses.hh"
#include "hipchain.hh"
CLICK_DECLS

/*
 * ClickPacketOps -- the packet operations trait of hipclasses.hh over
 * Click's Packet: each is one Packet call.
 */
struct ClickPacketOps {
    static Packet *uniqueify(Packet *p)		{ return p->uniqueify(); }
    static Packet *clone(Packet *p)		{ return p->clone(); }
    static void kill(Packet *p)			{ p->kill(); }
    static uint8_t *data(Packet *p)		{ return const_cast<unsigned char *>(p->data()); }
    static uint32_t length(Packet *p)		{ return p->length(); }
    static bool has_network_header(Packet *p)	{ return p->has_network_header(); }
    static const uint8_t *network_header(Packet *p)	{ return p->network_header(); }
    static int32_t network_header_offset(Packet *p)	{ return p->network_header_offset(); }
    static int network_length(Packet *p)	{ return p->network_length(); }
    static void set_ip_header(Packet *p, const uint8_t *ip, uint32_t hlen) {
	p->set_ip_header(reinterpret_cast<const click_ip *>(ip), hlen);
    }
    static void take(Packet *p, uint32_t n)	{ p->take(n); }
    static void pull(Packet *p, uint32_t n)	{ p->pull(n); }
    static void set_dst_ip_anno(Packet *p, uint32_t a)	{ p->set_dst_ip_anno(IPAddress(a)); }
    static uint32_t paint(Packet *p)		{ return PAINT_ANNO(p); }
    static void set_paint(Packet *p, uint32_t c)	{ SET_PAINT_ANNO(p, c); }
    static bool fix_ip_src(Packet *p)		{ return FIX_IP_SRC_ANNO(p); }
    static void clear_fix_ip_src(Packet *p)	{ SET_FIX_IP_SRC_ANNO(p, 0); }
    static void set_icmp_paramprob(Packet *p, uint32_t v)	{ SET_ICMP_PARAMPROB_ANNO(p, v); }
    static bool broadcast_or_multicast(Packet *p) {
	return p->packet_type_anno() == Packet::BROADCAST || p->packet_type_anno() == Packet::MULTICAST;
    }
    static void copy_annotations(Packet *to, Packet *from)	{ to->copy_annotations(from); }
    static Packet *make(uint32_t headroom, uint32_t len) {
	return headroom ? Packet::make(headroom, 0, len, 0) : Packet::make(len);
    }
};

/*
 * HIPBatchElement -- what every GPU-backed checksum element of this group
 * shares (not an element itself): Click's side of the core in hipcore.hh,
 * which holds the packets while their batch is on the GPU, routes the
 * results, keeps the runcount and the latency deadline, retries a failed
 * flush and batches in pull context.  The subclasses (one per reference
 * class) do what the reference element's simple_action() does around its
 * checksum: prepare() before staging (uniqueify, PaintTee clone) and
 * finish() with the result (annotations, trims; the output to push to).
 *
 * Processing: the reference's.  CheckIPHeader, CheckUDPHeader,
 * CheckTCPHeader, CheckICMPHeader, DecIPTTL, SetUDPChecksum and IPGWOptions
 * are PROCESSING_A_AH (checkipheader.hh:114); SetIPChecksum, SetTCPChecksum,
 * FixIPSrc and IPInputCombo AGNOSTIC (element.cc:1127); IPOutputCombo and
 * IPFragmenter PUSH.  In pull context pull() batches what input 0 has (up to
 * BATCH packets) and hands the output-0 packets out one per call; the drop
 * output stays push, as checked_output_push.
 *
 * Adapter keywords (removed before the rest of the configuration goes to the
 * glue, which parses the reference element's keywords itself):
 *   LATENCY  ms   flush a partial batch this long after its first packet
 *                 (default 1)
 *   DEVICE   n    the GPU (default: RouterThread id % gfx950 devices; the
 *                 glue validates it: CLK_ENODEV for a GPU that is not there)
 *   RETRIES  n    failed flushes of a batch before its packets are killed
 *                 (default 3)
 *   CHAIN    bool join the GPU-backed elements after this one into one batch
 *                 (default true; see Chains below)
 * Glue keywords passed through: BATCH (default here ADAPTER_BATCH = 2048,
 * where the glue's own default is 65536; in push context a batch is
 * launched after at most hipcore::Core::INFLIGHT = 2048 packets whatever
 * BATCH, so that held packets stay in the host caches), ZEROCOPY, and the
 * element's own.
 *
 * Threads (click -j N): one hipcore::State (context, glue element, held
 * packets) per RouterThread, chosen by click_current_cpu_id()
 * (glue.hh:409-429), each created the first time its thread uses it and
 * driven by that thread alone, so without a lock (State::shared false); a
 * thread id past them shares one catch-all state, which is locked.  Each
 * state has a Task moved to its RouterThread (Task::move_thread,
 * task.hh:275): while the state holds packets the Task polls its latency
 * deadline (hipcore::Core::poll), so a partial batch is flushed, and its
 * packets pushed downstream, on the thread that pushed them.  No output is
 * pushed while a lock is held.
 *
 * The element classes' own logic (what the reference element does around
 * its checksum) is hipclasses.hh's, instantiated with ClickPacketOps;
 * HIPClassElement<C> forwards the core's hooks to it.
 *
 * Chains (the GPU analogue of click-xform's combos): when this element's
 * output 0 pushes into a GPU-backed element's input 0 that nothing else
 * pushes into, on the same DEVICE, both with CHAIN true, the second joins
 * the first one's batch -- and so on down output 0 (an IPFragmenter ends a
 * chain, an IPOutputCombo only starts one: its PaintTee clones the packet
 * as it arrives).  The head's thread states run the members as one
 * clk_chain: a packet is staged once, each member's kernel runs over what
 * the members before it passed, and each result is finished by the member
 * it leaves (its class logic) and pushed on that member's output.  The
 * head makes a packet writable when any member may write it, and stages
 * the annotations every member reads.  The members' handlers count what
 * they did in the chains too.  A chain that cannot be created (e.g. ZEROCOPY
 * on some members only) is left as separate elements, with one message.
 * The rules are hipchain.hh's (HIPChainGraph answers its graph questions).
 */
class HIPBatchElement;

// deliver_run's output: member m's checked_output_push (element.hh)
struct ClickPush {
    Element *e;
    explicit ClickPush(Element *e_) : e(e_) { }
    void operator()(int port, Packet *p) const	{ e->checked_output_push(port, p); }
};

class HIPBatchElement : public Element { public:

    enum { ADAPTER_BATCH = 2048 };	// = hipcore::Core::INFLIGHT

    typedef hipcore::State<Packet, Spinlock> PerThread;
    typedef hipcore::Routed<Packet> Routed;

    HIPBatchElement() CLICK_COLD;
    ~HIPBatchElement() CLICK_COLD;

    const char *processing() const	{ return PROCESSING_A_AH; }
    int configure(Vector<String> &conf, ErrorHandler *errh) CLICK_COLD;
    int initialize(ErrorHandler *errh) CLICK_COLD;
    void cleanup(CleanupStage stage) CLICK_COLD;
    void add_handlers() CLICK_COLD;

    void push(int port, Packet *p);
    Packet *pull(int port);

    void *cast(const char *n);

    // ---- the class hooks (hipclasses.hh): the plain check elements' here,
    // HIPClassElement<C> forwards them to its class
    virtual Packet *cls_prepare(Packet *p, uint32_t *anno, Packet **extra)	{ return _plain.prepare(p, anno, extra); }
    virtual int32_t cls_nh_offset(Packet *p)	{ return _plain.nh_offset(p); }
    virtual bool cls_primary(int32_t port, uint32_t aux) const	{ return _plain.primary(port, aux); }
    virtual Packet *cls_make_packet(clk_element *e, uint32_t key)	{ return _plain.make_packet(e, key); }
    typedef hipcore::Chunk<Packet> Chunk;
    virtual void cls_deliver(PerThread &t, const Chunk &c, uint32_t i, uint32_t j, std::vector<Packet *> *ready) {
	hipcore::deliver_run<Packet, hipcore::Plain<Packet, ClickPacketOps>, PerThread, ClickPacketOps>(
	    _plain, t, c, i, j, ready, ClickPush(this));
    }
    virtual void cls_end_of_batch(PerThread &t)	{ _plain.end_of_batch(t); }
    virtual bool cls_extra_results() const	{ return false; }
    virtual bool cls_may_write() const		{ return false; }
    virtual bool cls_chain_last() const		{ return false; }
    virtual bool cls_chain_head_only() const	{ return false; }
    virtual bool cls_pass_effects() const	{ return false; }
    // reads the transport header annotation (the L4 classes): runs alone,
    // never in a chain, whose batches take no transport header
    virtual bool cls_reads_transport() const	{ return false; }

    // ---- the core's host interface (hipcore.hh); m: the chain member ---------
    Packet *prepare(Packet *p, uint32_t *anno, Packet **extra);
    int32_t nh_offset(Packet *p)		{ return cls_nh_offset(p); }
    int32_t th_offset(Packet *p) {		// udp_header() / tcp_header() / icmp_header()'s annotation
	return !cls_reads_transport() ? -1 : p->has_transport_header() ? p->transport_header_offset() : -2;
    }
    bool primary(int m, int32_t port, uint32_t aux) const	{ return _chain[m]->cls_primary(port, aux); }
    Packet *make_packet(int m, clk_element *e, uint32_t key)	{ return _chain[m]->cls_make_packet(e, key); }
    bool extra_results(int m) const	{ return _chain[m]->cls_extra_results(); }
    void deliver(int m, PerThread &t, const Chunk &c, uint32_t i, uint32_t j, std::vector<Packet *> *ready) {
	_chain[m]->cls_deliver(t, c, i, j, ready);	// one call per run of member m's results
    }
    void end_of_batch(int m, PerThread &t)	{ _chain[m]->cls_end_of_batch(t); }
    uint8_t *data(Packet *p)		{ return ClickPacketOps::data(p); }
    uint32_t length(Packet *p)		{ return p->length(); }
    Packet *input_pull()			{ return input(0).pull(); }
    void kill(Packet *p)			{ p->kill(); }
    void adjust_runcount(int delta);
    uint64_t now_ns()			{ return Timestamp::now_steady().nsecval(); }
    void wake(PerThread &t)		{ _tasks[t.id].reschedule(); }
    void chatter(const char *text);
    void message(int m, const char *line);
    bool run_task(Task *task);

  protected:

    // the glue class (default: the reference class name this adapter takes)
    virtual const char *glue_class() const	{ return class_name(); }
    // glue handler text of the home thread's element (the element's
    // configuration, e.g. OFFSET, COLOR, MTU)
    String glue_handler(const char *name) const;
    // the router attachment naming a once-per-router message, if the
    // reference element has one (SetUDPChecksum); 0: once per element
    virtual const char *message_attachment() const	{ return 0; }
    // the per-thread states made by initialize() (0 before it, or when
    // configuration failed)
    int nstates() const			{ return _pt ? _npt + 1 : 0; }

    String _glue_conf;
    int _device;		// -1: per thread
    uint32_t _latency_ms;
    uint32_t _retries;
    PerThread *_pt;
    Task *_tasks;			// one per state, on its RouterThread
    int _npt;
    clk_element *_gate;		// whose once-only chatter the thread elements share
    bool _chain_conf;		// CHAIN
    bool _chain_writes;		// a member after this head may write packets
    Vector<HIPBatchElement *> _chain;	// [0] this; then the members this head runs
    bool *_chain_tried;		// per state: its chain was set up (or refused)
    Vector<clk_element *> _borrowed;	// this element's glue copies in chains of heads before it
    Spinlock _borrow_lock;
    hipcore::Core<Packet, HIPBatchElement, Spinlock> _core;
    hipcore::Plain<Packet, ClickPacketOps> _plain;

  private:

    PerThread &state();
    int ensure(PerThread &t, ErrorHandler *errh);
    void ensure_chain(PerThread &t);
    static String read_handler(Element *e, void *thunk) CLICK_COLD;

    friend struct HIPChainGraph;

};

/*
 * HIPClassElement<C> -- a GPU-backed element whose reference behaviour is
 * class C of hipclasses.hh (instantiated with ClickPacketOps).
 */
template <class C>
class HIPClassElement : public HIPBatchElement { public:
    Packet *cls_prepare(Packet *p, uint32_t *anno, Packet **extra)	{ return _cls.prepare(p, anno, extra); }
    int32_t cls_nh_offset(Packet *p)	{ return _cls.nh_offset(p); }
    bool cls_primary(int32_t port, uint32_t aux) const	{ return _cls.primary(port, aux); }
    Packet *cls_make_packet(clk_element *e, uint32_t key)	{ return _cls.make_packet(e, key); }
    void cls_deliver(PerThread &t, const Chunk &c, uint32_t i, uint32_t j, std::vector<Packet *> *ready) {
	hipcore::deliver_run<Packet, C, PerThread, ClickPacketOps>(_cls, t, c, i, j, ready, ClickPush(this));
    }
    void cls_end_of_batch(PerThread &t)	{ _cls.end_of_batch(t); }
    bool cls_extra_results() const	{ return C::extra_results != 0; }
    bool cls_may_write() const		{ return C::may_write != 0; }
    bool cls_chain_last() const		{ return C::chain_last != 0; }
    bool cls_chain_head_only() const	{ return C::chain_head_only != 0; }
    bool cls_pass_effects() const	{ return C::pass_effects != 0; }
  protected:
    C _cls;
};

CLICK_ENDDECLS
#endif
