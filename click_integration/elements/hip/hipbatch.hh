#ifndef CLICK_HIPBATCH_HH
#define CLICK_HIPBATCH_HH
#include <click/element.hh>
#include <click/timer.hh>
#include <click/sync.hh>
#include "click_amd_elements.h"
#include "hipcore.hh"
CLICK_DECLS

/*
 * HIPBatchElement -- what every GPU-backed checksum element of this group
 * shares (not an element itself): Click's side of the core in hipcore.hh,
 * which holds the packets while their batch is on the GPU, routes the
 * results, keeps the runcount and the latency timer, retries a failed
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
 * Glue keywords passed through: BATCH, ZEROCOPY, and the element's own.
 *
 * Threads (click -j N): one hipcore::State (context, glue element, held
 * packets, lock) per RouterThread, chosen by click_current_cpu_id()
 * (glue.hh:409-429), each created the first time its thread uses it.  Timers
 * run on the element's home thread (timer.cc:238-247), as in ToDPDKDevice's
 * per-thread queues (todpdkdevice.cc:85-86,176-179); the state's Spinlock
 * serialises them with that thread's pushes.  No output is pushed while a
 * lock is held.
 */
class HIPBatchElement : public Element { public:

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
    void run_timer(Timer *t);

    // ---- the core's host interface (hipcore.hh) ------------------------------
    // before staging: uniqueify if the element writes the packet (as the
    // reference element does), fill *anno (CLK_ANNO_*), optionally hold a
    // second packet in *extra; return the packet to stage (0: consumed)
    virtual Packet *prepare(Packet *p, uint32_t *anno, Packet **extra);
    uint8_t *data(Packet *p)		{ return const_cast<unsigned char *>(p->data()); }
    uint32_t length(Packet *p)		{ return p->length(); }
    // the byte offset of the header the glue looks at (network header)
    virtual int32_t nh_offset(Packet *p);
    // false for a result that comes with another (IPOutputCombo's clone,
    // IPFragmenter's extra fragments): the held packet stays
    virtual bool primary(int32_t port, uint32_t aux) const	{ (void) port; (void) aux; return true; }
    virtual Packet *make_packet(clk_element *e, uint32_t key);
    // one result: the reference's side effects; returns the output port of
    // *out (core pushes it, or hands it out in pull context), -1 for none
    virtual int finish(PerThread &t, Routed &r, Packet **out);
    virtual void end_of_batch(PerThread &t)	{ (void) t; }
    void output_push(int port, Packet *p)	{ checked_output_push(port, p); }
    Packet *input_pull()			{ return input(0).pull(); }
    void kill(Packet *p)			{ p->kill(); }
    void adjust_runcount(int delta);
    void schedule(PerThread &t, unsigned ms)	{ _timers[t.id].schedule_after_msec(ms); }
    void unschedule(PerThread &t)		{ _timers[t.id].unschedule(); }
    bool scheduled(PerThread &t)		{ return _timers[t.id].scheduled(); }
    void chatter(const char *text);
    void message(const char *line);

  protected:

    // the glue class (default: the reference class name this adapter takes)
    virtual const char *glue_class() const	{ return class_name(); }
    // glue handler text of the home thread's element (the element's
    // configuration, e.g. OFFSET, COLOR, MTU)
    String glue_handler(const char *name) const;
    // the default finish(): output port as routed, killed on CLK_PORT_KILL
    int pass(Routed &r, Packet **out);
    // the router attachment naming a once-per-router message, if the
    // reference element has one (SetUDPChecksum); 0: once per element
    virtual const char *message_attachment() const	{ return 0; }

    String _glue_conf;
    int _device;		// -1: per thread
    uint32_t _latency_ms;
    uint32_t _retries;
    PerThread *_pt;
    Timer *_timers;
    int _npt;
    clk_element *_gate;		// whose once-only chatter the thread elements share
    hipcore::Core<Packet, HIPBatchElement, Spinlock> _core;

  private:

    PerThread &state();
    int ensure(PerThread &t, ErrorHandler *errh);
    static String read_handler(Element *e, void *thunk) CLICK_COLD;

};

CLICK_ENDDECLS
#endif
