#ifndef CLICK_HIPBATCH_HH
#define CLICK_HIPBATCH_HH
#include <click/element.hh>
#include <click/timer.hh>
#include <click/deque.hh>
#include <click/sync.hh>
#include "click_amd_elements.h"
CLICK_DECLS

/*
 * HIPBatchElement -- what every GPU-backed checksum element of this group
 * shares (not an element itself).
 *
 * Click's Element API hands over one packet at a time (element.cc:2891-2972);
 * the GPU wants batches.  The adapter stages each pushed packet into the
 * batched element glue (include/click_amd_elements.h), holds the Packet
 * until its batch comes back, and then does what the reference element's
 * simple_action() does after its checksum: the annotations, trims and
 * output pushes (the hooks deliver() and prepare() below, one subclass per
 * reference class).
 *
 * Adapter keywords (removed before the rest of the configuration goes to the
 * glue, which parses the reference element's keywords itself):
 *   LATENCY  ms   flush a partial batch this long after its first packet
 *                 (default 1)
 *   DEVICE   n    the GPU (default: RouterThread id % gfx950 devices; the
 *                 glue validates it: CLK_ENODEV for a GPU that is not there)
 * Glue keywords passed through: BATCH, ZEROCOPY, and the element's own.
 *
 * Threads (click -j N): one (context, glue element, held packets) per
 * RouterThread, chosen by click_current_cpu_id() (glue.hh:409-429), each
 * created the first time its thread pushes.  A Spinlock per thread state
 * serialises that thread's pushes with a flush from the home thread's timer
 * (timers run on the element's home thread, timer.cc:238-247, as in
 * ToDPDKDevice's per-thread queues, todpdkdevice.cc:85-86,176-179).
 *
 * Stop safety: while a thread state holds packets it holds one runcount
 * reference (Router::adjust_runcount, router.cc:832-846), so the driver
 * cannot stop the router (master.cc:283-303) before the batch is routed;
 * cleanup() flushes whatever is left.
 */
class HIPBatchElement : public Element { public:

    HIPBatchElement() CLICK_COLD;
    ~HIPBatchElement() CLICK_COLD;

    const char *processing() const	{ return PUSH; }
    int configure(Vector<String> &conf, ErrorHandler *errh) CLICK_COLD;
    int initialize(ErrorHandler *errh) CLICK_COLD;
    void cleanup(CleanupStage stage) CLICK_COLD;
    void add_handlers() CLICK_COLD;

    void push(int port, Packet *p);
    void run_timer(Timer *t);

  protected:

    struct Held {
	Packet *p;		// the packet pushed (made writable if the element writes it)
	Packet *extra;		// a second packet held with it (IPOutputCombo's PaintTee clone)
	uint32_t anno;		// the CLK_ANNO_* bits it was staged with
    };

    struct PerThread {
	clk_ctx *ctx;
	clk_element *e;
	Deque<Held> held;	// held[k] is token base + k
	uint64_t base;
	uint64_t next;
	Packet *frag_parent;	// IPFragmenter: the packet whose fragments follow
	bool counted;		// holds a runcount reference
	Timer timer;
	Spinlock lock;
	PerThread() : ctx(0), e(0), base(0), next(0), frag_parent(0), counted(false) { }
    };

    // the glue class (default: the reference class name this adapter takes)
    virtual const char *glue_class() const	{ return class_name(); }
    // before staging: uniqueify if the element writes the packet (as the
    // reference element does), fill *anno (CLK_ANNO_*), optionally hold a
    // second packet in *extra; return the packet to stage (0: consumed)
    virtual Packet *prepare(Packet *p, uint32_t *anno, Packet **extra);
    // the byte offset of the header the glue looks at (network header)
    virtual int nh_offset(const Packet *p) const;
    // route one result (the reference's side effects, then the push)
    virtual void deliver(PerThread &t, Held &h, int32_t port, uint32_t len, uint32_t aux) = 0;
    // false for a result that comes with another (IPOutputCombo's clone,
    // IPFragmenter's extra fragments): the held packet stays
    virtual bool primary(int32_t port, uint32_t aux) const	{ (void) port; (void) aux; return true; }
    // after a batch's results: release per-batch state
    virtual void end_of_batch(PerThread &t)	{ (void) t; }
    // glue handler text of the home thread's element (the element's
    // configuration, e.g. OFFSET, COLOR, MTU)
    String glue_handler(const char *name) const;
    void kill_or_output1(Packet *p, int32_t port);

    String _glue_conf;
    int _device;		// -1: per thread
    uint32_t _latency_ms;
    PerThread *_pt;
    int _npt;

  private:

    int ensure(PerThread &t, int thread, ErrorHandler *errh);
    void flush(PerThread &t, bool wait);
    void route_results(PerThread &t);
    void release_front(PerThread &t);
    static String read_handler(Element *e, void *thunk) CLICK_COLD;

};

CLICK_ENDDECLS
#endif
