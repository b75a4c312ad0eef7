// -*- c-basic-offset: 4 -*-
/*
 * hipbatch.{cc,hh} -- Click's side of the GPU-backed checksum elements'
 * shared adapter (see hipbatch.hh; the logic is hipcore.hh's).  Drop this
 * directory into Click's elements/ as the "hip" group; INTEGRATION.md has
 * the build hooks.
 */
#include <click/config.h>
#include "hipbatch.hh"
#include <click/args.hh>
#include <click/confparse.hh>
#include <click/error.hh>
#include <click/glue.hh>
#include <click/router.hh>
#include <click/routervisitor.hh>
#include <click/straccum.hh>
#include <ctype.h>
#include <stdlib.h>
#include <string.h>
#include <new>
#include <malloc.h>
CLICK_DECLS

namespace {
// the output ports connected to one input port
struct UpstreamPorts : public RouterVisitor {
    int n;
    Element *first;
    UpstreamPorts() : n(0), first(0) { }
    bool visit(Element *e, bool isoutput, int, Element *, int, int distance) {
	if (isoutput && distance == 1 && n++ == 0)
	    first = e;
	return false;
    }
};

HIPBatchElement *
gpu_backed(Element *e)
{
    return e ? static_cast<HIPBatchElement *>(e->cast("HIPBatchElement")) : 0;
}
}

// hipchain.hh's graph trait over the router's connections: the chain rules
// themselves are hipchain.hh's (tested natively)
struct HIPChainGraph {
    typedef HIPBatchElement *Node;
    Node push_next(Node x) const {
	if (x->noutputs() < 1 || !x->output_is_push(0) || x->output(0).port() != 0)
	    return 0;
	return gpu_backed(x->output(0).element());
    }
    Node sole_upstream(Node y) const {
	if (y->ninputs() < 1 || !y->input_is_push(0))
	    return 0;
	UpstreamPorts up;
	y->router()->visit_upstream(y, 0, &up);
	return up.n == 1 ? gpu_backed(up.first) : 0;
    }
    bool chain_conf(Node x) const	{ return x->_chain_conf && !x->cls_reads_transport(); }
    int device(Node x) const		{ return x->_device; }
    bool may_write(Node x) const	{ return x->cls_may_write(); }
    bool chain_last(Node x) const	{ return x->cls_chain_last(); }
    bool chain_head_only(Node x) const	{ return x->cls_chain_head_only(); }
    bool pass_effects(Node x) const	{ return x->cls_pass_effects(); }
};

HIPBatchElement::HIPBatchElement()
    : _device(-1), _latency_ms(1), _retries(3), _pt(0), _tasks(0), _npt(0), _gate(0), _chain_conf(true),
      _chain_writes(false), _chain_tried(0)
{
}

HIPBatchElement::~HIPBatchElement()
{
    delete[] _pt;
    delete[] _chain_tried;
    if (_tasks) {
	for (int k = 0; k <= _npt; k++)
	    _tasks[k].~Task();
	operator delete[](static_cast<void *>(_tasks));
    }
}

int
HIPBatchElement::configure(Vector<String> &conf, ErrorHandler *errh)
{
    // the adapter's keywords; the rest (the reference element's keywords,
    // BATCH, ZEROCOPY) is parsed by the glue, as the element's configure()
    // would parse it, and its errors come back through clk_last_error
    _device = -1;
    if (Args(this, errh).bind(conf)
	.read("LATENCY", _latency_ms)
	.read("DEVICE", _device)
	.read("RETRIES", _retries)
	.read("CHAIN", _chain_conf)
	.consume() < 0)
	return -1;
    // BATCH: the glue's (65536, sized for the device batch) unless given;
    // the adapter's default is the core's in-flight cap, so a batch's
    // packets stay in the host caches between staging and delivery
    // (hipcore.hh Core::INFLIGHT; profiles/r06/click_batch_tcache_r06l.json)
    bool batch = false;
    for (int i = 0; i < conf.size(); i++) {
	String w = cp_uncomment(conf[i]);
	batch = batch || (w.length() >= 5 && strncmp(w.data(), "BATCH", 5) == 0 && (w.length() == 5 || isspace((unsigned char) w[5])));
    }
    if (!batch)
	conf.push_back(String("BATCH ") + String((int) ADAPTER_BATCH));
    _glue_conf = cp_unargvec(conf);
    // the glue's keywords checked now, without a GPU, so a bad one is a
    // configure-time error as in the reference element (Args' wording)
    int nout = noutputs() < 1 ? 1 : (noutputs() > 5 ? 5 : noutputs());
    if (clk_element_check_config(glue_class(), _glue_conf.c_str(), name().c_str(), nout) != CLK_SUCCESS) {
	String m(clk_last_error(0)), pre = name() + ": ";
	if (m.starts_with(pre))		// errh names the element already
	    m = m.substring(pre.length());
	return errh->error("%s", m.c_str());
    }
    _core.set_latency(_latency_ms);
    _core.set_max_retries(_retries);
    return 0;
}

int
HIPBatchElement::ensure(PerThread &t, ErrorHandler *errh)
{
    if (t.e)
	return 0;
    int ndev = clk_device_count();
    if (ndev <= 0) {
	const char *why = clk_last_error(0);
	return errh ? errh->error(why && *why ? "no gfx950 GPU: %s" : "no gfx950 GPU%s", why ? why : "") : -1;
    }
    int dev = _device >= 0 ? _device : t.id % ndev;
    if (dev >= ndev)
	return errh ? errh->error("DEVICE %d: no such GPU (%d gfx950 devices)", dev, ndev) : -1;
    if (clk_ctx_create(dev, &t.ctx) != CLK_SUCCESS)
	return errh ? errh->error("%s", clk_last_error(0)) : -1;
    if (clk_element_create(t.ctx, glue_class(), _glue_conf.c_str(), name().c_str(),
			   noutputs(), &t.e) != CLK_SUCCESS) {
	int r = errh ? errh->error("%s", clk_last_error(t.ctx)) : -1;
	clk_ctx_destroy(t.ctx);
	t.ctx = 0;
	return r;
    }
    clk_element_hold_packets(t.e, 1);	// the core holds each Packet until its result
    t.xmask = cls_extra_results() ? 1 : 0;	// primary() asked only for such a class
    // this thread's element speaks its once-only chatter (first drop...)
    // together with the home thread's, as the one reference element does
    if (_gate && _gate != t.e)
	clk_element_share_messages(t.e, _gate);
    return 0;
}

int
HIPBatchElement::initialize(ErrorHandler *errh)
{
    // one state per RouterThread, driven by that thread alone (no lock:
    // hipcore State::shared), plus a locked catch-all state for a push from
    // a thread id past them
    // A state holds up to three batches of packets (hipcore INFLIGHT), past
    // what Click's packet pool keeps (packet.cc:238, 1000 per thread): the
    // clones and copies beyond it come from malloc and go back with free,
    // and glibc returned the heap's top to the kernel at every such free and
    // took it back at the next malloc -- a third of the samples of a drop-in
    // Click in malloc, free and brk (profiles/r06/click_samples_*_r06h.txt).
    // Freed memory stays in the heap instead (once per process).
    static bool heap_kept = false;
    if (!heap_kept) {
	mallopt(M_TRIM_THRESHOLD, 256 << 20);
	mallopt(M_TOP_PAD, 64 << 20);
	heap_kept = true;
    }
    _npt = click_max_cpu_ids();
    _pt = new PerThread[_npt + 1];
    for (int k = 0; k < _npt; k++)
	_pt[k].shared = false;
    _pt[_npt].id = _npt;
    _pt[_npt].shared = true;
    // one Task per state, moved to its RouterThread (task.hh:275), not
    // scheduled until the state holds packets (hipcore: wake / poll); the
    // catch-all state's stays on the element's home thread
    _tasks = static_cast<Task *>(operator new[](sizeof(Task) * (_npt + 1)));
    for (int k = 0; k <= _npt; k++) {
	_pt[k].id = k;
	new (&_tasks[k]) Task(this);
	_tasks[k].initialize(this, false);
	if (k < _npt)
	    _tasks[k].move_thread(k);
    }
    // the home thread's glue element now: configuration errors surface at
    // initialize time, as the reference element's configure() errors do
    int home = router()->home_thread_id(this);
    if (home < 0 || home >= _npt)
	home = 0;
    if (ensure(_pt[home], errh) < 0)
	return -1;
    _gate = _pt[home].e;
    if (const char *att = message_attachment()) {
	// a router-wide once-only message (setudpchecksum.cc:53-57): the
	// first such element's glue element counts for every one of them
	void *&x = router()->force_attachment(att);
	if (!x)
	    x = _gate;
	else
	    clk_element_share_messages(_gate, static_cast<clk_element *>(x));
    }
    char buf[64];			// BATCH, parsed by the glue
    clk_element_read_handler(_pt[home].e, "batch", buf, sizeof(buf));
    _core.set_batch(strtoul(buf, 0, 10));
    // a chain head collects the members down output 0 (the connections and
    // every element's configuration exist now; the states set their chains
    // up on first use, when every member is initialized)
    _chain_tried = new bool[_npt + 1];
    for (int k = 0; k <= _npt; k++)
	_chain_tried[k] = false;
    HIPChainGraph g;
    hipcore::form_chain(g, this, _chain);
    _chain_writes = hipcore::chain_writes(g, _chain);
    return 0;
}

void *
HIPBatchElement::cast(const char *n)
{
    if (strcmp(n, "HIPBatchElement") == 0)
	return this;
    return Element::cast(n);
}

// State t runs the chain (under t's lock): each member's glue element on t's
// context, counted in the member's handlers.  If the glue refuses the chain
// the elements stay separate (output 0 pushes into the next one).
void
HIPBatchElement::ensure_chain(PerThread &t)
{
    _chain_tried[t.id] = true;
    if (_chain.size() < 2 || !t.e || t.chain)
	return;
    t.mem.push_back(t.e);
    for (int m = 1; m < _chain.size(); m++) {
	HIPBatchElement *y = _chain[m];
	clk_element *me = 0;
	if (clk_element_create(t.ctx, y->glue_class(), y->_glue_conf.c_str(), y->name().c_str(),
			       y->noutputs(), &me) != CLK_SUCCESS)
	    break;
	clk_element_hold_packets(me, 1);
	if (y->_gate)
	    clk_element_share_messages(me, y->_gate);
	t.mem.push_back(me);
    }
    if (t.mem.size() == (size_t) _chain.size()
	&& clk_chain_create(t.mem.data(), (int) t.mem.size(), &t.chain) == CLK_SUCCESS) {
	HIPChainGraph g;
	clk_chain_report_passes(t.chain, hipcore::chain_report(g, _chain));
	t.xmask = 0;
	for (int m = 0; m < _chain.size(); m++)
	    if (_chain[m]->cls_extra_results())
		t.xmask |= uint64_t(1) << m;
	for (int m = 1; m < _chain.size(); m++) {
	    _chain[m]->_borrow_lock.acquire();
	    _chain[m]->_borrowed.push_back(t.mem[m]);
	    _chain[m]->_borrow_lock.release();
	}
	return;
    }
    click_chatter("%p{element}: running separately from the elements after it: %s", this,
		  t.mem.size() == (size_t) _chain.size() ? clk_last_error(0) : clk_last_error(t.ctx));
    for (size_t m = 1; m < t.mem.size(); m++)
	clk_element_destroy(t.mem[m]);
    t.mem.clear();
    t.chain = 0;
}

Packet *
HIPBatchElement::prepare(Packet *p, uint32_t *anno, Packet **extra)
{
    if (!(p = cls_prepare(p, anno, extra)))
	return 0;
    if (_chain.size() > 1)		// readied for every member
	p = hipcore::chain_ready<Packet, ClickPacketOps>(p, _chain_writes, anno);
    return p;
}

HIPBatchElement::PerThread &
HIPBatchElement::state()
{
    int thread = click_current_cpu_id();
    PerThread &t = _pt[thread >= 0 && thread < _npt ? thread : _npt];
    if (!t.e) {
	t.lock.acquire();
	ensure(t, 0);			// no GPU for this thread: the core kills its packets
	t.lock.release();
    }
    return t;
}

void
HIPBatchElement::push(int, Packet *p)
{
    PerThread &t = state();
    if (!_chain_tried[t.id]) {
	t.lock.acquire();
	ensure_chain(t);
	t.lock.release();
    }
    _core.push(*this, t, p);
}

Packet *
HIPBatchElement::pull(int)
{
    return _core.pull(*this, state());
}

bool
HIPBatchElement::run_task(Task *task)
{
    // state k's latency deadline, on state k's RouterThread
    int k = task - _tasks;
    if (k < 0 || k > _npt)
	return false;
    if (_core.poll(*this, _pt[k]))
	task->fast_reschedule();	// still holding packets: look again
    return true;
}

void
HIPBatchElement::adjust_runcount(int delta)
{
    router()->adjust_runcount(delta);	// router.cc:832-846
}

void
HIPBatchElement::chatter(const char *text)
{
    click_chatter("%p{element}: %s", this, text);
}

void
HIPBatchElement::message(int, const char *line)
{
    click_chatter("%s", line);		// already worded as the reference element's
}

void
HIPBatchElement::cleanup(CleanupStage)
{
    // nothing is pushed downstream: held, routed-but-undelivered and ready
    // packets are killed, the glue elements and contexts destroyed (the
    // members' copies taken out of their handler sums first); no states when
    // configure() or an earlier element's initialize() failed
    for (int k = 0; k < nstates(); k++) {
	for (size_t m = 1; m < _pt[k].mem.size() && (int) m < _chain.size(); m++) {
	    HIPBatchElement *y = _chain[m];
	    y->_borrow_lock.acquire();
	    for (int i = 0; i < y->_borrowed.size(); i++)
		if (y->_borrowed[i] == _pt[k].mem[m]) {
		    y->_borrowed[i] = y->_borrowed.back();
		    y->_borrowed.pop_back();
		    break;
		}
	    y->_borrow_lock.release();
	}
	_core.cleanup(*this, _pt[k]);
    }
}

String
HIPBatchElement::glue_handler(const char *hname) const
{
    for (int k = 0; k < nstates(); k++)
	if (_pt[k].e) {
	    char buf[4096];
	    clk_element_read_handler(_pt[k].e, hname, buf, sizeof(buf));
	    return String(buf);
	}
    return String();
}

// Counters are summed over the per-thread glue elements; drop_details sums
// line by line (same reason order in every thread).
String
HIPBatchElement::read_handler(Element *e, void *thunk)
{
    HIPBatchElement *he = static_cast<HIPBatchElement *>(e);
    const char *hname = static_cast<const char *>(thunk);
    // this element's glue elements: its states' and its copies in chains
    Vector<clk_element *> els;
    for (int k = 0; k < he->nstates(); k++)
	if (he->_pt[k].e)
	    els.push_back(he->_pt[k].e);
    he->_borrow_lock.acquire();
    for (int i = 0; i < he->_borrowed.size(); i++)
	els.push_back(he->_borrowed[i]);
    he->_borrow_lock.release();
    if (strcmp(hname, "drop_details") == 0) {
	Vector<unsigned long long> sum;
	Vector<String> text;
	for (int k = 0; k < els.size(); k++) {
	    char buf[4096];
	    clk_element_read_handler(els[k], hname, buf, sizeof(buf));
	    int line = 0;
	    for (char *s = buf, *nl; *s; s = nl, line++) {
		if (!(nl = strchr(s, '\n')))
		    nl = s + strlen(s);
		else
		    *nl++ = 0;
		char *tab = strchr(s, '\t');
		if (line >= sum.size()) {
		    sum.push_back(0);
		    text.push_back(String(tab ? tab + 1 : ""));
		}
		sum[line] += strtoull(s, 0, 10);
	    }
	}
	StringAccum sa;
	for (int i = 0; i < sum.size(); i++)
	    sa << sum[i] << '\t' << text[i] << '\n';
	return sa.take_string();
    }
    if (strcmp(hname, "device") == 0 || strcmp(hname, "color") == 0 || strcmp(hname, "active") == 0)
	return he->glue_handler(hname);
    unsigned long long total = 0;
    for (int k = 0; k < els.size(); k++) {
	char buf[64];
	clk_element_read_handler(els[k], hname, buf, sizeof(buf));
	total += strtoull(buf, 0, 10);
    }
    return String(total);
}

void
HIPBatchElement::add_handlers()
{
    // the reference element's handlers (e.g. checkipheader.cc:238-244)
    // plus the glue's batches / packets / gpu_ns / lost and the GPU in use
    static const char *const names[] = {"drops", "drop_details", "fragments", "batches", "packets",
					"gpu_ns", "lost", "device", "color", "active"};
    for (unsigned i = 0; i < sizeof(names) / sizeof(names[0]); i++)
	add_read_handler(String(names[i]), read_handler, static_cast<const void *>(names[i]));
}

CLICK_ENDDECLS
// (click-buildtool splits this line at ':' and ')': the library directories
// come from LDFLAGS at configure time, tools/click_scratch_build.sh)
ELEMENT_LIBS((-lclick_amd_cksum -lamdhip64))
ELEMENT_PROVIDES(HIPBatchElement)
