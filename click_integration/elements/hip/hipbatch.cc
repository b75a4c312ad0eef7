// -*- c-basic-offset: 4 -*-
/*
 * hipbatch.{cc,hh} -- shared adapter of the GPU-backed checksum elements
 * (see hipbatch.hh).  Drop this directory into Click's elements/ as the
 * "hip" group; INTEGRATION.md has the build hooks.
 */
#include <click/config.h>
#include "hipbatch.hh"
#include <click/args.hh>
#include <click/confparse.hh>
#include <click/error.hh>
#include <click/glue.hh>
#include <click/router.hh>
#include <click/straccum.hh>
#include <stdlib.h>
#include <string.h>
CLICK_DECLS

HIPBatchElement::HIPBatchElement()
    : _device(-1), _latency_ms(1), _pt(0), _npt(0)
{
}

HIPBatchElement::~HIPBatchElement()
{
    delete[] _pt;
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
	.consume() < 0)
	return -1;
    _glue_conf = cp_unargvec(conf);
    return 0;
}

int
HIPBatchElement::ensure(PerThread &t, int thread, ErrorHandler *errh)
{
    if (t.e)
	return 0;
    int ndev = clk_device_count();
    if (ndev <= 0)
	return errh ? errh->error("no gfx950 GPU: %s", clk_last_error(0)) : -1;
    int dev = _device >= 0 ? _device : thread % ndev;
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
    return 0;
}

int
HIPBatchElement::initialize(ErrorHandler *errh)
{
    _npt = click_max_cpu_ids();
    _pt = new PerThread[_npt];
    for (int k = 0; k < _npt; k++) {
	_pt[k].timer.assign(this);
	_pt[k].timer.initialize(this);
    }
    // the home thread's glue element now: configuration errors surface at
    // initialize time, as the reference element's configure() errors do
    int home = router()->home_thread_id(this);
    if (home < 0 || home >= _npt)
	home = 0;
    return ensure(_pt[home], home, errh);
}

int
HIPBatchElement::nh_offset(const Packet *p) const
{
    return p->has_network_header() ? p->network_header_offset() : -1;
}

Packet *
HIPBatchElement::prepare(Packet *p, uint32_t *anno, Packet **extra)
{
    (void) anno, (void) extra;
    return p;
}

void
HIPBatchElement::push(int, Packet *p)
{
    int thread = click_current_cpu_id();
    PerThread &t = _pt[thread < _npt ? thread : 0];
    t.lock.acquire();
    if (!t.e && ensure(t, thread, 0) < 0) {
	t.lock.release();
	p->kill();			// no GPU for this thread: as a failed uniqueify
	return;
    }
    uint32_t anno = 0;
    Packet *extra = 0;
    if (!(p = prepare(p, &anno, &extra))) {
	t.lock.release();
	return;
    }
    Held h;
    h.p = p;
    h.extra = extra;
    h.anno = anno;
    t.held.push_back(h);
    if (!t.counted) {		// keep the router running until this batch is routed
	router()->adjust_runcount(1);
	t.counted = true;
	t.timer.schedule_after_msec(_latency_ms);
    }
    int r = clk_element_push_anno(t.e, const_cast<unsigned char *>(p->data()), p->length(),
				  nh_offset(p), anno, t.next);
    if (r < 0) {			// not staged (e.g. ZEROCOPY memory not registered)
	click_chatter("%p{element}: %s", this, clk_element_last_error(t.e));
	t.held.pop_back();
	p->kill();
	if (extra)
	    extra->kill();
	if (t.held.empty() && t.counted) {
	    t.counted = false;
	    t.timer.unschedule();
	    router()->adjust_runcount(-1);
	}
    } else {
	t.next++;
	if (r == 1)			// batch full: launch it, route the one before
	    flush(t, false);
    }
    t.lock.release();
}

void
HIPBatchElement::run_timer(Timer *timer)
{
    for (int k = 0; k < _npt; k++)
	if (&_pt[k].timer == timer) {
	    PerThread &t = _pt[k];
	    t.lock.acquire();
	    flush(t, true);
	    t.lock.release();
	    return;
	}
}

// wait: route everything staged (timer, cleanup); otherwise double-buffered
// (launch the staged batch, route the previous one, return)
void
HIPBatchElement::flush(PerThread &t, bool wait)
{
    if (!t.e)
	return;
    int r = wait ? clk_element_flush(t.e) : clk_element_flush_async(t.e);
    if (r != CLK_SUCCESS)
	// nothing of the failed batch was routed; it stays staged and the
	// next flush retries it (include/click_amd_elements.h)
	click_chatter("%p{element}: GPU batch failed: %s", this, clk_element_last_error(t.e));
    route_results(t);
    if (t.held.empty()) {
	if (t.counted) {
	    t.counted = false;
	    t.timer.unschedule();
	    router()->adjust_runcount(-1);	// stop may now proceed
	}
    } else if (!t.timer.scheduled())
	t.timer.schedule_after_msec(_latency_ms);
}

void
HIPBatchElement::route_results(PerThread &t)
{
    enum { CAP = 256 };
    uint64_t tok[CAP];
    int32_t port[CAP];
    uint32_t len[CAP], aux[CAP];
    uint64_t n;
    bool any = false;
    while ((n = clk_element_results_aux(t.e, tok, port, len, aux, CAP)) > 0) {
	any = true;
	for (uint64_t i = 0; i < n; i++) {
	    // a result that follows its packet's own (IPFragmenter's extra
	    // fragments) may come after the entry was released
	    Held gone = {0, 0, 0};
	    Held &h = tok[i] >= t.base ? t.held[(int) (tok[i] - t.base)] : gone;
	    deliver(t, h, port[i], len[i], aux[i]);
	    if (primary(port[i], aux[i]))
		h.p = 0;
	}
	release_front(t);
	if (n < CAP)
	    break;
    }
    if (any)
	end_of_batch(t);
    char buf[8192];
    if (clk_element_take_messages(t.e, buf, sizeof(buf)) > 0)
	for (char *s = buf, *e; *s; s = e) {
	    if (!(e = strchr(s, '\n')))
		e = s + strlen(s);
	    else
		*e++ = 0;
	    click_chatter("%s", s);
	}
}

void
HIPBatchElement::release_front(PerThread &t)
{
    while (t.held.size() && !t.held.front().p && !t.held.front().extra) {
	t.held.pop_front();
	t.base++;
    }
}

void
HIPBatchElement::kill_or_output1(Packet *p, int32_t port)
{
    if (port == CLK_PORT_OUT1)
	checked_output_push(1, p);
    else
	p->kill();
}

void
HIPBatchElement::cleanup(CleanupStage)
{
    for (int k = 0; k < _npt; k++) {
	PerThread &t = _pt[k];
	if (t.e) {
	    flush(t, true);
	    clk_element_destroy(t.e);
	    clk_ctx_destroy(t.ctx);
	    t.e = 0;
	    t.ctx = 0;
	}
	while (t.held.size()) {		// a failed GPU: nothing can route them
	    Held &h = t.held.front();
	    if (h.p)
		h.p->kill();
	    if (h.extra)
		h.extra->kill();
	    t.held.pop_front();
	}
    }
}

String
HIPBatchElement::glue_handler(const char *hname) const
{
    for (int k = 0; k < _npt; k++)
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
    if (strcmp(hname, "drop_details") == 0) {
	Vector<unsigned long long> sum;
	Vector<String> text;
	for (int k = 0; k < he->_npt; k++) {
	    if (!he->_pt[k].e)
		continue;
	    char buf[4096];
	    clk_element_read_handler(he->_pt[k].e, hname, buf, sizeof(buf));
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
    for (int k = 0; k < he->_npt; k++)
	if (he->_pt[k].e) {
	    char buf[64];
	    clk_element_read_handler(he->_pt[k].e, hname, buf, sizeof(buf));
	    total += strtoull(buf, 0, 10);
	}
    return String(total);
}

void
HIPBatchElement::add_handlers()
{
    // the reference element's handlers (e.g. checkipheader.cc:238-244)
    // plus the glue's batches / packets / gpu_ns and the GPU in use
    static const char *const names[] = {"drops", "drop_details", "fragments", "batches", "packets",
					"gpu_ns", "device", "color", "active"};
    for (unsigned i = 0; i < sizeof(names) / sizeof(names[0]); i++)
	add_read_handler(String(names[i]), read_handler, static_cast<const void *>(names[i]));
}

CLICK_ENDDECLS
ELEMENT_LIBS((-L$(CLICK_AMD)/click_amd -lclick_amd_cksum -L/opt/rocm/lib -lamdhip64))
ELEMENT_PROVIDES(HIPBatchElement)
