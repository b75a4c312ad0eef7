// -*- c-basic-offset: 4 -*-
/*
 * hipoutput.{cc,hh} -- GPU-backed IPGWOptions, FixIPSrc, IPOutputCombo and
 * IPFragmenter.  The glue rewrites the header bytes and writes them back
 * into the (writable) packet when the batch is routed; the adapter keeps
 * the reference's annotations and output pushes.
 */
#include <click/config.h>
#include "hipoutput.hh"
#include <click/packet_anno.hh>
#include <clicknet/ip.h>
#include <stdlib.h>
CLICK_DECLS

// ---- IPGWOptions ------------------------------------------------------------

Packet *
HIPIPGWOptions::prepare(Packet *p, uint32_t *, Packet **)
{
    // only packets with options are touched (simple_action, ipgwoptions.cc:167-169)
    if (p->has_network_header() && p->ip_header()->ip_hl > 5)
	return p->uniqueify();
    return p;
}

int
HIPIPGWOptions::finish(PerThread &, Routed &r, Packet **out)
{
    if (r.p && r.port == CLK_PORT_OUT1)		// send_error (162-165)
	SET_ICMP_PARAMPROB_ANNO(r.p, r.aux);
    return pass(r, out);
}

// ---- FixIPSrc ---------------------------------------------------------------

Packet *
HIPFixIPSrc::prepare(Packet *p, uint32_t *anno, Packet **)
{
    if (FIX_IP_SRC_ANNO(p) && p->has_network_header()) {	// simple_action (69-73)
	*anno = CLK_ANNO_FIX_IP_SRC;
	return p->uniqueify();
    }
    return p;
}

int
HIPFixIPSrc::finish(PerThread &, Routed &r, Packet **out)
{
    if (r.p && (r.anno & CLK_ANNO_FIX_IP_SRC))
	SET_FIX_IP_SRC_ANNO(r.p, 0);		// fix_it (fixipsrc.cc:59)
    return pass(r, out);
}

// ---- IPOutputCombo ----------------------------------------------------------

int
HIPIPOutputCombo::initialize(ErrorHandler *errh)
{
    if (HIPBatchElement::initialize(errh) < 0)
	return -1;
    _color = atoi(glue_handler("color").c_str());		// COLOR, parsed by the glue
    return 0;
}

Packet *
HIPIPOutputCombo::prepare(Packet *p, uint32_t *anno, Packet **extra)
{
    // DropBroadcasts (50-53): the glue kills it; no clone, no copy
    if (p->packet_type_anno() == Packet::BROADCAST || p->packet_type_anno() == Packet::MULTICAST) {
	*anno = CLK_ANNO_BCAST;
	return p;
    }
    *anno = CLK_ANNO_PAINT(PAINT_ANNO(p)) | (FIX_IP_SRC_ANNO(p) ? CLK_ANNO_FIX_IP_SRC : 0);
    // PaintTee (56-57): the clone is taken before anything is rewritten;
    // uniqueify then gives the original its own bytes (60)
    if (PAINT_ANNO(p) == _color)
	*extra = p->clone();
    WritablePacket *q = p->uniqueify();
    if (!q && *extra) {
	// out of memory: the reference pushed the clone before the copy
	// failed; prepare() runs under the thread state's lock, where nothing
	// is pushed downstream (a re-entrant push would deadlock), so it dies
	(*extra)->kill();
	*extra = 0;
    }
    return q;
}

int
HIPIPOutputCombo::finish(PerThread &, Routed &r, Packet **out)
{
    if (r.extra && !r.p) {			// the PaintTee clone, before the packet
	*out = r.extra;
	return 1;
    }
    Packet *p = r.p;
    if (!p)
	return -1;
    if (r.port == CLK_PORT_KILL) {		// DropBroadcasts (50-53)
	p->kill();
	if (r.extra)
	    r.extra->kill();
	return -1;
    }
    if (r.port == CLK_PORT_OUT2)		// ipgw_send_error (202-204)
	SET_ICMP_PARAMPROB_ANNO(p, r.aux);
    else if (r.anno & CLK_ANNO_FIX_IP_SRC)	// FixIPSrc step (169-170)
	SET_FIX_IP_SRC_ANNO(p, 0);
    *out = p;
    return r.port;				// 0, 2, 3 (TTL expired), 4 (longer than the MTU)
}

// ---- IPFragmenter -----------------------------------------------------------

int
HIPIPFragmenter::initialize(ErrorHandler *errh)
{
    if (HIPBatchElement::initialize(errh) < 0)
	return -1;
    _mtu = strtoul(glue_handler("mtu").c_str(), 0, 10);		// MTU / HEADROOM, parsed by the glue
    _headroom = strtoul(glue_handler("headroom").c_str(), 0, 10);
    return 0;
}

Packet *
HIPIPFragmenter::prepare(Packet *p, uint32_t *, Packet **)
{
    // push (163-166): only a packet longer than the MTU is fragmented, and
    // made writable first (106-109)
    if (p->network_length() > (int) _mtu)
	return p->uniqueify();
    return p;
}

Packet *
HIPIPFragmenter::make_packet(clk_element *e, uint32_t key)
{
    // a fragment after the first (129-159): a new packet with the glue's
    // bytes and the element's HEADROOM; its annotations come in finish()
    int64_t n = clk_element_take_packet(e, key, 0, 0);
    WritablePacket *q = n >= 0 ? Packet::make(_headroom, 0, n, 0) : 0;
    if (!q) {				// out of memory: release the glue's copy, drop it
	unsigned char one;
	if (n >= 0)
	    clk_element_take_packet(e, key, &one, 1);
	return 0;
    }
    clk_element_take_packet(e, key, q->data(), n);
    q->set_network_header(q->data(), (q->data()[0] & 0xF) << 2);
    return q;
}

int
HIPIPFragmenter::finish(PerThread &t, Routed &r, Packet **out)
{
    if (r.made) {				// a fragment: annotations of the original (153)
	if (r.parent)
	    r.made->copy_annotations(r.parent);
	*out = r.made;
	return 0;
    }
    Packet *p = r.p;
    if (!p)
	return -1;
    if (r.port == CLK_PORT_OUT0 && r.len < (uint32_t) p->length()) {
	// the first fragment: the rewritten header is already in the packet
	// (112-120); a clone cut to its length goes out first (121-124), the
	// original stays for the annotations of the fragments that follow
	Packet *first = p->clone();
	if (t.frag_parent)
	    t.frag_parent->kill();
	t.frag_parent = p;
	if (!first)
	    return -1;
	first->take(p->length() - r.len);
	*out = first;
	return 0;
    }
    return pass(r, out);		// untouched, or DF with HONOR_DF / tiny MTU (96-102)
}

void
HIPIPFragmenter::end_of_batch(PerThread &t)
{
    if (t.frag_parent) {		// p->kill() after its fragments (169)
	t.frag_parent->kill();
	t.frag_parent = 0;
    }
}

CLICK_ENDDECLS
ELEMENT_REQUIRES(HIPBatchElement)
ELEMENT_PROVIDES(HIPOutputImpl)
// the classes are exported by hipdropin.cc (reference names) and
// hipparity.cc (HIP-prefixed names, for parity graphs beside the CPU ones)
