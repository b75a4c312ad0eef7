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

void
HIPIPGWOptions::deliver(PerThread &, Held &h, int32_t port, uint32_t, uint32_t aux)
{
    Packet *p = h.p;
    if (port == CLK_PORT_OUT0)
	output(0).push(p);
    else if (port == CLK_PORT_OUT1) {		// send_error (162-165)
	SET_ICMP_PARAMPROB_ANNO(p, aux);
	checked_output_push(1, p);
    } else
	p->kill();
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

void
HIPFixIPSrc::deliver(PerThread &, Held &h, int32_t, uint32_t, uint32_t)
{
    if (h.anno & CLK_ANNO_FIX_IP_SRC)
	SET_FIX_IP_SRC_ANNO(h.p, 0);		// fix_it (fixipsrc.cc:59)
    output(0).push(h.p);
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
    if (!q && *extra) {			// the reference pushed the clone before the copy failed
	output(1).push(*extra);
	*extra = 0;
    }
    return q;
}

void
HIPIPOutputCombo::deliver(PerThread &, Held &h, int32_t port, uint32_t, uint32_t aux)
{
    if (aux == CLK_AUX_CLONE) {			// the PaintTee clone, before the packet
	output(1).push(h.extra);
	h.extra = 0;
	return;
    }
    Packet *p = h.p;
    if (port == CLK_PORT_KILL) {
	p->kill();
	return;
    }
    if (port == CLK_PORT_OUT2) {		// ipgw_send_error (202-204)
	SET_ICMP_PARAMPROB_ANNO(p, aux);
	output(2).push(p);
	return;
    }
    if (h.anno & CLK_ANNO_FIX_IP_SRC)		// FixIPSrc step (169-170)
	SET_FIX_IP_SRC_ANNO(p, 0);
    output(port).push(p);			// 0, 3 (TTL expired), 4 (longer than the MTU)
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

void
HIPIPFragmenter::deliver(PerThread &t, Held &h, int32_t port, uint32_t len, uint32_t aux)
{
    if (aux != 0) {
	// a fragment after the first (129-159): a new packet with the
	// glue's bytes, annotations copied from the original
	int64_t n = clk_element_take_packet(t.e, aux, 0, 0);
	WritablePacket *q = n >= 0 ? Packet::make(_headroom, 0, n, 0) : 0;
	if (!q) {			// out of memory: release the glue's copy, drop it
	    unsigned char one;
	    if (n >= 0)
		clk_element_take_packet(t.e, aux, &one, 1);
	    return;
	}
	clk_element_take_packet(t.e, aux, q->data(), n);
	q->set_network_header(q->data(), (q->data()[0] & 0xF) << 2);
	if (t.frag_parent)
	    q->copy_annotations(t.frag_parent);
	output(0).push(q);
	return;
    }
    Packet *p = h.p;
    if (port == CLK_PORT_OUT0 && len < (uint32_t) p->length()) {
	// the first fragment: the rewritten header is already in the packet
	// (112-120); a clone cut to its length goes out first (121-124), the
	// original stays for the annotations of the fragments that follow
	Packet *first = p->clone();
	if (first) {
	    first->take(p->length() - len);
	    output(0).push(first);
	}
	if (t.frag_parent)
	    t.frag_parent->kill();
	t.frag_parent = p;
    } else if (port == CLK_PORT_OUT0)
	output(0).push(p);
    else				// DF with HONOR_DF or tiny MTU: checked_output_push(1) (96-102)
	kill_or_output1(p, port);
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
