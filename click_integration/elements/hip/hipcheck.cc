// -*- c-basic-offset: 4 -*-
/*
 * hipcheck.{cc,hh} -- GPU-backed CheckIPHeader, CheckIPHeader2,
 * IPInputCombo, CheckUDPHeader, CheckTCPHeader and CheckICMPHeader.
 * The verdict comes from the GPU batch; what the reference does with a
 * passing packet after its checksum is done here, on the host.
 */
#include <click/config.h>
#include "hipcheck.hh"
#include <click/packet_anno.hh>
#include <clicknet/ip.h>
#include <stdlib.h>
CLICK_DECLS

int
HIPCheckIPHeader::initialize(ErrorHandler *errh)
{
    if (HIPBatchElement::initialize(errh) < 0)
	return -1;
    _offset = atoi(glue_handler("offset").c_str());		// OFFSET, parsed by the glue
    return 0;
}

int
HIPCheckIPHeader::finish(PerThread &, Routed &r, Packet **out)
{
    Packet *p = r.p;
    if (!p || r.port != CLK_PORT_OUT0)		// drop(): output 1 if connected, else kill (143-159)
	return pass(r, out);
    // checkipheader.cc:213-223: network header, trim to ip_len, dst annotation
    const click_ip *ip = reinterpret_cast<const click_ip *>(p->data() + _offset);
    p->set_ip_header(ip, ip->ip_hl << 2);
    if (p->length() > r.len)			// len: the packet's length after the trim
	p->take(p->length() - r.len);
    p->set_dst_ip_anno(ip->ip_dst);
    *out = p;
    return 0;
}

int
HIPIPInputCombo::initialize(ErrorHandler *errh)
{
    if (HIPBatchElement::initialize(errh) < 0)
	return -1;
    _color = atoi(glue_handler("color").c_str());		// COLOR, parsed by the glue
    return 0;
}

int
HIPIPInputCombo::finish(PerThread &, Routed &r, Packet **out)
{
    Packet *p = r.p;
    if (!p)
	return -1;
    if (r.port != CLK_PORT_OUT0) {		// bad: killed (ipinputcombo.cc:134-139)
	p->kill();
	return -1;
    }
    SET_PAINT_ANNO(p, _color);			// Paint (71)
    p->pull(14);				// Strip(14) (74)
    const click_ip *ip = reinterpret_cast<const click_ip *>(p->data());
    p->set_ip_header(ip, ip->ip_hl << 2);	// 125
    if (p->length() > r.len)			// 128-129
	p->take(p->length() - r.len);
    p->set_dst_ip_anno(ip->ip_dst);		// 132
    *out = p;
    return 0;
}

CLICK_ENDDECLS
ELEMENT_REQUIRES(HIPBatchElement)
ELEMENT_PROVIDES(HIPCheckImpl)
// the classes are exported by hipdropin.cc (reference names) and
// hipparity.cc (HIP-prefixed names, for parity graphs beside the CPU ones)
