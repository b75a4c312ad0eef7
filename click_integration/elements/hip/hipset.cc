// -*- c-basic-offset: 4 -*-
/*
 * hipset.{cc,hh} -- GPU-backed SetIPChecksum, SetUDPChecksum,
 * SetTCPChecksum and DecIPTTL.
 */
#include <click/config.h>
#include "hipset.hh"
#include <clicknet/ip.h>
CLICK_DECLS

Packet *
HIPSetChecksum::prepare(Packet *p, uint32_t *, Packet **)
{
    // setipchecksum.cc:77, setudpchecksum.cc:40, settcpchecksum.cc:47; the
    // result routes by HIPBatchElement::pass(): output 0, SetUDPChecksum's
    // output 1 (setudpchecksum.cc:60), killed on bad lengths
    return p->uniqueify();
}

Packet *
HIPDecIPTTL::prepare(Packet *p, uint32_t *, Packet **)
{
    // decipttl.cc:59: writable only when the TTL is decremented; a packet
    // that leaves untouched (expired, ACTIVE false, multicast) may be
    // uniqueified here needlessly, which changes nothing but sharing
    if (p->has_network_header() && p->ip_header()->ip_ttl > 1)
	return p->uniqueify();
    return p;
}


CLICK_ENDDECLS
ELEMENT_REQUIRES(HIPBatchElement)
ELEMENT_PROVIDES(HIPSetImpl)
// the classes are exported by hipdropin.cc (reference names) and
// hipparity.cc (HIP-prefixed names, for parity graphs beside the CPU ones)
