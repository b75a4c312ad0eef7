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
    // setipchecksum.cc:77, setudpchecksum.cc:40, settcpchecksum.cc:47
    return p->uniqueify();
}

void
HIPSetChecksum::deliver(PerThread &, Held &h, int32_t port, uint32_t, uint32_t)
{
    if (port == CLK_PORT_OUT0)
	output(0).push(h.p);
    else				// SetUDPChecksum: output 1 (setudpchecksum.cc:60); bad lengths: killed
	kill_or_output1(h.p, port);
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

void
HIPDecIPTTL::deliver(PerThread &, Held &h, int32_t port, uint32_t, uint32_t)
{
    if (port == CLK_PORT_OUT0)
	output(0).push(h.p);
    else				// expired: checked_output_push(1, p) (54-57)
	kill_or_output1(h.p, port);
}

CLICK_ENDDECLS
ELEMENT_REQUIRES(HIPBatchElement)
ELEMENT_PROVIDES(HIPSetImpl)
// the classes are exported by hipdropin.cc (reference names) and
// hipparity.cc (HIP-prefixed names, for parity graphs beside the CPU ones)
