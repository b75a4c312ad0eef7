#ifndef CLICK_HIPSET_HH
#define CLICK_HIPSET_HH
#include "hipbatch.hh"
CLICK_DECLS

/*
 * GPU-backed checksum writers, under the reference class names:
 *
 *   SetIPChecksum   setipchecksum.cc:74-95
 *   SetUDPChecksum  setudpchecksum.cc:37-69
 *   SetTCPChecksum  settcpchecksum.cc:44-75 (FIXOFF)
 *   DecIPTTL        decipttl.cc:45-77 (RFC 1624 update of ip_sum)
 *
 * As the reference does, the packet is made writable (uniqueify()) before
 * it is staged; the glue writes the new checksum (and TTL) into that
 * writable packet when its batch is routed.
 */

typedef HIPClassElement<hipcore::SetChecksumClass<Packet, ClickPacketOps> > HIPSetChecksum;

class HIPSetIPChecksum : public HIPSetChecksum { public:
    const char *class_name() const	{ return "SetIPChecksum"; }
    const char *port_count() const	{ return PORTS_1_1; }
    const char *processing() const	{ return AGNOSTIC; }
};

class HIPSetUDPChecksum : public HIPSetChecksum { public:
    const char *class_name() const	{ return "SetUDPChecksum"; }
    bool cls_reads_transport() const	{ return true; }
    const char *message_attachment() const	{ return "HIPSetUDPChecksum_message"; }
    const char *port_count() const	{ return PORTS_1_1X2; }
};

class HIPSetTCPChecksum : public HIPSetChecksum { public:
    const char *class_name() const	{ return "SetTCPChecksum"; }
    bool cls_reads_transport() const	{ return true; }
    const char *port_count() const	{ return PORTS_1_1; }
    const char *processing() const	{ return AGNOSTIC; }
};

class HIPDecIPTTL : public HIPClassElement<hipcore::DecIPTTLClass<Packet, ClickPacketOps> > { public:
    const char *class_name() const	{ return "DecIPTTL"; }
    const char *port_count() const	{ return PORTS_1_1X2; }
};

CLICK_ENDDECLS
#endif
