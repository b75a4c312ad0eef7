// -*- c-basic-offset: 4 -*-
/*
 * hipset.{cc,hh} -- GPU-backed SetIPChecksum, SetUDPChecksum,
 * SetTCPChecksum and DecIPTTL.
 */
#include <click/config.h>
#include "hipset.hh"
CLICK_DECLS

// The classes are hipclasses.hh's SetChecksumClass (uniqueify before
// staging: setipchecksum.cc:77, setudpchecksum.cc:40, settcpchecksum.cc:47)
// and DecIPTTLClass (writable only when the TTL is decremented,
// decipttl.cc:59); nothing to configure on the Click side.

CLICK_ENDDECLS
ELEMENT_REQUIRES(HIPBatchElement)
ELEMENT_PROVIDES(HIPSetImpl)
// the classes are exported by hipdropin.cc (reference names) and
// hipparity.cc (HIP-prefixed names, for parity graphs beside the CPU ones)
