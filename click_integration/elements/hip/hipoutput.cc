// -*- c-basic-offset: 4 -*-
/*
 * hipoutput.{cc,hh} -- GPU-backed IPGWOptions, FixIPSrc, IPOutputCombo and
 * IPFragmenter.  The glue rewrites the header bytes and writes them back
 * into the (writable) packet when the batch is routed; the reference's
 * annotations, clones and output choices are hipclasses.hh's class logic.
 */
#include <click/config.h>
#include "hipoutput.hh"
#include <stdlib.h>
CLICK_DECLS

// IPGWOptions and FixIPSrc: hipclasses.hh's classes, nothing to configure
// on the Click side (the glue parsed MYADDR / IPADDR).

int
HIPIPOutputCombo::initialize(ErrorHandler *errh)
{
    if (HIPBatchElement::initialize(errh) < 0)
	return -1;
    _cls.color = atoi(glue_handler("color").c_str());		// COLOR, parsed by the glue
    return 0;
}

int
HIPIPFragmenter::initialize(ErrorHandler *errh)
{
    if (HIPBatchElement::initialize(errh) < 0)
	return -1;
    _cls.mtu = strtoul(glue_handler("mtu").c_str(), 0, 10);		// MTU / HEADROOM, parsed by the glue
    _cls.headroom = strtoul(glue_handler("headroom").c_str(), 0, 10);
    return 0;
}

CLICK_ENDDECLS
ELEMENT_REQUIRES(HIPBatchElement)
ELEMENT_PROVIDES(HIPOutputImpl)
// the classes are exported by hipdropin.cc (reference names) and
// hipparity.cc (HIP-prefixed names, for parity graphs beside the CPU ones)
