// -*- c-basic-offset: 4 -*-
/*
 * hipcheck.{cc,hh} -- GPU-backed CheckIPHeader, CheckIPHeader2,
 * IPInputCombo, CheckUDPHeader, CheckTCPHeader and CheckICMPHeader.
 * The verdict comes from the GPU batch; what the reference does with a
 * passing packet after its checksum is hipclasses.hh's class logic; here
 * only the configuration it needs is read back from the glue.
 */
#include <click/config.h>
#include "hipcheck.hh"
#include <stdlib.h>
CLICK_DECLS

int
HIPCheckIPHeader::initialize(ErrorHandler *errh)
{
    if (HIPBatchElement::initialize(errh) < 0)
	return -1;
    _cls.offset = atoi(glue_handler("offset").c_str());	// OFFSET, parsed by the glue
    return 0;
}

int
HIPIPInputCombo::initialize(ErrorHandler *errh)
{
    if (HIPBatchElement::initialize(errh) < 0)
	return -1;
    _cls.color = atoi(glue_handler("color").c_str());		// COLOR, parsed by the glue
    return 0;
}

CLICK_ENDDECLS
ELEMENT_REQUIRES(HIPBatchElement)
ELEMENT_PROVIDES(HIPCheckImpl)
// the classes are exported by hipdropin.cc (reference names) and
// hipparity.cc (HIP-prefixed names, for parity graphs beside the CPU ones)
