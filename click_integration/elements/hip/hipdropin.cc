// -*- c-basic-offset: 4 -*-
/*
 * hipdropin.cc -- exports the GPU-backed elements under the REFERENCE class
 * names (CheckIPHeader, SetUDPChecksum, ...), so an unchanged .click graph
 * runs them.  Build with the CPU versions skipped:
 *   ./configure --enable-hip --enable-skip-elements=CheckIPHeader,\
 *     CheckIPHeader2,SetIPChecksum,CheckUDPHeader,SetUDPChecksum,\
 *     CheckTCPHeader,SetTCPChecksum,CheckICMPHeader,DecIPTTL,IPInputCombo,\
 *     IPGWOptions,FixIPSrc,IPOutputCombo,IPFragmenter,HIPParity
 * (configure.in:573,584-587; click-buildtool findelem -x drops the files that
 * export those names, and hipparity.cc, which provides HIPParity).
 */
#include <click/config.h>
#include "hipdropin.hh"
CLICK_DECLS
CLICK_ENDDECLS
ELEMENT_REQUIRES(HIPCheckImpl HIPSetImpl HIPOutputImpl)
EXPORT_ELEMENT(HIPCheckIPHeader)
EXPORT_ELEMENT(HIPCheckIPHeader2)
EXPORT_ELEMENT(HIPIPInputCombo)
EXPORT_ELEMENT(HIPCheckUDPHeader)
EXPORT_ELEMENT(HIPCheckTCPHeader)
EXPORT_ELEMENT(HIPCheckICMPHeader)
EXPORT_ELEMENT(HIPSetIPChecksum)
EXPORT_ELEMENT(HIPSetUDPChecksum)
EXPORT_ELEMENT(HIPSetTCPChecksum)
EXPORT_ELEMENT(HIPDecIPTTL)
EXPORT_ELEMENT(HIPIPGWOptions)
EXPORT_ELEMENT(HIPFixIPSrc)
EXPORT_ELEMENT(HIPIPOutputCombo)
EXPORT_ELEMENT(HIPIPFragmenter)
ELEMENT_MT_SAFE(HIPCheckIPHeader)
ELEMENT_MT_SAFE(HIPCheckIPHeader2)
ELEMENT_MT_SAFE(HIPIPInputCombo)
ELEMENT_MT_SAFE(HIPCheckUDPHeader)
ELEMENT_MT_SAFE(HIPCheckTCPHeader)
ELEMENT_MT_SAFE(HIPCheckICMPHeader)
ELEMENT_MT_SAFE(HIPSetIPChecksum)
ELEMENT_MT_SAFE(HIPSetUDPChecksum)
ELEMENT_MT_SAFE(HIPSetTCPChecksum)
ELEMENT_MT_SAFE(HIPDecIPTTL)
ELEMENT_MT_SAFE(HIPIPGWOptions)
ELEMENT_MT_SAFE(HIPFixIPSrc)
ELEMENT_MT_SAFE(HIPIPOutputCombo)
ELEMENT_MT_SAFE(HIPIPFragmenter)
