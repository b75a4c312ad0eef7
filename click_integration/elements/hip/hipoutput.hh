#ifndef CLICK_HIPOUTPUT_HH
#define CLICK_HIPOUTPUT_HH
#include "hipbatch.hh"
CLICK_DECLS

/*
 * GPU-backed IP output path, under the reference class names:
 *
 *   IPGWOptions    ipgwoptions.cc:53-172
 *   FixIPSrc       fixipsrc.cc:52-72
 *   IPOutputCombo  ipoutputcombo.cc:44-205 (ports 0-4)
 *   IPFragmenter   ipfragmenter.cc:88-171 (fragments after the first are
 *                  new packets the glue made; the adapter copies them into
 *                  Packet::make(HEADROOM, ...) packets)
 */

class HIPIPGWOptions : public HIPClassElement<hipcore::IPGWOptionsClass<Packet, ClickPacketOps> > { public:
    const char *class_name() const	{ return "IPGWOptions"; }
    const char *port_count() const	{ return PORTS_1_1X2; }
};

class HIPFixIPSrc : public HIPClassElement<hipcore::FixIPSrcClass<Packet, ClickPacketOps> > { public:
    const char *class_name() const	{ return "FixIPSrc"; }
    const char *port_count() const	{ return PORTS_1_1; }
    const char *processing() const	{ return AGNOSTIC; }
};

class HIPIPOutputCombo : public HIPClassElement<hipcore::IPOutputComboClass<Packet, ClickPacketOps> > { public:
    const char *class_name() const	{ return "IPOutputCombo"; }
    const char *port_count() const	{ return "1/5"; }
    const char *processing() const	{ return PUSH; }
    int initialize(ErrorHandler *errh) CLICK_COLD;
};

class HIPIPFragmenter : public HIPClassElement<hipcore::IPFragmenterClass<Packet, ClickPacketOps> > { public:
    const char *class_name() const	{ return "IPFragmenter"; }
    const char *port_count() const	{ return PORTS_1_1X2; }
    const char *processing() const	{ return PUSH; }
    int initialize(ErrorHandler *errh) CLICK_COLD;
};

CLICK_ENDDECLS
#endif
