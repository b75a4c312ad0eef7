#ifndef CLICK_HIPCHECK_HH
#define CLICK_HIPCHECK_HH
#include "hipbatch.hh"
CLICK_DECLS

/*
 * GPU-backed header checks, registered under the reference class names so
 * an unchanged .click graph uses them (build with
 * --enable-skip-elements=CheckIPHeader,... : INTEGRATION.md).  Each keeps the
 * reference's keywords (parsed by the glue), ports, handlers and messages;
 * PROCESSING is push only (batching holds packets).
 *
 *   CheckIPHeader   checkipheader.cc:161-226    (glue CheckIPHeader)
 *   CheckIPHeader2  checkipheader2.cc:27-31     (glue CheckIPHeader2)
 *   IPInputCombo    ipinputcombo.cc:66-140      (glue IPInputCombo)
 *   CheckUDPHeader  checkudpheader.cc:84-107
 *   CheckTCPHeader  checktcpheader.cc:85-107
 *   CheckICMPHeader checkicmpheader.cc:83-141
 */

class HIPCheckIPHeader : public HIPClassElement<hipcore::CheckIPHeaderClass<Packet, ClickPacketOps> > { public:
    const char *class_name() const	{ return "CheckIPHeader"; }
    const char *port_count() const	{ return PORTS_1_1X2; }
    const char *flags() const		{ return "A"; }
    int initialize(ErrorHandler *errh) CLICK_COLD;
};

class HIPCheckIPHeader2 : public HIPCheckIPHeader { public:
    const char *class_name() const	{ return "CheckIPHeader2"; }
};

class HIPIPInputCombo : public HIPClassElement<hipcore::IPInputComboClass<Packet, ClickPacketOps> > { public:
    const char *class_name() const	{ return "IPInputCombo"; }
    const char *port_count() const	{ return PORTS_1_1; }
    const char *processing() const	{ return AGNOSTIC; }
    const char *flags() const		{ return "A"; }
    int initialize(ErrorHandler *errh) CLICK_COLD;
};

class HIPCheckL4Header : public HIPBatchElement { public:
    const char *port_count() const	{ return PORTS_1_1X2; }
    bool cls_reads_transport() const	{ return true; }
};

class HIPCheckUDPHeader : public HIPCheckL4Header { public:
    const char *class_name() const	{ return "CheckUDPHeader"; }
};

class HIPCheckTCPHeader : public HIPCheckL4Header { public:
    const char *class_name() const	{ return "CheckTCPHeader"; }
};

class HIPCheckICMPHeader : public HIPCheckL4Header { public:
    const char *class_name() const	{ return "CheckICMPHeader"; }
};

CLICK_ENDDECLS
#endif
