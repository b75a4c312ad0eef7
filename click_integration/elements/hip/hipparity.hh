#ifndef CLICK_HIPPARITY_HH
#define CLICK_HIPPARITY_HH
#include "hipcheck.hh"
#include "hipset.hh"
#include "hipoutput.hh"
CLICK_DECLS

/*
 * The same GPU-backed elements under HIP-prefixed class names, for graphs
 * that run them BESIDE the CPU reference elements (no --enable-skip-elements
 * of the CPU classes; skip HIPCheckIPHeader... via hipdropin.cc instead), e.g.
 * the Tee -> {CPU element, GPU element} -> ComparePackets parity graphs of
 * click_integration/conf/.  The glue is told the reference class name.
 */

class HIPCheckIPHeaderX : public HIPCheckIPHeader { public:
    const char *class_name() const	{ return "HIPCheckIPHeader"; }
    const char *glue_class() const	{ return "CheckIPHeader"; }
};

class HIPCheckIPHeader2X : public HIPCheckIPHeader2 { public:
    const char *class_name() const	{ return "HIPCheckIPHeader2"; }
    const char *glue_class() const	{ return "CheckIPHeader2"; }
};

class HIPIPInputComboX : public HIPIPInputCombo { public:
    const char *class_name() const	{ return "HIPIPInputCombo"; }
    const char *glue_class() const	{ return "IPInputCombo"; }
};

class HIPCheckUDPHeaderX : public HIPCheckUDPHeader { public:
    const char *class_name() const	{ return "HIPCheckUDPHeader"; }
    const char *glue_class() const	{ return "CheckUDPHeader"; }
};

class HIPCheckTCPHeaderX : public HIPCheckTCPHeader { public:
    const char *class_name() const	{ return "HIPCheckTCPHeader"; }
    const char *glue_class() const	{ return "CheckTCPHeader"; }
};

class HIPCheckICMPHeaderX : public HIPCheckICMPHeader { public:
    const char *class_name() const	{ return "HIPCheckICMPHeader"; }
    const char *glue_class() const	{ return "CheckICMPHeader"; }
};

class HIPSetIPChecksumX : public HIPSetIPChecksum { public:
    const char *class_name() const	{ return "HIPSetIPChecksum"; }
    const char *glue_class() const	{ return "SetIPChecksum"; }
};

class HIPSetUDPChecksumX : public HIPSetUDPChecksum { public:
    const char *class_name() const	{ return "HIPSetUDPChecksum"; }
    const char *glue_class() const	{ return "SetUDPChecksum"; }
};

class HIPSetTCPChecksumX : public HIPSetTCPChecksum { public:
    const char *class_name() const	{ return "HIPSetTCPChecksum"; }
    const char *glue_class() const	{ return "SetTCPChecksum"; }
};

class HIPDecIPTTLX : public HIPDecIPTTL { public:
    const char *class_name() const	{ return "HIPDecIPTTL"; }
    const char *glue_class() const	{ return "DecIPTTL"; }
};

class HIPIPGWOptionsX : public HIPIPGWOptions { public:
    const char *class_name() const	{ return "HIPIPGWOptions"; }
    const char *glue_class() const	{ return "IPGWOptions"; }
};

class HIPFixIPSrcX : public HIPFixIPSrc { public:
    const char *class_name() const	{ return "HIPFixIPSrc"; }
    const char *glue_class() const	{ return "FixIPSrc"; }
};

class HIPIPOutputComboX : public HIPIPOutputCombo { public:
    const char *class_name() const	{ return "HIPIPOutputCombo"; }
    const char *glue_class() const	{ return "IPOutputCombo"; }
};

class HIPIPFragmenterX : public HIPIPFragmenter { public:
    const char *class_name() const	{ return "HIPIPFragmenter"; }
    const char *glue_class() const	{ return "IPFragmenter"; }
};

CLICK_ENDDECLS
#endif
