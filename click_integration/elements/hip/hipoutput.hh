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

class HIPIPGWOptions : public HIPBatchElement { public:
    const char *class_name() const	{ return "IPGWOptions"; }
    const char *port_count() const	{ return PORTS_1_1X2; }
    Packet *prepare(Packet *p, uint32_t *anno, Packet **extra);
    int finish(PerThread &t, Routed &r, Packet **out);
};

class HIPFixIPSrc : public HIPBatchElement { public:
    const char *class_name() const	{ return "FixIPSrc"; }
    const char *port_count() const	{ return PORTS_1_1; }
    const char *processing() const	{ return AGNOSTIC; }
    Packet *prepare(Packet *p, uint32_t *anno, Packet **extra);
    int finish(PerThread &t, Routed &r, Packet **out);
};

class HIPIPOutputCombo : public HIPBatchElement { public:
    const char *class_name() const	{ return "IPOutputCombo"; }
    const char *port_count() const	{ return "1/5"; }
    const char *processing() const	{ return PUSH; }
    int initialize(ErrorHandler *errh) CLICK_COLD;
    Packet *prepare(Packet *p, uint32_t *anno, Packet **extra);
    int finish(PerThread &t, Routed &r, Packet **out);
    bool primary(int32_t port, uint32_t aux) const	{ (void) port; return aux != CLK_AUX_CLONE; }
  protected:
    int _color;
};

class HIPIPFragmenter : public HIPBatchElement { public:
    const char *class_name() const	{ return "IPFragmenter"; }
    const char *port_count() const	{ return PORTS_1_1X2; }
    const char *processing() const	{ return PUSH; }
    int initialize(ErrorHandler *errh) CLICK_COLD;
    Packet *prepare(Packet *p, uint32_t *anno, Packet **extra);
    Packet *make_packet(clk_element *e, uint32_t key);
    int finish(PerThread &t, Routed &r, Packet **out);
    bool primary(int32_t port, uint32_t aux) const	{ (void) port; return aux == 0; }
    void end_of_batch(PerThread &t);
  protected:
    uint32_t _mtu;
    uint32_t _headroom;
};

CLICK_ENDDECLS
#endif
