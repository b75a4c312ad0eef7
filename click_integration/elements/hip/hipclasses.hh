// -*- c-basic-offset: 4 -*-
#ifndef CLICK_HIPCLASSES_HH
#define CLICK_HIPCLASSES_HH
/*
 * hipclasses.hh -- what each GPU-backed element does around its batched
 * checksum, as the reference element's simple_action()/push() does it: the
 * packet made writable before staging, the PaintTee clone, and on the way out
 * the annotations, trims, Strip and the first-fragment clone.  Click-
 * independent: every class is a template over the packet type P and a packet
 * operations trait O, so the SAME code runs in Click (P = Packet, O =
 * ClickPacketOps in hipbatch.hh, whose functions are single Packet calls) and
 * in tests/native/hipcore_test.cc (its own packet with shared buffers and an
 * annotation area), where it is driven on the GPU against the oracle.
 *
 * The trait O (all static):
 *   P *uniqueify(P *p)          Packet::uniqueify(): writable, 0 on failure (p gone)
 *   P *clone(P *p)              Packet::clone(), 0 on failure
 *   void kill(P *p)
 *   uint8_t *data(P *p); uint32_t length(P *p)
 *   bool has_network_header(P *p); const uint8_t *network_header(P *p)
 *   int32_t network_header_offset(P *p); int network_length(P *p)
 *   void set_ip_header(P *p, const uint8_t *ip, uint32_t hlen)
 *   void take(P *p, uint32_t n)  (trim the tail); void pull(P *p, uint32_t n) (Strip)
 *   void set_dst_ip_anno(P *p, uint32_t addr)   (network byte order, as read)
 *   uint32_t paint(P *p); void set_paint(P *p, uint32_t c)
 *   bool fix_ip_src(P *p); void clear_fix_ip_src(P *p)
 *   void set_icmp_paramprob(P *p, uint32_t v)
 *   bool broadcast_or_multicast(P *p)           (packet_type_anno)
 *   void copy_annotations(P *to, P *from)
 *   P *make(uint32_t headroom, uint32_t len)    Packet::make(headroom, 0, len, 0)
 *
 * A class's hooks (called by hipcore::Core through the host):
 *   prepare(p, &anno, &extra)  under the thread state's lock, before staging;
 *        returns the packet to stage, 0 when it is consumed.  A consumed
 *        packet may leave a result behind in *extra (IPOutputCombo's clone
 *        when the copy fails): the core delivers it as an output-1 result.
 *   nh_offset(p)               the offset of the header the glue looks at
 *   primary(port, aux)         false for a result that comes with its
 *                              packet's own (a clone, an extra fragment)
 *   make_packet(e, key)        a packet the glue made (a fragment)
 *   finish(t, r, &out)         no lock held: side effects of one result,
 *                              returns the output port of *out, -1 for none
 *   end_of_batch(t)            after a batch's results
 *
 * And four traits for chains (hipcore.hh; the adapter forms them):
 *   may_write        the element may rewrite a packet's bytes (a chain makes
 *                    the packet writable at its head)
 *   chain_last       extra results after a packet (fragments): only the last
 *                    member of a chain
 *   chain_head_only  its prepare() clones the packet as it arrives
 *                    (PaintTee): only the first member
 *   pass_effects     its finish() changes a packet it passes on (network
 *                    header, trim, Strip, annotations): the chain reports
 *                    those passes (clk_chain_report_passes)
 * and extra_results  results besides its packets' own (a clone, fragments):
 *                    the core asks primary() only for such a class
 */
#include <stdint.h>
#include <string.h>
#include "click_amd_elements.h"
#include "hipcore.hh"

namespace hipcore {

// The glue's drop(): output 1 if it exists, killed otherwise (the port comes
// routed; checkipheader.cc:143-159, checked_output_push).
template <class P, class O> struct Plain {
    enum { may_write = 0, chain_last = 0, chain_head_only = 0, pass_effects = 0, extra_results = 0 };
    P *prepare(P *p, uint32_t *anno, P **extra) { (void) anno, (void) extra; return p; }
    int32_t nh_offset(P *p) const { return O::has_network_header(p) ? O::network_header_offset(p) : -1; }
    bool primary(int32_t port, uint32_t aux) const { (void) port, (void) aux; return true; }
    P *make_packet(clk_element *e, uint32_t key) const { return take_glue_packet(e, key, 0); }
    template <class S> int finish(S &t, Routed<P> &r, P **out) { (void) t; return pass(r, out); }
    template <class S> void end_of_batch(S &t) { (void) t; }

    static int pass(Routed<P> &r, P **out)
    {
        if (!r.p)
            return -1;
        if (r.port == CLK_PORT_KILL) {
            O::kill(r.p);
            return -1;
        }
        *out = r.p;
        return r.port;
    }
    // a packet of the glue's bytes, with `headroom` (0: the default); on
    // failure the glue's copy is released and 0 returned
    static P *take_glue_packet(clk_element *e, uint32_t key, uint32_t headroom)
    {
        int64_t n = clk_element_take_packet(e, key, 0, 0);
        P *q = n >= 0 ? O::make(headroom, (uint32_t) n) : 0;
        if (!q) {
            unsigned char one;
            if (n >= 0)
                clk_element_take_packet(e, key, &one, 1);
            return 0;
        }
        clk_element_take_packet(e, key, O::data(q), (size_t) n);
        return q;
    }
};

// CheckIPHeader / CheckIPHeader2 (checkipheader.cc:161-226): a passing
// packet gets its network header set, is trimmed to ip_len, and carries
// ip_dst as its destination annotation (213-223).
template <class P, class O> struct CheckIPHeaderClass : Plain<P, O> {
    enum { may_write = 0, chain_last = 0, chain_head_only = 0, pass_effects = 1 };
    uint32_t offset = 0;            // OFFSET (the glue parsed it)
    template <class S> int finish(S &t, Routed<P> &r, P **out)
    {
        (void) t;
        P *p = r.p;
        if (!p || r.port != CLK_PORT_OUT0)
            return Plain<P, O>::pass(r, out);
        const uint8_t *ip = O::data(p) + offset;
        O::set_ip_header(p, ip, (uint32_t) (ip[0] & 0xF) << 2);
        if (O::length(p) > r.len)                  // r.len: the length after the trim
            O::take(p, O::length(p) - r.len);
        uint32_t dst;
        memcpy(&dst, ip + 16, 4);
        O::set_dst_ip_anno(p, dst);
        *out = p;
        return 0;
    }
};

// IPInputCombo (ipinputcombo.cc:66-140): Paint (71), Strip(14) (74), the
// CheckIPHeader steps (125-132); a bad packet is killed (134-139).
template <class P, class O> struct IPInputComboClass : Plain<P, O> {
    enum { may_write = 0, chain_last = 0, chain_head_only = 0, pass_effects = 1 };
    uint32_t color = 0;             // COLOR
    int32_t nh_offset(P *p) const { (void) p; return 14; }   // the header sits behind the 14 bytes Strip removes
    template <class S> int finish(S &t, Routed<P> &r, P **out)
    {
        (void) t;
        P *p = r.p;
        if (!p)
            return -1;
        if (r.port != CLK_PORT_OUT0) {
            O::kill(p);
            return -1;
        }
        O::set_paint(p, color);
        O::pull(p, 14);
        const uint8_t *ip = O::data(p);
        O::set_ip_header(p, ip, (uint32_t) (ip[0] & 0xF) << 2);
        if (O::length(p) > r.len)
            O::take(p, O::length(p) - r.len);
        uint32_t dst;
        memcpy(&dst, ip + 16, 4);
        O::set_dst_ip_anno(p, dst);
        *out = p;
        return 0;
    }
};

// SetIPChecksum / SetUDPChecksum / SetTCPChecksum: uniqueify first
// (setipchecksum.cc:77, setudpchecksum.cc:40, settcpchecksum.cc:47); the
// results route as the glue decided (output 1: SetUDPChecksum's fragments).
template <class P, class O> struct SetChecksumClass : Plain<P, O> {
    enum { may_write = 1, chain_last = 0, chain_head_only = 0, pass_effects = 0 };
    P *prepare(P *p, uint32_t *anno, P **extra) { (void) anno, (void) extra; return O::uniqueify(p); }
};

// DecIPTTL (decipttl.cc:45-77): writable only when the TTL is decremented.
template <class P, class O> struct DecIPTTLClass : Plain<P, O> {
    enum { may_write = 1, chain_last = 0, chain_head_only = 0, pass_effects = 0 };
    P *prepare(P *p, uint32_t *anno, P **extra)
    {
        (void) anno, (void) extra;
        if (O::has_network_header(p) && O::network_header(p)[8] > 1)
            return O::uniqueify(p);
        return p;
    }
};

// IPGWOptions (ipgwoptions.cc:53-172): only packets with options are made
// writable (167-169); a parameter problem goes to output 1 with its pointer
// as the ICMP annotation (161-165).
template <class P, class O> struct IPGWOptionsClass : Plain<P, O> {
    enum { may_write = 1, chain_last = 0, chain_head_only = 0, pass_effects = 0 };
    P *prepare(P *p, uint32_t *anno, P **extra)
    {
        (void) anno, (void) extra;
        if (O::has_network_header(p) && (O::network_header(p)[0] & 0xF) > 5)
            return O::uniqueify(p);
        return p;
    }
    template <class S> int finish(S &t, Routed<P> &r, P **out)
    {
        (void) t;
        if (r.p && r.port == CLK_PORT_OUT1)
            O::set_icmp_paramprob(r.p, r.aux);
        return Plain<P, O>::pass(r, out);
    }
};

// FixIPSrc (fixipsrc.cc:52-72): a packet with the annotation is made
// writable, rewritten by the glue, and its annotation cleared (59).
template <class P, class O> struct FixIPSrcClass : Plain<P, O> {
    enum { may_write = 1, chain_last = 0, chain_head_only = 0, pass_effects = 1 };
    P *prepare(P *p, uint32_t *anno, P **extra)
    {
        (void) extra;
        if (O::fix_ip_src(p) && O::has_network_header(p)) {
            *anno = CLK_ANNO_FIX_IP_SRC;
            return O::uniqueify(p);
        }
        return p;
    }
    template <class S> int finish(S &t, Routed<P> &r, P **out)
    {
        (void) t;
        if (r.p && (r.anno & CLK_ANNO_FIX_IP_SRC))
            O::clear_fix_ip_src(r.p);
        return Plain<P, O>::pass(r, out);
    }
};

// IPOutputCombo (ipoutputcombo.cc:44-205), ports 0-4.  Alone or at the head
// of a chain its prepare() takes the PaintTee clone as the packet arrives;
// as a chain member after the head, the glue keeps the bytes as the packet
// reaches it and the clone comes as a new packet (aux CLK_AUX_CLONE | key).
template <class P, class O> struct IPOutputComboClass : Plain<P, O> {
    enum { may_write = 1, chain_last = 0, chain_head_only = 0, pass_effects = 1, extra_results = 1 };
    uint32_t color = 0;             // COLOR
    P *prepare(P *p, uint32_t *anno, P **extra)
    {
        // DropBroadcasts (50-53): the glue kills it, no clone, no copy
        if (O::broadcast_or_multicast(p)) {
            *anno = CLK_ANNO_BCAST;
            return p;
        }
        *anno = CLK_ANNO_PAINT(O::paint(p)) | (O::fix_ip_src(p) ? CLK_ANNO_FIX_IP_SRC : 0);
        // PaintTee (56-57): the clone is taken before anything is rewritten;
        // uniqueify (60) then gives the original bytes of its own
        P *clone = O::paint(p) == color ? O::clone(p) : 0;
        P *q = O::uniqueify(p);
        if (!q) {
            // the copy failed (out of memory): the reference has pushed the
            // clone already; it leaves on output 1, the packet is gone
            *extra = clone;
            return 0;
        }
        *extra = clone;
        return q;
    }
    bool primary(int32_t port, uint32_t aux) const { (void) port; return !(aux & CLK_AUX_CLONE); }
    // a chain member's clone: the bytes the glue kept, the IP header at data()
    P *make_packet(clk_element *e, uint32_t aux) const
    {
        P *q = Plain<P, O>::take_glue_packet(e, aux & ~CLK_AUX_CLONE, 0);
        if (q)
            O::set_ip_header(q, O::data(q), (uint32_t) (O::data(q)[0] & 0xF) << 2);
        return q;
    }
    template <class S> int finish(S &t, Routed<P> &r, P **out)
    {
        (void) t;
        if (r.extra && !r.p) {                     // the PaintTee clone, before its packet
            *out = r.extra;
            return 1;
        }
        if (r.made) {                              // the same, kept by a chain: the packet's
            if (r.parent)                          // annotations as it reached this member
                O::copy_annotations(r.made, r.parent);
            *out = r.made;
            return 1;
        }
        P *p = r.p;
        if (!p)
            return -1;
        if (r.port == CLK_PORT_KILL) {             // DropBroadcasts
            O::kill(p);
            if (r.extra)
                O::kill(r.extra);
            return -1;
        }
        if (r.port == CLK_PORT_OUT2)               // ipgw_send_error (202-204)
            O::set_icmp_paramprob(p, r.aux);
        else if (r.anno & CLK_ANNO_FIX_IP_SRC)     // the FixIPSrc step (169-170)
            O::clear_fix_ip_src(p);
        *out = p;
        return r.port;                             // 0, 2, 3 (TTL expired), 4 (longer than the MTU)
    }
};

// IPFragmenter (ipfragmenter.cc:88-171).
template <class P, class O> struct IPFragmenterClass : Plain<P, O> {
    enum { may_write = 1, chain_last = 1, chain_head_only = 0, pass_effects = 0, extra_results = 1 };
    uint32_t mtu = 0, headroom = 0; // MTU / HEADROOM
    P *prepare(P *p, uint32_t *anno, P **extra)
    {
        (void) anno, (void) extra;
        // push (163-166): only a packet longer than the MTU is fragmented,
        // made writable first (106-109)
        if (O::network_length(p) > (int) mtu)
            return O::uniqueify(p);
        return p;
    }
    bool primary(int32_t port, uint32_t aux) const { (void) port; return aux == 0; }
    // a fragment after the first (129-159): the glue's bytes in a new packet
    // with HEADROOM; its annotations come in finish()
    P *make_packet(clk_element *e, uint32_t key) const
    {
        P *q = Plain<P, O>::take_glue_packet(e, key, headroom);
        if (q)
            O::set_ip_header(q, O::data(q), (uint32_t) (O::data(q)[0] & 0xF) << 2);
        return q;
    }
    template <class S> int finish(S &t, Routed<P> &r, P **out)
    {
        if (r.made) {                              // annotations of the original (153)
            if (r.parent)
                O::copy_annotations(r.made, r.parent);
            *out = r.made;
            return 0;
        }
        P *p = r.p;
        if (!p)
            return -1;
        if (r.port == CLK_PORT_OUT0 && r.len < O::length(p)) {
            // the first fragment: its header is already rewritten in the
            // packet (112-120); a clone cut to its length leaves first
            // (121-124), the original stays for the annotations of the
            // fragments that follow
            P *first = O::clone(p);
            if (t.frag_parent)
                O::kill(t.frag_parent);
            t.frag_parent = p;
            if (!first)
                return -1;
            O::take(first, O::length(p) - r.len);
            *out = first;
            return 0;
        }
        return Plain<P, O>::pass(r, out);          // untouched, or DF with HONOR_DF (96-102)
    }
    template <class S> void end_of_batch(S &t)
    {
        if (t.frag_parent) {                       // p->kill() after its fragments (169)
            O::kill(t.frag_parent);
            t.frag_parent = 0;
        }
    }
};

} // namespace hipcore
#endif
