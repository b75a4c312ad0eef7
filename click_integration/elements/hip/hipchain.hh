// -*- c-basic-offset: 4 -*-
#ifndef CLICK_HIPCHAIN_HH
#define CLICK_HIPCHAIN_HH
/*
 * hipchain.hh -- which GPU-backed elements of a router configuration run as
 * one clk_chain, and what a chain's head does for its members.  Click-
 * independent: templates over a graph trait G, so the SAME rules run in
 * Click (hipbatch.cc's ClickGraph: Router connections, Element::cast) and in
 * tests/native/chain_form_test.cc (a graph of plain structs), where they are
 * checked on the CPU against the configurations they must and must not join.
 *
 * The rules: a GPU-backed element's output 0 pushing into the input 0 of a
 * GPU-backed element that nothing else pushes into, both with CHAIN true, on
 * the same DEVICE, makes the second a member of the first one's chain -- and
 * so on down output 0.  A chain_last class (IPFragmenter: its fragments are
 * extra results) ends a chain; a chain_head_only class never joins one, it
 * starts its own (no shipped class is one now: IPOutputCombo's PaintTee
 * clone, ipoutputcombo.cc:50-60, is taken by the glue from the bytes as the
 * packet reaches it when it is a member after the head).  At most CHAIN_MAX members (the pass report
 * is a 64-bit member mask, clk_chain_report_passes).  The first element of a
 * run that is not itself a member heads it; every other element runs alone.
 *
 * The graph trait G (N = G::Node, a handle; N() = none):
 *   N push_next(N x)      the GPU-backed element that x's output 0 pushes
 *                         into at its input 0; none when output 0 is missing
 *                         or pull, goes to another input, or into an element
 *                         that is not GPU-backed
 *   N sole_upstream(N y)  the GPU-backed element whose output is the only one
 *                         feeding y's input 0 in push; none otherwise (no
 *                         input, pull, several outputs, not GPU-backed)
 *   bool chain_conf(N)    CHAIN
 *   int device(N)         DEVICE (-1: per thread)
 *   bool may_write(N), chain_last(N), chain_head_only(N), pass_effects(N)
 *                         the class traits of hipclasses.hh
 */
#include <stdint.h>
#include "click_amd_elements.h"

namespace hipcore {

enum { CHAIN_MAX = 64 };

// The element after x in x's chain, if it can join one x is in
template <class G>
typename G::Node chain_next(G &g, typename G::Node x)
{
    typedef typename G::Node N;
    if (!g.chain_conf(x))
	return N();
    N y = g.push_next(x);
    if (!y || y == x || !g.chain_conf(y) || g.device(y) != g.device(x) || g.chain_head_only(y))
	return N();
    return g.sole_upstream(y) == x ? y : N();
}

// y is a member of the chain of the element before it (which runs it)
template <class G>
bool chain_member(G &g, typename G::Node y)
{
    typename G::Node u = g.sole_upstream(y);
    return u && !g.chain_last(u) && chain_next(g, u) == y;
}

// The chain e runs: [e] and the members after it (only [e] when e is a
// member of an earlier chain, or heads none).  V: push_back / clear / size.
template <class G, class V>
void form_chain(G &g, typename G::Node e, V &chain)
{
    typedef typename G::Node N;
    chain.clear();
    chain.push_back(e);
    if (!g.chain_conf(e) || chain_member(g, e))
	return;
    N x = e, y;
    while ((int) chain.size() < CHAIN_MAX && !g.chain_last(x) && (y = chain_next(g, x)) && y != e) {
	chain.push_back(y);
	x = y;
    }
}

// A member after the head may write the packet: the head makes it writable
template <class G, class V>
bool chain_writes(G &g, const V &chain)
{
    for (int m = 1; m < (int) chain.size(); m++)
	if (g.may_write(chain[m]))
	    return true;
    return false;
}

// The members whose finish() changes a packet they pass on
// (clk_chain_report_passes)
template <class G, class V>
uint64_t chain_report(G &g, const V &chain)
{
    uint64_t mask = 0;
    for (int m = 0; m < (int) chain.size() && m < CHAIN_MAX; m++)
	if (g.pass_effects(chain[m]))
	    mask |= uint64_t(1) << m;
    return mask;
}

// The head readies a packet for every member, after its own prepare():
// writable if any member may write (the reference makes it writable in the
// element that writes it: setipchecksum.cc:77, decipttl.cc:59), and the
// annotations the members read staged with it -- FixIPSrc's and
// IPOutputCombo's FIX_IP_SRC, IPOutputCombo's paint and packet type
// (fixipsrc.cc:52-56, ipoutputcombo.cc:50-60).  O: hipclasses.hh's packet
// operations trait.  0 when the copy fails (the packet is gone).
template <class P, class O>
P *chain_ready(P *p, bool writes, uint32_t *anno)
{
    if (writes && !(p = O::uniqueify(p)))
	return 0;
    *anno |= (O::fix_ip_src(p) ? CLK_ANNO_FIX_IP_SRC : 0u)
	| (O::broadcast_or_multicast(p) ? CLK_ANNO_BCAST : 0u)
	| CLK_ANNO_PAINT(O::paint(p));
    return p;
}

}   // namespace hipcore
#endif
