/*
 * click_amd_elements.h -- C ABI of the batched, GPU-backed checksum elements.
 *
 * The host-side element glue (click_amd/host/elements.{hh,cc}, C++) keeps
 * the semantics of Click's element classes -- configuration keywords,
 * output-0/output-1/kill routing, `drops`/`drop_details` handlers and the
 * click_chatter messages -- while the checksum work runs on the GPU through
 * include/click_amd_cksum.h.  Packets are HOST packets (Click's Packet
 * data(), as a DPDK/pcap source hands them over): push() gathers their
 * bytes into a pinned struct-of-arrays staging batch, flush() copies the
 * batch to HBM, runs the element kernel, copies verdicts/checksums back,
 * writes Set results into the host packets and routes every packet.
 *
 * Click's Element API is one packet at a time (element.cc:2891-2972); the
 * Click-side adapter that turns push(port, Packet*) into these calls --
 * holding packets until flush, flushing on batch-full, timer and
 * router stop -- is in INTEGRATION.md.
 *
 * Classes (same names and keywords as the reference):
 *   CheckIPHeader   INTERFACES, BADSRC, GOODDST, OFFSET, VERBOSE, DETAILS,
 *                   CHECKSUM; legacy positional [BADSRC,] OFFSET
 *                                      (elements/ip/checkipheader.cc:87-141)
 *   CheckIPHeader2  as CheckIPHeader, never checksums (checkipheader2.cc)
 *   SetIPChecksum   (no keywords)      (elements/ip/setipchecksum.cc)
 *   CheckUDPHeader  VERBOSE, DETAILS   (elements/tcpudp/checkudpheader.cc:50-64)
 *   SetUDPChecksum  (no keywords)      (elements/tcpudp/setudpchecksum.cc)
 *   CheckTCPHeader  VERBOSE, DETAILS   (elements/tcpudp/checktcpheader.cc:50-64)
 *   SetTCPChecksum  [FIXOFF]           (elements/tcpudp/settcpchecksum.cc:36-42)
 *   CheckICMPHeader VERBOSE, DETAILS   (elements/icmp/checkicmpheader.cc:49-60)
 *   DecIPTTL        ACTIVE, MULTICAST  (elements/ip/decipttl.cc:36-41); handlers
 *                   drops, active; expired packets to output 1 or killed
 *   IPInputCombo    COLOR, [BADSRC,] INTERFACES, BADSRC, GOODDST
 *                   (elements/ip/ipinputcombo.cc:38-64): CheckIPHeader at
 *                   OFFSET 14, bad packets killed; the result length is the
 *                   length after Strip(14) and the ip_len trim, and the
 *                   adapter paints COLOR ("color" handler) and pulls 14 bytes
 *   IPGWOptions     MYADDR, [OTHERADDRS] (elements/ip/ipgwoptions.cc:38-48);
 *                   handler drops; parameter problems to output 1 (aux =
 *                   ICMP_PARAMPROB_ANNO)
 *   FixIPSrc        IPADDR             (elements/ip/fixipsrc.cc:40-49); acts
 *                   on packets pushed with CLK_ANNO_FIX_IP_SRC (the adapter
 *                   clears that annotation)
 *   IPOutputCombo   COLOR, IPADDR, MTU (elements/ip/ipoutputcombo.cc:34-41);
 *                   ports 0-4: broadcast/multicast killed, a painted clone to
 *                   1 (aux CLK_AUX_CLONE), parameter problems to 2 (aux =
 *                   offset), expired TTL to 3, longer than MTU to 4
 *   IPFragmenter    MTU, [HONOR_DF], [VERBOSE], HEADROOM
 *                   (elements/ip/ipfragmenter.cc:41-55); handlers drops,
 *                   fragments; each fragment beyond the first is a new
 *                   packet (aux = its key for clk_element_take_packet)
 * plus glue keywords BATCH (packets per GPU batch, default 65536), DEVICE
 * (the GPU, see clk_element_create; handler "device") and
 * ZEROCOPY (bool, default false): the kernels read -- and the Set /
 * rewriting elements write -- the packets where they lie, in host memory
 * registered with clk_host_register, instead of gathering them into a
 * staging batch and copying it to HBM.
 * Elements that rewrite header bytes (IPGWOptions, FixIPSrc, IPOutputCombo,
 * IPFragmenter) write them back into `data` at flush().
 */
#ifndef CLICK_AMD_ELEMENTS_H
#define CLICK_AMD_ELEMENTS_H
#include <stdint.h>
#include <stddef.h>
#include "click_amd_cksum.h"
#ifdef __cplusplus
extern "C" {
#endif

typedef struct clk_element clk_element;

/* Where a flushed packet goes (the reference's routing). */
enum clk_port {
    CLK_PORT_OUT0 = 0,        /* output(0).push(p)                          */
    CLK_PORT_OUT1 = 1,        /* output(1).push(p) (drop port / SetUDP short) */
    CLK_PORT_OUT2 = 2,        /* IPOutputCombo: parameter problem           */
    CLK_PORT_OUT3 = 3,        /* IPOutputCombo: TTL expired                 */
    CLK_PORT_OUT4 = 4,        /* IPOutputCombo: longer than the MTU         */
    CLK_PORT_KILL = -1,       /* p->kill()                                   */
    CLK_PORT_NEXT = 8         /* chains (clk_chain_report_passes): the packet
                                 goes on to the next member                  */
};

/* name: the element's name in messages (Click's name(); NULL = class name);
 * noutputs: how many outputs are connected (1 or 2; IPOutputCombo 5).
 * ctx: the context (device + stream) the element's batches run on; NULL
 * makes the element create (and destroy) its own, on the GPU its DEVICE
 * keyword names (default 0).  With a context, DEVICE must be the
 * context's device.  DEVICE past the gfx950 devices present: CLK_ENODEV.
 * Returns CLK_EINVAL with clk_last_error(ctx) (clk_last_error(NULL) when
 * ctx is NULL) set on a configure error, worded like the reference's
 * ErrorHandler messages.                                                  */
int clk_element_create(clk_ctx *ctx, const char *class_name, const char *config,
                       const char *name, int noutputs, clk_element **out);
int clk_element_destroy(clk_element *e);
/* Configuration check without a GPU: the class's keywords parsed as
 * clk_element_create parses them (DEVICE's value checked for form only),
 * nothing allocated.  CLK_SUCCESS, or CLK_EINVAL with clk_last_error(NULL)
 * set as clk_element_create would set it -- so an adapter reports a bad
 * keyword at configure time, as the reference element does, on a host
 * whatever its GPUs.                                                      */
int clk_element_check_config(const char *class_name, const char *config, const char *name, int noutputs);
/* Why the element's last flush / push failed.  A flush that fails (a HIP
 * runtime error, or a kernel's internal fault report) routes nothing: the
 * batch stays staged, exactly as pushed, and the next flush retries it
 * (except a ZEROCOPY batch of a rewriting element: clk_element_abandon). */
const char *clk_element_last_error(clk_element *e);

/* Stage one host packet.  data/length = Packet::data()/length();
 * nh_offset = network_header_offset() (-1 = no network header: the IP
 * elements then use data(), as SetIPChecksum does, setipchecksum.cc:78).
 * Set elements write their result into `data` at flush(), so for them the
 * packet memory must stay valid until then; the other elements copy what
 * their kernel reads at the push (unless clk_element_hold_packets).
 * Returns 1 when the batch is full and should be flushed, 0 otherwise,
 * < 0 on error.                                                            */
int clk_element_push(clk_element *e, uint8_t *data, uint32_t length, int32_t nh_offset,
                     uint64_t token);

/* on != 0: the caller keeps every packet it pushes valid and unchanged
 * until the packet's result is popped (the Click adapter holds its Packets
 * so), and the element may then gather a long span (>= 256 B) of a packet
 * pushed alone at the flush, with the batch, rather than in the push.
 * Default off.  CLK_EINVAL for a null element.                            */
int clk_element_hold_packets(clk_element *e, int on);

/* Stage a burst of n host packets (an rte_eth_rx_burst-style array of
 * packet pointers; fromdpdkdevice.cc:98-115); token of packet k is
 * first_token + k.  nh_offsets may be NULL (= -1 for all).  Flushes by
 * itself whenever the batch fills.  Returns 0 or < 0 on error.           */
int clk_element_push_burst(clk_element *e, uint8_t *const *datas, const uint32_t *lengths,
                           const int32_t *nh_offsets, uint64_t first_token, uint32_t n);

/* Packet annotations the output-path elements read (push_anno's `anno`). */
#define CLK_ANNO_FIX_IP_SRC 0x1u       /* FIX_IP_SRC_ANNO (packet_anno.hh)           */
#define CLK_ANNO_BCAST 0x2u            /* packet_type_anno() BROADCAST or MULTICAST  */
#define CLK_ANNO_PAINT(c) (((uint32_t)(c) & 0xFFu) << 8)   /* PAINT_ANNO            */

/* clk_element_push with the packet's annotations (CLK_ANNO_*). */
int clk_element_push_anno(clk_element *e, uint8_t *data, uint32_t length, int32_t nh_offset,
                          uint32_t anno, uint64_t token);

/* clk_element_push_anno with the packet's transport header annotation:
 * th_offset = Packet::transport_header_offset(), -2 when the packet has
 * none, -1 unknown (taken to be at ip_hl).  The L4 elements read the
 * segment where the annotation says, as the reference's udp_header() /
 * tcp_header() / icmp_header() do (checkudpheader.cc:87,
 * checktcpheader.cc:88, checkicmpheader.cc:85, setudpchecksum.cc:45,
 * settcpchecksum.cc:49), and the lengths' ip_hl from the header bytes: the
 * two differ when ip_hl changed after the header was marked.  Such a packet
 * is staged as a canonical copy (not with ZEROCOPY: CLK_EINVAL); SetTCPChecksum
 * kills a packet with no transport header (settcpchecksum.cc:53).  The other
 * classes ignore th_offset.                                               */
int clk_element_push_th(clk_element *e, uint8_t *data, uint32_t length, int32_t nh_offset,
                        int32_t th_offset, uint32_t anno, uint64_t token);

/* Run the staged batch on the GPU and route it (synchronous).  Results are
 * appended to the element's result queue in push order.                  */
int clk_element_flush(clk_element *e);

/* Double-buffered flush: route the batch still on the GPU (if any), launch
 * the staged one, and return without waiting, so the caller stages the
 * next batch while this one runs (push_burst flushes this way).  Results
 * of the launched batch arrive at the next flush / flush_async.           */
int clk_element_flush_async(clk_element *e);

/* Give up on the element's staged and in-flight packets (an adapter's retry
 * limit after flushes keep failing): each is routed as CLK_PORT_KILL, in
 * push order, and counted by the "lost" handler.  Returns how many.  A
 * ZEROCOPY batch of an element that rewrites packets in place and is not
 * idempotent (DecIPTTL, IPGWOptions, IPOutputCombo, IPFragmenter) is
 * abandoned this way by the failing flush itself: its kernel may already
 * have written the host packets, so it is never run twice.               */
uint64_t clk_element_abandon(clk_element *e);

/* Count e's once-only chatter together with `with`'s: the first drop's
 * reason of the Check elements and IPInputCombo (checkipheader.cc:145-147,
 * ipinputcombo.cc:135-137), SetUDPChecksum's fragment warning
 * (setudpchecksum.cc:52-58, once per router there) and IPFragmenter's first
 * five DF lines (ipfragmenter.cc:96-102).  The Click adapter keeps one glue
 * element per RouterThread; sharing makes them speak once, as the one
 * reference element does.  CLK_EINVAL for a null element. */
int clk_element_share_messages(clk_element *e, const clk_element *with);

/* Pop up to `cap` results: token, port (enum clk_port) and the packet's
 * new length (CheckIPHeader trims to ip_len, checkipheader.cc:216-217;
 * otherwise unchanged).  Returns the number popped.                        */
uint64_t clk_element_results(clk_element *e, uint64_t *tokens, int32_t *ports,
                             uint32_t *lengths, uint64_t cap);

/* clk_element_results plus a per-result auxiliary word: the
 * ICMP_PARAMPROB_ANNO offset of a parameter problem (IPGWOptions port 1,
 * IPOutputCombo port 2), CLK_AUX_CLONE for IPOutputCombo's painted clone
 * (a clone of the packet as pushed, before any rewrite), or for
 * IPFragmenter the key of a new fragment packet (0 = the pushed packet
 * itself, now the first fragment).                                         */
#define CLK_AUX_CLONE 0x80000000u
uint64_t clk_element_results_aux(clk_element *e, uint64_t *tokens, int32_t *ports,
                                 uint32_t *lengths, uint32_t *aux, uint64_t cap);

/* Copy out (and release) new packet `key` an element made (IPFragmenter's
 * fragments after the first): its bytes start at the IP header.  Returns
 * the packet length, or < 0 for an unknown key; copies min(len, cap).
 * buf == NULL only queries the length (the packet is kept).               */
int64_t clk_element_take_packet(clk_element *e, uint32_t key, uint8_t *buf, size_t cap);

/* Handler text, as Click's read handlers print it ("drops",
 * "drop_details", plus the glue's "batches", "packets", "gpu_ns").
 * Returns the full length (may exceed cap-1; output is NUL-terminated).   */
int clk_element_read_handler(clk_element *e, const char *handler, char *buf, size_t cap);

/* Pop the click_chatter lines the element produced, '\n'-separated. */
int clk_element_take_messages(clk_element *e, char *buf, size_t cap);

/* ---- chains: consecutive elements on one device-resident batch ----------
 * members[k+1] is connected to members[k]'s output 0, all in one thread and
 * on one context, all ZEROCOPY or none; an element with extra results after its
 * packet (IPFragmenter) only as the last member.  The members stay the
 * caller's (configuration, handlers, counters: each counts what it routed,
 * as if it had run alone); the chain never uses their own staging.  A packet
 * pushed into the chain is staged once (the bytes any member reads); a flush
 * copies the batch to the GPU once, runs member k's kernel over the packets
 * members 0..k-1 passed on output 0, copies the rewritten bytes back once and
 * routes each packet once, through every member it reaches, in order.  Each
 * result names the member it leaves and that member's output (enum
 * clk_port); a member's extra results (IPOutputCombo's clone before the
 * packet, IPFragmenter's fragments after it) come with their member; new
 * packets are taken with clk_element_take_packet(members[member], aux).
 * IPOutputCombo as member k > 0: its PaintTee clone (ipoutputcombo.cc:56-57)
 * must be the packet as it reaches the member, which the caller no longer
 * has once the chain copied the members' rewrites back; the chain keeps
 * those bytes before member k's kernel runs and the clone result names them:
 * aux = CLK_AUX_CLONE | key, the bytes from clk_element_take_packet(
 * members[k], key) (at member 0, aux = CLK_AUX_CLONE: the caller clones the
 * packet as it pushes it, as for the element alone).
 * The GPU analogue of click-xform's combos (ipinputcombo.cc:66-140,
 * ipoutputcombo.cc:44-205): one gather, one H2D, one D2H and one routing
 * pass per packet instead of one per element.  Each member's results come
 * in push order, as its outputs see them, and a packet's results at member
 * k before those at k+1; results of different members may interleave (a
 * packet a member decides on the host goes on to the next member at once,
 * while that member has no packet before it waiting for the GPU).  A flush
 * that fails at member k has routed what left the chain before k (their
 * bytes written back); the packets at k stay in the chain and the next
 * flush resumes there (a push retries that flush first; while it still
 * fails the push is refused with CLK_EHIP) -- except after
 * the kernel of a member that is not idempotent (DecIPTTL, IPGWOptions,
 * IPOutputCombo, IPFragmenter) was launched: its packets are then killed
 * (results with CLK_PORT_KILL, counted by its "lost" handler), never run
 * twice.                                                                   */
typedef struct clk_chain clk_chain;
int clk_chain_create(clk_element *const *members, int n, clk_chain **out);
int clk_chain_destroy(clk_chain *c);
const char *clk_chain_last_error(clk_chain *c);
int clk_chain_push_anno(clk_chain *c, uint8_t *data, uint32_t length, int32_t nh_offset, uint32_t anno,
                        uint64_t token);   /* 1: the batch is full, flush it */
int clk_chain_push_burst(clk_chain *c, uint8_t *const *datas, const uint32_t *lengths,
                         const int32_t *nh_offsets, uint64_t first_token, uint32_t n);
int clk_chain_flush(clk_chain *c);
/* Double-buffered flush (as clk_element_flush_async): launch the staged
 * batch's first GPU step, finish the batch flushed before it (its results
 * are handed out), move the staged one on to its next GPU step, and return;
 * pushes go to the other batch while it runs.  clk_chain_flush routes
 * everything pushed.  Results come out batch by batch, in push order of the
 * batches; a failure anywhere leaves the chain to be flushed again (or
 * abandoned) before it takes packets.                                      */
int clk_chain_flush_async(clk_chain *c);
/* A GPU that keeps failing: every packet still in the chain (staged, or at
 * the member a failed flush stopped at) becomes a CLK_PORT_KILL result at
 * the member it has reached, counted by that member's "lost" handler; so
 * does a packet routed out whose rewritten bytes could not be copied back
 * (results are only handed out once their bytes are back).  Returns the
 * packets killed.                                                          */
uint64_t clk_chain_abandon(clk_chain *c);
/* Bit k of `members` set: member k also reports each packet it passes on to
 * the next member (port CLK_PORT_NEXT, length as the next member sees it),
 * in its place among its results -- so a host that applies each element's
 * own side effects (the Click adapter: network header, trim, Strip,
 * annotations) can apply them member by member; ~0: every member.  A
 * packet a pass rule lets through a member unchanged (the member decides it
 * on the host and changes nothing) is not reported.                        */
int clk_chain_report_passes(clk_chain *c, uint64_t members);
uint64_t clk_chain_results(clk_chain *c, uint64_t *tokens, int32_t *members, int32_t *ports,
                           uint32_t *lengths, uint32_t *aux, uint64_t cap);
/* Host seconds the chain has spent, by phase: push (staging, and the packet
 * into member 0 and on through the members that decide it on the host),
 * rebuilding the batch of a member a failed flush stopped at, the members'
 * GPU round trips, (unused), the flush's H2D of the batch (pieces go while
 * it fills), D2H of the rewritten bytes, routing after each GPU step (with
 * the next members' descriptors and host decisions), copy-back into the
 * packets.  Returns 8.                                                     */
int clk_chain_stats(clk_chain *c, double *sec, int n);

#ifdef __cplusplus
}
#endif
#endif /* CLICK_AMD_ELEMENTS_H */
