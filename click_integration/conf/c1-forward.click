// c1-forward.click -- BASELINE config 1's forwarding work as one graph:
// fake-iprouter's frame (conf/fake-iprouter.click:38-50: 14 B Ethernet,
// 20 B IP, UDP to 2.0.0.2) through the element sequence its packets take
// from eth1 to eth0 (Paint, Strip, CheckIPHeader, the route, DropBroadcasts,
// PaintTee, IPGWOptions, FixIPSrc, DecIPTTL, IPFragmenter, EtherEncap),
// counted where they leave.  Written for this repository; the ARP side,
// the idle interface and the ICMP error generators, which no such packet
// reaches, are left out, and the interface queue is a Counter pushed to
// directly (a GPU element hands its results out a batch at a time; a
// Queue(200) in front of a pulling sink would drop most of a batch).
//
//   click c1-forward.click [LIMIT=n] [BURST=b] -h out.count -h out.rate
//
// The same file runs on a stock Click (the CPU elements) and on one built
// with the GPU group as a drop-in (tools/click_scratch_build.sh dropin):
// the element names are the reference's.  Every packet is forwarded:
// out.count == LIMIT.

define($LIMIT 600000, $BURST 1);

src :: InfiniteSource(DATA \<
  00 00 c0 ae 67 ef  00 00 00 00 00 00  08 00
  45 00 00 28  00 00 00 00  40 11 77 c3  01 00 00 01  02 00 00 02
  13 69 13 69  00 14 d6 41
  55 44 50 20  70 61 63 6b  65 74 21 0a  04 00 00 00  01 00 00 00
  01 00 00 00  00 00 00 00  00 80 04 08  00 80 04 08  53 53 00 00
  53 53 00 00  05 00 00 00  00 10 00 00  01 00 00 00  54 53 00 00
  54 e3 04 08  54 e3 04 08  d8 01 00 00
>, LIMIT $LIMIT, BURST $BURST, STOP true);

lookup :: StaticIPLookup(18.26.4.24/32 0, 18.26.7.1/32 0,
                         18.26.4.0/24 1, 18.26.7.0/24 2,
                         0.0.0.0/0 18.26.4.1 1);

src -> Paint(2)
    -> Strip(14)
    -> chk :: CheckIPHeader(INTERFACES 18.26.4.1/24 18.26.7.1/24)
    -> lookup;

lookup[1] -> DropBroadcasts
          -> paint :: PaintTee(1)
          -> gw :: IPGWOptions(18.26.4.24)
          -> FixIPSrc(18.26.4.24)
          -> ttl :: DecIPTTL
          -> frag :: IPFragmenter(300)
          -> EtherEncap(0x0800, 00:00:c0:ae:67:ef, 00:00:c0:4f:71:ef)
          -> out :: AverageCounter
          -> Discard;

lookup[0] -> local :: Counter -> Discard;
lookup[2] -> other :: Counter -> Discard;
chk[1] -> bad :: Counter -> Discard;
paint[1] -> redirect :: Counter -> Discard;
gw[1] -> Discard;
ttl[1] -> Discard;
frag[1] -> Discard;
