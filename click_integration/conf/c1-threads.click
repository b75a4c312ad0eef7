// c1-threads.click -- c1-forward.click's forwarding path fed by two sources
// on two RouterThreads (click -j 2): every GPU-backed element is pushed into
// from both threads at once (ELEMENT_MT_SAFE, setipchecksum.cc:105), so the
// adapter keeps a state per thread, each delivering on its own thread.
// Written for this repository.
//
//   click -j 2 c1-threads.click [LIMIT=n] [BURST=b] -h out.count
//   every packet is forwarded: out.count == 2 * LIMIT

define($LIMIT 300000, $BURST 32);

src0 :: InfiniteSource(DATA \<
  00 00 c0 ae 67 ef  00 00 00 00 00 00  08 00
  45 00 00 28  00 00 00 00  40 11 77 c3  01 00 00 01  02 00 00 02
  13 69 13 69  00 14 d6 41
  55 44 50 20  70 61 63 6b  65 74 21 0a  04 00 00 00  01 00 00 00
  01 00 00 00  00 00 00 00  00 80 04 08  00 80 04 08  53 53 00 00
  53 53 00 00  05 00 00 00  00 10 00 00  01 00 00 00  54 53 00 00
  54 e3 04 08  54 e3 04 08  d8 01 00 00
>, LIMIT $LIMIT, BURST $BURST);
src1 :: InfiniteSource(DATA \<
  00 00 c0 ae 67 ef  00 00 00 00 00 00  08 00
  45 00 00 28  00 00 00 00  40 11 77 c3  01 00 00 01  02 00 00 02
  13 69 13 69  00 14 d6 41
  55 44 50 20  70 61 63 6b  65 74 21 0a  04 00 00 00  01 00 00 00
  01 00 00 00  00 00 00 00  00 80 04 08  00 80 04 08  53 53 00 00
  53 53 00 00  05 00 00 00  00 10 00 00  01 00 00 00  54 53 00 00
  54 e3 04 08  54 e3 04 08  d8 01 00 00
>, LIMIT $LIMIT, BURST $BURST);
StaticThreadSched(src0 0, src1 1);

lookup :: StaticIPLookup(18.26.4.24/32 0, 18.26.7.1/32 0,
                         18.26.4.0/24 1, 18.26.7.0/24 2,
                         0.0.0.0/0 18.26.4.1 1);

src0 -> Paint(2) -> Strip(14) -> chk :: CheckIPHeader(INTERFACES 18.26.4.1/24 18.26.7.1/24);
src1 -> Paint(2) -> Strip(14) -> chk;
chk -> lookup;

lookup[1] -> DropBroadcasts
          -> paint :: PaintTee(1)
          -> gw :: IPGWOptions(18.26.4.24)
          -> FixIPSrc(18.26.4.24)
          -> ttl :: DecIPTTL
          -> frag :: IPFragmenter(300)
          -> EtherEncap(0x0800, 00:00:c0:ae:67:ef, 00:00:c0:4f:71:ef)
          -> out :: AverageCounter
          -> Discard;

lookup[0] -> Discard;
lookup[2] -> Discard;
chk[1] -> bad :: AverageCounter -> Discard;
paint[1] -> Discard;
gw[1] -> Discard;
ttl[1] -> Discard;
frag[1] -> Discard;

// the sources stop themselves at LIMIT; the router stops once every packet
// has left (the GPU elements hold a runcount reference while they hold any)
Script(label w, wait 10ms, goto w $(lt $(add $(out.count) $(bad.count)) $(mul 2 $LIMIT)), stop);
