// hip-parity-ip.click -- CheckIPHeader on the CPU (the reference element)
// and on the GPU (HIPCheckIPHeader, hipparity.cc) for every packet; the two
// output streams are compared packet by packet (data, length, header
// offsets: comparepackets.cc) and must not differ.
//
//   click -h cmp.diffs -h cmp.diff_details -h cpu.drops -h gpu.drops hip-parity-ip.click
//   expected: cmp.diffs 0, cpu.drops == gpu.drops
//
// Needs a Click built with the hip group and WITHOUT skipping the CPU
// elements (click_integration/README.md, "Parity builds").  The source is
// conf/fake-iprouter.click's frame (lines 38-50); RandomBitErrors flips
// bits so both checks drop the same packets (randomerror.hh).

src :: InfiniteSource(DATA \<
  00 00 c0 ae 67 ef  00 00 00 00 00 00  08 00
  45 00 00 28  00 00 00 00  40 11 77 c3  01 00 00 01  02 00 00 02
  13 69 13 69  00 14 d6 41
  55 44 50 20  70 61 63 6b  65 74 21 0a  04 00 00 00  01 00 00 00
  01 00 00 00  00 00 00 00  00 80 04 08  00 80 04 08  53 53 00 00
  53 53 00 00  05 00 00 00  00 10 00 00  01 00 00 00  54 53 00 00
  54 e3 04 08  54 e3 04 08  d8 01 00 00
>, LIMIT 600000)
  -> Strip(14)
  -> RandomBitErrors(0.0005)
  -> t :: Tee(2);

t[0] -> cpu :: CheckIPHeader(DETAILS true) -> q0 :: Queue(1000000) -> [0]cmp :: ComparePackets(TIMESTAMP false);
t[1] -> gpu :: HIPCheckIPHeader(DETAILS true, BATCH 65536, LATENCY 1) -> q1 :: Queue(1000000) -> [1]cmp;
cmp[0] -> d0 :: Discard(ACTIVE false);
cmp[1] -> d1 :: Discard(ACTIVE false);

// ComparePackets pairs the two streams as its outputs are pulled, and takes
// an input that is empty at that moment as "more packets in" the other: the
// GPU side arrives a batch at a time, so the sinks start only once the
// source is done and both queues hold every packet that passed
Script(label src, wait 5ms, goto src $(lt $(src.count) 600000),
       label gpu, wait 5ms, goto gpu $(ne $(q0.length) $(q1.length)),
       write d0.active true, write d1.active true,
       label cmp, wait 5ms, goto cmp $(gt $(add $(q0.length) $(q1.length)) 0),
       stop);
