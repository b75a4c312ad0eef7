// hip-parity-icmp.click -- CheckICMPHeader on the CPU (the reference
// element) and on the GPU (HIPCheckICMPHeader, hipparity.cc) for every
// packet of a pcap file; the two output streams are compared packet by
// packet (comparepackets.cc) and must not differ, and both must drop the
// same packets for the same reasons.
//
//   click hip-parity-icmp.click IN=icmp.pcap N=<records> \
//         -h cmp.diffs -h cpu.drop_details -h gpu.drop_details
//   expected: cmp.diffs 0, equal drop details
//
// tests/test_gpu_click.py writes the file: ICMP messages of every type
// class checkicmpheader.cc:96-132 tells apart, at lengths around each class's
// bound, with options before the ICMP header, bad checksums, trailing bytes
// past ip_len, and packets that are not ICMP.  MarkIPHeader sets the
// network and transport header annotations from ip_hl, as CheckIPHeader
// would, without dropping anything.

define($IN icmp.pcap, $N 0);

src :: FromDump($IN, STOP false);
src -> Strip(14) -> MarkIPHeader -> t :: Tee(2);

t[0] -> cpu :: CheckICMPHeader(DETAILS true) -> q0 :: Queue(1000000) -> [0]cmp :: ComparePackets(TIMESTAMP false);
t[1] -> gpu :: HIPCheckICMPHeader(DETAILS true, BATCH 4096, LATENCY 1) -> q1 :: Queue(1000000) -> [1]cmp;
cmp[0] -> d0 :: Discard(ACTIVE false);
cmp[1] -> d1 :: Discard(ACTIVE false);

// the sinks start once the source is done and the GPU side has caught up
// (ComparePackets takes a momentarily empty input as a missing packet)
Script(label src, wait 5ms, goto src $(lt $(src.count) $N),
       label gpu, wait 5ms, goto gpu $(ne $(add $(q0.length) $(cpu.drops)) $(add $(q1.length) $(gpu.drops))),
       write d0.active true, write d1.active true,
       label cmp, wait 5ms, goto cmp $(gt $(add $(q0.length) $(q1.length)) 0),
       stop);
