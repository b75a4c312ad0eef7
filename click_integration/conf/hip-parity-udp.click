// hip-parity-udp.click -- SetUDPChecksum and CheckUDPHeader, CPU and GPU side
// by side, each pair compared packet by packet (comparepackets.cc).
//
//   click -h setcmp.diffs -h chkcmp.diffs -h cpucheck.drops -h gpucheck.drops hip-parity-udp.click
//   expected: both diffs 0, equal drop counts
//
// Set: the GPU writes the same uh_sum bytes as setudpchecksum.cc:64-66 into
// its own copy of every packet.  Check: the packets are checksummed once,
// bits are flipped (randomerror.hh) BEFORE the Tee, so both checks see the
// same corrupted packets and must drop the same ones.  UDPIPEncap gets
// CHECKSUM false explicitly (udpipencap.cc:47,54,69 leaves it
// uninitialised otherwise).

RandomSeed(1);
src :: RandomSource(LENGTH 1472, LIMIT 200000)
  -> UDPIPEncap(10.0.0.1, 1234, 192.168.1.2, 5678, CHECKSUM false)
  -> ts :: Tee(3);

ts[0] -> SetUDPChecksum -> s0 :: Queue(1000000) -> [0]setcmp :: ComparePackets(TIMESTAMP false);
ts[1] -> HIPSetUDPChecksum(BATCH 16384) -> s1 :: Queue(1000000) -> [1]setcmp;
setcmp[0] -> d0 :: Discard(ACTIVE false);
setcmp[1] -> d1 :: Discard(ACTIVE false);

ts[2] -> SetUDPChecksum -> RandomBitErrors(0.00001) -> tc :: Tee(2);
tc[0] -> cpucheck :: CheckUDPHeader -> c0 :: Queue(1000000) -> [0]chkcmp :: ComparePackets(TIMESTAMP false);
tc[1] -> gpucheck :: HIPCheckUDPHeader(BATCH 16384) -> c1 :: Queue(1000000) -> [1]chkcmp;
chkcmp[0] -> d2 :: Discard(ACTIVE false);
chkcmp[1] -> d3 :: Discard(ACTIVE false);

// the sinks start once the source is done and the GPU side has caught up
// (ComparePackets takes a momentarily empty input as a missing packet)
Script(label src, wait 5ms, goto src $(lt $(src.count) 200000),
       label gpu, wait 5ms, goto gpu $(or $(ne $(s0.length) $(s1.length)) $(ne $(c0.length) $(c1.length))),
       write d0.active true, write d1.active true, write d2.active true, write d3.active true,
       label cmp, wait 5ms, goto cmp $(gt $(add $(s0.length) $(s1.length) $(c0.length) $(c1.length)) 0),
       stop);
