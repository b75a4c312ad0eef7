// hip-parity-mix.click -- five more reference elements beside their GPU
// versions (hipparity.cc) in one router, over the IPv4 packets of a pcap
// file; each pair's outputs are compared packet by packet
// (comparepackets.cc) and counted:
//   CheckTCPHeader, SetTCPChecksum(FIXOFF true), SetIPChecksum,
//   CheckIPHeader2, IPInputCombo (over the Ethernet frames), IPOutputCombo
//   (MTU 576, painted with its COLOR: output 0 compared, outputs 1-4 counted).
//
//   click hip-parity-mix.click IN=mix.pcap N=<records> -h tcpchk.diffs ...
//   expected: every *.diffs 0, every cpu/gpu counter pair equal
//
// tests/test_gpu_click.py writes the file: TCP (header offsets 0-15, options,
// payloads), UDP, ICMP and other protocols, IP options, bad checksums,
// ip_len above and below the captured length, a few short packets.
// MarkIPHeader sets the network and transport header annotations from
// ip_hl without dropping anything.  Each GPU element holds its packets up
// to LATENCY 1 ms, so the sinks start 300 ms after the source is done.

define($IN mix.pcap, $N 0);

src :: FromDump($IN, STOP false);
src -> fr :: Tee(2);
fr[0] -> Strip(14) -> MarkIPHeader -> t :: Tee(9);

t[0] -> CheckTCPHeader -> k0 :: Counter -> Queue(1000000) -> [0]tcpchk :: ComparePackets(TIMESTAMP false);
t[1] -> HIPCheckTCPHeader(BATCH 4096, LATENCY 1) -> k1 :: Counter -> Queue(1000000) -> [1]tcpchk;
t[2] -> SetTCPChecksum(FIXOFF true) -> k2 :: Counter -> Queue(1000000) -> [0]tcpset :: ComparePackets(TIMESTAMP false);
t[3] -> HIPSetTCPChecksum(FIXOFF true, BATCH 4096, LATENCY 1) -> k3 :: Counter -> Queue(1000000) -> [1]tcpset;
t[4] -> SetIPChecksum -> k4 :: Counter -> Queue(1000000) -> [0]ipset :: ComparePackets(TIMESTAMP false);
t[5] -> HIPSetIPChecksum(BATCH 4096, LATENCY 1) -> k5 :: Counter -> Queue(1000000) -> [1]ipset;
t[6] -> CheckIPHeader2 -> k6 :: Counter -> Queue(1000000) -> [0]ip2 :: ComparePackets(TIMESTAMP false);
t[7] -> HIPCheckIPHeader2(BATCH 4096, LATENCY 1) -> k7 :: Counter -> Queue(1000000) -> [1]ip2;
fr[1] -> cb :: Tee(2);
t[8] -> Paint(1) -> GetIPAddress(16) -> oc :: Tee(2);
oc[0] -> co :: IPOutputCombo(1, 10.0.0.1, 576);
oc[1] -> go :: HIPIPOutputCombo(1, 10.0.0.1, 576, BATCH 4096, LATENCY 1);
co[0] -> o0 :: Counter -> Queue(1000000) -> [0]outc :: ComparePackets(TIMESTAMP false);
go[0] -> o1 :: Counter -> Queue(1000000) -> [1]outc;
co[1] -> o2 :: Counter -> Discard;  go[1] -> o3 :: Counter -> Discard;
co[2] -> o4 :: Counter -> Discard;  go[2] -> o5 :: Counter -> Discard;
co[3] -> o6 :: Counter -> Discard;  go[3] -> o7 :: Counter -> Discard;
co[4] -> o8 :: Counter -> Discard;  go[4] -> o9 :: Counter -> Discard;
cb[0] -> IPInputCombo(1) -> k8 :: Counter -> Queue(1000000) -> [0]combo :: ComparePackets(TIMESTAMP false);
cb[1] -> HIPIPInputCombo(1, BATCH 4096, LATENCY 1) -> k9 :: Counter -> Queue(1000000) -> [1]combo;

tcpchk[0] -> s0 :: Discard(ACTIVE false);  tcpchk[1] -> s1 :: Discard(ACTIVE false);
tcpset[0] -> s2 :: Discard(ACTIVE false);  tcpset[1] -> s3 :: Discard(ACTIVE false);
ipset[0] -> s4 :: Discard(ACTIVE false);   ipset[1] -> s5 :: Discard(ACTIVE false);
ip2[0] -> s6 :: Discard(ACTIVE false);     ip2[1] -> s7 :: Discard(ACTIVE false);
combo[0] -> s8 :: Discard(ACTIVE false);   combo[1] -> s9 :: Discard(ACTIVE false);
outc[0] -> s10 :: Discard(ACTIVE false);   outc[1] -> s11 :: Discard(ACTIVE false);

Script(label src, wait 5ms, goto src $(lt $(src.count) $N),
       wait 300ms,
       write s0.active true, write s1.active true, write s2.active true, write s3.active true,
       write s4.active true, write s5.active true, write s6.active true, write s7.active true,
       write s8.active true, write s9.active true, write s10.active true, write s11.active true,
       wait 300ms,
       stop);
