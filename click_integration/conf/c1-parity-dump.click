// c1-parity-dump.click -- c1-forward.click's element sequence over frames
// read from a pcap file, every output written to a pcap file of its own, so
// a stock Click (the CPU elements) and a drop-in build (the GPU elements
// under the same names) can be compared byte for byte, timestamps included
// (FromDump keeps each record's timestamp, ToDump writes it back).
//
//   click c1-parity-dump.click IN=frames.pcap OUT=dir
//   writes dir/{fwd,bad,redirect,gwopt,ttl,frag,local,other}.pcap
//
// Used by tests/test_gpu_click.py with fuzzed frames: IP options (record
// route), bad checksums and lengths, expiring TTLs, packets longer than the
// MTU.

define($IN frames.pcap, $OUT .);

src :: FromDump($IN, STOP true);

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
          -> ToDump($OUT/fwd.pcap, ENCAP IP);

lookup[0] -> ToDump($OUT/local.pcap, ENCAP IP);
lookup[2] -> ToDump($OUT/other.pcap, ENCAP IP);
chk[1] -> ToDump($OUT/bad.pcap, ENCAP IP);
paint[1] -> ToDump($OUT/redirect.pcap, ENCAP IP);
gw[1] -> ToDump($OUT/gwopt.pcap, ENCAP IP);
ttl[1] -> ToDump($OUT/ttl.pcap, ENCAP IP);
frag[1] -> ToDump($OUT/frag.pcap, ENCAP IP);
