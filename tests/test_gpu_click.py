"""Click itself, on the GPU: the userlevel driver built with the GPU element
group (tools/click_scratch_build.sh) runs graphs whose elements are the
reference's class names, and its results are compared with the stock build's
(the reference's CPU elements) on the same graph and input:

- the parity graphs (click_integration/conf/hip-parity-{ip,udp}.click):
  Tee -> {CPU element, GPU element} -> ComparePackets, diffs == 0
  (elements/test/comparepackets.cc:150-152) and equal drop counts;
- config 1's forwarding path (c1-forward.click: fake-iprouter's frame,
  600000 forwarded as iprouter-01 expects, every counter equal);
- the same element sequence over fuzzed frames from a pcap file, every
  output port written to a pcap file (c1-parity-dump.click), the files of the
  drop-in build byte-identical to the stock build's: IP options rewritten by
  IPGWOptions, bad headers, expiring TTLs, fragments.

Skipped when the binaries were not built."""
import os

import struct

import numpy as np
import pytest

from tests import click_run, fuzz, oracle_lib

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not (click_run.binary("cpu") and click_run.binary("dropin") and
                                      click_run.binary("parity")),
                                 reason="Click binaries not built (tools/click_scratch_build.sh)")]

MY_IP = 0x18041A12                              # 18.26.4.24, IPGWOptions' / FixIPSrc's address


@pytest.fixture(scope="module", autouse=True)
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def test_parity_graph_ip():
    rc, h, err = click_run.run("parity", "hip-parity-ip.click",
                               handlers=("cmp.diffs", "cmp.diff_details", "cpu.drops", "gpu.drops"), timeout=120)
    assert rc == 0, err
    assert h["cmp.diffs"] == "0", (h, err)
    assert h["cpu.drops"] == h["gpu.drops"] and int(h["cpu.drops"]) > 0, h


def test_parity_graph_udp():
    rc, h, err = click_run.run("parity", "hip-parity-udp.click",
                               handlers=("setcmp.diffs", "chkcmp.diffs", "setcmp.diff_details", "chkcmp.diff_details",
                                         "cpucheck.drops", "gpucheck.drops"),
                               timeout=120)
    assert rc == 0, err
    assert h["setcmp.diffs"] == "0" and h["chkcmp.diffs"] == "0", (h, err)
    assert h["cpucheck.drops"] == h["gpucheck.drops"] and int(h["cpucheck.drops"]) > 0, h


def inet_cksum(b):
    """RFC 1071 checksum of bytes (the value to store; test helper)."""
    if len(b) & 1:
        b += b"\0"
    s = sum(struct.unpack(">%dH" % (len(b) // 2), b))
    s = (s & 0xFFFF) + (s >> 16)
    s += s >> 16
    return ~s & 0xFFFF


def icmp_pcap(path, seed, n):
    """Ethernet frames of IPv4 packets for CheckICMPHeader's rules
    (checkicmpheader.cc:89-138): ICMP types of each length class at lengths
    around its bound (8, 36, exactly 20, exactly 8), other types at any
    length including under 8, NOP options before the ICMP header on some,
    a bad checksum on some, bytes past ip_len on some, a few not ICMP."""
    rng = np.random.default_rng(seed)
    bounds = {3: 36, 4: 36, 5: 36, 11: 36, 12: 36, 13: 20, 14: 20, 15: 8, 16: 8}
    types = list(bounds) + [0, 8, 9, 10, 17, 18, 30, 255]
    frames = []
    for k in range(n):
        t = types[int(rng.integers(len(types)))]
        b = bounds.get(t, 8)
        ilen = int(rng.choice([b - 1, b, b + 1, b + int(rng.integers(2, 120)), int(rng.integers(0, 8))]))
        ilen = max(ilen, 0)
        hl = 5 if rng.random() < 0.85 else int(rng.integers(6, 9))
        icmp = bytearray(rng.integers(0, 256, ilen, dtype=np.uint8).tobytes())
        if ilen >= 1:
            icmp[0] = t
        if ilen >= 4:
            icmp[2:4] = b"\0\0"
            if rng.random() < 0.85:
                icmp[2:4] = struct.pack(">H", inet_cksum(bytes(icmp)))
        ip = bytearray(4 * hl)
        ip[0] = 0x40 | hl
        ip[2:4] = struct.pack(">H", 4 * hl + ilen)
        ip[8] = 64
        ip[9] = 1 if rng.random() < 0.95 else 17
        ip[12:16] = bytes([10, 0, 0, 1])
        ip[16:20] = bytes([10, 0, 0, 2])
        ip[20:] = b"\x01" * (4 * hl - 20)               # NOPs
        ip[10:12] = struct.pack(">H", inet_cksum(bytes(ip)))
        tail = rng.integers(0, 256, int(rng.integers(1, 6)), dtype=np.uint8).tobytes() if rng.random() < 0.1 else b""
        eth = bytes.fromhex("0000c0ae67ef") + bytes(6) + b"\x08\x00"
        frames.append(eth + bytes(ip) + bytes(icmp) + tail)
    click_run.write_pcap(path, frames)


def test_parity_graph_icmp(tmp_path):
    """CheckICMPHeader's length classes and checksum on the GPU against the
    reference element in one router: ComparePackets sees no difference, and
    both drop the same packets for the same reasons (parity pinned by Click
    itself, where the reference's tests hold no ICMP bytes)."""
    n = 30000
    icmp_pcap(str(tmp_path / "icmp.pcap"), 23, n)
    rc, h, err = click_run.run("parity", "hip-parity-icmp.click", {"IN": str(tmp_path / "icmp.pcap"), "N": n},
                               handlers=("cmp.diffs", "cmp.diff_details", "cpu.drops", "gpu.drops",
                                         "cpu.drop_details", "gpu.drop_details"), timeout=120)
    assert rc == 0, err
    assert h["cmp.diffs"] == "0", (h, err)
    assert h["cpu.drops"] == h["gpu.drops"] and 0 < int(h["cpu.drops"]) < n, h
    said = {ln.split(" :: ")[0]: ln.split("failed: ")[-1] for ln in err.splitlines() if "header check failed" in ln}
    assert said.get("cpu") and said.get("cpu") == said.get("gpu"), err    # the first drop's reason
    # the reference's drop_details counters start uninitialised
    # (checkicmpheader.cc:58, new atomic_uint32_t[NREASONS]): only the GPU
    # element's are read, each reason seen, summing to the drops
    det = [int(ln.split()[0]) for ln in h["gpu.drop_details"].splitlines()]
    assert len(det) == 3 and all(x > 0 for x in det) and sum(det) == int(h["gpu.drops"]), h


def mix_pcap(path, seed, n):
    """Ethernet frames of fuzzed IPv4 packets for hip-parity-mix.click: TCP
    (th_off 0-15, payload 0-600 B), UDP, ICMP and protocol 47, ip_hl 5-7 with
    NOP options, the IP, TCP and UDP checksums right on most, ip_len equal to,
    above or below the captured length, some packets shorter than 40 B."""
    rng = np.random.default_rng(seed)
    frames = []
    for k in range(n):
        proto = int(rng.choice([6, 6, 6, 17, 1, 47]))
        hl = 5 if rng.random() < 0.8 else int(rng.integers(6, 8))
        if proto == 6:
            doff = int(rng.integers(5, 11)) if rng.random() < 0.9 else int(rng.integers(0, 16))
            l4 = bytearray(rng.integers(0, 256, max(4 * doff, 20) + int(rng.integers(0, 600)), dtype=np.uint8).tobytes())
            l4[12] = (doff << 4) | (l4[12] & 0x0F)
            sum_at = 16
        elif proto == 17:
            l4 = bytearray(rng.integers(0, 256, 8 + int(rng.integers(0, 400)), dtype=np.uint8).tobytes())
            l4[4:6] = struct.pack(">H", len(l4))
            sum_at = 6
        else:
            l4 = bytearray(rng.integers(0, 256, int(rng.integers(0, 200)), dtype=np.uint8).tobytes())
            sum_at = None
        ip = bytearray(4 * hl)
        ip[0] = 0x40 | hl
        total = 4 * hl + len(l4)
        ip[2:4] = struct.pack(">H", total)
        ip[6] = 0x40 if rng.random() < 0.5 else 0
        ip[8] = int(rng.integers(1, 255))
        ip[9] = proto
        ip[12:16] = bytes([10, 0, int(rng.integers(0, 4)), int(rng.integers(1, 255))])
        ip[16:20] = bytes([192, 168, int(rng.integers(0, 4)), int(rng.integers(1, 255))])
        ip[20:] = b"\x01" * (4 * hl - 20)
        if sum_at is not None and len(l4) >= sum_at + 2:
            l4[sum_at:sum_at + 2] = b"\0\0"
            if rng.random() < 0.85:
                ph = bytes(ip[12:20]) + bytes([0, proto]) + struct.pack(">H", len(l4))
                c = inet_cksum(ph + bytes(l4))
                l4[sum_at:sum_at + 2] = struct.pack(">H", c if (c or proto != 17) else 0xFFFF)
        r = rng.random()
        if r < 0.05:                                          # ip_len above the packet
            ip[2:4] = struct.pack(">H", total + int(rng.integers(1, 40)))
        elif r < 0.10 and len(l4) > 4:                        # ip_len below the packet
            ip[2:4] = struct.pack(">H", total - int(rng.integers(1, min(len(l4), 40))))
        ip[10:12] = b"\0\0"
        if rng.random() < 0.9:
            ip[10:12] = struct.pack(">H", inet_cksum(bytes(ip)))
        pkt = bytes(ip) + bytes(l4)
        if rng.random() < 0.03:                               # short packets
            pkt = pkt[:4 * hl + int(rng.integers(0, 20))]     # (MarkIPHeader needs the IP header)
        eth = bytes.fromhex("0000c0ae67ef") + bytes(6) + b"\x08\x00"
        frames.append(eth + pkt)
    click_run.write_pcap(path, frames)


MIX_PAIRS = ("tcpchk", "tcpset", "ipset", "ip2", "combo", "outc")


def test_parity_graph_mix(tmp_path):
    """CheckTCPHeader, SetTCPChecksum(FIXOFF), SetIPChecksum, CheckIPHeader2,
    IPInputCombo and IPOutputCombo beside their GPU versions in one router
    over 20000 fuzzed packets: every pair's outputs equal packet by packet,
    in number, bytes and header offsets (ComparePackets), IPOutputCombo's
    other four outputs equal in number."""
    n = 20000
    mix_pcap(str(tmp_path / "mix.pcap"), 29, n)
    hs = (tuple("%s.diffs" % c for c in MIX_PAIRS) + tuple("k%d.count" % k for k in range(10))
          + tuple("o%d.count" % k for k in range(10)))
    rc, h, err = click_run.run("parity", "hip-parity-mix.click", {"IN": str(tmp_path / "mix.pcap"), "N": n},
                               handlers=hs, timeout=120)
    assert rc == 0, err[-2000:]
    for c in MIX_PAIRS:
        assert h["%s.diffs" % c] == "0", (c, h)
    for k in range(0, 10, 2):
        assert h["k%d.count" % k] == h["k%d.count" % (k + 1)], (k, h)
        assert 0 < int(h["k%d.count" % k]) <= n, (k, h)
    assert sum(int(h["k%d.count" % k]) < n for k in range(0, 10, 2)) >= 4, h   # drops seen on four of the five
    for k in range(0, 10, 2):                            # IPOutputCombo's five outputs
        assert h["o%d.count" % k] == h["o%d.count" % (k + 1)], (k, h)
    assert all(int(h["o%d.count" % k]) > 0 for k in (0, 2, 6, 8)), h   # forwarded/fragments, PaintTee, TTL, DF


C1_HANDLERS = ("out.count", "local.count", "other.count", "bad.count", "redirect.count", "gw.drops", "ttl.drops",
               "frag.fragments", "frag.drops", "chk.drops")


@pytest.mark.parametrize("burst", [1, 32])
def test_dropin_config1_forward(burst):
    """fake-iprouter's 600000 frames through the drop-in's GPU elements:
    all forwarded, every counter as the stock elements'."""
    d = {"BURST": burst}
    rc, gpu, err = click_run.run("dropin", "c1-forward.click", d, C1_HANDLERS, timeout=120)
    assert rc == 0, err
    rc, cpu, err2 = click_run.run("cpu", "c1-forward.click", d, C1_HANDLERS, timeout=120)
    assert rc == 0, err2
    assert gpu["out.count"] == "600000", (gpu, err)
    assert gpu == cpu


def fuzzed_pcap(path, seed, n):
    """Ethernet frames of fuzzed IPv4 packets for the forwarding path:
    record-route options (timestamps need the wall clock), TTLs 0-2, flipped
    header bits, truncations, lengths past IPFragmenter(300)'s MTU."""
    from tests.test_gpu_chain import no_timestamps
    rng = np.random.default_rng(seed)
    a3, o3, c3, _ = fuzz.gw_batch(rng, n, MY_IP, max_total=1400)
    no_timestamps(a3, o3, c3)
    for i in range(0, n, 7):
        o, c = int(o3[i]), int(c3[i])
        if c >= 20:
            a3[o + 8] = i % 3
            oracle_lib.batch("set_ip", a3[o:o + c], 1, fixed_len=c)
    for i in range(3, n, 11):
        if c3[i] > 12:
            a3[int(o3[i]) + 12] ^= 0x02
    frames = []
    for i in range(n):
        eth = bytes.fromhex("0000c0ae67ef") + rng.integers(0, 256, 6, dtype=np.uint8).tobytes() + b"\x08\x00"
        frames.append(eth + a3[int(o3[i]):int(o3[i]) + int(c3[i])].tobytes())
    click_run.write_pcap(path, frames)


OUTS = ("fwd", "local", "other", "bad", "redirect", "gwopt", "ttl", "frag")


def test_dropin_config1_pcap_bytes(tmp_path):
    """The forwarding path over 20000 fuzzed frames: every output's pcap
    file from the drop-in build equals the stock build's byte for byte."""
    fuzzed_pcap(str(tmp_path / "in.pcap"), 61, 20000)
    said = {}
    for mode in ("cpu", "dropin"):
        d = tmp_path / mode
        d.mkdir()
        rc, _, err = click_run.run(mode, "c1-parity-dump.click", {"IN": str(tmp_path / "in.pcap"), "OUT": str(d)},
                                   timeout=120)
        assert rc == 0, (mode, err)
        said[mode] = err
    assert said["dropin"] == said["cpu"]            # the elements' chatter (first drop, ...)
    seen = 0
    for o in OUTS:
        a = click_run.read_pcap(str(tmp_path / "cpu" / (o + ".pcap")))
        b = click_run.read_pcap(str(tmp_path / "dropin" / (o + ".pcap")))
        assert len(a) == len(b), (o, len(a), len(b))
        for k, (x, y) in enumerate(zip(a, b)):
            assert x == y, (o, k, x[:3], y[:3], x[3].hex(), y[3].hex())
        seen += len(a) > 0
    assert seen >= 4                                # forwarded, bad headers, option problems, TTLs


@pytest.mark.skipif(not (click_run.binary("cpu-mt") and click_run.binary("dropin-mt")),
                    reason="multithreaded Click binaries not built (tools/click_scratch_build.sh cpu-mt / dropin-mt)")
def test_dropin_two_router_threads():
    """click -j 2 (--enable-user-multithread): two sources on two
    RouterThreads push into the same GPU-backed elements at once; the
    adapter keeps a state per thread (glue element, context, held packets,
    Task moved to the thread).  Every packet forwarded, every counter as the
    stock build's."""
    hs = ("out.count", "bad.count", "chk.drops", "gw.drops", "ttl.drops", "frag.drops", "frag.fragments")
    rc, gpu, err = click_run.run("dropin-mt", "c1-threads.click", {"LIMIT": 300000}, hs, timeout=120, threads=2)
    assert rc == 0, err
    rc, cpu, err2 = click_run.run("cpu-mt", "c1-threads.click", {"LIMIT": 300000}, hs, timeout=120, threads=2)
    assert rc == 0, err2
    assert gpu["out.count"] == "600000", (gpu, err)
    assert gpu == cpu
