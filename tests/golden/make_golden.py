#!/usr/bin/env python3
"""Extract golden vectors for the checksum path from the reference's own files.

Run once in the development container (it reads /root/reference, which does
not exist on the GPU box); the output, tests/golden/golden_vectors.json, is
committed.  Only DATA is extracted: packet bytes and the expected results the
reference's tests state.  Every vector records where it came from and how its
expectation is pinned:

  pin = "reference-output"   the bytes were produced by Click itself and the
                             reference test expects them (e.g. IPFragmenter
                             rewrote ip_sum with click_in_cksum,
                             elements/ip/ipfragmenter.cc:120,150)
  pin = "reference-accepts"  the reference test pushes the packet through a
                             checking element and expects it to pass
  pin = "captured"           checksum fields written by the capturing host's
                             stack in a pcap the reference's tests hold
  pin = "survey-ref-run"     value measured by running the reference's
                             lib/in_cksum.c during the survey
  pin = "tcpdump-ok"         tcpdump printed "[tcp sum ok]" for Click's output
                             on a packet with these IP options
                             (test/analysis/FromIPSummaryDump-ipopt-01.clicktest)

Usage: python3 tests/golden/make_golden.py [--reference /root/reference]
"""
import argparse
import json
import os
import re
import struct

HERE = os.path.dirname(os.path.abspath(__file__))


def hexbytes(s):
    return bytes.fromhex(re.sub(r"[^0-9a-fA-F]", "", s))


def line_of(text, needle):
    return text[: text.index(needle)].count("\n") + 1


def clicktest_sections(path):
    text = open(path, encoding="latin-1").read()
    return text


def vec(name, source, pin, op, l3, expect, caplen=None, arg=None, note=None):
    v = {"name": name, "source": source, "pin": pin, "op": op,
         "l3": l3.hex(), "caplen": len(l3) if caplen is None else caplen,
         "expect": expect}
    if arg is not None:
        v["arg"] = arg
    if note:
        v["note"] = note
    return v


def le16(b, off):
    return struct.unpack_from("<H", b, off)[0]


def zero_field(b, off):
    b = bytearray(b)
    b[off:off + 2] = b"\0\0"
    return bytes(b)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--out", default=os.path.join(HERE, "golden_vectors.json"))
    args = ap.parse_args()
    R = args.reference
    out = []
    frag_cases = []

    # 1. IPFragmenter-01/02: input packets with IP options (ip_hl = 6) whose
    #    IP and TCP checksums the reference accepts, and the fragment headers
    #    IPFragmenter wrote with click_in_cksum.
    for tname in ("IPFragmenter-01", "IPFragmenter-02"):
        rel = "test/ip/%s.clicktest" % tname
        text = clicktest_sections(os.path.join(R, rel))
        m = re.search(r'DATA "\\<([0-9a-fA-F ]+)>"', text)
        pkt = hexbytes(m.group(1))
        src = "%s:%d" % (rel, line_of(text, m.group(0)))
        hl = (pkt[0] & 0xF) * 4
        # CheckIPHeader accepts it (IPFragmenter-02 pipes it through CheckIPHeader)
        out.append(vec(tname + "-in-ip-check", src, "reference-accepts", "check_ip", pkt, 0))
        out.append(vec(tname + "-in-ip-set", src, "reference-accepts", "set_ip", pkt, le16(pkt, 10),
                       note="stored ip_sum reproduced by SetIPChecksum"))
        out.append(vec(tname + "-in-ip-cksum", src, "reference-accepts", "in_cksum", pkt[:hl], 0))
        out.append(vec(tname + "-in-tcp-check", src, "reference-accepts", "check_tcp", pkt, 0,
                       note="ip_hl=6: pseudo-header via click_in_cksum_pseudohdr_hard"))
        out.append(vec(tname + "-in-tcp-set", src, "reference-accepts", "set_tcp", pkt, le16(pkt, hl + 16),
                       arg=0))
        exp = re.search(r"%expect stderr\n(.*?)\n\n", text, re.S).group(1)
        # the whole case for the fragmenter: input, configuration, every
        # fragment Click printed (Print(CONTENTS true): length | bytes)
        fm = re.search(r"IPFragmenter\((\d+), HONOR_DF (true|false)\)", text)
        frag_cases.append({"name": tname, "source": "%s:%d" % (rel, line_of(text, fm.group(0))),
                           "pin": "reference-output", "in": pkt.hex(), "mtu": int(fm.group(1)),
                           "honor_df": fm.group(2) == "true",
                           "fragments": [hexbytes(ln.split("|")[1]).hex() for ln in exp.strip().splitlines()]})
        for k, line in enumerate(exp.strip().splitlines()):
            n, hx = line.split("|")
            frag = hexbytes(hx)
            assert len(frag) == int(n)
            fsrc = "%s:%d" % (rel, line_of(text, line))
            fhl = (frag[0] & 0xF) * 4
            # IPFragmenter set ip_sum = click_in_cksum(header) (ipfragmenter.cc:120,150)
            out.append(vec("%s-frag%d-ip-set" % (tname, k), fsrc, "reference-output", "set_ip",
                           zero_field(frag, 10), le16(frag, 10)))
            out.append(vec("%s-frag%d-ip-cksum-zeroed" % (tname, k), fsrc, "reference-output", "in_cksum",
                           zero_field(frag, 10)[:fhl], le16(frag, 10)))
            out.append(vec("%s-frag%d-ip-check" % (tname, k), fsrc, "reference-output", "check_ip", frag, 0))

    # 2. conf/fake-iprouter.click: the BASELINE config-1 frame.  Every copy
    #    passes CheckIPHeader (test/userlevel/iprouter-01.clicktest expects
    #    600000 forwarded).  Its UDP checksum field is as the file states.
    rel = "conf/fake-iprouter.click"
    text = open(os.path.join(R, rel), encoding="latin-1").read()
    m = re.search(r"InfiniteSource\(DATA \\<(.*?)>", text, re.S)
    body = "\n".join(re.sub(r"//.*", "", ln) for ln in m.group(1).splitlines())
    frame = hexbytes(body)
    src = "%s:%d" % (rel, line_of(text, m.group(0)))
    l3 = frame[14:]
    out.append(vec("fake-iprouter-ip-check", src, "reference-accepts", "check_ip", l3, 0))
    out.append(vec("fake-iprouter-ip-set", src, "reference-accepts", "set_ip", zero_field(l3, 10), le16(l3, 10)))
    out.append(vec("fake-iprouter-udp-check", src, "captured", "check_udp", l3, 0,
                   note="uh_sum d641 as written in the config; verified through the reference object in the survey"))
    out.append(vec("fake-iprouter-udp-set", src, "captured", "set_udp", zero_field(l3, 20 + 6), le16(l3, 26)))

    # 3. test/analysis/IPSummaryDump-02.clicktest holds a 431-byte pcap
    #    (dump.trace): four captured TCP/IPv4 frames and one hand-made frame
    #    with zero checksums.
    rel = "test/analysis/IPSummaryDump-02.clicktest"
    data = open(os.path.join(R, rel), "rb").read()
    hdr = b"%file +431 dump.trace\n"
    i = data.index(hdr) + len(hdr)
    blob = data[i:i + 431]
    src = "%s:%d" % (rel, data[:i].count(b"\n"))
    # the file itself, for the pcap ingest tests (tests/test_ingest.py)
    with open(os.path.join(HERE, "dump_trace.pcap"), "wb") as f:
        f.write(blob)
    p = 24
    k = 0
    while p < len(blob):
        _, _, cap, _ = struct.unpack_from("<IIII", blob, p)
        p += 16
        fr = blob[p:p + cap]
        p += cap
        l3 = fr[14:]
        hl = (l3[0] & 0xF) * 4
        if le16(l3, 10) != 0:
            out.append(vec("dumptrace%d-ip-check" % k, src, "captured", "check_ip", l3, 0))
            out.append(vec("dumptrace%d-ip-set" % k, src, "captured", "set_ip", zero_field(l3, 10), le16(l3, 10)))
            out.append(vec("dumptrace%d-tcp-check" % k, src, "captured", "check_tcp", l3, 0))
            out.append(vec("dumptrace%d-tcp-set" % k, src, "captured", "set_tcp", zero_field(l3, hl + 16),
                           le16(l3, hl + 16), arg=0))
        else:
            # hand-made frame, all checksums zero: header words are nonzero,
            # so the zero checksum cannot verify (RFC 1071).
            out.append(vec("dumptrace%d-ip-check-zero-sum" % k, src, "derived", "check_ip", l3, 5,
                           note="ip_sum 0 on a nonzero header -> BAD_CHECKSUM"))
            out.append(vec("dumptrace%d-tcp-check-zero-sum" % k, src, "derived", "check_tcp", l3, 3))
        k += 1

    # 4. Survey run of the reference lib/in_cksum.c: the u32 accumulator wraps
    #    at 131,074 bytes; 200,000 x 0xFF -> 0x0001 (a true one's-complement
    #    sum would give 0x0000).  SURVEY.md §7 "Bit-exactness corner cases".
    out.append({"name": "survey-overflow-200000xff", "source": "SURVEY.md §7", "pin": "survey-ref-run",
                "op": "in_cksum", "fill": 255, "caplen": 200000, "expect": 0x0001})
    # all-zero data -> 0xFFFF (in_cksum.c:45-49)
    out.append({"name": "survey-allzero-1500", "source": "SURVEY.md Appendix A.6", "pin": "survey-ref-run",
                "op": "in_cksum", "fill": 0, "caplen": 1500, "expect": 0xFFFF})

    # 5. FromIPSummaryDump-ipopt-01.clicktest: tcpdump printed "[tcp sum ok]"
    #    for SetTCPChecksum's output on packets carrying these options; the
    #    pseudo-header destination is the LAST address of an SSRR/LSRR
    #    (in_cksum.c:101-105), the header dst otherwise.  Options as encoded
    #    on the wire (RFC 791) for the test's ip_opt strings.
    rel = "test/analysis/FromIPSummaryDump-ipopt-01.clicktest"
    text = open(os.path.join(R, rel), encoding="latin-1").read()

    def ip4(s):
        return bytes(int(x) for x in s.split("."))
    cases = [
        ("ssrr", bytes([137, 19, 12]) + ip4("128.4.45.60") + ip4("128.4.49.61") + ip4("1.1.1.1")
         + ip4("2.2.2.2") + b"\0", "10.0.0.8", 20, 80, "2.2.2.2"),
        ("nopnopeol", bytes([1, 1, 0, 0]), "10.0.0.4", 30, 40, None),
        ("rr", bytes([7, 19, 8]) + ip4("2.3.4.5") + b"\0" * 12 + b"\0", "10.0.0.8", 10, 80, None),
        ("lsrr", bytes([131, 11, 4]) + ip4("9.9.9.9") + ip4("7.7.7.7") + b"\0", "10.0.0.8", 21, 80, "7.7.7.7"),
    ]
    for nm, opt, dst, sport, dport, final in cases:
        hl = 20 + len(opt)
        total = hl + 20
        ip = bytearray(total)
        ip[0] = 0x40 | (hl // 4)
        struct.pack_into(">H", ip, 2, total)
        ip[9] = 6
        ip[12:16] = ip4("18.26.4.44")
        ip[16:20] = ip4(dst)
        ip[20:hl] = opt
        struct.pack_into(">HH", ip, hl, sport, dport)
        ip[hl + 12] = 0x50
        needle = {"ssrr": "ssrr{", "nopnopeol": "nop;nop;eol", "rr": "rr{2.3.4.5}"}.get(nm)
        if needle:
            source, pin = "%s:%d" % (rel, line_of(text, needle)), "tcpdump-ok"
        else:  # LSRR is not in the test: same rule, in_cksum.c:101
            source, pin = "lib/in_cksum.c:101-105", "derived"
        out.append({"name": "ipopt-%s-tcp-set-then-check" % nm, "source": source,
                    "pin": pin, "op": "set_tcp_then_rfc1071", "l3": bytes(ip).hex(),
                    "caplen": total, "final_dst": final or dst, "expect": 0})

    with open(args.out, "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "reference": "kohler/click 2.1",
                   "vectors": out, "fragment_cases": frag_cases}, f, indent=1)
    print("wrote %d vectors to %s" % (len(out), args.out))


if __name__ == "__main__":
    main()
