"""CPU tests of the pcap ingest (include/click_amd_ingest.h, host code):
FromDump's file/record handling and FORCE_IP, checked against the
reference's own trace (test/analysis/IPSummaryDump-02.clicktest's
dump.trace, extracted by tests/golden/make_golden.py) and against the
Python restatement (tests/pyref.py) on synthetic files of every link type
FORCE_IP knows."""
import os
import struct

import numpy as np
import pytest

import click_amd
from click_amd import _abi
from tests import oracle_lib, pyref

HERE = os.path.dirname(os.path.abspath(__file__))
TRACE = os.path.join(HERE, "golden", "dump_trace.pcap")


def _records(p):
    return [bytes(p.arena[int(o):int(o) + int(c)]) for o, c in zip(p.off, p.caplen)]


def _check_against_pyref(path, data, force_ip=True):
    info, recs = pyref.read_pcap(data, force_ip)
    p = click_amd.read_pcap(path, force_ip=force_ip)
    for k in ("linktype", "nanosecond", "swapped", "force_ip"):
        assert p.info[k] == info[k], k
    assert (p.info["stopped"] is not None) == info["stopped"]
    assert p.info["records"] == len(recs)
    assert _records(p) == [r[0] for r in recs]
    assert list(p.wire_len) == [r[1] for r in recs]
    assert list(p.ts_ns) == [r[2] & 0xFFFFFFFFFFFFFFFF for r in recs]
    assert list(p.nh) == [r[3] for r in recs]
    assert all(int(o) % 16 == 0 for o in p.off)
    return p


def test_reference_trace():
    """dump.trace: five Ethernet records, every one IP at offset 14; the
    IP packets verify as the golden vectors say (four captured TCP/IPv4
    frames pass CheckIPHeader, the hand-made fifth has ip_sum 0)."""
    data = open(TRACE, "rb").read()
    p = _check_against_pyref(TRACE, data)
    assert p.info["linktype"] == 1 and p.info["records"] == 5 and p.info["ip_records"] == 5
    assert list(p.nh) == [14] * 5 and list(p.caplen) == [66, 66, 66, 66, 63]
    off, ln = p.ip_layout()
    arena = p.arena.copy()
    codes, _ = oracle_lib.batch("check_ip", arena, len(off), off=off, length=ln)
    assert list(codes) == [0, 0, 0, 0, 5]
    codes, _ = oracle_lib.batch("check_tcp", arena, len(off), off=off, length=ln)
    assert list(codes[:4]) == [0, 0, 0, 0]


def _ip4(rng, payload=20, hl=5):
    h = bytearray(rng.integers(0, 256, 4 * hl + payload, dtype=np.uint8).tobytes())
    h[0] = 0x40 | hl
    return bytes(h)


def _framings(rng, ip):
    """(linktype, record) pairs that put `ip` behind each link header FORCE_IP
    parses, plus near-miss variants."""
    eth = bytes(12)
    out = [
        (1, eth + b"\x08\x00" + ip), (1, eth + b"\x86\xdd" + bytes([0x60]) + ip[1:] + bytes(40)),
        (1, eth + b"\x81\x00\x00\x05\x08\x00" + ip), (1, eth + b"\x81\x00\x00\x05\x08\x06" + ip),
        (1, eth + b"\x08\x06" + ip), (1, eth[:10]),
        (101, ip), (12, ip), (101, b""), (101, bytes([0x45]) + bytes(10)),
        (113, bytes(14) + b"\x08\x00" + ip), (113, bytes(14) + b"\x00\x01" + ip),
        (104, b"\x0f\x00\x08\x00" + ip), (50, b"\xff\x03\x00\x21" + ip), (50, b"\x8f\x00\x08\x00" + ip),
        (50, b"\xff\x03\x00\x57" + ip), (9, b"\xff\x03\x00\x21" + ip), (9, b"\x21" + ip), (9, b"\xff\x03\x57" + ip),
        (0, b"\x02\x00\x00\x00" + ip), (0, b"\x00\x00\x00\x02" + ip), (0, b"\x07\x00\x00\x00" + ip),
        (100, b"\xaa\xaa\x03\x00\x00\x00\x08\x00" + ip), (100, b"\x06\x06\x03\x00" + ip),
        (100, b"\xaa\xaa\x03\x00\x00\x00\x08\x00"[:6] + b"\x08\x00" + ip),
        (100, b"\xaa\xaa\x03\x00\x80\xc2\x00\x07" + eth + b"\x08\x00" + ip),
        (100, b"\xaa\xaa\x03\x00\x80\xc2\x00\x04" + b"\x00" + b"\x50" + bytes(12) + b"\xaa\xaa\x03\x00\x00\x00\x08\x00"
         + ip),
        (100, b"\xaa\xaa\x03\x00\x00\xf8\x08\x00" + ip),
        (123, bytes(4) + b"\xaa\xaa\x03\x00\x00\x00\x08\x00" + ip),
        (10, b"\x50" + bytes(12) + b"\xaa\xaa\x03\x00\x00\x00\x08\x00" + ip), (10, b"\x40" + bytes(20) + ip),
        (105, b"\x08\x00" + bytes(22) + b"\xaa\xaa\x03\x00\x00\x00\x08\x00" + ip),
        (105, b"\x08\x03" + bytes(28) + b"\xaa\xaa\x03\x00\x00\x00\x08\x00" + ip),
        (105, b"\x04\x00" + bytes(22) + b"\xaa\xaa\x03\x00\x00\x00\x08\x00" + ip),
        (119, bytes(144) + b"\x08\x00" + bytes(22) + b"\x06\x06\x03\x00" + ip),
        (127, b"\x00\x00\x0c\x00" + bytes(8) + b"\x08\x00" + bytes(22) + b"\x06\x06\x03\x00" + ip),
        (127, b"\x00\x00\x04\x00" + ip),
    ]
    # random bytes behind every link type: whatever FORCE_IP decides, both agree
    for dlt in sorted(pyref.FORCE_IPABLE):
        for _ in range(6):
            out.append((dlt, rng.integers(0, 256, int(rng.integers(0, 200)), dtype=np.uint8).tobytes()))
    return out


def test_force_ip_every_linktype(tmp_path):
    rng = np.random.default_rng(5)
    L = _abi.load()
    n = 0
    for hl in (5, 6, 15):
        ip = _ip4(rng, hl=hl)
        for dlt, rec in _framings(rng, ip):
            buf = np.frombuffer(rec, np.uint8).copy() if rec else np.zeros(1, np.uint8)
            got = L.clk_pcap_force_ip(buf.ctypes.data, len(rec), dlt)
            assert got == pyref.force_ip(rec, dlt), (dlt, rec[:24].hex())
            n += 1
    # short IP headers: ip_hl < 5, or the header longer than the record
    for rec in (bytes([0x44]) + bytes(30), bytes([0x4f]) + bytes(30), bytes([0x60]) + bytes(20)):
        buf = np.frombuffer(rec, np.uint8).copy()
        assert L.clk_pcap_force_ip(buf.ctypes.data, len(rec), 101) == -1
    assert n > 150


@pytest.mark.parametrize("magic,big", [(0xA1B2C3D4, False), (0xA1B2C3D4, True), (0xA1B23C4D, False),
                                       (0xA1B23C4D, True), (0xA1B2CD34, False), (0xA1B2CD34, True)])
def test_file_formats(tmp_path, magic, big):
    """Byte order, nanosecond and Linux-modified headers, per-link records."""
    rng = np.random.default_rng(magic & 0xFF ^ big)
    for dlt in (1, 101, 113, 0):
        recs = []
        for k in range(40):
            ip = _ip4(rng, payload=int(rng.integers(0, 300)))
            fr = [r for d, r in _framings(rng, ip)[:40] if d == dlt] or [ip]
            recs.append((fr[int(rng.integers(0, len(fr)))], int(rng.integers(-5, 2 ** 31 - 1)),
                         int(rng.integers(0, 999999))))
        data = pyref.write_pcap(recs, linktype=dlt, magic=magic, big_endian=big)
        path = tmp_path / ("t%d.pcap" % dlt)
        path.write_bytes(data)
        p = _check_against_pyref(str(path), data)
        assert p.info["records"] == 40


def test_record_header_quirks(tmp_path):
    """fromdump.cc:348-368: caplen/len swapped before pcap 2.3 (and at 2.3
    when caplen > len); caplen > len repaired by skipping the excess;
    caplen > 65535 stops the read; a short final record ends it."""
    rng = np.random.default_rng(9)
    ip = _ip4(rng, payload=60)
    fr = bytes(12) + b"\x08\x00" + ip
    cases = [
        (2, [(fr, 1, 2)], [(len(fr) + 100, len(fr))]),           # old file: words swapped -> caplen = len(fr)
        (3, [(fr, 1, 2)], [(len(fr), len(fr) + 100)]),           # 2.3, caplen <= len: as written
        (3, [(fr, 1, 2)], [(len(fr) + 100, len(fr))]),           # 2.3, caplen > len: swapped
        (4, [(fr + bytes(7), 1, 2)], [(len(fr) + 7, len(fr))]),   # caplen > len: 7 bytes skipped
        (4, [(fr, 1, 2), (fr, 3, 4)], [None, (70000, 70000)]),   # bad header: stop after record 0
    ]
    for vmin, recs, raw in cases:
        data = pyref.write_pcap(recs, vmin=vmin, raw_headers=raw)
        path = tmp_path / "q.pcap"
        path.write_bytes(data)
        p = _check_against_pyref(str(path), data)
    assert p.info["stopped"] and "bad packet header; giving up" in p.info["stopped"]
    data = pyref.write_pcap([(fr, 1, 2), (fr, 3, 4)])[:-5]            # truncated final record
    path.write_bytes(data)
    p = _check_against_pyref(str(path), data)
    assert p.info["records"] == 1


def test_errors_match_fromdump(tmp_path):
    rng = np.random.default_rng(1)
    ip = _ip4(rng)
    path = tmp_path / "e.pcap"
    for data, msg in [(b"\xd4\xc3\xb2\xa1", "not a tcpdump file (too short)"),
                      (b"\x00" * 40, "not a tcpdump file (bad magic number)"),
                      (struct.pack("<IHHiIII", 0xA1B2C3D4, 3, 0, 0, 0, 65535, 1), "unknown major version 3"),
                      (pyref.write_pcap([(ip, 0, 0)], linktype=147), "unknown linktype 147; can't force IP packets")]:
        path.write_bytes(data)
        with pytest.raises(click_amd.ClickAmdError, match=msg.replace("(", r"\(").replace(")", r"\)")):
            click_amd.read_pcap(str(path))
    # without FORCE_IP an unknown linktype reads (nh = -1), and DLT_RAW forces IP (fromdump.cc:256-257)
    path.write_bytes(pyref.write_pcap([(ip, 0, 0)], linktype=147))
    p = click_amd.read_pcap(str(path), force_ip=False)
    assert p.info["records"] == 1 and list(p.nh) == [-1]
    path.write_bytes(pyref.write_pcap([(ip, 0, 0)], linktype=12))
    p = click_amd.read_pcap(str(path), force_ip=False)
    assert p.info["force_ip"] == 1 and p.info["linktype"] == 101 and list(p.nh) == [0]
    with pytest.raises(click_amd.ClickAmdError):
        click_amd.read_pcap(str(tmp_path / "missing.pcap"))


def test_sizing_and_small_arena(tmp_path):
    import ctypes
    L = _abi.load()
    info = _abi.clk_pcap_info()
    assert L.clk_pcap_read(TRACE.encode(), 1, None, 0, None, None, None, None, None, 0, ctypes.byref(info)) == 0
    assert info.records == 5 and info.arena_bytes == 384 and info.ip_records == 5
    arena = np.zeros(100, np.uint8)
    off = np.zeros(5, np.uint64)
    cap = np.zeros(5, np.uint32)
    nh = np.zeros(5, np.int32)
    rc = L.clk_pcap_read(TRACE.encode(), 1, arena.ctypes.data, arena.size, off.ctypes.data, cap.ctypes.data,
                         None, None, nh.ctypes.data, 5, ctypes.byref(info))
    assert rc == _abi.CLK_EINVAL if hasattr(_abi, "CLK_EINVAL") else rc < 0
    assert b"arena too small" in L.clk_last_error(None)
    p = click_amd.read_pcap(TRACE, max_records=2)
    assert p.info["records"] == 5 and len(p.off) == 2


def test_parser_under_sanitizers(tmp_path):
    """The pcap reader parses untrusted files: build it with ASan + UBSan
    (host code; tests/native/pcap_fuzz_main.cc) and run it over mutated
    files of every link type -- flipped bytes, truncations, huge lengths."""
    import shutil
    import subprocess
    gxx = shutil.which("g++")
    if not gxx:
        pytest.skip("no g++")
    root = os.path.dirname(HERE)
    exe = str(tmp_path / "pcap_fuzz")
    r = subprocess.run([gxx, "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                        "-I", os.path.join(root, "include"), os.path.join(HERE, "native", "pcap_fuzz_main.cc"),
                        os.path.join(root, "click_amd", "host", "ingest.cc"), "-o", exe],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    rng = np.random.default_rng(77)
    paths = []
    for dlt in sorted(pyref.FORCE_IPABLE) + [147]:
        for v in range(12):
            recs = []
            for _ in range(int(rng.integers(0, 12))):
                ip = _ip4(rng, payload=int(rng.integers(0, 80)), hl=int(rng.integers(5, 16)))
                fr = [rec for d, rec in _framings(rng, ip) if d == dlt] or [ip]
                recs.append((fr[int(rng.integers(0, len(fr)))], 1, 2))
            data = bytearray(pyref.write_pcap(recs, linktype=dlt, magic=[0xA1B2C3D4, 0xA1B23C4D, 0xA1B2CD34][v % 3],
                                              big_endian=bool(v & 4), vmin=int(rng.integers(1, 5))))
            for _ in range(int(rng.integers(0, 6))):                   # byte flips (headers included)
                if data:
                    data[int(rng.integers(0, len(data)))] = int(rng.integers(0, 256))
            if v % 5 == 4 and len(data) > 24:                          # a record length far past the file
                struct.pack_into("<I", data, min(24 + 8, len(data) - 4), int(rng.integers(0, 2 ** 32)))
            if v % 3 == 2:
                data = data[:int(rng.integers(0, len(data) + 1))]        # truncation
            p = tmp_path / ("f%d_%d.pcap" % (dlt, v))
            p.write_bytes(bytes(data))
            paths.append(str(p))
    r = subprocess.run([exe] + paths, capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1"))
    assert r.returncode == 0, (r.returncode, r.stderr[-3000:])
    assert int(r.stdout.strip()) > 0
