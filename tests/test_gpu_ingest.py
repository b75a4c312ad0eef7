"""pcap ingest -> GPU: a tcpdump file read by
clk_pcap_read into a page-aligned host arena, registered for zero-copy,
checked by the kernels where the records lie -- the
FromDump(FORCE_IP true) -> CheckIPHeader / CheckTCPHeader graph of the
reference's test/analysis tests -- and, through the element glue, with the
records' network-header offsets.  Every verdict is compared with the oracle
over the same bytes."""
import os

import numpy as np
import pytest

from tests import fuzz, oracle_lib, pyref

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def ctx():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import click_amd
    c = click_amd.Context(0)
    yield c
    c.close()


def _synthetic_trace(path, n, proto, seed):
    """Ethernet records around fuzzed IPv4 packets: plain, 802.1Q-tagged,
    and non-IP (ARP) frames that FORCE_IP rejects."""
    rng = np.random.default_rng(seed)
    arena, off, caplen, _ = fuzz.make_batch(rng, n, proto, max_total=1500)
    recs = []
    for k in range(n):
        ip = arena[int(off[k]):int(off[k]) + int(caplen[k])].tobytes()
        r = rng.random()
        if r < 0.1:
            fr = bytes(12) + b"\x81\x00\x00\x07\x08\x00" + ip
        elif r < 0.15:
            fr = bytes(12) + b"\x08\x06" + ip
        else:
            fr = bytes(12) + b"\x08\x00" + ip
        recs.append((fr, 1000 + k, k))
    data = pyref.write_pcap(recs, linktype=1)
    with open(path, "wb") as f:
        f.write(data)


@pytest.mark.parametrize("op,proto", [("check_ip", 17), ("check_tcp", 6), ("check_udp", 17), ("set_udp", 17)])
def test_pcap_zero_copy(ctx, tmp_path, op, proto):
    import torch
    import click_amd
    path = str(tmp_path / "t.pcap")
    _synthetic_trace(path, 4000, proto, 300 + proto)
    p = click_amd.read_pcap(path)
    off, ln = p.ip_layout()
    assert 0 < len(off) < 4000
    ref = p.arena.copy()
    dev = ctx.host_register(p.arena)
    try:
        b = click_amd.Batch(dev, len(off), off=torch.from_numpy(off.view(np.int64)).cuda(),
                            length=torch.from_numpy(ln.view(np.int32)).cuda(), max_len=int(ln.max()))
        codes = {"check_ip": lambda: ctx.check_ip_header(b), "check_tcp": lambda: ctx.check_tcp_header(b),
                 "check_udp": lambda: ctx.check_udp_header(b),
                 "set_udp": lambda: ctx.set_udp_checksum(b)[0]}[op]()
        ctx.sync()
        rc, _ = oracle_lib.batch(op, ref, len(off), off=off, length=ln)
        assert np.array_equal(codes.cpu().numpy(), rc)
        assert np.array_equal(p.arena, ref)
    finally:
        ctx.host_unregister(p.arena)


def test_reference_trace_through_glue(ctx):
    """dump.trace (IPSummaryDump-02.clicktest) into CheckIPHeader(OFFSET 14)
    and CheckTCPHeader, records pushed with their FORCE_IP network header."""
    import click_amd
    from click_amd.elements import Element
    p = click_amd.read_pcap(os.path.join(HERE, "golden", "dump_trace.pcap"))
    ports = {}
    for cls, conf in (("CheckIPHeader", "OFFSET 14"), ("CheckTCPHeader", "")):
        e = Element(ctx, cls, conf, noutputs=2)
        for k in range(len(p.off)):
            e.push_ptr(p.arena.ctypes.data + int(p.off[k]), int(p.caplen[k]), int(p.nh[k]), token=k)
        e.flush()
        tok, port, _ = e.results()
        assert list(tok) == list(range(5))
        ports[cls] = list(port)
    assert ports["CheckIPHeader"] == [0, 0, 0, 0, 1]      # the fifth frame's ip_sum is 0 (golden vectors)
    assert ports["CheckTCPHeader"] == [0, 0, 0, 0, 1]     # ... and th_sum 0 (BAD_CHECKSUM)


def test_c_example_on_reference_trace(ctx):
    """The plain-C program (examples/pcap_check.c): pcap -> zero-copy ->
    CheckIPHeader + CheckTCPHeader, no Python in the data path."""
    import subprocess
    exe = os.path.join(os.path.dirname(HERE), "examples", "bin", "pcap_check")
    if not os.path.exists(exe):
        pytest.skip("examples not built (python -m click_amd.build --examples)")
    r = subprocess.run([exe, os.path.join(HERE, "golden", "dump_trace.pcap")], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 0, r.stderr
    # record, CheckIPHeader verdict, CheckTCPHeader verdict (the golden vectors: the fifth
    # frame's ip_sum and th_sum are 0 -> BAD_CHECKSUM, 1 + Reason = 5 and 3)
    assert r.stdout.split("\n")[:5] == ["0 0 0", "1 0 0", "2 0 0", "3 0 0", "4 5 3"]
