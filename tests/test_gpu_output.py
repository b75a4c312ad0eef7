"""GPU parity for the IP output path: IPGWOptions, FixIPSrc and
IPOutputCombo (elements/ip/ipgwoptions.cc, fixipsrc.cc, ipoutputcombo.cc)
through the C ABI against the CPU oracle, bit-exact on codes, parameter-
problem offsets, stored ip_sum and every arena byte; and the fake-iprouter
data path (test/userlevel/iprouter-01.clicktest) run on the device both as
separate elements and as the click-xform combos."""
import json
import os

import numpy as np
import pytest

from tests import fuzz, oracle_lib

pytestmark = pytest.mark.gpu

MY_IP = 0x18041A12          # 18.26.4.24, raw s_addr
TS = 0x40E20100


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


@pytest.fixture(scope="module")
def ctx(torch):
    import click_amd
    c = click_amd.Context(0)
    yield c
    c.close()


def _dev(torch, a, dtype=None):
    return torch.from_numpy(a if dtype is None else a.view(dtype)).to("cuda:0")


@pytest.mark.parametrize("op", ["ip_gw_options", "fix_ip_src", "ip_output_combo"])
@pytest.mark.parametrize("seed", [1, 2])
def test_ip_output_path_parity(torch, ctx, op, seed):
    import click_amd
    rng = np.random.default_rng(seed * 17)
    arena, off, caplen, flags = fuzz.gw_batch(rng, 4000, MY_IP)
    n = len(off)
    addrs = np.array([MY_IP, 0x01020304], np.uint32)
    b = click_amd.Batch(_dev(torch, arena), n, off=_dev(torch, off, np.int64), length=_dev(torch, caplen, np.int32))
    fl = _dev(torch, flags)
    if op == "ip_gw_options":
        codes, prob, sums = ctx.ip_gw_options(b, MY_IP, ts=TS, my_addrs=_dev(torch, addrs, np.int32))
    elif op == "fix_ip_src":
        sums = ctx.fix_ip_src(b, MY_IP, anno=fl)
        codes = prob = None
    else:
        codes, prob, sums = ctx.ip_output_combo(b, MY_IP, 120, ts=TS, flags=fl)
    ctx.sync()
    ref = arena.copy()
    rc, rp, rs = oracle_lib.ip_out_batch(op, ref, n, off=off, length=caplen, flags=flags, my_ip=MY_IP,
                                         my_addrs=addrs, ts=TS, mtu=120)
    if codes is not None:
        assert np.array_equal(codes.cpu().numpy(), rc)
        assert np.array_equal(prob.cpu().numpy(), rp)
    assert np.array_equal(sums.cpu().numpy(), rs)
    after = b.base.cpu().numpy()
    diff = np.nonzero(after != ref)[0]
    assert diff.size == 0, (op, diff[:10])


def test_ip_output_combo_full_size(torch, ctx):
    """IPOutputCombo over a C2-sized batch (16M x 64 B slots, no options, no
    FIX_IP_SRC): every TTL drops by one, the headers still check, MTU 40
    sends every 46 B packet to port 4."""
    import click_amd
    n, L, stride = 16 << 20, 46, 64
    arena = torch.empty(n * stride, dtype=torch.uint8, device="cuda:0")
    b = click_amd.Batch(arena, n, stride=stride, fixed_len=L)
    ctx.gen_packets(b, proto=17)
    ctx.set_ip_checksum(b, want_sums=False)
    port, prob, _ = ctx.ip_output_combo(b, MY_IP, 1500)
    assert int(port.ne(0).sum()) == 0 and int(prob.ne(0).sum()) == 0
    assert int(ctx.check_ip_header(b).ne(0).sum()) == 0
    assert int(arena.view(n, stride)[:, 8].ne(63).sum()) == 0
    port, _, _ = ctx.ip_output_combo(b, MY_IP, 40)
    assert int(port.ne(4).sum()) == 0
    del arena
    torch.cuda.empty_cache()


def _fake_frame():
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden_vectors.json")))["vectors"]
    for v in g:
        if v["name"] == "fake-iprouter-ip-check":        # conf/fake-iprouter.click:42-50
            return bytes.fromhex("0000c0ae67ef00000000000008 00".replace(" ", "")) + bytes.fromhex(v["l3"])
    raise AssertionError("fake-iprouter frame missing from the golden vectors")


def test_fake_iprouter_data_path(torch, ctx):
    """conf/fake-iprouter.click's forwarding path for its 600,000 frames
    (iprouter-01.clicktest expects 600000 forwarded, OUTA == OUTB):
    Strip(14) + CheckIPHeader(INTERFACES ...) -> [route] -> IPGWOptions ->
    FixIPSrc -> DecIPTTL versus IPInputCombo -> IPOutputCombo, both on the
    device; every frame passes, both give identical bytes, and the result
    matches the oracle."""
    import click_amd
    frame = np.frombuffer(_fake_frame(), np.uint8)
    n, stride = 600000, 128
    host = np.zeros(n * stride, np.uint8)
    host.reshape(n, stride)[:, :len(frame)] = frame
    out = []
    for combo in (False, True):
        arena = _dev(torch, host)
        eth = click_amd.Batch(arena, n, stride=stride, fixed_len=len(frame))
        bad = _dev(torch, np.array([0xFF041A12, 0x00041A12, 0xFF071A12, 0x00071A12], np.uint32), np.int32)
        v = ctx.check_ip_header(eth, offset=14, badsrc=bad)      # INTERFACES 18.26.4.1/24 18.26.7.1/24
        assert int(v.ne(0).sum()) == 0
        ipb = click_amd.Batch(arena[14:], n, stride=stride, fixed_len=len(frame) - 14)
        if combo:
            port, _, _ = ctx.ip_output_combo(ipb, MY_IP, 300, ts=TS)
            assert int(port.ne(0).sum()) == 0
        else:
            st, _, _ = ctx.ip_gw_options(ipb, MY_IP, ts=TS)
            assert int(st.ne(0).sum()) == 0
            ctx.fix_ip_src(ipb, MY_IP, anno=torch.zeros(n, dtype=torch.uint8, device="cuda:0"))
            st, _ = ctx.dec_ip_ttl(ipb)
            assert int(st.ne(0).sum()) == 0
        ctx.sync()
        out.append(arena.cpu().numpy())
    assert np.array_equal(out[0], out[1])
    ref = frame.copy()
    oracle_lib.batch("dec_ttl", ref[14:], 1, stride=0, fixed_len=len(frame) - 14)
    assert np.array_equal(out[1].reshape(n, stride)[:, :len(frame)], np.broadcast_to(ref, (n, len(frame))))
