"""GPU parity for IPFragmenter (elements/ip/ipfragmenter.cc:88-171) through
the C ABI: the reference's own IPFragmenter-01/02 outputs, fuzzed batches
against the oracle (ports, first-fragment rewrite in place, every appended
fragment byte, descriptors), capacity limits, and a full-size batch whose
fragments all pass CheckIPHeader and reassemble to the original payload.
Every test runs on each write path: the flat payload pass, the 16-lane
groups (CLK_TUNE_FRAG_FLAT_MIN), and the flat pass in tile ranges on two
streams (CLK_TUNE_FRAG_CHUNKS)."""
import json
import os

import numpy as np
import pytest

from tests import fuzz, oracle_lib

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


@pytest.fixture(scope="module", params=["flat", "groups", "flat_ranges"])
def ctx(torch, request):
    """Every write path at every size: the flat payload pass
    (frag_flat_kernel) for every batch, the 16-lane groups only, and the
    flat pass in 5 tile ranges overlapping the plans (batches of 10+ tiles)."""
    import click_amd
    c = click_amd.Context(0).tune(frag_flat_min=1 << 62 if request.param == "groups" else 0,
                                  frag_chunks=5 if request.param == "flat_ranges" else 1)
    yield c
    c.close()


def gpu_fragment(torch, ctx, arena, off, caplen, mtu, honor_df, new_id=None, slack=0):
    """Two calls (size, then write), as a host would.  Returns host arrays."""
    import click_amd
    n = len(off)
    base = torch.from_numpy(arena).to("cuda:0")
    b = click_amd.Batch(base, n, off=torch.from_numpy(off.view(np.int64)).to("cuda:0"),
                        length=torch.from_numpy(caplen.view(np.int32)).to("cuda:0"))
    nid = torch.from_numpy(new_id.view(np.int16)).to("cuda:0") if new_id is not None else None
    probe = base.clone()
    pb = click_amd.Batch(probe, n, off=b.off, length=b.length)
    r = ctx.ip_fragment(pb, mtu, honor_df, nid)
    ctx.sync()
    nf, nb = (int(x) for x in r["totals"].cpu())
    out = torch.zeros(max(nb - slack, 1), dtype=torch.uint8, device="cuda:0")
    r = ctx.ip_fragment(b, mtu, honor_df, nid, arena=out, max_frags=max(nf - (1 if slack else 0), 0))
    ctx.sync()
    h = {k: v.cpu().numpy() for k, v in r.items()}
    h["arena"] = out.cpu().numpy()
    h["base"] = base.cpu().numpy()
    h["nf"], h["nb"] = nf, nb
    return h


def test_reference_fragmenter_cases(torch, ctx):
    cases = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden_vectors.json")))
    for case in cases["fragment_cases"]:
        pkt = bytes.fromhex(case["in"])
        for shift in (0, 1, 2, 3, 13):
            arena = np.zeros(shift + len(pkt) + 16, np.uint8)
            arena[shift:shift + len(pkt)] = np.frombuffer(pkt, np.uint8)
            h = gpu_fragment(torch, ctx, arena, np.array([shift], np.uint64), np.array([len(pkt)], np.uint32),
                             case["mtu"], case["honor_df"])
            assert h["port"][0] == 2
            got = [h["base"][shift:shift + int(h["first_len"][0])].tobytes()]
            for k in range(h["nf"]):
                o, l = int(h["frag_off"][k]), int(h["frag_len"][k])
                got.append(h["arena"][o:o + l].tobytes())
            assert [g.hex() for g in got] == case["fragments"], (case["name"], shift)


@pytest.mark.parametrize("mtu,honor_df", [(576, False), (1500, True), (68, False), (40, True), (1006, False)])
def test_fragment_fuzz_parity(torch, ctx, mtu, honor_df):
    rng = np.random.default_rng(7 * mtu + honor_df)
    arena, off, caplen = fuzz.frag_batch(rng, 2500)
    n = len(off)
    nid = rng.integers(0, 65536, n).astype(np.uint16)
    h = gpu_fragment(torch, ctx, arena.copy(), off, caplen, mtu, honor_df, nid)
    ref = arena.copy()
    r = oracle_lib.ip_fragment(ref, n, mtu, honor_df, off=off, length=caplen, new_id=nid)
    assert np.array_equal(h["port"], r["port"])
    assert np.array_equal(h["first_len"].view(np.uint32), r["first_len"])
    assert np.array_equal(h["frag_first"].view(np.uint64), r["frag_first"])
    assert (h["nf"], h["nb"]) == (len(r["frags"]), r["arena_bytes"])
    assert np.array_equal(h["frag_off"][:h["nf"]].view(np.uint64), r["frag_off"])
    assert np.array_equal(h["frag_len"][:h["nf"]].view(np.uint32), r["frag_len"])
    assert np.array_equal(h["frag_src"][:h["nf"]].view(np.uint32), r["frag_src"])
    for k in range(h["nf"]):
        o, l = int(r["frag_off"][k]), int(r["frag_len"][k])
        assert h["arena"][o:o + l].tobytes() == r["frags"][k], k
    diff = np.nonzero(h["base"] != ref)[0]
    assert diff.size == 0, diff[:10]


def test_fragment_capacity_limit(torch, ctx):
    """A packet whose fragments do not all fit the caller's arena /
    max_frags is left whole (port CLK_FRAG_NOROOM = 3, bytes untouched,
    nothing of it written); every packet that fits is exact; totals still
    report the need."""
    rng = np.random.default_rng(5)
    arena, off, caplen = fuzz.frag_batch(rng, 300)
    h = gpu_fragment(torch, ctx, arena.copy(), off, caplen, 300, False, slack=40)
    ref = arena.copy()
    r = oracle_lib.ip_fragment(ref, len(off), 300, False, off=off, length=caplen)
    assert (h["nf"], h["nb"]) == (len(r["frags"]), r["arena_bytes"])
    cap_b, cap_f = h["nb"] - 40, h["nf"] - 1
    nfr = np.bincount(r["frag_src"].astype(np.int64), minlength=len(off))
    fitted = noroom = 0
    for i in range(len(off)):
        o, c = int(off[i]), int(caplen[i])
        ks = range(int(r["frag_first"][i]), int(r["frag_first"][i]) + int(nfr[i]))
        fits = all(k < cap_f and int(r["frag_off"][k]) + ((int(r["frag_len"][k]) + 15) & ~15) <= cap_b for k in ks)
        if r["port"][i] != 2 or fits:
            assert h["port"][i] == r["port"][i], i
            assert np.array_equal(h["base"][o:o + c], ref[o:o + c]), i
            for k in ks:
                fo, fl = int(r["frag_off"][k]), int(r["frag_len"][k])
                assert h["arena"][fo:fo + fl].tobytes() == r["frags"][k]
            fitted += r["port"][i] == 2
        else:
            assert h["port"][i] == 3, i
            assert np.array_equal(h["base"][o:o + c], arena[o:o + c]), i     # untouched
            for k in ks:
                fo = int(r["frag_off"][k])
                assert not h["arena"][fo:min(fo + int(r["frag_len"][k]), len(h["arena"]))].any()
            noroom += 1
    assert fitted > 0 and noroom > 0


def test_fragment_many_tiles_uneven(torch, ctx):
    """The single-pass look-back over more than 64 predecessor tiles (1024
    packets each) with uneven tile sums: a fuzzed batch of 70,000 packets of
    mixed lengths, options, DF/MF and fragment counts, exact against the
    oracle (ports, first lengths, fragment indices and every fragment)."""
    rng = np.random.default_rng(70)
    arena, off, caplen = fuzz.frag_batch(rng, 70000, max_total=1600)
    n = len(off)
    nid = rng.integers(0, 65536, n).astype(np.uint16)
    h = gpu_fragment(torch, ctx, arena.copy(), off, caplen, 296, False, nid)
    ref = arena.copy()
    r = oracle_lib.ip_fragment(ref, n, 296, False, off=off, length=caplen, new_id=nid)
    assert np.array_equal(h["port"], r["port"])
    assert np.array_equal(h["first_len"].view(np.uint32), r["first_len"])
    assert np.array_equal(h["frag_first"].view(np.uint64), r["frag_first"])
    assert (h["nf"], h["nb"]) == (len(r["frags"]), r["arena_bytes"])
    assert np.array_equal(h["frag_off"][:h["nf"]].view(np.uint64), r["frag_off"])
    assert np.array_equal(h["frag_len"][:h["nf"]].view(np.uint32), r["frag_len"])
    assert np.array_equal(h["frag_src"][:h["nf"]].view(np.uint32), r["frag_src"])
    assert np.array_equal(h["arena"][:r["arena_bytes"]], r["arena"])
    assert np.array_equal(h["base"], ref)
    tiles = np.bincount(np.arange(n) // 1024, weights=np.bincount(r["frag_src"].astype(np.int64), minlength=n))
    assert len(tiles) > 65 and tiles.min() != tiles.max()


def test_fragment_full_size(torch, ctx):
    """1M x 1500 B UDP packets to MTU 576 (3 fragments each): every
    fragment passes CheckIPHeader, offsets/MF are consistent, and the
    payloads reassemble to the original bytes."""
    import click_amd
    n, L, stride = 1 << 20, 1500, 1536
    arena = torch.empty(n * stride, dtype=torch.uint8, device="cuda:0")
    b = click_amd.Batch(arena, n, stride=stride, fixed_len=L)
    ctx.gen_packets(b, proto=17)
    ctx.set_ip_checksum(b, want_sums=False)
    ctx.set_udp_checksum(b, want_sums=False)
    orig = arena.view(n, stride)[:, 20:L].clone()
    out = torch.empty(n * 2 * 576, dtype=torch.uint8, device="cuda:0")
    r = ctx.ip_fragment(b, 576, True, arena=out, max_frags=2 * n)
    ctx.sync()
    assert [int(x) for x in r["totals"].cpu()] == [2 * n, n * (576 + 400)]    # slots of 572 + 396 B
    assert int(r["port"].ne(2).sum()) == 0
    assert int(r["first_len"].ne(572).sum()) == 0
    first = click_amd.Batch(arena, n, stride=stride, fixed_len=572)
    assert int(ctx.check_ip_header(first).ne(0).sum()) == 0
    nf = int(r["totals"][0])
    fb = click_amd.Batch(out, nf, off=r["frag_off"][:nf], length=r["frag_len"][:nf])
    assert int(ctx.check_ip_header(fb).ne(0).sum()) == 0
    # reassemble: fragment k of packet i is 2i + k
    fo = r["frag_off"][:nf].view(n, 2)
    p1 = out[(fo[:, 0:1] + 20 + torch.arange(552, device="cuda:0")).reshape(-1)].view(n, 552)
    p2 = out[(fo[:, 1:2] + 20 + torch.arange(376, device="cuda:0")).reshape(-1)].view(n, 376)
    assert torch.equal(orig[:, 552:1104], p1)
    assert torch.equal(orig[:, 1104:1480], p2)
    del arena, out
    torch.cuda.empty_cache()


def test_fragment_tune_knobs_range(torch):
    """CLK_TUNE_FRAG_CHUNKS takes 1..64 and CLK_TUNE_FRAG_FLAT_MIN any
    count; anything else is CLK_EINVAL and leaves the setting as it was."""
    import click_amd
    from click_amd import ClickAmdError
    c = click_amd.Context(0)
    try:
        c.tune(frag_chunks=64, frag_flat_min=0)
        for bad in ({"frag_chunks": 0}, {"frag_chunks": 65}, {"frag_flat_min": -1}):
            with pytest.raises(ClickAmdError):
                c.tune(**bad)
    finally:
        c.close()
