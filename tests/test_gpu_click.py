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
