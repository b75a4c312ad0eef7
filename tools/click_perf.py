"""Click-level rates of the drop-in GPU elements against the stock CPU
elements, on the same graph and host (click_integration/bin/click-{cpu,
dropin}, tools/click_scratch_build.sh).  Graphs:

  c1     click_integration/conf/c1-forward.click (config 1's forwarding work)
  c3chk  a 1500 B UDP frame (InfiniteSource clones) -> Strip(14) ->
         CheckIPHeader -> CheckUDPHeader -> AverageCounter -> Discard
  c3set  ... -> MarkIPHeader -> SetUDPChecksum -> AverageCounter -> Discard

Variants rewrite the GPU elements' configurations (BATCH, CHAIN) for the
adapter's knobs; the stock build runs the graph as written.  Each run is
timed by its AverageCounter (first to last packet) and by the wall clock of
the process.  Used by bench.py (--click) and from the command line:

  python tools/click_perf.py [--limit N] [--reps R] [--out file.json]
"""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests import click_run  # noqa: E402

GPU_CLASSES = ("CheckIPHeader", "CheckIPHeader2", "SetIPChecksum", "CheckUDPHeader", "SetUDPChecksum",
               "CheckTCPHeader", "SetTCPChecksum", "CheckICMPHeader", "DecIPTTL", "IPInputCombo", "IPGWOptions",
               "FixIPSrc", "IPOutputCombo", "IPFragmenter")


def csum16(b):
    if len(b) % 2:
        b = b + b"\0"
    s = sum(int.from_bytes(b[i:i + 2], "big") for i in range(0, len(b), 2))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return (~s) & 0xFFFF


def udp_frame(total=1500, seed=7):
    """Ethernet + IPv4 (total bytes) + UDP with valid checksums."""
    import random
    r = random.Random(seed)
    pay = bytes(r.getrandbits(8) for _ in range(total - 28))
    src, dst = bytes([1, 0, 0, 1]), bytes([2, 0, 0, 2])
    ulen = total - 20
    udp = (4660).to_bytes(2, "big") + (22136).to_bytes(2, "big") + ulen.to_bytes(2, "big") + b"\0\0" + pay
    ph = src + dst + b"\0\x11" + ulen.to_bytes(2, "big")
    us = csum16(ph + udp) or 0xFFFF
    udp = udp[:6] + us.to_bytes(2, "big") + udp[8:]
    ip = bytearray(b"\x45\x00" + total.to_bytes(2, "big") + b"\0\0\0\0\x40\x11\0\0" + src + dst)
    ip[10:12] = csum16(bytes(ip)).to_bytes(2, "big")
    eth = bytes.fromhex("0000c0ae67ef000000000000") + b"\x08\x00"
    return eth + bytes(ip) + udp


def c3_conf(kind):
    hexd = " ".join("%02x" % x for x in udp_frame())
    # (SetUDPChecksum reads the network header: MarkIPHeader sets it, on the CPU)
    tail = "CheckIPHeader -> CheckUDPHeader" if kind == "c3chk" else "MarkIPHeader -> SetUDPChecksum"
    return ("define($LIMIT 2000000, $BURST 32);\n"
            "InfiniteSource(DATA \\<%s>, LIMIT $LIMIT, BURST $BURST, STOP true)\n"
            "  -> Strip(14) -> %s -> out :: AverageCounter -> Discard;\n" % (hexd, tail))


def with_gpu_conf(text, extra):
    """Add `extra` keywords to every GPU-backed element's configuration."""
    if not extra:
        return text
    pat = re.compile(r"\b(%s)\s*(\(([^()]*)\))?" % "|".join(GPU_CLASSES))

    def rep(m):
        args = (m.group(3) or "").strip()
        return "%s(%s)" % (m.group(1), (args + ", " + extra) if args else extra)
    return "\n".join(ln if ln.lstrip().startswith("//") else pat.sub(rep, ln) for ln in text.split("\n"))


def conf_text(graph):
    if graph == "c1":
        return open(os.path.join(click_run.CONF, "c1-forward.click")).read()
    return c3_conf(graph)


# glibc's per-thread cache of freed chunks, deep enough for the packets a
# GPU element holds (Click's own pool keeps 1000, packet.cc:238)
TCACHE = {"GLIBC_TUNABLES": "glibc.malloc.tcache_count=65535"}


def run_one(mode, graph, extra="", limit=None, burst=None, timeout=180, extra_env=None):
    text = conf_text(graph)
    if mode != "cpu":
        text = with_gpu_conf(text, extra)
    with tempfile.NamedTemporaryFile("w", suffix=".click", delete=False) as f:
        f.write(text)
        path = f.name
    d = {}
    if limit:
        d["LIMIT"] = limit
    if burst:
        d["BURST"] = burst
    t0 = time.perf_counter()
    rc, h, err = click_run.run(mode, path, d, ("out.count", "out.rate"), timeout=timeout, extra_env=extra_env)
    wall = time.perf_counter() - t0
    os.unlink(path)
    if rc != 0:
        return {"rc": rc, "err": err[-400:]}
    n = int(h["out.count"])
    return {"count": n, "mpps_counter": float(h["out.rate"]) / 1e6, "mpps_wall": n / wall / 1e6, "wall_s": wall}


def sweep(limit_c1=6000000, limit_c3=2000000, reps=3, variants=None, bursts=(1, 32)):
    variants = variants if variants is not None else [("cpu", ""), ("dropin", "")]
    out = {}
    for graph, limit in (("c1", limit_c1), ("c3chk", limit_c3), ("c3set", limit_c3)):
        for burst in bursts:
            for mode, extra in variants:
                key = "%s/burst%d/%s%s" % (graph, burst, mode, ("/" + extra.replace(" ", "")) if extra else "")
                ex = extra.replace("@tcache", "").strip(" ,")
                runs = [run_one(mode, graph, ex, limit, burst, extra_env=TCACHE if "@tcache" in extra else None)
                        for _ in range(reps)]
                ok = [r for r in runs if "count" in r]
                rec = {"runs": runs}
                if ok:
                    rates = sorted(r["mpps_counter"] for r in ok)
                    rec["mpps_median"] = rates[len(rates) // 2]
                out[key] = rec
                print(key, rec.get("mpps_median"), "" if ok else runs[0], flush=True)
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--limit", type=int, default=6000000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out")
    ap.add_argument("--bursts", default="1,32")
    ap.add_argument("--variants", default="cpu:;dropin:;dropin:LATENCY 20;dropin:BATCH 1024;dropin:BATCH 32768, LATENCY 50;dropin:CHAIN false, LATENCY 20")
    a = ap.parse_args()
    v = [tuple(x.split(":", 1)) for x in a.variants.split(";")]
    res = sweep(a.limit, a.limit // 3, a.reps, v, tuple(int(b) for b in a.bursts.split(",")))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
