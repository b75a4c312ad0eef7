"""Debug: which fragment bytes differ from the oracle (fuzzed batch, MTU 576)."""
import sys
import numpy as np
sys.path.insert(0, ".")
from tests import fuzz, oracle_lib
from tests.test_gpu_fragment import gpu_fragment
import torch
import click_amd

ctx = click_amd.Context(0)
for mtu, hd in ((576, False), (1500, True)):
    rng = np.random.default_rng(7 * mtu + hd)
    arena, off, caplen = fuzz.frag_batch(rng, 2500)
    n = len(off)
    nid = rng.integers(0, 65536, n).astype(np.uint16)
    h = gpu_fragment(torch, ctx, arena.copy(), off, caplen, mtu, hd, nid)
    ref = arena.copy()
    r = oracle_lib.ip_fragment(ref, n, mtu, hd, off=off, length=caplen, new_id=nid)
    bad = 0
    for k in range(h["nf"]):
        o, l = int(r["frag_off"][k]), int(r["frag_len"][k])
        g = h["arena"][o:o + l]
        e = np.frombuffer(r["frags"][k], np.uint8)
        d = np.nonzero(g != e)[0]
        if d.size:
            bad += 1
            if bad <= 25:
                i = int(r["frag_src"][k])
                print("mtu", mtu, "frag", k, "k%8", k % 8, "len", l, "off", o, "diff", d[0], d[-1], d.size,
                      "zeros", int((g[d] == 0).all()), "pkt", i, "caplen", int(caplen[i]), "hl", arena[int(off[i])] & 15,
                      "base8", int(r["frag_off"][k - k % 8]), "chunk", (o - int(r["frag_off"][k - k % 8]) + d[0]) // 16)
    print("mtu", mtu, "bad", bad, "of", h["nf"])
