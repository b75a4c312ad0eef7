#!/usr/bin/env python3
"""A/B tuning of kernel variants, interleaved in ONE process (guide rule 24).

  python tools/tune.py --build                 # here: compile variant .so files
  python tools/tune.py --workload c3 ...       # on the GPU box (via gpurun)

Variants are compile-time flags (-DCLK_K, -DCLK_NT_LOADS, ...) built into
their own library under tools/variants/, and/or the speed-only context knobs
of clk_ctx_tune (Context.tune: max_blocks, scatter_blocks, set_mode,
stream_min, group).  Nothing is read from the environment by the library.
Every variant runs the same element over the same device-resident batch;
rounds interleave the variants; the median and min kernel time per variant
are printed as JSON, with the variants whose status output differs from the
first one's (all must be bit-identical).
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VDIR = os.path.join(ROOT, "tools", "variants")          # git-ignored; travels to the GPU box

# name -> (compile flags, Context.tune knobs)
VARIANTS = {
    "base": ([], {}),
    "prev": (["<tools/build_prev.sh>"], {}),     # the last commit's sources
    "k6": (["-DCLK_K=6"], {}),
    "k16_8": (["-DCLK_K16=8"], {}),
    "nt": (["-DCLK_NT_LOADS=1"], {}),
    "nont": (["-DCLK_NT_LOADS=0"], {}),
    "g16": ([], {"group": 16}),
    "g32": ([], {"group": 32}),
    "fused": ([], {"set_mode": 0}),
    "two": ([], {"set_mode": 1}),
    "mb1280": ([], {"max_blocks": 1280}),
    "mb2560": ([], {"max_blocks": 2560}),
    "mb4k": ([], {"max_blocks": 4096}),
    "mb8k": ([], {"max_blocks": 8192}),
    "mb16k": ([], {"max_blocks": 16384}),
    "mb32k": ([], {"max_blocks": 32768}),
    "mb64k": ([], {"max_blocks": 65536}),
    "sb8k": ([], {"scatter_blocks": 8192}),
    "sb64k": ([], {"scatter_blocks": 65536}),
    "two_stream": ([], {"set_mode": 1}),
    "skv3": (["-DCLK_SKV=3"], {}),
    "ck2w8": (["-DCLK_SKV_CHECK=2", "-DCLK_SWPE_CHECK=8"], {}),
    "ck3w7": (["-DCLK_SKV_CHECK=3", "-DCLK_SWPE_CHECK=7"], {}),
    "runs0": (["-DCLK_L4_RUNS=0"], {}),
    "sw5": (["-DCLK_L4_WPE_SET=5"], {}),
    "cw5": (["-DCLK_L4_WPE_CHECK=5"], {}),
    "r32": (["-DCLK_L4_RUNS_SET_G=32"], {}),
    "occ6": (["-DCLK_SET_OCC_PAD=0"], {}),
    "regblk0": (["-DCLK_SET_REGBLK=0"], {}),
    "hdrc0": (["-DCLK_HDR_FROM_CHUNKS=0"], {}),
    "ffu0": (["-DCLK_FRAG_FUSED=0"], {}),
    "ft512": (["-DCLK_FRAG_TILE=512"], {}),
    "fusednt": (["-DCLK_NT_LOADS=1"], {"set_mode": 0}),
    "dense0": (["-DCLK_DENSE=0", "-DCLK_SKV_CHECK=3", "-DCLK_SWPE_CHECK=6"], {}),
    "dk3w6": (["-DCLK_SKV_CHECK=3", "-DCLK_SWPE_CHECK=6"], {}),
    "dk5": (["-DCLK_SKV_CHECK=5", "-DCLK_SWPE_CHECK=5"], {}),
    "dk2w8": (["-DCLK_SKV_CHECK=2", "-DCLK_SWPE_CHECK=8"], {}),
    "dk6w4": (["-DCLK_SKV_CHECK=6", "-DCLK_SWPE_CHECK=4"], {}),
    "dset": (["-DCLK_DENSE_SET=1"], {}),
    "dsetk3": (["-DCLK_DENSE_SET=1", "-DCLK_SKV=3"], {}),
    "dsetk4": (["-DCLK_DENSE_SET=1", "-DCLK_SKV=4", "-DCLK_SWPE=4"], {}),
    "fusedsw5": (["-DCLK_L4_WPE_SET=5"], {"set_mode": 0}),
    "fusedrb0": (["-DCLK_SET_REGBLK=0"], {"set_mode": 0}),
    "fusedrb0nt": (["-DCLK_SET_REGBLK=0", "-DCLK_NT_LOADS=1"], {"set_mode": 0}),
    "fusedrb0nts": (["-DCLK_SET_REGBLK=0", "-DCLK_NT_LOADS=1", "-DCLK_NT_STORES=1"], {"set_mode": 0}),
    "occ4": (["-DCLK_SET_OCC_PAD=36864"], {}),
    "xcd": (["-DCLK_XCD_BLOCKS=1"], {}),
    "xcdset0": (["-DCLK_XCD_SET=0"], {}),
    "fusedxcd": (["-DCLK_XCD_BLOCKS=1"], {"set_mode": 0}),
    "ffu0xcd": (["-DCLK_FRAG_FUSED=0", "-DCLK_FRAG_XCD=1"], {}),
    "oldset": (["-DCLK_DENSE_SET=0", "-DCLK_SKV=2", "-DCLK_SWPE=8"], {}),
    "dsetk5": (["-DCLK_DENSE_SET=1", "-DCLK_SKV=5", "-DCLK_SWPE=4"], {}),
    "dsetk6w3": (["-DCLK_DENSE_SET=1", "-DCLK_SKV=6", "-DCLK_SWPE=3"], {}),
    "ch2": ([], {"set_chunks": 2}),
    "ch4": ([], {"set_chunks": 4}),
    "ch8": ([], {"set_chunks": 8}),
    "ch16": ([], {"set_chunks": 16}),
    "fw5": (["-DCLK_FRAG_WPE=5"], {}),
    "fw5u2": (["-DCLK_FRAG_WPE=5", "-DCLK_FRAG_U=2"], {}),
    "fu2": (["-DCLK_FRAG_U=2"], {}),
    "fg32": (["-DCLK_FRAG_G=32"], {}),
    "fw5u3": (["-DCLK_FRAG_WPE=5", "-DCLK_FRAG_U=3"], {}),
    "flat0": (["-DCLK_FRAG_FLAT=0"], {}),            # payloads in frag_write_kernel (round 5)
    "flatf16": (["-DCLK_FRAG_FLAT_F=16"], {}),
    "flatf4": (["-DCLK_FRAG_FLAT_F=4"], {}),
    "flatu2": (["-DCLK_FRAG_FLAT_U=2"], {}),
    "flatu8": (["-DCLK_FRAG_FLAT_U=8"], {}),
    "flatf16u8": (["-DCLK_FRAG_FLAT_F=16", "-DCLK_FRAG_FLAT_U=8"], {}),
    "flatf16u8t512": (["-DCLK_FRAG_FLAT_F=16", "-DCLK_FRAG_FLAT_U=8", "-DCLK_FRAG_TILE=512"], {}),
    "flatf32u8": (["-DCLK_FRAG_FLAT_F=32", "-DCLK_FRAG_FLAT_U=8"], {}),
    "hx4off": (["-DCLK_FRAG_HDR_X4=0"], {}),
    "hx4t512": (["-DCLK_FRAG_TILE=512"], {}),
    "hx4w5": (["-DCLK_FRAG_WPE=5"], {}),
    "flatnt0": (["-DCLK_FRAG_FLAT_NT=0"], {}),
    "flatf12u6": (["-DCLK_FRAG_FLAT_F=12", "-DCLK_FRAG_FLAT_U=6"], {}),
    "flatf6u3": (["-DCLK_FRAG_FLAT_F=6", "-DCLK_FRAG_FLAT_U=3"], {}),
    "hdrnt": (["-DCLK_FRAG_HDR_NT=1"], {}),
    "fch2": ([], {"frag_chunks": 2}),
    "fch4": ([], {"frag_chunks": 4}),
    "fch8": ([], {"frag_chunks": 8}),
}


def lib_for(name):
    flags, _ = VARIANTS[name]
    if not flags or os.environ.get("TUNE_NO_VARIANT_LIBS"):
        return os.path.join(ROOT, "click_amd", "libclick_amd_cksum.so")
    return os.path.join(VDIR, "lib_%s.so" % name)


def build(names):
    from click_amd import build as b
    b.build_library()
    os.makedirs(VDIR, exist_ok=True)
    for n in names:
        flags, _ = VARIANTS[n]
        if not flags or flags[0].startswith("<"):
            continue
        out = lib_for(n)
        cmd = [b._hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
               "-I" + os.path.join(ROOT, "include")] + flags + ["-o", out] + b.SOURCES
        print(" ".join(cmd))
        subprocess.run(cmd, check=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--variants", default=",".join(VARIANTS))
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--launches", type=int, default=5)
    args = ap.parse_args()
    names = args.variants.split(",")
    if args.build:
        build(names)
        return
    import torch
    import click_amd
    import bench
    w = bench.WORKLOADS[args.workload]
    n = w["n"]
    base_ctx = click_amd.Context(0)
    if args.workload == "c4":
        off, ln, total, sum_l = bench.imix_layout(torch, n, 0x5EED, 0)
        arena = torch.empty(total, dtype=torch.uint8, device="cuda")
        b = click_amd.Batch(arena, n, off=off, length=ln, max_len=1500)
    else:
        arena = torch.empty(n * w["stride"], dtype=torch.uint8, device="cuda")
        b = click_amd.Batch(arena, n, stride=w["stride"], fixed_len=w["L"])
    base_ctx.gen_packets(b, proto=w["proto"])
    base_ctx.set_ip_checksum(b, want_sums=False)
    status = torch.empty(n, dtype=torch.uint8, device="cuda")
    sums16 = torch.empty(n, dtype=torch.uint16, device="cuda")
    bench.run_element(base_ctx, "SetTCPChecksum" if w["proto"] == 6 else "SetUDPChecksum", b, status)
    ctxs = {}
    for nm in names:
        _, knobs = VARIANTS[nm]
        ctxs[nm] = click_amd.Context(0, lib_path=lib_for(nm)).tune(**knobs)
    elements = {"SetUDPChecksum": lambda c: c.set_udp_checksum(b, status=status, want_sums=False),
                "SetTCPChecksum": lambda c: c.set_tcp_checksum(b, status=status, want_sums=False),
                "SetIPChecksum": lambda c: c.set_ip_checksum(b, status=status, want_sums=False),
                "CheckUDPHeader": lambda c: c.check_udp_header(b, out=status),
                "CheckTCPHeader": lambda c: c.check_tcp_header(b, out=status),
                "CheckIPHeader": lambda c: c.check_ip_header(b, out=status),
                "DecIPTTL": lambda c: c.dec_ip_ttl(b, status=status, want_sums=False),
                "InCksum": lambda c: c.in_cksum(b, out=sums16),
                "IPFragmenter": lambda c: frag(c)}
    if os.environ.get("TUNE_ELEMENT") == "IPFragmenter":       # C3 to MTU 576; headers restored per call
        hdr = arena.view(n, w["stride"])[:, :12]
        saved = hdr.clone()
        fout = torch.empty(n * 976, dtype=torch.uint8, device="cuda")
        ff = torch.empty(n, dtype=torch.int64, device="cuda")
        fl = torch.empty(n, dtype=torch.int32, device="cuda")

        def frag(c):
            hdr.copy_(saved)
            c.ip_fragment(b, 576, True, arena=fout, max_frags=2 * n, port=status, first_len=fl, frag_first=ff)
    element = os.environ.get("TUNE_ELEMENT", w["elements"][-1])
    run = elements[element]
    times = {nm: [] for nm in names}
    ref_status, mismatch = None, []
    for r in range(args.rounds):
        for nm in names:
            c = ctxs[nm]
            status.fill_(0xEE)
            run(c)
            torch.cuda.synchronize()
            if ref_status is None:
                ref_status = status.clone()
            elif not torch.equal(status, ref_status) and nm not in mismatch:
                mismatch.append(nm)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(args.launches):
                run(c)
            e.record()
            torch.cuda.synchronize()
            times[nm].append(s.elapsed_time(e) / args.launches)
    if element == "IPFragmenter":
        alg = 1924 * n
    elif element == "InCksum":
        alg = (w["L"] + 2) * n
    else:
        alg = bench.ALG[element](w["L"]) * n if args.workload != "c4" else sum_l + (bench.ALG[element](0) + 12) * n
    out = {nm: {"median_ms": round(statistics.median(t), 4), "min_ms": round(min(t), 4),
                "GBs": round(alg / (statistics.median(t) * 1e-3) / 1e9, 1)} for nm, t in times.items()}
    print(json.dumps({"workload": args.workload, "element": element,
                      "variants": out, "status_mismatch": mismatch}))


if __name__ == "__main__":
    main()
