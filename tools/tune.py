#!/usr/bin/env python3
"""A/B tuning of kernel variants, interleaved in ONE process (guide rule 24).

  python tools/tune.py --build                 # here: compile variant .so files
  python tools/tune.py --workload c3 ...       # on the GPU box (via gpurun)

Variants are compile-time flags (-DCLK_K, -DCLK_NT_LOADS) and/or the
runtime tuning knobs read at context creation (CLK_MAX_BLOCKS,
CLK_FORCE_GROUP).  Every variant runs the same element over the same
device-resident batch; rounds interleave the variants; the median and min
kernel time per variant are printed as JSON.
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VDIR = os.path.join(ROOT, "build", "variants")

# name -> (compile flags, runtime env)
VARIANTS = {
    "base": ([], {}),
    "k8": (["-DCLK_K=8"], {}),
    "k16": (["-DCLK_K=16"], {}),
    "nt": (["-DCLK_NT_LOADS=1"], {}),
    "nont": (["-DCLK_NT_LOADS=0"], {}),
    "g16": ([], {"CLK_FORCE_GROUP": "16"}),
    "g32": ([], {"CLK_FORCE_GROUP": "32"}),
    "fused": ([], {"CLK_SET_MODE": "0"}),
    "fusednt": (["-DCLK_NT_LOADS=1"], {"CLK_SET_MODE": "0"}),
    "two": ([], {"CLK_SET_MODE": "1"}),
    "mb8k": ([], {"CLK_MAX_BLOCKS": "8192"}),
    "mb16k": ([], {"CLK_MAX_BLOCKS": "16384"}),
    "sb8k": ([], {"CLK_SCATTER_BLOCKS": "8192"}),
    "scu4": (["-DCLK_SCATTER_UNROLL=4"], {}),
    "scu4sb4k": (["-DCLK_SCATTER_UNROLL=4"], {"CLK_SCATTER_BLOCKS": "4096"}),
    "sb64k": ([], {"CLK_SCATTER_BLOCKS": "65536"}),
    "sb4k": ([], {"CLK_SCATTER_BLOCKS": "4096"}),
    "mb32k": ([], {"CLK_MAX_BLOCKS": "32768"}),
    "iphpair": (["-DCLK_IPH_PAIR=1"], {}),
    "sntc": (["-DCLK_STREAM_NT_CHECK=1"], {}),
    "ck3w7": (["-DCLK_SKV_CHECK=3", "-DCLK_SWPE_CHECK=7"], {}),
    "ck3w5": (["-DCLK_SKV_CHECK=3", "-DCLK_SWPE_CHECK=5"], {}),
    "mb64k": ([], {"CLK_MAX_BLOCKS": "65536"}),
    "mb1m": ([], {"CLK_MAX_BLOCKS": "1048576"}),
    "diag_nofield": (["-DCLK_DIAG_NO_FIELD_STORE=1"], {}),
    "kv1": (["-DCLK_KV=1"], {}),
    "kv2": (["-DCLK_KV=2"], {}),
    "k1u2": (["-DCLK_KV=1", "-DCLK_VU=2"], {}),
    "kv4": (["-DCLK_KV=4"], {}),
    "u2": (["-DCLK_VU=2"], {}),
    "u3": (["-DCLK_VU=3"], {}),
    "u4": (["-DCLK_VU=4"], {}),
    "k1u4": (["-DCLK_KV=1", "-DCLK_VU=4"], {}),
    "k1u8": (["-DCLK_KV=1", "-DCLK_VU=8"], {}),
    "kv8": (["-DCLK_KV=8"], {}),
    "bins": ([], {"CLK_VARLEN": "0"}),
    "range": ([], {"CLK_VARLEN": "1"}),
    "stream": ([], {"CLK_VARLEN": "2"}),
    "skv1": (["-DCLK_SKV=1"], {"CLK_VARLEN": "2"}),
    "skv4": (["-DCLK_SKV=4"], {"CLK_VARLEN": "2"}),
    "skv3": (["-DCLK_SKV=3"], {"CLK_VARLEN": "2"}),
    "skv4w7": (["-DCLK_SKV=4", "-DCLK_SWPE=7"], {"CLK_VARLEN": "2"}),
    "skv3w7": (["-DCLK_SKV=3", "-DCLK_SWPE=7"], {"CLK_VARLEN": "2"}),
    "skv8": (["-DCLK_SKV=8"], {"CLK_VARLEN": "2"}),
    "fused_stream": ([], {"CLK_SET_MODE": "0", "CLK_VARLEN": "2"}),
    "two_stream": ([], {"CLK_SET_MODE": "1", "CLK_VARLEN": "2"}),
    "prev": (["(built by hand from the previous commit's sources)"], {}),
    "sw5": (["-DCLK_L4_WPE_SET=5"], {}),
    "sw1": (["-DCLK_L4_WPE_SET=1"], {}),
    "sw6": (["-DCLK_L4_WPE_SET=6"], {}),
    "cw6": (["-DCLK_L4_WPE_CHECK=6"], {}),
    "cw8": (["-DCLK_L4_WPE_CHECK=8"], {}),
    "ffu0": (["-DCLK_FRAG_FUSED=0"], {}),
    "fpro0": (["-DCLK_FRAG_PRO=0"], {}),
    "ft256": (["-DCLK_FRAG_TILE=256"], {}),
    "ft512": (["-DCLK_FRAG_TILE=512"], {}),
    "ft2048": (["-DCLK_FRAG_TILE=2048"], {}),
    "fua": (["-DCLK_FRAG_UA=1"], {}),
    "fuah": (["-DCLK_FRAG_UA=1", "-DCLK_FRAG_HDR_FIRST=1"], {}),
    "fuahu2": (["-DCLK_FRAG_UA=1", "-DCLK_FRAG_HDR_FIRST=1", "-DCLK_FRAG_U=2"], {}),
    "fuau8": (["-DCLK_FRAG_UA=1", "-DCLK_FRAG_U=8"], {}),
    "fuau2": (["-DCLK_FRAG_UA=1", "-DCLK_FRAG_U=2"], {}),
    "fnts": (["-DCLK_FRAG_NT_STORE=1"], {}),
    "fntl": (["-DCLK_FRAG_NT_LOAD=1"], {}),
    "fnt": (["-DCLK_FRAG_NT_STORE=1", "-DCLK_FRAG_NT_LOAD=1"], {}),
    "fw6": (["-DCLK_FRAG_WPE=6"], {}),
    "fw8": (["-DCLK_FRAG_WPE=8"], {}),
    "fu2w6": (["-DCLK_FRAG_U=2", "-DCLK_FRAG_WPE=6"], {}),
    "fu2w8": (["-DCLK_FRAG_U=2", "-DCLK_FRAG_WPE=8"], {}),
    "fg32": (["-DCLK_FRAG_G=32"], {}),
    "fg64": (["-DCLK_FRAG_G=64"], {}),
    "fu2": (["-DCLK_FRAG_U=2"], {}),
    "fu8": (["-DCLK_FRAG_U=8"], {}),
    "fg32u8": (["-DCLK_FRAG_G=32", "-DCLK_FRAG_U=8"], {}),
    "hc2": (["-DCLK_SHC_EXTRA=0"], {}),
    "hc2w8": (["-DCLK_SHC_EXTRA=0", "-DCLK_SWPE=8"], {}),
    "w8": (["-DCLK_SWPE=8"], {}),
    "smark": (["-DCLK_SMARK=1"], {}),
    "smark_kv4": (["-DCLK_SMARK=1", "-DCLK_SKV=4"], {}),
    "spf": (["-DCLK_SPF=1"], {}),
    "spf_kv1": (["-DCLK_SPF=1", "-DCLK_SKV=1"], {}),
    "spf_kv4": (["-DCLK_SPF=1", "-DCLK_SKV=4"], {}),
    "block": (["-DCLK_BLOCK_WRITE=1"], {}),
    "fused_block": (["-DCLK_BLOCK_WRITE=1"], {"CLK_SET_MODE": "0"}),
    "g8": ([], {"CLK_FORCE_GROUP": "8"}),
    "k4": (["-DCLK_K=4"], {}),
    "k12": (["-DCLK_K=12"], {}),
    "k9": (["-DCLK_K=9"], {}),
    "k10": (["-DCLK_K=10"], {}),
    "k6": (["-DCLK_K=6"], {}),
    "k7": (["-DCLK_K=7"], {}),
    "regblk0": (["-DCLK_SET_REGBLK=0"], {}),
    "hdrc0": (["-DCLK_HDR_FROM_CHUNKS=0"], {}),
    "cw1": (["-DCLK_L4_WPE_CHECK=1"], {}),
    "ntst": (["-DCLK_NT_STORES=1"], {}),
    "nt_ntst": (["-DCLK_NT_LOADS=1", "-DCLK_NT_STORES=1"], {}),
    "two_nt": (["-DCLK_NT_LOADS=1"], {"CLK_SET_MODE": "1"}),
    "regblk_fused": ([], {"CLK_SET_MODE": "0"}),
    "two_stream_nt": (["-DCLK_NT_LOADS=1"], {"CLK_SET_MODE": "1", "CLK_VARLEN": "2"}),
    "regblk0_fused": (["-DCLK_SET_REGBLK=0"], {"CLK_SET_MODE": "0"}),
    "runs0": (["-DCLK_L4_RUNS=0"], {}),
    "cw5": (["-DCLK_L4_WPE_CHECK=5"], {}),
    "setruns16": (["-DCLK_L4_RUNS_SET_G=16"], {}),
    "k16_8": (["-DCLK_K16=8"], {}),
    "diag_nowork": (["-DCLK_DIAG_NO_WORK_STORE=1"], {}),
    "sw4": (["-DCLK_L4_WPE_SET=4"], {}),
    "setruns16sw4": (["-DCLK_L4_RUNS_SET_G=16", "-DCLK_L4_WPE_SET=4"], {}),
    "scnt": (["-DCLK_SCATTER_ST=1"], {}),
    "scst0": (["-DCLK_SCATTER_ST=0"], {}),
    "fieldnt": (["-DCLK_FIELD_NT=1"], {}),
    "scoal": (["-DCLK_STASH_COALESCE=1"], {}),
    "fh4": (["-DCLK_FRAG_HDR16=0"], {}),
    "scblk": (["-DCLK_SCATTER_BLOCK=1"], {}),
    "occ5": (["-DCLK_SET_OCC_PAD=28672"], {}),
    "occ6": (["-DCLK_SET_OCC_PAD=0"], {}),
    "skv4w5": (["-DCLK_SKV=4", "-DCLK_SWPE=5"], {}),
    "skv4w6": (["-DCLK_SKV=4", "-DCLK_SWPE=6"], {}),
    "skv3w6": (["-DCLK_SKV=3", "-DCLK_SWPE=6"], {}),
    "skv8w4": (["-DCLK_SKV=8", "-DCLK_SWPE=4"], {}),
    "occ4": (["-DCLK_SET_OCC_PAD=36864"], {}),
    "occ64_4": (["-DCLK_SET_OCC_PAD64=36864"], {}),
    "occ64_3": (["-DCLK_SET_OCC_PAD64=49152"], {}),
    "fhnt": (["-DCLK_FRAG_HDR_NT=1"], {}),
    "scoalnt": (["-DCLK_STASH_COALESCE=1", "-DCLK_STASH_NT=1"], {}),
    "r32": (["-DCLK_L4_RUNS_SET_G=32"], {}),
    "two_stream_scst0": (["-DCLK_SCATTER_ST=0"], {"CLK_SET_MODE": "1", "CLK_VARLEN": "2"}),
    "scsc": (["-DCLK_SCATTER_ST=2"], {}),
    "scscnt": (["-DCLK_SCATTER_ST=3"], {}),
    "r16scnt": (["-DCLK_L4_RUNS_SET_G=16", "-DCLK_SCATTER_ST=1"], {}),
    "r16scsc": (["-DCLK_L4_RUNS_SET_G=16", "-DCLK_SCATTER_ST=2"], {}),
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
        if not flags:
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
        _, env = VARIANTS[nm]
        saved = {k: os.environ.get(k) for k in ("CLK_MAX_BLOCKS", "CLK_FORCE_GROUP", "CLK_SET_MODE", "CLK_VARLEN",
                                                "CLK_SCATTER_BLOCKS")}
        for k in saved:
            os.environ.pop(k, None)
        os.environ.update(env)
        ctxs[nm] = click_amd.Context(0, lib_path=lib_for(nm))
        for k, v in saved.items():
            if v is not None:
                os.environ[k] = v
            else:
                os.environ.pop(k, None)
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
            elif not torch.equal(status, ref_status) and nm not in mismatch and not nm.startswith("d"):
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
