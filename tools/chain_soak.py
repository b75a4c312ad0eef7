"""Chain parity soak (tools only): tests/test_gpu_chain.py's comparison --
the chain against the same elements one by one, every result in each
member's push order, bytes, clones and handlers -- over many fuzzed frame
sets, batch sizes and flush modes.
    python3 tools/chain_soak.py SEEDS FRAMES
Prints one JSON line: cases run, failures (seed, chain, error)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import click_amd
    from click_amd.elements import ANNO_BCAST, anno_paint
    from tests import test_gpu_chain as T
    seeds, frames = int(sys.argv[1]), int(sys.argv[2])
    ctx = click_amd.Context(0)
    runs, fails, t0 = 0, [], time.time()
    for seed in range(1000, 1000 + seeds):
        rng = np.random.default_rng(seed)
        batch = int(rng.choice([257, 1000, 4096, 65536]))
        async_flush = bool(seed & 1)
        for which in ("elements", "combos"):
            _, arena, foff, flen = T.fuzzed_frames(seed, n=frames)
            n = len(foff)
            if which == "elements":
                anno = (rng.random(n) < 0.3).astype(np.uint32)
                spec = [("CheckIPHeader", "OFFSET 14, DETAILS true, BATCH %d" % batch, 2),
                        ("IPGWOptions", T.MY_IP_TXT, 2), ("FixIPSrc", T.MY_IP_TXT, 1), ("DecIPTTL", "", 2),
                        ("IPFragmenter", "576, HONOR_DF true", 2)]
                handlers = ("drops", "fragments", "packets", "lost")
            else:
                anno = np.array([anno_paint(int(p)) for p in rng.integers(0, 3, n)], np.uint32) + \
                    (rng.random(n) < 0.05) * ANNO_BCAST + (rng.random(n) < 0.2).astype(np.uint32)
                spec = [("IPInputCombo", "1, BATCH %d" % batch, 1), ("IPOutputCombo", "1, %s, 120" % T.MY_IP_TXT, 5)]
                handlers = ("drops", "packets", "lost")
            runs += 1
            try:
                T.compare_chain(ctx, spec, arena, foff, flen, anno=anno, async_flush=async_flush, handlers=handlers)
            except AssertionError as e:
                fails.append({"seed": seed, "chain": which, "batch": batch, "async": async_flush,
                              "error": str(e)[:200]})
        print("seed %d done (%d runs, %d failures, %.0f s)" % (seed, runs, len(fails), time.time() - t0), flush=True)
    ctx.close()
    print(json.dumps({"cases": runs, "frames_per_case": frames, "failures": fails}))


if __name__ == "__main__":
    main()
