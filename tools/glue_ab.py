"""A/B of glue library builds on bench.py's E2E legs (tools only):
    python3 tools/glue_ab.py ROUNDS LIB.so [LIB.so ...]
Each round runs bench.e2e (C3 CheckUDPHeader) once per library, in turn, and
prints the staged and ZEROCOPY glue rates per library."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import click_amd
    import bench
    rounds, libs = int(sys.argv[1]), sys.argv[2:]
    res = {l: {"staged": [], "zerocopy": []} for l in libs}
    for _ in range(rounds):
        for l in libs:
            ctx = click_amd.Context(0, lib_path=l)
            r = bench.e2e(torch, ctx, "c3", "CheckUDPHeader")
            res[l]["staged"].append(r["element_glue"]["mpps"])
            res[l]["zerocopy"].append(r["element_glue_zero_copy"]["mpps"])
            ctx.close()
            print(os.path.basename(l), res[l]["staged"][-1], res[l]["zerocopy"][-1], flush=True)
    print(json.dumps({os.path.basename(l): v for l, v in res.items()}))


if __name__ == "__main__":
    main()
