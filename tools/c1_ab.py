"""A/B of glue library builds on bench.py's config-1 legs (tools only):
    python3 tools/c1_ab.py ROUNDS LIB.so [LIB.so ...]
Each round runs bench.config1 once per library, in turn; prints each leg's
Mpps per library."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import click_amd
    import bench
    rounds, libs = int(sys.argv[1]), sys.argv[2:]
    res = {l: {} for l in libs}
    for _ in range(rounds):
        for l in libs:
            ctx = click_amd.Context(0, lib_path=l)
            r = bench.config1(ctx)
            for k, v in r.items():
                if isinstance(v, dict) and "mpps" in v:
                    res[l].setdefault(k, []).append(v["mpps"])
            ctx.close()
            print(l, {k: v[-1] for k, v in res[l].items()}, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
