"""Fold preload_sampler.c's samples into functions (tools only).

    python tools/core_profile/fold.py SAMPLES [--map OBJ=UNSTRIPPED ...] [--top N]

Each sample is "object offset"; offsets are resolved with addr2line -f -C
against the object (or the unstripped copy given with --map).
"""
import argparse
import collections
import subprocess


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("samples")
    ap.add_argument("--map", action="append", default=[])
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    remap = dict(m.split("=", 1) for m in a.map)
    by_obj = collections.defaultdict(list)
    for ln in open(a.samples):
        obj, off = ln.split()
        by_obj[obj].append(off)
    total = sum(len(v) for v in by_obj.values())
    fn_count = collections.Counter()
    for obj, offs in by_obj.items():
        uniq = sorted(set(offs))
        names = {}
        path = remap.get(obj, obj)
        if obj != "?":
            r = subprocess.run(["addr2line", "-f", "-C", "-e", path] + uniq, capture_output=True, text=True)
            out = r.stdout.splitlines()
            for i, o in enumerate(uniq):
                names[o] = out[2 * i] if 2 * i < len(out) else "?"
        short = obj.rsplit("/", 1)[-1]
        for o in offs:
            fn_count["%s  [%s]" % (names.get(o, "?")[:110], short)] += 1
    print("%d samples" % total)
    for fn, c in fn_count.most_common(a.top):
        print("%6.2f%%  %s" % (100.0 * c / total, fn))


if __name__ == "__main__":
    main()
