"""Resolve chain_prof's PC samples (tools only): top source lines and
functions, inlined frames attributed to the innermost line and to the
outermost function they were inlined into.
    python3 tools/chain_prof/resolve.py BINARY SAMPLES [TOP]"""
import collections
import subprocess
import sys


def main():
    binary, path = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    pcs = collections.Counter(l.strip() for l in open(path) if l.strip())
    total = sum(pcs.values())
    # offsets from the executable's start: add its first segment's address
    # (0 for a position-independent executable)
    hdr = subprocess.run(["readelf", "-lW", binary], capture_output=True, text=True).stdout
    base = int([l.split()[2] for l in hdr.splitlines() if l.strip().startswith("LOAD")][0], 16)
    pcs = collections.Counter({("0x%x" % (int(a, 16) + base) if a.startswith("0x") else a): c
                               for a, c in pcs.items()})
    addrs = [a for a in pcs if a.startswith("0x")]
    out = subprocess.run(["addr2line", "-f", "-C", "-i", "-a", "-e", binary] + addrs,
                         capture_output=True, text=True).stdout.splitlines()
    frames, cur = {}, None
    for l in out:
        if l.startswith("0x") and all(c in "0123456789abcdefx" for c in l):
            cur = "0x%x" % int(l, 16)
            frames[cur] = []
        else:
            frames[cur].append(l)
    lines, funcs = collections.Counter(), collections.Counter()
    for a, c in pcs.items():
        if not a.startswith("0x"):
            lines[a] += c
            funcs[a] += c
            continue
        f = frames.get("0x%x" % int(a, 16), ["?", "?"])
        pairs = list(zip(f[0::2], f[1::2]))
        inner_fn, inner_ln = pairs[0]
        outer_fn = pairs[-1][0]
        lines["%s  [%s]" % (inner_ln.split(" (")[0].replace("/root/repo/", ""), inner_fn[:70])] += c
        funcs[outer_fn[:150]] += c
    print("samples %d" % total)
    print("-- functions (inlined code counted to its caller)")
    for k, c in funcs.most_common(top):
        print("%6.2f%%  %s" % (100.0 * c / total, k))
    print("-- lines (innermost)")
    for k, c in lines.most_common(top):
        print("%6.2f%%  %s" % (100.0 * c / total, k))


if __name__ == "__main__":
    main()
