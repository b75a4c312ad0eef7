#!/usr/bin/env python3
"""Record the object code of the CPU baseline's checksum loop.

SURVEY §6 describes the reference's lib/in_cksum.c compiled with Click's
flags (-g -O2, gcc 11.4) as a scalar loop that adds one 16-bit word per
iteration (movzwl + add) and is not vectorized.  The reference cannot be
compiled here (it needs the configure-generated <click/config.h>; DESIGN.md
"Oracle"), so this checks the restatement the GPU box times instead, built
by oracle/Makefile with the same compiler and flags: oracle_in_cksum must be
that loop, and the element functions must call it (no inlined or vector
copy), as Click's elements call click_in_cksum in another object file.

    python oracle/objdump_check.py            # prints the check, writes oracle/objdump_in_cksum.txt
"""
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libcksum_oracle.so")
ELEMENTS = ("oracle_check_ip_header", "oracle_set_ip_checksum", "oracle_check_udp_header",
            "oracle_set_udp_checksum", "oracle_check_tcp_header", "oracle_set_tcp_checksum")


def disasm(fn, lib=LIB):
    out = subprocess.run(["objdump", "-d", "--no-show-raw-insn", lib], check=True, capture_output=True,
                         text=True).stdout
    m = re.search(r"^[0-9a-f]+ <%s>:\n(.*?)(?:\n\n|\Z)" % re.escape(fn), out, re.S | re.M)
    if not m:
        raise KeyError(fn)
    return [l.split("\t", 1)[1].strip() for l in m.group(1).splitlines() if "\t" in l]


def check(lib=LIB):
    """Returns (ok, report lines)."""
    rep = []
    body = disasm("oracle_in_cksum", lib)
    vec = [i for i in body if re.search(r"%[xyz]mm|\bv?p(add|shuf|unpck)", i)]
    # the word loop loads one zero-extended 16-bit word per iteration and adds it
    word_loop = any("movzwl" in i for i in body) and sum(1 for i in body if i.startswith("add")) >= 2
    rep.append("oracle_in_cksum: %d instructions, %d vector, movzwl word loads: %s"
               % (len(body), len(vec), "yes" if word_loop else "no"))
    ok = not vec and word_loop
    for fn in ELEMENTS:
        b = disasm(fn, lib)
        calls = [i for i in b if i.startswith("call")]
        v = [i for i in b if re.search(r"%[xyz]mm", i)]
        calls_it = any("oracle_in_cksum" in c and "pseudohdr" not in c for c in calls)
        rep.append("%s: calls oracle_in_cksum: %s, vector instructions: %d" % (fn, calls_it, len(v)))
        ok = ok and calls_it and not v
    return ok, rep, body


def main():
    ok, rep, body = check()
    cc = subprocess.run(["gcc", "--version"], capture_output=True, text=True).stdout.splitlines()[0]
    text = ["# oracle_in_cksum as built by oracle/Makefile (%s, -g -O2 -W -Wall)" % cc,
            "# SURVEY §6: the reference's click_in_cksum at -O2 is a scalar movzwl/add loop, one",
            "# 16-bit word per iteration, not vectorized.  Check: %s" % ("PASS" if ok else "FAIL")] + \
           ["# " + r for r in rep] + [""] + body
    with open(os.path.join(HERE, "objdump_in_cksum.txt"), "w") as f:
        f.write("\n".join(text) + "\n")
    print("\n".join(rep))
    print("PASS" if ok else "FAIL")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
