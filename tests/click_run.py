"""Running Click userlevel drivers built by tools/click_scratch_build.sh
(click_integration/bin/click-{cpu,dropin,parity}) from the tests and the
bench: the reference's elements (click-cpu), the GPU elements under the
reference names (click-dropin) and both side by side (click-parity).  The
binaries are built in this container from a scratch copy of the reference
with click_integration/elements/hip overlaid; they travel to the GPU box with
the tree (git-ignored)."""
import os
import struct
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "click_integration", "bin")
CONF = os.path.join(ROOT, "click_integration", "conf")


def binary(mode):
    """Path of click-<mode>, or None when it was not built."""
    p = os.path.join(BIN, "click-" + mode)
    return p if os.access(p, os.X_OK) else None


def env(extra=None):
    e = dict(os.environ, **(extra or {}))
    libs = [os.path.join(ROOT, "click_amd"), "/opt/rocm/lib"]
    e["LD_LIBRARY_PATH"] = ":".join(libs + ([e["LD_LIBRARY_PATH"]] if e.get("LD_LIBRARY_PATH") else []))
    return e


def run(mode, conf=None, defines=None, handlers=(), expr=None, timeout=300, cwd=None, extra_env=None, threads=0):
    """Run click-<mode> on a config file (or -e expr) with NAME=value
    defines (threads: click -j N); returns (returncode, {handler: text},
    stderr)."""
    cmd = [binary(mode)] + (["-j", str(threads)] if threads else [])
    if expr is not None:
        cmd += ["-e", expr]
    else:
        cmd += [conf if os.path.isabs(conf) else os.path.join(CONF, conf)]
    for k, v in (defines or {}).items():
        cmd.append("%s=%s" % (k, v))
    for h in handlers:
        cmd += ["-h", h]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env(extra_env), cwd=cwd)
    vals = {}
    # click -h prints "NAME:\nVALUE" blocks (one line values: "NAME: VALUE")
    lines = p.stdout.splitlines()
    i = 0
    while i < len(lines):
        ln = lines[i]
        for h in handlers:
            if ln.startswith(h + ":"):
                rest = ln[len(h) + 1:].strip()
                if rest:
                    vals[h] = rest
                else:
                    body = []
                    while i + 1 < len(lines) and not any(lines[i + 1].startswith(x + ":") for x in handlers):
                        i += 1
                        body.append(lines[i])
                    vals[h] = "\n".join(body).strip()
                break
        i += 1
    return p.returncode, vals, p.stderr


def write_pcap(path, frames, linktype=1, t0=1000000000):
    """frames: list of bytes; record k stamped t0 s + k us (distinct)."""
    with open(path, "wb") as f:
        f.write(struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 65535, linktype))
        for k, fr in enumerate(frames):
            f.write(struct.pack("<IIII", t0 + k // 1000000, k % 1000000, len(fr), len(fr)))
            f.write(fr)


def read_pcap(path):
    """[(ts_sec, ts_usec, orig_len, bytes)] of a little-endian pcap file."""
    out = []
    with open(path, "rb") as f:
        b = f.read()
    magic = struct.unpack_from("<I", b, 0)[0]
    assert magic in (0xA1B2C3D4, 0xA1B23C4D), hex(magic)
    o = 24
    while o + 16 <= len(b):
        s, us, incl, orig = struct.unpack_from("<IIII", b, o)
        out.append((s, us, orig, b[o + 16:o + 16 + incl]))
        o += 16 + incl
    return out
