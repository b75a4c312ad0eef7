"""Build the gfx950 shared library (and the test oracle) in-tree.

    python -m click_amd.build            # product library only
    python -m click_amd.build --oracle   # also oracle/libcksum_oracle.so

The product library is click_amd/libclick_amd_cksum.so: the C ABI of
include/click_amd_cksum.h over the hand-written kernels in click_amd/csrc.
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "click_amd")
LIB = os.path.join(PKG, "libclick_amd_cksum.so")
SOURCES = [os.path.join(PKG, "csrc", "cksum_api.hip"), os.path.join(PKG, "host", "elements.cc"),
           os.path.join(PKG, "host", "chain.cc"), os.path.join(PKG, "host", "ingest.cc")]
DEPS = SOURCES + [os.path.join(PKG, "csrc", f) for f in ("cksum_kernels.hh", "cksum_device.hh", "frag_kernels.hh",
                                                                    "internal.hh")] + [
    os.path.join(PKG, "host", "elements.hh")] + [
    os.path.join(ROOT, "include", f) for f in ("click_amd_cksum.h", "click_amd_elements.h", "click_amd_ingest.h")]
ARCH = "gfx950"


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.sep not in c or os.path.exists(c)):
            return c
    raise RuntimeError("hipcc not found")


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build_library(force=False, verbose=False):
    if not force and not _stale(LIB, DEPS):
        return LIB
    cmd = [_hipcc(), "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wall", "-I" + os.path.join(ROOT, "include"), "-o", LIB + ".tmp"] + SOURCES
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(LIB + ".tmp", LIB)
    return LIB


def build_oracle(force=False):
    odir = os.path.join(ROOT, "oracle")
    target = os.path.join(odir, "libcksum_oracle.so")
    deps = [os.path.join(odir, f) for f in ("cksum_oracle.c", "cksum_oracle.h", "Makefile")]
    if force or _stale(target, deps):
        subprocess.run(["make", "-s", "-C", odir, "-B" if force else "all"], check=True)
    return target


EXAMPLES = ["pcap_check"]


def build_examples(force=False):
    """Plain-C programs over the ABI (examples/*.c) -> examples/bin/, linked
    against the in-tree library (rpath relative to the binary)."""
    lib = build_library()
    edir = os.path.join(ROOT, "examples")
    os.makedirs(os.path.join(edir, "bin"), exist_ok=True)
    out = []
    for name in EXAMPLES:
        src = os.path.join(edir, name + ".c")
        exe = os.path.join(edir, "bin", name)
        deps = [src, lib] + [os.path.join(ROOT, "include", h) for h in ("click_amd_cksum.h", "click_amd_ingest.h")]
        if force or _stale(exe, deps):
            subprocess.run(["gcc", "-std=c11", "-O2", "-Wall", "-Wextra", "-Werror", "-D__HIP_PLATFORM_AMD__",
                            "-I" + os.path.join(ROOT, "include"), "-I/opt/rocm/include", src,
                            "-L" + PKG, "-lclick_amd_cksum", "-L/opt/rocm/lib", "-lamdhip64",
                            "-Wl,-rpath,$ORIGIN/../../click_amd", "-Wl,-rpath,/opt/rocm/lib", "-o", exe], check=True)
        out.append(exe)
    return out


NATIVE_TESTS = ["hipcore_test", "pull_bench", "mt_glue"]
NATIVE_ORACLE = {"hipcore_test"}          # the measurement programs never link the oracle


def build_native_tests(force=False):
    """Host-only C++ test programs (tests/native/*.cc) -> tests/native/bin/,
    linked against the in-tree library and the test oracle (built here, on
    the CPU; the GPU tests only run them)."""
    lib = build_library()
    oracle = build_oracle()
    ndir = os.path.join(ROOT, "tests", "native")
    os.makedirs(os.path.join(ndir, "bin"), exist_ok=True)
    out = []
    for name in NATIVE_TESTS:
        src = os.path.join(ndir, name + ".cc")
        exe = os.path.join(ndir, "bin", name)
        hip = os.path.join(ROOT, "click_integration", "elements", "hip")
        deps = [src, lib, os.path.join(ndir, "harness.hh"), os.path.join(hip, "hipcore.hh"),
                os.path.join(hip, "hipclasses.hh"), os.path.join(hip, "hipchain.hh")] + [
            os.path.join(ROOT, "include", h) for h in ("click_amd_cksum.h", "click_amd_elements.h")]
        orc = name in NATIVE_ORACLE
        if orc:
            deps.append(oracle)
        if force or _stale(exe, deps):
            subprocess.run(["g++", "-std=c++17", "-O2", "-g", "-Wall", "-Wextra", "-pthread",
                            "-I" + os.path.join(ROOT, "include"), src, "-L" + PKG, "-lclick_amd_cksum"] +
                           (["-L" + os.path.join(ROOT, "oracle"), "-lcksum_oracle",
                             "-Wl,-rpath,$ORIGIN/../../../oracle"] if orc else []) +
                           ["-L/opt/rocm/lib", "-Wl,-rpath-link,/opt/rocm/lib",
                            "-Wl,-rpath,$ORIGIN/../../../click_amd", "-Wl,-rpath,/opt/rocm/lib", "-o", exe], check=True)
        out.append(exe)
    return out


if __name__ == "__main__":
    force = "--force" in sys.argv
    print(build_library(force=force, verbose=True))
    if "--oracle" in sys.argv:
        print(build_oracle(force=force))
    if "--examples" in sys.argv:
        print(build_examples(force=force))
    if "--native-tests" in sys.argv:
        print(build_native_tests(force=force))
