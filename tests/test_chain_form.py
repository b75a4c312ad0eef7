"""The Click adapter's chain rules on the CPU.

`click_integration/elements/hip/hipchain.hh` decides which GPU-backed
elements run as one clk_chain (hipbatch.cc applies it over Click's Router at
initialize()).  `tests/native/chain_form_test.cc` instantiates the same
templates over router graphs built in the test -- conf/fake-iprouter.click's
interface path, the five elements back to back, the combos (IPOutputCombo a member), a head-only class, two upstreams,
DEVICE and CHAIN differences, other ports, pull context, a ring, a line
longer than the pass report's 64 members -- with the shipped class traits
(hipclasses.hh), and checks each chain and the head's packet readying.
No GPU and no glue library: the header compiles with g++ alone.
"""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_chain_formation_rules(tmp_path):
    exe = str(tmp_path / "chain_form_test")
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Wextra", "-Werror", "-I" + os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "native", "chain_form_test.cc"), "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = r.stdout.splitlines()
    assert lines[-1] == "ALL OK"
    assert sum(ln.startswith("PASS ") for ln in lines) == 19
