"""The adapter core's containers on the CPU: `tests/native/core_units_test.cc`
checks the held-packet ring (`hipcore::HeldRing`, a power-of-two ring with a
kept mask, grown by doubling while its packets wrap) against a std::deque
model over 400 rounds of bursts, and a result chunk's put / at round trip.
No GPU and no glue library: the header compiles with g++ alone."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_core_containers(tmp_path):
    exe = str(tmp_path / "core_units_test")
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Wextra", "-Werror", "-I" + os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "native", "core_units_test.cc"), "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = r.stdout.splitlines()
    assert lines[-1] == "ALL OK"
    assert sum(ln.startswith("PASS ") for ln in lines) == 2
