"""CPU tests of bench.py's host logic: the multi-rank launch contract, the
corruption picks the timed Check passes are verified against, and the CPU
baseline legs on a small sample."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_refuses_mislabelled_world():
    """WORLD_SIZE != --gpus must fail before anything touches a GPU."""
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
    assert "refusing" in r.stderr


def test_corrupt_picks_match_the_kernel_hash(oracle):
    """bench.corrupt_picks restates corrupt_kernel's pick: the low bits of
    splitmix64(seed ^ (first + i) * C) (oracle_splitmix64 is the same hash
    as the device's, tests/test_oracle.py)."""
    import bench
    first, n = 123456789, 5000
    picks = bench.corrupt_picks(first, n)
    C = 0xD1B54A32D192ED03
    exp = [(oracle.oracle_splitmix64(bench.CORRUPT_SEED ^ (((first + i) * C) & (2**64 - 1))) & 1023) == 0
           for i in range(n)]
    assert np.array_equal(picks, np.array(exp))
    assert 0 < picks.sum() < n // 100


def test_cpu_baseline_legs_small(monkeypatch):
    """Every leg runs pinned, processes every packet of its sample and
    reports the median of 5 passes."""
    import bench
    monkeypatch.setenv("CLK_CPU_SAMPLE_BYTES", str(24 << 20))
    monkeypatch.setenv("CLK_CPU_THREADS", "2")
    r = bench.cpu_baseline(legs=("c2", "c3", "c4", "c5"))
    assert r["threads"] == 2
    for wl, leg in r["legs"].items():
        for label in ("single_thread", "all_cores"):
            x = leg[label]
            assert x["ok"] == x["packets"] > 0, (wl, label)
            assert x["pinned"] == x["threads"]
            assert x["min_s"] <= x["median_s"] <= x["max_s"]
            assert x["value"] > 0 and x["mpps"] > 0


def test_config1_cpu_forwards_everything():
    import bench
    r = bench.config1_cpu(20000)
    assert r["elements"]["forwarded"] == 20000 and r["combos"]["forwarded"] == 20000


def test_cpu_baseline_object_code(oracle):
    """The timed restatement is the scalar movzwl/add word loop SURVEY §6
    describes for the reference at -O2, called (not inlined or vectorized)
    by every element function (oracle/objdump_check.py; the committed
    oracle/objdump_in_cksum.txt is its output)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("objdump_check", os.path.join(ROOT, "oracle", "objdump_check.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    ok, rep, body = m.check()
    assert ok, rep
    assert any(i.startswith("movzwl") for i in body)
