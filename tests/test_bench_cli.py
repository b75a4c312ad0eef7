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


def test_line_summary_is_last_and_complete(monkeypatch):
    """The bench line ends with `summary`: one entry per timed element of
    every workload section plus the fragmenter and config 1, so the tail of
    the line alone carries them (the driver keeps only the last few KB);
    cpu_baseline legs are compact; comm names the communicator."""
    import json
    import bench
    monkeypatch.setenv("CLK_CPU_SAMPLE_BYTES", str(8 << 20))
    monkeypatch.setenv("CLK_CPU_THREADS", "2")
    el = lambda ms, fr, m: {"roofline": {"kernel_ms": ms, "frac": fr},
                            "verify": {"drops_exact": True, "oracle": {"oracle_match": m}}}
    line = {"config": {"workload": "C3: x"},
            "elements": {"CheckUDPHeader": el(3.68, 0.855, True), "SetUDPChecksum": el(4.4, 0.71, True)},
            "c2_64b": {"workload": "C2: y", "elements": {"CheckIPHeader": el(0.17, 0.25, True)}},
            "c4_imix": {"workload": "C4: z", "elements": {"CheckUDPHeader": el(3.8, 0.82, True),
                                                         "SetUDPChecksum": el(5.3, 0.58, False)}},
            "fragmenter": {"kernel_ms": 8.9, "roofline": {"frac": 0.45},
                           "verify": {"fragmented": 5, "packets": 5, "appended_fragments": 10}},
            "c1_fake_iprouter": {"ok": True, "elements": {"mpps": 20.1}, "combos": {"mpps": 40.2}}}
    s = bench.bench_summary(line)
    assert s["C3 CheckUDPHeader"] == [3.68, 0.855, True, True]
    assert s["C4 SetUDPChecksum"][2] is False and s["C2 CheckIPHeader"][1] == 0.25
    assert s["C3 IPFragmenter"][2] is True and s["C1 mpps"] == {"elements": 20.1, "combos": 40.2}
    legs = bench.compact_legs(dict(bench.cpu_baseline(legs=("c2", "c3"))["legs"], c1=bench.config1_cpu(2000)))
    assert set(legs) == {"c2", "c3", "c1"} and len(legs["c3"]["all"]) == 3 and legs["c1"]["combos"] > 0
    assert len(json.dumps(legs)) + len(json.dumps(s)) < 2000
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert 'line["summary"] = bench_summary(line)\n        print(json.dumps(line)' in src
