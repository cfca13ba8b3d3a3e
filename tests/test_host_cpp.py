"""Runs tests/cpp/host_test (the C++ host mirror, include/reflow_host.hpp)
which restates the reference's digest tests -- flow_test.go:24-58,
executor_test.go:62-86, syntax/digest_test.go:13-29 -- against the device."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "host_test")


def test_host_test_built_and_linked():
    assert os.path.exists(BIN), "run __graft_entry__.build()"
    out = subprocess.run(["ldd", BIN], capture_output=True, text=True).stdout
    assert "libreflow_hip.so" in out and "not found" not in out.split("libreflow_hip.so")[1].split("\n")[0]


@pytest.mark.gpu
def test_host_mirror_reference_goldens():
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "PASS"


@pytest.mark.gpu
def test_lower_bench_collapsed_hand_over():
    """tools/lower_bench on a small 1000align Flow graph, once with the shared
    reference chain and once with a copy per sample: Canonicalize collapses
    3 x (samples - 1) copies and hands over its Eval with their jobs dropped;
    the canonical root, the job count and the incremental step (checked
    against a full recompute inside) equal the shared-chain run's."""
    import json
    exe = os.path.join(ROOT, "tools", "lower_bench")
    runs = []
    for extra in ([], ["dup"]):
        r = subprocess.run([exe, "40", "4"] + extra, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
        runs.append(json.loads(r.stdout.strip().splitlines()[-1]))
    shared, dup = runs
    assert shared["collapsed"] == 0 and dup["collapsed"] == 3 * 39
    assert dup["canonicalize_handed_over"] and dup["incremental_equals_full"]
    assert dup["root"] == shared["root"]
    assert dup["jobs"] == shared["jobs"] and dup["jobs_rehashed"] == shared["jobs_rehashed"]
