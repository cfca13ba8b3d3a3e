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
