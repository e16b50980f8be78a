"""The C++ header API (include/neo/fft.hpp, include/neo/convolution.hpp) compiles
against libneo_hip.so and passes the reference's hot-path tests re-expressed in
tests/cpp/test_api.cpp (GPU part on the device)."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPP = os.path.join(REPO, "tests", "cpp")
BIN = os.path.join(CPP, "bin", "test_api")


def build():
    subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle"), "liboracle.so"])
    subprocess.check_call(["make", "-s", "-C", CPP, "bin/test_api", "bin/test_group"])
    return BIN


def test_cpp_api_builds_and_host_checks():
    b = build()
    r = subprocess.run([b], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.gpu
def test_cpp_api_on_gpu():
    b = build()
    r = subprocess.run([b], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "all C++ API tests passed" in r.stdout


@pytest.mark.gpu
def test_cpp_convolver_groups_on_gpu():
    """The plugin's std::vector<upols_convolver> pattern with the group-backed alias
    (NEO_HIP_CONVOLVER_GROUPS, tests/cpp/test_group.cpp): 256 instances equal one
    upols_multichannel bit for bit, one launch per frame after three watched frames."""
    build()
    r = subprocess.run([os.path.join(CPP, "bin", "test_group")], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "group test passed" in r.stdout
