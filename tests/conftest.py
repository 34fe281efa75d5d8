"""Test configuration: `-m gpu` tests need a real MI355X; everything else runs on CPU.

The oracle under oracle/ is test infrastructure (parity checker); the product is the HIP
library under amc-slam_amd/ loaded through amc_lba (no CPU fallback).
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "amc-slam_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD GPU (MI355X) and the built HIP library")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def harness():
    """Host build of the product's per-observation math (tests/native/math_harness.cpp)."""
    import ctypes
    import subprocess
    src = os.path.join(ROOT, "tests", "native", "math_harness.cpp")
    out = os.path.join(ROOT, "tests", "native", "_build", "libmath_harness.so")
    deps = [src, os.path.join(ROOT, "amc-slam_amd", "csrc", "lba_math.hpp")]
    if not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(d) for d in deps):
        os.makedirs(os.path.dirname(out), exist_ok=True)
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", src, "-o", out])
    return ctypes.CDLL(out)


@pytest.fixture(scope="session")
def plan_harness():
    """Host build of the reduced camera system's ordering / symbolic factorisation (lba_plan.hpp)."""
    import ctypes
    import subprocess
    src = os.path.join(ROOT, "tests", "native", "plan_harness.cpp")
    out = os.path.join(ROOT, "tests", "native", "_build", "libplan_harness.so")
    deps = [src, os.path.join(ROOT, "amc-slam_amd", "csrc", "lba_plan.hpp")]
    if not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(d) for d in deps):
        os.makedirs(os.path.dirname(out), exist_ok=True)
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", src, "-o", out])
    return ctypes.CDLL(out)
