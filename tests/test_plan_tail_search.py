"""make_plan's loop-closure tail search (amc-slam_amd/csrc/lba_plan.hpp) was rewritten from a scan per (c, a) to
a running max over the envelope's first panels (O(NP^2)); scripts/micro/tail_search_eq.cpp holds both forms and
compares them on 20000 random envelopes (banded, with random loop-closure rows).  Host only."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_tail_search_forms_agree(tmp_path):
    exe = tmp_path / "tail_eq"
    subprocess.run(["g++", "-O2", "-o", str(exe), os.path.join(ROOT, "scripts", "micro", "tail_search_eq.cpp")],
                   check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    assert out.strip() == "mismatches 0"
