"""The multi-device simulation's frame partition and ordered stop rule (fpldpc_sim_plan.hpp, used by
fpldpc_ber_sim and fpldpc_ber_sim_multi) against the reference's serial frame loop
(PerfTest.cpp:97-135), on the CPU: 20000 random trials over rank counts 1-8, chunk sizes, frame
offsets, frame-error and frame-count limits (tests/cpp/sim_plan_test.cpp)."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_partition_and_stop_rule(tmp_path):
    exe = str(tmp_path / "sim_plan_test")
    subprocess.run(["g++", "-std=c++17", "-O2", "-I", os.path.join(ROOT, "fixedpointldpc_amd", "csrc"), "-o", exe,
                    os.path.join(ROOT, "tests", "cpp", "sim_plan_test.cpp")], check=True, timeout=300)
    p = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    assert " 0 mismatches" in p.stdout
