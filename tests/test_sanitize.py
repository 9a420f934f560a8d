"""ASan + UBSan run of the host-only code (SURVEY §5 "Race detection / sanitizers"): the library's
host translation units (alist parser, channel model, encoder) and the oracle restatement, built by
tests/sanitize/Makefile and driven by tests/sanitize/san_driver.cpp -- including truncated and
hostile alist text, the input the reference's unchecked ReadH (ArrayLDPC_Decoder.cpp:642-674)
would read out of bounds on.  GPU sanitizers are not available on this pool."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("make") is None, reason="needs g++ and make")
def test_host_code_under_asan_ubsan(tmp_path):
    env = {**os.environ, "OUT": str(tmp_path)}
    p = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "sanitize"), "-j4", "run"], capture_output=True,
                       text=True, timeout=600, env=env)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    assert "all checks passed" in p.stdout
    assert "ERROR: AddressSanitizer" not in p.stderr and "runtime error" not in p.stderr, p.stderr[-3000:]
