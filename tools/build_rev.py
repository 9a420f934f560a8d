#!/usr/bin/env python3
"""Build libfpldpc.so from the sources of a git revision into OUT (A/B runs against an earlier
state of the kernels: FPLDPC_LIB_PATH=OUT).  usage: tools/build_rev.py REV OUT"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(rev, out):
    with tempfile.TemporaryDirectory() as td:
        tar = subprocess.run(["git", "-C", ROOT, "archive", rev, "fixedpointldpc_amd", "include"], check=True,
                             capture_output=True).stdout
        subprocess.run(["tar", "-x", "-C", td], input=tar, check=True)
        sys.path.insert(0, td)
        from fixedpointldpc_amd import _build
        _build.build_variant(os.path.abspath(out), [])
    print(out)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
