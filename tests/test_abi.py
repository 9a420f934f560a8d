"""The C ABI library (libfpldpc.so) loads and exports every symbol include/*.h declares; without a
GPU, decoder creation fails loudly (there is no CPU decode path).  CPU only."""
import ctypes
import glob
import os
import re

import pytest

from conftest import ROOT


def _declared():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names |= set(re.findall(r"\b(fpldpc_[a-z0-9_]+)\s*\(", src))
    return sorted(names)


def test_every_declared_symbol_is_exported(F):
    lib = F.lib()
    names = _declared()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    from fixedpointldpc_amd import _lib
    assert sorted(_lib.EXPORTED) == names


def test_per_kernel_translation_units():
    """The A and W kernels are built in translation units of their own with their own code-generation
    options (DESIGN §5 "Code generation per kernel"): the sources, their flags and the build-id
    hashing all name them, and the main unit takes their host stubs from there instead of
    instantiating the kernels."""
    from fixedpointldpc_amd import _build
    assert "fpldpc_kernels_a1.hip" in _build.SOURCES and "fpldpc_kernels_a1.hip" in _build.DEVICE_TUS
    for src, flags in _build.SOURCE_FLAGS.items():
        assert src in _build.SOURCES, src
        # device-side only (-Xarch_device before each -mllvm=): the host compile stays plain
        assert all(f == "-Xarch_device" for f in flags[0::2]) and all(f.startswith("-mllvm=") for f in flags[1::2])
    a1 = open(os.path.join(_build.CSRC, "fpldpc_kernels_a1.hip")).read()
    assert "#define FPLDPC_TU_ARRAY1 1" in a1 and '#include "fpldpc_kernels.hip"' in a1
    main = open(os.path.join(_build.CSRC, "fpldpc_kernels.hip")).read()
    assert "reinterpret_cast<KernelFn>(const_cast<void *>(array47_pair_kernel()))" in main
    w1 = open(os.path.join(_build.CSRC, "fpldpc_kernels_w1.hip")).read()
    assert "#define FPLDPC_TU_TABLE1 1" in w1 and '#include "fpldpc_kernels.hip"' in w1
    assert "fpldpc_kernels_w1.hip" in _build.SOURCES and "fpldpc_kernels_w1.hip" in _build.DEVICE_TUS
    assert "reinterpret_cast<KernelFn>(const_cast<void *>(table8_pair_kernel()))" in main
    out = __import__("subprocess").run(["nm", "-DC", _build.LIB], capture_output=True, text=True).stdout
    assert "fpldpc::array47_pair_kernel()" in out and "fpldpc::table8_pair_kernel()" in out


def test_version_and_defaults(F):
    lib = F.lib()
    assert b"gfx950" in lib.fpldpc_version()
    from fixedpointldpc_amd._lib import Params
    p = Params()
    lib.fpldpc_params_default(ctypes.byref(p))
    assert (p.max_iter, p.frac_bits, p.width_mask, p.early_term, p.precheck, p.device) == (30, 4, 0xFF, 1, 0, -1)


def test_rng_skip_matches_stepping(F, O):
    import ctypes as C
    s = C.c_int64(123456789)
    for _ in range(1000):
        O.lib().orc_random(C.byref(s))
    assert F.rng_skip(123456789, 1000) == s.value
    assert F.rng_skip(1, 10000) == 399268537  # rngs.cpp:154-180 CHECK


def test_decoder_without_gpu_fails_loudly(F):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(F.FpldpcError) as e:
        F.Decoder(F.Code.array(47, 5))
    assert e.value.code == -5


def test_channel_int16_overflow_is_an_error(F):
    import numpy as np
    with pytest.raises(F.FpldpcError):
        F.channel_llr(123456789, 0, 2, 64, 5000.0, 0.01, 4, dtype=np.int16)


def test_compat_header_cpu_program(F, tmp_path):
    """include/fpldpc_compat.hpp compiled into a C++ program against libfpldpc.so; exercises the
    reference API members that need no GPU (tests/cpp/compat_cpu.cpp)."""
    import subprocess
    F.lib()
    pkg = os.path.join(ROOT, "fixedpointldpc_amd")
    exe = str(tmp_path / "compat_cpu")
    subprocess.run(["g++", "-std=c++17", "-O1", "-I", os.path.join(ROOT, "include"), "-I", "/opt/rocm/include",
                    "-D__HIP_PLATFORM_AMD__", os.path.join(ROOT, "tests", "cpp", "compat_cpu.cpp"), "-o", exe,
                    "-L", pkg, "-lfpldpc", f"-Wl,-rpath,{pkg}", "-Wl,-rpath,/opt/rocm/lib"], check=True)
    p = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and p.stdout.strip() == "ok", p.stderr
