"""Build libfpldpc.so in-tree with hipcc for gfx950 (no JIT, no site-packages install)."""
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libfpldpc.so")
CLI = os.path.join(PKG, "fpldpc_perftest")
CLI_SRC = os.path.join(PKG, "tools", "fpldpc_perftest.cpp")
SOURCES = [
    "fpldpc_code.cpp",
    "fpldpc_decoder.cpp",
    "fpldpc_channel.cpp",
    "fpldpc_sim.cpp",
    "fpldpc_encoder.cpp",
    "fpldpc_perftest.cpp",
    "fpldpc_kernels.hip",
    "fpldpc_gen.hip",
    "fpldpc_float.hip",
]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# the sources that decide what runs on the device (kernels, their launch front-end and kernel
# choice, the ABI structs): their hash is the library's kernel build id
KERNEL_SOURCES = ["fpldpc_kernels.hip", "fpldpc_float.hip", "fpldpc_gen.hip", "fpldpc_internal.hpp"]
ARCH = "gfx950"


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(verbose=False, force=False):
    srcs = [os.path.join(CSRC, s) for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]
    deps = srcs + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hpp", ".h"))]
    deps += [os.path.join(ROOT, "include", f) for f in os.listdir(os.path.join(ROOT, "include"))]
    if force or _stale(LIB, deps):
        _build_lib(srcs, verbose)
    if force or _stale(CLI, [LIB, CLI_SRC] + deps):
        # the PerfTest driver links the library in place (rpath $ORIGIN: both travel together)
        cmd = [HIPCC, "-O2", "-std=c++17", "-I", os.path.join(ROOT, "include"), "-o", CLI + f".tmp{os.getpid()}", CLI_SRC,
               "-L", PKG, "-lfpldpc", "-Wl,-rpath,$ORIGIN"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        os.replace(CLI + f".tmp{os.getpid()}", CLI)
    return LIB


BASE_FLAGS = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-Wall",
              "-Wno-unused-function"]


def kernel_build_id(defines=(), flags=()):
    """sha256 over the device sources, include/fpldpc.h and the compile flags (16 hex digits)."""
    import hashlib
    h = hashlib.sha256()
    for f in KERNEL_SOURCES:
        h.update(f.encode() + b"\0" + open(os.path.join(CSRC, f), "rb").read())
    h.update(open(os.path.join(ROOT, "include", "fpldpc.h"), "rb").read())
    h.update(" ".join([*BASE_FLAGS, *defines, *flags]).encode())
    return h.hexdigest()[:16]


def _build_lib(srcs, verbose, out=LIB, defines=(), flags=()):
    bid = kernel_build_id(defines, flags)
    cmd = [HIPCC, *BASE_FLAGS, *[f"-D{d}" for d in defines], *flags, f'-DFPLDPC_KERNEL_BUILD_ID="{bid}"',
           "-I", os.path.join(ROOT, "include"), "-I", CSRC, "-o", out + f".tmp{os.getpid()}"] + srcs + [
               "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib", "-lpthread"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(out + f".tmp{os.getpid()}", out)  # atomic: concurrent ranks may build at once


def build_variant(out, defines, verbose=False, flags=()):
    """Experiments only: the same sources with extra -D defines (and compiler flags) into `out`
    (loaded through FPLDPC_LIB_PATH by bench.py / tools/gpu_ab.sh for A/B runs)."""
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    srcs = [os.path.join(CSRC, s) for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]
    _build_lib(srcs, verbose, out=out, defines=defines, flags=flags)
    return out


if __name__ == "__main__":
    print(build(verbose=True, force="--force" in sys.argv))
