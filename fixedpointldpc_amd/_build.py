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
    "fpldpc_kernels_a1.hip",
    "fpldpc_kernels_w1.hip",
    "fpldpc_gen.hip",
    "fpldpc_float.hip",
]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
# Translation units that hold device code (and the host code that picks and launches it)
DEVICE_TUS = ["fpldpc_kernels.hip", "fpldpc_kernels_a1.hip", "fpldpc_kernels_w1.hip", "fpldpc_float.hip", "fpldpc_gen.hip"]
# Per-source code-generation options (profiles/r5/ab/post_ra.txt).  The A kernel's translation unit
# runs without the post-RA machine scheduler (+3.3 % / +3.8 % on A at 0 / 4.5 dB, while W and R lose
# 5 % / 2 % with it off) and with the generic bottom-up max-ILP machine scheduler (+1.4 % / +1.3 % on
# top).  The other kernels' unit schedules with the AMDGPU register-pressure trackers: R +1.2 %, W
# unchanged (A -3 % with them).  The W kernel's unit (with its split tail, round 6) runs without the
# post-RA scheduler too: W +0.3 % / W @ 2 dB +1.1 % over the trackers, whose W split build lost 0.6 % at
# 30 iterations (profiles/r6/ab/w_split_options.txt).  -mllvm= joined form under -Xarch_device: device
# compile only.
SOURCE_FLAGS = {"fpldpc_kernels_a1.hip": ["-Xarch_device", "-mllvm=-disable-post-ra", "-Xarch_device", "-mllvm=-misched=ilpmax"],
                "fpldpc_kernels.hip": ["-Xarch_device", "-mllvm=-amdgpu-use-amdgpu-trackers"],
                "fpldpc_kernels_w1.hip": ["-Xarch_device", "-mllvm=-disable-post-ra"]}
HASHED_TUS = DEVICE_TUS + ["fpldpc_decoder.cpp"]  # + the tables and launch arguments the kernels read
_PROBED = {}


def _option_ok(opt):
    """One trial device compile per LLVM-internal option (checked on ROCm 7.2's hipcc): such options
    are not a stable interface, and one that a later LLVM renames or drops must cost only its tuning,
    not the whole library build (it is left out with a warning; tests/test_codegen.py then names the
    lost option through the A unit's ISA)."""
    if opt not in _PROBED:
        import tempfile
        with tempfile.TemporaryDirectory() as d:
            src = os.path.join(d, "probe.hip")
            with open(src, "w") as f:
                f.write("#include <hip/hip_runtime.h>\n__global__ void k(int *p) { p[threadIdx.x] = 1; }\n")
            r = subprocess.run([HIPCC, f"--offload-arch={ARCH}", "--offload-device-only", "-c", src, "-o", os.devnull,
                                "-Xarch_device", opt], capture_output=True, text=True)
        _PROBED[opt] = r.returncode == 0
        if r.returncode:
            print(f"fpldpc build: {opt} rejected by {HIPCC}, building without it:\n{r.stderr.strip()}", file=sys.stderr)
    return _PROBED[opt]


def source_flags(name):
    """SOURCE_FLAGS[name] without the options this hipcc rejects."""
    fl = SOURCE_FLAGS.get(name, [])
    return [x for pair in zip(fl[0::2], fl[1::2]) if _option_ok(pair[1]) for x in pair]


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(verbose=False, force=False):
    srcs = [os.path.join(CSRC, s) for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]
    deps = srcs + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hpp", ".h"))]
    deps += [os.path.join(ROOT, "include", f) for f in os.listdir(os.path.join(ROOT, "include"))]
    deps.append(os.path.abspath(__file__))  # the flags (SOURCE_FLAGS) are part of the build
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


BASE_FLAGS = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wall",
              "-Wno-unused-function"]


def _alloc_sections(obj):
    """(name, bytes) of every allocated section with contents in an ELF64 relocatable object, in
    file order: code (.text and its per-function / template sections), constants (.rodata*), the
    initialised tables (.data*, .data.rel.ro*: e.g. the kernel-variant table, function pointers
    under -fPIC), the GPU code object (.hip_fatbin)."""
    import struct
    b = open(obj, "rb").read()
    assert b[:4] == b"\x7fELF" and b[4] == 2, obj
    shoff, = struct.unpack_from("<Q", b, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", b, 0x3A)
    hdrs = [struct.unpack_from("<IIQQQQIIQQ", b, shoff + i * shentsize) for i in range(shnum)]
    stroff = hdrs[shstrndx][4]

    def name(off):
        return b[stroff + off:b.index(b"\0", stroff + off)].decode()
    SHF_ALLOC, SHT_NOBITS = 0x2, 8
    return [(name(h[0]), b[h[4]:h[4] + h[5]]) for h in hdrs if h[2] & SHF_ALLOC and h[1] != SHT_NOBITS]


def _relocations(obj):
    """Every relocation that applies to an allocated section, as text: target section, offset, type,
    symbol NAME (section symbols by their section's name) and addend.  In a -fPIC relocatable object
    a call target or a function pointer in a table (e.g. kVariants in .data.rel.ro) is zero bytes in
    its section; which kernel it names lives only here.  Names, not symbol indices, so the text does
    not depend on symbol-table order."""
    import struct
    b = open(obj, "rb").read()
    shoff, = struct.unpack_from("<Q", b, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", b, 0x3A)
    hdrs = [struct.unpack_from("<IIQQQQIIQQ", b, shoff + i * shentsize) for i in range(shnum)]

    def cstr(off):
        return b[off:b.index(b"\0", off)].decode()
    secname = [cstr(hdrs[shstrndx][4] + h[0]) for h in hdrs]
    SHT_RELA, SHT_REL, SHF_ALLOC, STT_SECTION = 4, 9, 0x2, 3
    out = []
    for h in hdrs:
        if h[1] not in (SHT_RELA, SHT_REL) or not hdrs[h[7]][2] & SHF_ALLOC:
            continue
        sym = hdrs[h[6]]  # the symbol table (sh_link), its string table at sym's sh_link
        strtab = hdrs[sym[6]][4]
        esz = 24 if h[1] == SHT_RELA else 16
        for i in range(h[5] // esz):
            if h[1] == SHT_RELA:
                off, info, add = struct.unpack_from("<QQq", b, h[4] + i * esz)
            else:
                (off, info), add = struct.unpack_from("<QQ", b, h[4] + i * esz), 0
            st_name, st_info, _, st_shndx = struct.unpack_from("<IBBH", b, sym[4] + (info >> 32) * 24)
            nm = secname[st_shndx] if (st_info & 0xF) == STT_SECTION and st_shndx < len(hdrs) else cstr(strtab + st_name)
            out.append(f"{secname[h[7]]}+{off:x}:{info & 0xffffffff}:{nm}{add:+d}")
    return out


def kernel_build_id(objs):
    """sha256 (16 hex digits) of the machine code and tables of the device translation units: every
    allocated section of their objects -- the GPU code objects (.hip_fatbin, compiled with a fixed
    -cuid so that it is reproducible) and the host code, constants and initialised data that choose
    and launch the kernels (variant table, launch bounds, fallback chains) -- and every relocation
    applied to them (which kernel a table entry or a launch names: ADVICE r4).  Comments, file names
    and the other translation units do not change it; any change to what runs on the GPU, or to how it
    is chosen and launched, does."""
    import hashlib
    h = hashlib.sha256()
    for o in sorted(objs, key=os.path.basename):
        src = os.path.basename(o).split(".")[0]  # the source's name (object names carry a pid)
        for sec, data in _alloc_sections(o):
            h.update(f"{src}:{sec}:{len(data)}:".encode() + data)
        h.update(f"{src}:relocations:".encode() + "\n".join(_relocations(o)).encode())
    return h.hexdigest()[:16]


def _build_lib(srcs, verbose, out=LIB, defines=(), flags=()):
    """Each source to an object (in parallel), the kernel build id from the device objects, then
    fpldpc_code.cpp (which returns the id) and the shared library."""
    import concurrent.futures
    import hashlib
    tag = hashlib.sha256((out + "|" + " ".join(defines) + "|" + " ".join(flags)).encode()).hexdigest()[:10]
    objdir = os.path.join(ROOT, "build", "obj", tag)
    os.makedirs(objdir, exist_ok=True)
    common = [HIPCC, *BASE_FLAGS, *[f"-D{d}" for d in defines], *flags, "-I", os.path.join(ROOT, "include"), "-I", CSRC]

    def compile_one(src, extra=()):
        obj = os.path.join(objdir, os.path.basename(src) + f".{os.getpid()}.o")
        # a fixed compilation-unit id per file (hipcc's default is random), so that the device code
        # object, and with it the kernel build id, is reproducible
        cuid = "fpldpc_" + os.path.basename(src).replace(".", "_")
        cmd = [*common, f"-cuid={cuid}", *extra, "-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        return obj

    first = [x for x in srcs if os.path.basename(x) != "fpldpc_code.cpp"]
    with concurrent.futures.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        objs = list(ex.map(lambda x: compile_one(x, source_flags(os.path.basename(x))), first))
    bid = kernel_build_id([o for o, x in zip(objs, first) if os.path.basename(x) in HASHED_TUS])
    objs.append(compile_one(os.path.join(CSRC, "fpldpc_code.cpp"), (f'-DFPLDPC_KERNEL_BUILD_ID="{bid}"',)))
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out + f".tmp{os.getpid()}", *objs,
           "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib", "-lpthread"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    for o in objs:
        os.remove(o)
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
