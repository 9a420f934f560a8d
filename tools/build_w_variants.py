"""A/B builds of the W split form (FPLDPC_W_SPLIT=1) under different code-generation options for W's
translation unit (fpldpc_kernels_w1.hip) only: build/ab/<name>.so, loaded by FPLDPC_LIB_PATH."""
import os, sys; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sys
from fixedpointldpc_amd import _build as b
base = dict(b.SOURCE_FLAGS)
V = {
 "wsplit": (["FPLDPC_W_SPLIT=1"], ["-Xarch_device", "-mllvm=-amdgpu-use-amdgpu-trackers"]),
 "ws_notrk": (["FPLDPC_W_SPLIT=1"], []),
 "ws_ilp": (["FPLDPC_W_SPLIT=1"], ["-Xarch_device", "-mllvm=-misched=ilpmax"]),
 "ws_npr": (["FPLDPC_W_SPLIT=1"], ["-Xarch_device", "-mllvm=-disable-post-ra"]),
 "ws_trk_npr": (["FPLDPC_W_SPLIT=1"], ["-Xarch_device", "-mllvm=-amdgpu-use-amdgpu-trackers", "-Xarch_device", "-mllvm=-disable-post-ra"]),
}
for name, (defs, wflags) in V.items():
    b.SOURCE_FLAGS = dict(base); b.SOURCE_FLAGS["fpldpc_kernels_w1.hip"] = wflags
    b.build_variant(f"build/ab/{name}.so", defs)
    print(name, "ok")
