"""A/B builds of the main kernel translation unit (fpldpc_kernels.hip: R's MixChecks kernel, the
fallbacks, the per-frame kernels) under other code-generation options: build/ab/<name>.so."""
import os, sys; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fixedpointldpc_amd import _build as b
base = dict(b.SOURCE_FLAGS)
X = "-Xarch_device"
V = {
    "m_trk_npr": [X, "-mllvm=-amdgpu-use-amdgpu-trackers", X, "-mllvm=-disable-post-ra"],
    "m_npr": [X, "-mllvm=-disable-post-ra"],
    "m_none": [],
    "m_npr_ilp": [X, "-mllvm=-disable-post-ra", X, "-mllvm=-misched=ilpmax"],
}
for name in sys.argv[1:] or V:
    b.SOURCE_FLAGS = dict(base)
    b.SOURCE_FLAGS["fpldpc_kernels.hip"] = V[name]
    b.build_variant(f"build/ab/{name}.so", [])
    print(name, "ok")
