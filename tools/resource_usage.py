#!/usr/bin/env python3
"""Per-kernel register / scratch / occupancy table of a .hip file (hipcc -Rpass-analysis=
kernel-resource-usage, device-only compile for gfx950): the quick check that a kernel change did not
add spills or drop occupancy, before any GPU run.

usage: tools/resource_usage.py [file.hip] [name-filter] [-D...]"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _source_flags(src):
    """The per-source options the library build uses (fixedpointldpc_amd/_build.py SOURCE_FLAGS)."""
    sys.path.insert(0, ROOT)
    from fixedpointldpc_amd._build import SOURCE_FLAGS
    return SOURCE_FLAGS.get(os.path.basename(src), [])


def usage(src, defines=()):
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
           "-I", os.path.join(ROOT, "include"), "-I", os.environ.get("RU_INC", os.path.join(ROOT, "fixedpointldpc_amd", "csrc")),
           "--offload-device-only", "-c", src, "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage",
           *_source_flags(src), *defines]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark: (.*?) \[-Rpass", line)
        if not m:
            continue
        t = m.group(1).strip()
        if t.startswith("Function Name:"):
            cur = {"name": t.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in t:
            k, v = t.split(":", 1)
            cur[k.strip()] = v.strip()
    return rows


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("-D")]
    defs = [a for a in sys.argv[1:] if a.startswith("-D")]
    src = args[0] if args else os.path.join(ROOT, "fixedpointldpc_amd", "csrc", "fpldpc_kernels.hip")
    filt = args[1] if len(args) > 1 else ""
    for r in usage(src, defs):
        if filt not in r["name"]:
            continue
        nm = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
        nm = nm.replace("fpldpc::(anonymous namespace)::", "")
        print(f"{nm[:90]:90s} VGPR {r.get('VGPRs','?'):>4} AGPR {r.get('AGPRs','?'):>3} "
              f"scratch {r.get('ScratchSize [bytes/lane]','?'):>4} occ {r.get('Occupancy [waves/SIMD]','?'):>2} "
              f"spill v/s {r.get('VGPRs Spill','?')}/{r.get('SGPRs Spill','?')}")


if __name__ == "__main__":
    main()
