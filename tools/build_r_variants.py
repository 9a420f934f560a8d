"""A/B builds of R's MixChecks kernel with the three 256-thread blocks of waves in other roles
(FPLDPC_R_ROLES digit b = role of block b: 0 two whole checks, 1 one check + split units, 2 one check;
the default 0x210).  build/ab/r<roles>.so, loaded by FPLDPC_LIB_PATH."""
import os, sys; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fixedpointldpc_amd import _build as b
for roles in sys.argv[1:] or ["0x012", "0x201", "0x120", "0x102", "0x021"]:
    b.build_variant(f"build/ab/r{roles[2:]}.so", [f"FPLDPC_R_ROLES={roles}"])
    print(roles, "ok")
