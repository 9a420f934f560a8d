"""A/B builds of R's MixChecks kernel: the three 256-thread blocks of waves in other roles
(FPLDPC_R_ROLES digit b = role of block b: 0 two whole checks, 1 one check + the split units, 2 one
check; default 0x210) and with per-block wave priorities (FPLDPC_R_PRIO digit b = s_setprio of block
b).  Arguments: name=ROLES[,PRIO] ...; build/ab/<name>.so, loaded by FPLDPC_LIB_PATH."""
import os, sys; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fixedpointldpc_amd import _build as b
for arg in sys.argv[1:]:
    name, spec = arg.split("=")
    roles, *prio = spec.split(",")
    defs = [f"FPLDPC_R_ROLES={roles}"] + ([f"FPLDPC_R_PRIO={prio[0]}"] if prio else [])
    b.build_variant(f"build/ab/{name}.so", defs)
    print(name, defs, "ok")
