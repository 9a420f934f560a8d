#!/usr/bin/env python3
"""Issue-stall attribution of the flood kernels from tools/gpu_attr.sh's three --pmc passes per config.

Per config: every counter per launch of the main flood kernel (the fallback kernels' empty launches
are excluded; per-launch mean over the profiled launches), and the ratios that locate the stalls:
  wait_inst_any / wave_cycles   waves waiting on an instruction dependency (s_waitcnt)
  wait_inst_lds / wave_cycles   ... of which on LDS results
  wait_any / wave_cycles        waves waiting for anything (incl. barriers)
  active_valu / wave_cycles     cycles a wave issues VALU
  salu, smem, branch, lds per VALU instruction
  lds bank-conflict share of LDS-active cycles
usage: tools/pmc_attr.py gpurun_out/<tag> [out.json]
"""
import csv
import json
import os
import sys


def per_launch(d):
    rows = list(csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))))
    # the main kernel: the flood kernel with the most time (the fallbacks run empty)
    dur = {}
    for r in rows:
        if "flood" in r["Kernel_Name"]:
            dur.setdefault(r["Kernel_Name"], []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    main = max(dur, key=lambda k: sum(dur[k]) / len(dur[k]))
    acc = {}
    for r in rows:
        if r["Kernel_Name"] == main:
            acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    out = {k: sum(v) / len(v) for k, v in acc.items()}
    out["_launch_ns"] = sum(dur[main]) / len(dur[main])
    return main, out


def main(src, dst=None):
    res = {}
    for cfg in ("A", "W", "R"):
        c, kern = {}, None
        for p in (1, 2, 3):
            d = os.path.join(src, f"{cfg}_p{p}")
            if os.path.isdir(d):
                kern, v = per_launch(d)
                c.update(v)
        if not c:
            continue
        wc = c["SQ_WAVE_CYCLES"]
        valu = c["SQ_INSTS_VALU"]
        r = {
            "kernel": kern,
            "wait_inst_any_per_wave_cycle": c["SQ_WAIT_INST_ANY"] / wc,
            "wait_inst_lds_per_wave_cycle": c["SQ_WAIT_INST_LDS"] / wc,
            "wait_any_per_wave_cycle": c["SQ_WAIT_ANY"] / wc,
            "active_inst_any_per_wave_cycle": c["SQ_ACTIVE_INST_ANY"] / wc,
            "active_valu_per_wave_cycle": c["SQ_ACTIVE_INST_VALU"] / wc,
            "active_sca_per_wave_cycle": c.get("SQ_ACTIVE_INST_SCA", 0) / wc,
            "active_lds_per_wave_cycle": c.get("SQ_ACTIVE_INST_LDS", 0) / wc,
            "active_misc_per_wave_cycle": c.get("SQ_ACTIVE_INST_MISC", 0) / wc,
            "salu_per_valu": c.get("SQ_INSTS_SALU", 0) / valu,
            "smem_per_valu": c.get("SQ_INSTS_SMEM", 0) / valu,
            "branch_per_valu": c.get("SQ_INSTS_BRANCH", 0) / valu,
            "lds_per_valu": c.get("SQ_INSTS_LDS", 0) / valu,
            "lds_atomic_per_lds": c.get("SQ_INSTS_LDS_ATOMIC", 0) / max(c.get("SQ_INSTS_LDS", 1), 1),
            "lds_bank_conflict_per_active": c.get("SQ_LDS_BANK_CONFLICT", 0) / max(c.get("SQ_LDS_IDX_ACTIVE", 1), 1),
            "lds_addr_conflict_per_active": c.get("SQ_LDS_ADDR_CONFLICT", 0) / max(c.get("SQ_LDS_IDX_ACTIVE", 1), 1),
            "thread_valu_lanes_per_inst": c["SQ_THREAD_CYCLES_VALU"] / max(c.get("SQ_ACTIVE_INST_VALU", 1), 1),
            "ifetch_per_valu": c.get("SQ_IFETCH", 0) / valu,
            "counters": c,
        }
        res[cfg] = r
        print(cfg, kern)
        for k, v in r.items():
            if k not in ("counters", "kernel"):
                print(f"   {k:34s} {v:.4f}")
    if dst:
        json.dump(res, open(dst, "w"), indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:])
