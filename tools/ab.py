#!/usr/bin/env python3
"""A/B runs of bench.py on the GPU box: every (case, variant) pair, interleaved over reps, each run
a child process under its own time limit; one summary line per run and a JSON record.

usage: tools/ab.py OUT_DIR REPS 'case=<bench args>' ... -- 'variant=<ENV=V,ENV2=V>' ...
  e.g. tools/ab.py gpurun_out/pre 2 'A=--config A' 'A45=--ebn0 4.5' -- 'off=FPLDPC_PRE_T=0' 'on='
Assignments in a variant are separated by '|' (values may hold commas).  A variant's env may name
FPLDPC_LIB_PATH (an alternative build of the same sources)."""
import json
import os
import subprocess
import sys
import time


def main():
    out, reps = sys.argv[1], int(sys.argv[2])
    rest = sys.argv[3:]
    k = rest.index("--")
    cases = [c.split("=", 1) for c in rest[:k]]
    variants = []
    for v in rest[k + 1:]:
        name, envs = v.split("=", 1)
        env = dict(e.split("=", 1) for e in envs.split("|") if e)
        variants.append((name, env))
    os.makedirs(out, exist_ok=True)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    rec = []
    for rep in range(reps):
        for cname, cargs in cases:
            for vname, venv in variants:
                tag = f"{cname}_{vname}_{rep}"
                t = time.time()
                p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--no-cpu", *cargs.split()],
                                   env={**os.environ, **venv}, capture_output=True, text=True, timeout=300)
                open(os.path.join(out, tag + ".err"), "w").write(p.stderr)
                if p.returncode != 0:
                    print(tag, "FAILED rc", p.returncode, p.stderr[-800:], flush=True)
                    sys.exit(1)
                line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1]
                open(os.path.join(out, tag + ".json"), "w").write(line + "\n")
                d = json.loads(line)
                r = {"case": cname, "variant": vname, "rep": rep, "value": d["value"],
                     "launch_ms": d["roofline"]["avg_launch_ms"], "avg_iters": d["ber"]["avg_iters"],
                     "parity": d["parity_vs_cpu_oracle"], "kernel": d["config"]["kernel"].split(" ")[0],
                     "wall_s": round(time.time() - t, 1)}
                rec.append(r)
                print(json.dumps(r), flush=True)
    json.dump(rec, open(os.path.join(out, "ab.json"), "w"), indent=1)
    print("summary (mean value per case / variant):")
    for cname, _ in cases:
        for vname, _ in variants:
            v = [r["value"] for r in rec if r["case"] == cname and r["variant"] == vname]
            ms = [r["launch_ms"] for r in rec if r["case"] == cname and r["variant"] == vname]
            print(f"  {cname:8s} {vname:10s} {sum(v) / len(v):10.1f} Mb/s  {sum(ms) / len(ms):.4f} ms  "
                  f"parity {all(r['parity'] is True for r in rec if r['case'] == cname and r['variant'] == vname)}")


if __name__ == "__main__":
    main()
