#!/usr/bin/env python3
"""Headline benchmark: decoded information Mb/s of the fixed-point flooding decoder.

Workload (BASELINE.json configs[1]): the p=47, r=5 array code (2209, 1978) -- BASELINE's
"(2209,1974)" is a mislabel, k = 1978 -- 4096 frames per GPU, MAX_ITER 30, Q4.4
(FRAC 4), sxor mask 0xff.  Inputs are the reference harness's own channel (BPSK/AWGN, all-zero
codeword, Lehmer seed 123456789, Odeh-Evans normals, PerfTest.cpp:168-169) at Eb/N0 0 dB, where
every frame runs the full 30 iterations, quantised to int16 and resident in HBM
before the timed region.  One step = one fpldpc_decode launch over the batch.

Multi-GPU: one process per GPU (torchrun), rank r decodes frames [r*B, (r+1)*B) of the same
stream (skip-ahead), no data-path collective; one all-reduce of the BER counters at the end.

Prints ONE JSON line (rank 0) with roofline and cpu_baseline (the oracle's C restatement of
decode_general_fp, one core, timed on this host; calibrated against the reference's own decoder in
the newest profiles/r*/cpu_calibration.json, tools/cpu_calibrate.py, carried as
cpu_baseline.calibration).

roofline: the decoder keeps every message on chip (measured HBM traffic ~1/570 of an HBM-streaming
decoder's bytes), so its binding bound is VALU issue: "achieved" = wave-level VALU instructions per
launch (rocprofv3 SQ_INSTS_VALU, committed in profiles/r*/pmc_traffic.json for the kernel this run
uses) / this run's mean launch time, "peak" = one wave64 VALU instruction per 2 cycles per SIMD at
2.4 GHz (MI355X_MICROARCH.md).  Beside it: "algorithmic" (SURVEY 8d's 45 int ops per
edge-iteration over the int32 VALU lane peak) and "hbm_streaming_equivalent" (SURVEY 8d's
B_cw bytes over 8 TB/s, informational: > 1 means the on-chip design outruns HBM streaming).
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "decoded info Mb/s @ 30 iter, (2209,1974) array code; BER match vs CPU ref"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
VALU_CLOCK_GHZ = 2.4   # peak engine clock (MI355X_MICROARCH.md)
ALG_OPS_PER_EDGE_ITER = 45  # ~13 ops per sxor x (3d-4)/d sxor per edge + v2c/posterior/hard/syndrome
SEED = 123456789


def algorithmic_bytes_per_frame(n, e, iters):
    """B_cw = I*(8E + 4N) + 2N + ceil(N/8) (int16 messages, flooding schedule)."""
    return iters * (8 * e + 4 * n) + 2 * n + math.ceil(n / 8)


def _kernel_sig(name):
    """'flood_reg<DC=47,CPL=1,regular>' and 'fpldpc::(anonymous namespace)::flood_reg<47, 1, true>' -> ('flood_reg', (47, 1))."""
    import re
    m = re.search(r"(\w+)<([^>]*)>", name)
    return (m.group(1), tuple(int(x) for x in re.findall(r"\d+", m.group(2)))) if m else (name, ())


def find_profile(wkey, kernel_build_id, frames, ebn0, describe):
    """The newest committed rocprofv3 PMC summary (profiles/r*/pmc_traffic.json, written by
    tools/pmc_summary.py) that measured exactly this workload: the same decoder/config key (`A`,
    `W_float`, ...), kernel build (the library's fpldpc_kernel_build_id, a hash of the device machine
    code), frames per launch, Eb/N0 and kernel variant.  Counters of any other run do different work
    and are refused, never reported."""
    import glob
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_traffic.json")), reverse=True):
        try:
            entries = json.load(open(p))
        except (OSError, ValueError):
            continue
        for key, d in entries.items():
            if (d.get("workload", key) == wkey and d.get("kernel_build_id") == kernel_build_id
                    and d.get("profiled_frames") == frames and d.get("profiled_ebn0_db") == ebn0
                    and d.get("describe") == describe):
                return dict(d, file=os.path.relpath(p, ROOT), key=key)
    return None


def count_gpus():
    """GPUs this process may use, counted without initialising HIP (a launcher must not touch the
    GPU before its ranks start): the KFD topology's GPU nodes (simd_count > 0), limited by
    ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES when set."""
    import glob
    n = 0
    for p in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties"):
        try:
            props = dict(line.split()[:2] for line in open(p) if len(line.split()) >= 2)
        except OSError:
            continue
        if int(props.get("simd_count", "0")) > 0:
            n += 1
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip() != ""]))
    return n


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def usable_cores():
    """(threads, info): every CPU in this process's affinity mask, reduced to the cgroup CPU quota
    when one is set (cpu.max), so the all-cores leg uses what the job is actually granted."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, math.ceil(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    cores = min(aff, quota) if quota else aff
    return cores, {"nproc": os.cpu_count(), "affinity_cpus": aff, "cgroup_cpu_quota": quota}


def calibration(cfg):
    """The committed CPU-baseline calibration (tools/cpu_calibrate.py): the restatement's time over
    the reference decoder's on the same core and frames, in the build container."""
    import glob
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "cpu_calibration.json")), reverse=True):
        try:
            d = json.load(open(p))
        except (OSError, ValueError):
            continue
        c = d.get("configs", {}).get(cfg)
        if c:
            return {"port_over_reference_time": c["port_over_reference_time"],
                    "port_over_reference_time_median_paired": c.get("port_over_reference_time_median_paired"),
                    "bit_exact": c["bit_exact"],
                    "reference_ns_per_edge_iter": c["reference_ns_per_edge_iter"], "host_cpu": d.get("host_cpu"),
                    "file": os.path.relpath(p, ROOT)}
    return None


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_command(gpus, argv, env, port, python=sys.executable, script=None):
    """The command that starts this benchmark as `gpus` ranks (one process per GPU, torchrun on
    127.0.0.1), or None when this process is itself a rank (WORLD_SIZE set by a launcher) or one
    GPU was asked for.  argv is passed through unchanged, so every rank parses the same flags."""
    if gpus <= 1 or "WORLD_SIZE" in env:
        return None
    return [python, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", script or os.path.abspath(__file__), *argv]


def self_launch(args, argv):
    """`bench.py --gpus N` without an outer torchrun: start N ranks as child processes (before
    anything here touches the GPU: the devices are counted from the KFD topology, not through HIP)
    and exit with their status.  Rank 0 prints the one JSON line after the max-over-ranks timing and the counter
    all-reduce; it reaches stdout unchanged."""
    import subprocess
    cmd = launch_command(args.gpus, argv, os.environ, _free_port())
    if cmd is None:
        return
    if args.backend == "nccl":
        have = count_gpus()
        if have < args.gpus:
            print(f"bench.py: --gpus {args.gpus} needs {args.gpus} visible GPUs, found {have} "
                  f"(--backend gloo rehearses N ranks on a shared GPU)", file=sys.stderr, flush=True)
            sys.exit(2)
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")  # the ranks' host threads are sized explicitly (nthreads=)
    sys.exit(subprocess.run(cmd, env=env).returncode)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--min-warmup-s", type=float, default=0.25,
                    help="untimed warm-up continues past --warmup steps until this much decode time has passed: "
                         "the GPU clock settles over the first tens of ms of a sustained decode (a 3-step warm-up "
                         "measured 1.5 %% below a 30-step one, profiles/r1/warmup)")
    ap.add_argument("--config", choices=["A", "W", "R"], default="A")
    ap.add_argument("--batch", type=int, default=0, help="frames per GPU (default: 4096 A, 8192 W, 4096 R)")
    ap.add_argument("--ebn0", type=float, default=None)
    ap.add_argument("--cpu-frames", type=int, default=None,
                    help="oracle frames timed for cpu_baseline (default: the A and W batches, 512 R frames: about 10 s on one core)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="collective backend for N > 1 (gloo: rehearsal with ranks sharing one GPU)")
    ap.add_argument("--llr-fill", type=int, default=None,
                    help="diagnostic only: replace the channel LLRs by this constant (data-activity experiments)")
    ap.add_argument("--inflight-steps", type=int, default=0,
                    help="steps of the supplementary two-batches-in-flight measurement (default 0: not run, so that "
                         "a profile of the default command sees only the headline's launches)")
    ap.add_argument("--decoder", choices=["fixed", "float"], default="fixed",
                    help="fixed: decode_general_fp (the headline); float: decode_general, double BP (SURVEY 8f row 3)")
    args = ap.parse_args()
    self_launch(args, sys.argv[1:])  # returns only in a rank (or at N = 1)

    import torch
    import torch.distributed as dist
    import fixedpointldpc_amd as F
    from fixedpointldpc_amd import dist as D

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.backend == "gloo":  # rehearsal of the N > 1 path on a 1-GPU box: ranks share the visible GPUs
        local %= max(1, torch.cuda.device_count())
    # started by a launcher (torchrun sets WORLD_SIZE): a process group even at one rank, so that
    # the counter all-reduce runs through RCCL exactly as on N GPUs
    pg = "WORLD_SIZE" in os.environ
    if pg:
        torch.cuda.set_device(local)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))  # RCCL over xGMI
        else:
            dist.init_process_group("gloo")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    cfg = args.config
    if cfg == "A":
        code, max_iter, mask, batch, ebn0 = F.Code.array(47, 5), 30, 0xFF, 4096, 0.0
        wl = "A: p47/r5 array code (2209,1978), 30 iter, Q4.4, mask 0xff"
    elif cfg == "W":
        code, max_iter, mask, batch, ebn0 = F.Code.wifi_1944_r12(), 30, 0xFF, 8192, -2.0
        wl = "W: 802.11n (1944,972) R=1/2 Z=81, 30 iter, Q4.4, mask 0xff"
    else:
        code, max_iter, mask, batch, ebn0 = F.Code.array(47, 24), 50, 0x3F, 4096, 2.0
        wl = "R: p47/r24 array code (2209,1104), 50 iter, Q4.4, mask 0x3f"
    if args.batch:
        batch = args.batch
    if args.ebn0 is not None:
        ebn0 = args.ebn0
    rate = 0.5 if cfg == "W" else code.rate  # the WiFi harness hard-codes R = 0.5 (PerfTest.cpp:62)
    snr, sigma = F.snr_sigma(ebn0, rate)
    k_info = code.n - code.rank

    # Synthetic reference-harness frames for this rank, resident in HBM (int16).
    first, _ = D.frame_range(rank, world, batch)  # this rank's frames of the one RNG stream
    fl = args.decoder == "float"
    llr_host = F.channel_llr(SEED, first, batch, code.n, snr, sigma, 4, None, np.float64 if fl else np.int16,
                             nthreads=16)
    if args.llr_fill is not None:
        llr_host[:] = args.llr_fill
    llr = torch.from_numpy(llr_host).to(dev)
    dec = F.Decoder(code, max_iter=max_iter, width_mask=mask, device=local)
    describe = ("bp_float (decode_general, double; register form for dc 47 / <= 8)" if fl else dec.describe())
    # BER bookkeeping against the all-zero codeword over the k information positions.
    dec.set_reference(np.arange(k_info, dtype=np.int32), np.zeros(k_info, np.uint8))
    hard = torch.empty((batch, dec.hard_words), dtype=torch.int32, device=dev)
    iters = torch.empty(batch, dtype=torch.int32, device=dev)
    ok = torch.empty(batch, dtype=torch.uint8, device=dev)
    bit_err = torch.empty(batch, dtype=torch.int32, device=dev)
    totals = torch.zeros(4, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)

    def step():
        if fl:
            F._lib._check(F.lib().fpldpc_decode_float(dec._h, llr.data_ptr(), batch, hard.data_ptr(), iters.data_ptr(),
                                                      ok.data_ptr(), None, bit_err.data_ptr(), totals.data_ptr(),
                                                      stream.cuda_stream))
            return
        dec.decode_ptrs(llr.data_ptr(), F.FPLDPC_LLR_I16, batch, hard.data_ptr(), iters.data_ptr(), ok.data_ptr(), 0,
                        bit_err.data_ptr(), totals.data_ptr(), stream.cuda_stream)

    t_w, n_w = time.perf_counter(), 0
    while n_w < args.warmup or time.perf_counter() - t_w < args.min_warmup_s:
        step()
        n_w += 1
        if n_w >= args.warmup and n_w % 8 == 0:
            torch.cuda.synchronize(dev)  # time the decodes, not their enqueueing
    torch.cuda.synchronize(dev)
    warm_s = time.perf_counter() - t_w
    totals.zero_()
    if pg:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        step()
        ev[i][1].record(stream)
    torch.cuda.synchronize(dev)
    if pg:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    launch_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))

    # Beside the headline (one batch at a time, each launch waiting for the last frame of the one
    # before): two decoders on two streams alternating over the same batches, as a caller that keeps
    # two batches in flight would run them -- the next launch's workgroups take the CUs that one
    # launch's tail leaves idle (its last frames, up to max_iter iterations, run alone on their CU).
    # Every step is the same full decode with all outputs; both decoders' iteration counts are
    # checked equal to the headline's.  Reported as `two_in_flight`, never as `value`.
    inflight = None
    n_if = args.inflight_steps
    if not fl and n_if > 0 and args.llr_fill is None:
        dec2 = F.Decoder(code, max_iter=max_iter, width_mask=mask, device=local)
        dec2.set_reference(np.arange(k_info, dtype=np.int32), np.zeros(k_info, np.uint8))
        st2 = [stream, torch.cuda.Stream(dev)]
        bufs = [(dec, hard, iters, ok, bit_err, torch.zeros(4, dtype=torch.int64, device=dev))]
        bufs.append((dec2, torch.empty_like(hard), torch.empty_like(iters), torch.empty_like(ok), torch.empty_like(bit_err),
                     torch.zeros(4, dtype=torch.int64, device=dev)))
        ref_iters = iters.clone()

        def step2(i):
            d, h, it, o, be, tt = bufs[i & 1]
            d.decode_ptrs(llr.data_ptr(), F.FPLDPC_LLR_I16, batch, h.data_ptr(), it.data_ptr(), o.data_ptr(), 0,
                          be.data_ptr(), tt.data_ptr(), st2[i & 1].cuda_stream)

        for i in range(max(2, args.warmup)):
            step2(i)
        torch.cuda.synchronize(dev)
        if pg:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        for i in range(n_if):
            step2(i)
        torch.cuda.synchronize(dev)
        if pg:
            dist.barrier()
        dt_if = time.perf_counter() - t
        same = bool(all(bool((b[2] == ref_iters).all()) for b in bufs))
        _, t_if = D.allreduce_counters(torch.zeros(4, dtype=torch.int64, device=dev), dt_if, device=dev)
        inflight = {"value": round(world * batch * n_if * k_info / t_if / 1e6, 3), "unit": "Mb/s",
                    "ms_per_step": round(t_if / n_if * 1e3, 4), "steps": n_if, "batches_in_flight": 2,
                    "iters_equal_headline": same,
                    "note": "two decoders on two streams alternating over the same batch; full decode and outputs "
                            "every step; not the headline"}
        del dec2, bufs

    # the host->device copy of one batch of LLRs (pinned), timed separately; the
    # PCIe-inclusive rate would be frames / (launch + copy) with no copy/compute overlap
    h2d = None
    if rank == 0:
        pinned = torch.from_numpy(llr_host).pin_memory()
        dst = torch.empty_like(llr)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        dst.copy_(pinned, non_blocking=True)
        e0.record(stream)
        for _ in range(3):
            dst.copy_(pinned, non_blocking=True)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        cms = e0.elapsed_time(e1) / 3
        h2d = {"bytes": int(pinned.numel() * pinned.element_size()), "ms": round(cms, 4),
               "GB_per_s": round(pinned.numel() * pinned.element_size() / (cms * 1e-3) / 1e9, 2),
               "pcie_inclusive_value": round(batch * k_info / ((launch_ms + cms) * 1e-3) / 1e6, 3)}
        del pinned, dst

    # the only collective: the BER/FER counters (sum) and the step time (max), fixedpointldpc_amd/dist.py
    tot, t_max = D.allreduce_counters(totals, elapsed, device=dev)
    frames_total = world * batch * args.steps
    value = frames_total * k_info / t_max / 1e6
    avg_iters = tot[3] / max(tot[2], 1)

    # Parity against the CPU oracle (the metric's "BER match") on a sample spread over the whole
    # batch: every (batch / 192)-th frame plus the last 64, so it holds first fills of the persistent
    # grid, refills and the last frames pulled.  Then, at N = 1 only, the CPU baseline (the bench
    # contract's rule; at N > 1 the parity sample still runs on rank 0 while the other ranks wait on a
    # gloo group, so that they block in a socket instead of spinning on the GPU stream of an RCCL
    # barrier).
    parity = parity_sample = None
    cpu = cpu_mt = None
    wait_group = dist.new_group(backend="gloo") if pg and world > 1 else None
    if rank == 0:
        try:
            from oracle import oracle as O
            ocode = O.OracleCode.from_alist_text(code.write_alist())
            sel = np.unique(np.concatenate([np.linspace(0, batch - 1, min(batch, 192)).astype(np.int64),
                                            np.arange(max(0, batch - 64), batch)]))
            if fl:
                ref = O.decode_float_batch(ocode, llr_host[sel], max_iter=max_iter, want_post=False)
            else:
                ref = O.decode_batch(ocode, llr_host[sel], max_iter=max_iter, mask=mask, want_post=False)
            g_it = iters.cpu().numpy()[sel]
            g_hard = F.unpack_hard(hard.cpu().numpy()[sel], code.n)
            g_ok = ok.cpu().numpy()[sel]
            parity = bool((g_it == ref["iters"]).all() and (g_hard == ref["hard"]).all()
                          and (g_ok == ref["syndrome_ok"]).all())
            parity_sample = {"frames": int(len(sel)), "first": int(sel[0]), "last": int(sel[-1]),
                             "rule": "every (batch/192)-th frame + the last 64 of rank 0's batch",
                             "checked": "iterations, hard decisions, syndrome verdict"}
            if not args.no_cpu and world == 1:
                cf = args.cpu_frames or {"A": 4096, "W": 8192, "R": 512}.get(cfg, 1024)
                nf = min(cf, batch) if not fl else min(cf, batch, 256)
                t = time.perf_counter()
                if fl:
                    O.decode_float_batch(ocode, llr_host[:nf], max_iter=max_iter, nthreads=1, want_post=False)
                else:
                    O.decode_batch(ocode, llr_host[:nf], max_iter=max_iter, mask=mask, nthreads=1, want_post=False)
                dt = time.perf_counter() - t
                cpu = {"value": round(nf * k_info / dt / 1e6, 4), "unit": "Mb/s", "cores": 1, "kind": "port",
                       "sample": f"{nf} frames of the same {cfg} batch (Eb/N0 {ebn0} dB, {max_iter} it), oracle "
                                 f"{'decode_general' if fl else 'decode_general_fp'} restatement, 1 thread, "
                                 f"{dt:.1f} s",
                       "host_cpu": cpu_model(), "host_nproc": os.cpu_count(),
                       "ns_per_edge_iter": round(dt / (nf * max_iter * code.edges) * 1e9, 3),
                       "calibration": None if fl else calibration(cfg)}
                # the same restatement, OpenMP over frames on every host core this
                # job may use (affinity mask, bounded by a cgroup CPU quota if one is set), on a
                # sample sized for a few seconds
                cores, core_info = usable_cores()
                # whole passes over the rank's batch (or the 1-core sample) until ~3 s have passed,
                # so that a many-core host still gets a sample long enough to time
                nm = min(batch, max(nf, nf * cores // 2))
                done, reps, t = 0, 0, time.perf_counter()
                while True:
                    if fl:
                        O.decode_float_batch(ocode, llr_host[:nm], max_iter=max_iter, nthreads=cores, want_post=False)
                    else:
                        O.decode_batch(ocode, llr_host[:nm], max_iter=max_iter, mask=mask, nthreads=cores,
                                       want_post=False)
                    done, reps = done + nm, reps + 1
                    dt = time.perf_counter() - t
                    if dt >= 3.0 or reps >= 200:
                        break
                cpu_mt = {"value": round(done * k_info / dt / 1e6, 4), "unit": "Mb/s", "cores": cores, "kind": "port",
                          "sample": f"{reps} x {nm} frames of the same batch, OpenMP over frames, {cores} threads, "
                                    f"{dt:.1f} s", **core_info}
        except Exception as e:  # report, never hide
            parity = f"error: {e}"
    if wait_group is not None:
        dist.barrier(group=wait_group)

    if rank == 0:
        e = code.edges
        bpf = algorithmic_bytes_per_frame(code.n, e, avg_iters) * (4 if fl else 1)  # 8-B vs 2-B messages
        hbm_eq = batch * bpf / (launch_ms * 1e-3) / 1e9
        # committed counters describe the profiled run (tools/gpu_round.sh: the default batch and Eb/N0
        # of this config); another batch or SNR does different work, so they are not reported then
        bid = F.lib().fpldpc_kernel_build_id().decode() if hasattr(F.lib(), "fpldpc_kernel_build_id") else None
        wkey = cfg + ("_float" if fl else "")
        prof = find_profile(wkey, bid, batch, ebn0, describe.split(" ")[0]) if args.llr_fill is None else None
        traffic = prof.get("hbm_bytes_per_launch") if prof else None
        sq = prof.get("sq") if prof else None
        simds = 4 * torch.cuda.get_device_properties(dev).multi_processor_count
        valu_peak = simds * VALU_CLOCK_GHZ / 2  # G wave64-instructions / s
        valu_ach = sq["SQ_INSTS_VALU"] / (launch_ms * 1e-3) / 1e9 if sq and sq.get("SQ_INSTS_VALU") else None
        # SURVEY 8d's operation count of the algorithm (frame-iterations actually run), int32 lane ops
        alg_ops = ALG_OPS_PER_EDGE_ITER * e * tot[3] / max(args.steps, 1) / max(world, 1)
        alg_ach = alg_ops / (launch_ms * 1e-3) / 1e12
        alg_peak = valu_peak * 64 / 1e3  # T int32 lane-ops / s
        roofline = {
            "bound": "valu", "achieved": None if valu_ach is None else round(valu_ach, 1), "peak": round(valu_peak, 1),
            "unit": "G wave-instr/s", "frac": None if valu_ach is None else round(valu_ach / valu_peak, 4),
            "traffic": traffic, "avg_launch_ms": round(launch_ms, 4),
            "valu_insts_per_launch": int(sq["SQ_INSTS_VALU"]) if sq else None,
            "profile": f"{prof['file']}:{prof['key']}" if prof else None,
            "basis": "rocprofv3 SQ_INSTS_VALU per launch (profiles pmc_traffic.json, same kernel build id / batch / "
                     "Eb/N0) over this run's mean launch time (HIP events on the decode stream)" if sq else
                     "no committed SQ_INSTS_VALU profile for this kernel build id / batch / Eb/N0",
            "clock_ghz_under_pmc": round(sq["clock_ghz"], 3) if sq and sq.get("clock_ghz") else None,
            # the kernel runs two frames per 32-bit lane (int16 halves), so an algorithm op on one
            # frame is half a lane-op: against that packed peak (2x the int32 lane peak) the fraction
            # halves; frac_int32_lanes keeps SURVEY 8d's int32 reading
            "algorithmic": {"ops_per_edge_iter": ALG_OPS_PER_EDGE_ITER, "ops_per_launch": int(alg_ops),
                            "achieved": round(alg_ach, 2), "peak": round(2 * alg_peak, 2),
                            "unit": "T frame-ops/s (16-bit halves, 2 per lane-op)",
                            "frac": round(alg_ach / (2 * alg_peak), 4),
                            "frac_int32_lanes": round(alg_ach / alg_peak, 4)},
            "hbm_streaming_equivalent": {"bytes_per_frame": int(bpf), "achieved": round(hbm_eq, 1),
                                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(hbm_eq / HBM_PEAK_GBS, 4),
                                         "note": "SURVEY 8d B_cw for an HBM-streaming decoder; this one keeps "
                                                 "messages on chip (traffic is the measured HBM bytes)"},
        }
        # north_star's "fraction of the HBM roofline", measured: the committed PMC pass's HBM bytes per
        # launch (FETCH_SIZE / WRITE_SIZE, tools/pmc_summary.py) over this run's launch time.  For the
        # fixed-point decoder that is its I/O alone (messages stay on chip); the float decoder streams
        # its c2v planes through L2 / HBM, so beside its FP64-issue bound this is its second bound.
        hbm_meas = None
        if traffic:
            gbs = traffic / (launch_ms * 1e-3) / 1e9
            hbm_meas = {"bytes_per_launch": int(traffic), "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(gbs / HBM_PEAK_GBS, 5),
                        "basis": "rocprofv3 FETCH_SIZE / WRITE_SIZE per launch (profiles pmc_traffic.json, same kernel "
                                 "build id / batch / Eb/N0) over this run's mean launch time"}
        roofline["hbm_measured"] = hbm_meas
        roofline["hbm_measured_frac"] = hbm_meas["frac"] if hbm_meas else None
        if fl:
            # The double-precision decoder issues FP64 arithmetic at half the rate of 32-bit VALU work
            # (4 SIMD cycles per wave64 instruction, v_rcp_f64 16: profiles/r3/float/f64_rate.txt), so
            # its bound is VALU issue CYCLES: 4 (FMA+ADD+MUL F64) + 16 TRANS_F64 + 2 (other VALU) per
            # launch over the SIMD cycles of the launch (1,024 SIMDs x 2.4 GHz).  FP64 compares,
            # min/max and ldexp count at 2 cycles here (they are 4): a lower bound on the fraction.
            f64 = sum(sq.get(k, 0) for k in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64")) if sq else 0
            tr = sq.get("SQ_INSTS_VALU_TRANS_F64", 0) if sq else 0
            cyc = 4 * f64 + 16 * tr + 2 * (sq["SQ_INSTS_VALU"] - f64 - tr) if sq and f64 else None
            peak_c = simds * VALU_CLOCK_GHZ
            ach_c = cyc / (launch_ms * 1e-3) / 1e9 if cyc else None
            roofline.update({
                "bound": "valu_fp64_issue", "unit": "G SIMD issue-cycles/s", "peak": round(peak_c, 1),
                "achieved": None if ach_c is None else round(ach_c, 1),
                "frac": None if ach_c is None else round(ach_c / peak_c, 4),
                "issue_cycles_per_launch": None if cyc is None else int(cyc),
                "fp64_insts_per_launch": int(f64) if f64 else None, "trans_f64_insts_per_launch": int(tr) if sq else None,
                "basis": "rocprofv3 SQ_INSTS_VALU{,_FMA_F64,_ADD_F64,_MUL_F64,_TRANS_F64} per launch (profiles "
                         "pmc_traffic.json, same kernel build id / batch / Eb/N0), cycle-weighted 4/4/4/16/2, over "
                         "this run's mean launch time" if cyc else "no committed FP64 issue profile for this kernel build "
                                                                    "id / batch / Eb/N0",
                "algorithmic": None,
                # the other bound of this kernel, measured: HBM bytes per launch over the launch time
                "hbm": hbm_meas})
        out = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Mb/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "warmup_steps_run": n_w,
            "warmup_s": round(warm_s, 3),
            "ms_per_step": round(t_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64" if fl else "int16",
            "dtype_note": None if fl else "two frames per 32-bit lane in exact int16 halves (int32-equivalent: frames that "
                                          "leave the int16 range are re-decoded by the int32 kernel in the same call)",
            "data": "synthetic: reference channel model (Lehmer/Odeh-Evans AWGN, all-zero codeword), "
                    + ("unquantised f64 LLRs in HBM" if fl else "int16 LLRs in HBM"),
            "config": {"workload": wl, "global_batch": world * batch, "frames_per_gpu": batch, "ebn0_db": ebn0,
                       "max_iter": max_iter, "info_bits_per_frame": k_info, "parallelism": f"dp{world}",
                       "kernel": describe, "kernel_build_id": bid},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "cpu_baseline_all_cores": cpu_mt,
            "h2d": h2d,
            "two_in_flight": inflight,
            "ber": {"bit_errors": tot[0], "frame_errors": tot[1], "frames": tot[2], "avg_iters": round(avg_iters, 3)},
            "parity_vs_cpu_oracle": parity,
            "parity_sample": parity_sample,
            "collective": ({"backend": dist.get_backend(), "world": world, "ops": "all_reduce SUM int64[4] + MAX elapsed"}
                           if pg else None),
        }
        print(json.dumps(out), flush=True)
    if pg:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
