"""bench.py's own N-rank launch on the GPU box: `bench.py --gpus 2 --backend gloo` with no outer
torchrun starts two ranks (sharing the box's one GPU), each decoding its own frame range of the
reference channel stream; rank 0 prints one line for the whole job."""
import json
import os
import subprocess
import sys

import pytest

from conftest import stale_profile_ok, ROOT

pytestmark = pytest.mark.gpu


def _bench(*args):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=240, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def test_bench_self_launches_two_ranks():
    """The N > 1 line: parity on rank 0's sample (checked after the timed region while rank 1
    waits), no CPU baseline (timed at N = 1 only, the bench contract's rule), and the VALU-issue
    roofline (the committed counters of the per-GPU workload, configs[1]'s 4096 frames, apply to
    every rank's launch)."""
    r = _bench("--gpus", "2", "--backend", "gloo", "--steps", "2", "--warmup", "1", "--min-warmup-s", "0",
               "--cpu-frames", "256")
    assert r["n_gpus"] == 2 and r["config"]["global_batch"] == 8192 and r["config"]["parallelism"] == "dp2"
    assert r["parity_vs_cpu_oracle"] is True and r["parity_sample"]["last"] == 4095
    assert r["ber"]["frames"] == 2 * 4096 * 2 and r["ber"]["avg_iters"] == 30.0
    assert r["value"] > 0 and r["collective"]["backend"] == "gloo" and r["collective"]["world"] == 2
    assert r["cpu_baseline"] is None and r["cpu_baseline_all_cores"] is None
    assert (r["roofline"]["frac"] is not None and 0 < r["roofline"]["frac"] < 1) or stale_profile_ok(r), r["roofline"]


def test_bench_one_rank_rccl():
    """bench.py under torchrun at one rank: the process group is RCCL (`nccl`) and the counter
    all-reduce runs through it (a 1-rank communicator), as every rank of an 8-GPU run does."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
                        "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "bench.py"),
                        "--batch", "1024", "--steps", "2", "--warmup", "1", "--no-cpu"],
                       capture_output=True, text=True, timeout=240, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    r = json.loads(lines[0])
    assert r["collective"] == {"backend": "nccl", "world": 1, "ops": r["collective"]["ops"]}
    assert r["n_gpus"] == 1 and r["parity_vs_cpu_oracle"] is True
    assert r["ber"]["frames"] == 1024 * 2 and r["ber"]["avg_iters"] == 30.0


def test_bench_single_gpu_line():
    r = _bench("--batch", "1024", "--steps", "2", "--warmup", "1", "--cpu-frames", "256", "--inflight-steps", "2")
    assert r["n_gpus"] == 1 and r["config"]["global_batch"] == 1024 and r["parity_vs_cpu_oracle"] is True
    # the CPU baseline (N = 1): 1 core, the port calibrated against the reference's own decoder
    # (BASELINE.md CPU-baseline plan, tools/cpu_calibrate.py): bit-exact, within +-15 % of its time
    assert r["cpu_baseline"]["value"] > 0 and r["cpu_baseline"]["cores"] == 1
    cal = r["cpu_baseline"]["calibration"]
    assert cal is not None and cal["bit_exact"] is True, r["cpu_baseline"]
    assert 0.85 <= cal["port_over_reference_time"] <= 1.15, cal
    assert r["cpu_baseline_all_cores"]["value"] > 0
    t = r["two_in_flight"]  # the supplementary two-streams measurement: same decodes, same results
    assert t["batches_in_flight"] == 2 and t["steps"] == 2 and t["iters_equal_headline"] is True and t["value"] > 0


def test_bench_two_in_flight_early_termination():
    """At 4.5 dB (frames stop at different iterations) both decoders of the two-streams
    measurement reproduce the headline's per-frame iteration counts."""
    r = _bench("--ebn0", "4.5", "--steps", "4", "--warmup", "2", "--no-cpu", "--inflight-steps", "4")
    assert r["parity_vs_cpu_oracle"] is True and r["ber"]["avg_iters"] < 10
    assert r["two_in_flight"]["iters_equal_headline"] is True
