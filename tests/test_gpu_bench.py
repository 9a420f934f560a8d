"""bench.py's own N-rank launch on the GPU box: `bench.py --gpus 2 --backend gloo` with no outer
torchrun starts two ranks (sharing the box's one GPU), each decoding its own frame range of the
reference channel stream; rank 0 prints one line for the whole job."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

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
    r = _bench("--gpus", "2", "--backend", "gloo", "--batch", "1024", "--steps", "2", "--warmup", "1")
    assert r["n_gpus"] == 2 and r["config"]["global_batch"] == 2048 and r["config"]["parallelism"] == "dp2"
    assert r["parity_vs_cpu_oracle"] is True
    assert r["ber"]["frames"] == 2 * 1024 * 2 and r["ber"]["avg_iters"] == 30.0
    assert r["value"] > 0 and r["cpu_baseline"] is None  # the CPU baseline is rank 0 at N = 1 only


def test_bench_single_gpu_line():
    r = _bench("--batch", "1024", "--steps", "2", "--warmup", "1", "--no-cpu", "--inflight-steps", "2")
    assert r["n_gpus"] == 1 and r["config"]["global_batch"] == 1024 and r["parity_vs_cpu_oracle"] is True
    t = r["two_in_flight"]  # the supplementary two-streams measurement: same decodes, same results
    assert t["batches_in_flight"] == 2 and t["steps"] == 2 and t["iters_equal_headline"] is True and t["value"] > 0


def test_bench_two_in_flight_early_termination():
    """At 4.5 dB (frames stop at different iterations) both decoders of the two-streams
    measurement reproduce the headline's per-frame iteration counts."""
    r = _bench("--ebn0", "4.5", "--steps", "4", "--warmup", "2", "--no-cpu", "--inflight-steps", "4")
    assert r["parity_vs_cpu_oracle"] is True and r["ber"]["avg_iters"] < 10
    assert r["two_in_flight"]["iters_equal_headline"] is True
