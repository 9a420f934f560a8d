"""The N > 1 bench path on the 1-GPU box: `torchrun --nproc-per-node 2 bench.py --gpus 2` with the
gloo backend standing in for RCCL (both ranks share the one GPU).  Checks the contract's weak
scaling bookkeeping: global batch = N x per-GPU batch, the all-reduced counters cover every rank's
frames, rank 0 alone prints the line, and rank 0's frames still match the CPU oracle."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("cfg", ["A", "W"])
def test_bench_two_ranks_gloo(cfg):
    batch, steps = 1024, 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend",
           "gloo", "--config", cfg, "--batch", str(batch), "--steps", str(steps), "--warmup", "1", "--no-cpu"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT,
                       env={**os.environ, "OMP_NUM_THREADS": "4"})
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak"
    assert d["config"]["global_batch"] == 2 * batch and d["config"]["parallelism"] == "dp2"
    assert d["ber"]["frames"] == 2 * batch * steps
    assert d["parity_vs_cpu_oracle"] is True
    assert d["value"] > 0


@pytest.mark.parametrize("ranks", [1, 2, 3])
def test_kat_w_sharded_over_ranks(ranks):
    """The published KAT-W (2732 / 100 / 393214) from tools/ber_dist.py on 1, 2 and 3 ranks (the
    harness's stop rule combined across ranks in frame order; ranks share the box's GPU, gloo)."""
    import json as _json
    kj = _json.load(open(os.path.join(ROOT, "tests", "golden", "kat_w.json")))
    script = os.path.join(ROOT, "tools", "ber_dist.py")
    if ranks == 1:
        cmd = [sys.executable, script, "--chunk", "32768"]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(ranks),
               "--master-addr", "127.0.0.1", "--master-port", str(_port()), script, "--backend", "gloo",
               "--chunk", "16384"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT,
                       env={**os.environ, "OMP_NUM_THREADS": "4"})
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    d = _json.loads(lines[0])
    assert (d["bit_errors"], d["frame_errors"], d["frames"]) == (kj["bit_errors"], kj["frame_errors"], kj["frames"])
    assert d["ranks"] == ranks
