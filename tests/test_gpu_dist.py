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
