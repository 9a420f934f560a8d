"""bench.py's self-launcher (CPU): `bench.py --gpus N` with no outer torchrun starts N ranks itself
(one process per GPU, torchrun on 127.0.0.1, the same flags on every rank); a rank (WORLD_SIZE set)
or N = 1 runs in place.  The launch itself is exercised on the GPU box (test_gpu_bench.py)."""
import importlib.util
import os
import subprocess
import sys

from conftest import ROOT


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_launch_command_n_ranks():
    b = _bench()
    argv = ["--gpus", "8", "--steps", "5", "--config", "R"]
    cmd = b.launch_command(8, argv, {}, 29512, python="py", script="/x/bench.py")
    assert cmd == ["py", "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=8",
                   "--master-addr=127.0.0.1", "--master-port=29512", "/x/bench.py", *argv]


def test_launch_command_in_place():
    b = _bench()
    assert b.launch_command(1, [], {}, 1) is None                      # N = 1: this process decodes
    assert b.launch_command(8, [], {"WORLD_SIZE": "8"}, 1) is None     # already a rank of a launcher


def test_missing_gpus_fail_loudly():
    # no HIP device here: --gpus 2 over RCCL must refuse (exit 2) before starting any rank
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 2, r.stderr
    assert "needs 2 visible GPUs, found 0" in r.stderr
    assert r.stdout == ""


def test_usable_cores():
    b = _bench()
    cores, info = b.usable_cores()
    assert 1 <= cores <= info["affinity_cpus"] <= info["nproc"]
