"""The N > 1 bench path on the 1-GPU box: `torchrun --nproc-per-node 2 bench.py --gpus 2` with the
gloo backend standing in for RCCL (both ranks share the one GPU).  Checks the contract's weak
scaling bookkeeping: global batch = N x per-GPU batch, the all-reduced counters cover every rank's
frames, rank 0 alone prints the line, and rank 0's frames still match the CPU oracle."""
import json
import math
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import stale_profile_ok, ROOT

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("cfg,batch", [("A", 1024), ("W", 1024), ("A", 8192), ("R", 4096)],
                         ids=["A", "W", "configs3_A_8192_per_rank", "configs4_R_50it_0x3f"])
def test_bench_two_ranks_gloo(cfg, batch):
    """Also BASELINE configs[3] (A, 8192 frames per rank: 65536 over 8 GPUs) and configs[4] (R: p47/r24,
    50 iterations, mask 0x3f, 4096 frames per rank) through the bench's multi-rank path, as far as one
    GPU allows: two ranks on the box's GPU, each its own frame range, gloo for the counter all-reduce.
    Their per-rank batches are the committed profiles' (profiles/r*/pmc_traffic.json), so the line
    carries the VALU-issue roofline fraction (the two ranks share the GPU: a lower fraction)."""
    steps = 2
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
    assert d["collective"]["world"] == 2 and d["collective"]["backend"] == "gloo"
    assert d["value"] > 0
    if cfg == "R":
        assert d["config"]["max_iter"] == 50 and "mask 0x3f" in d["config"]["workload"]
        assert d["ber"]["avg_iters"] == 50.0  # 2 dB: every frame runs all 50 iterations
    if batch in (4096, 8192):
        assert (d["roofline"]["frac"] is not None and 0 < d["roofline"]["frac"] < 1) or stale_profile_ok(d), d["roofline"]


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


# ---- the native multi-device simulation (fpldpc_ber_sim_multi, C++ threads + RCCL) -------------

def _kat_w_args(F):
    kw = np.load(os.path.join(ROOT, "tests", "golden", "kat_w.npz"), allow_pickle=False)
    snr = 2 * math.pow(10.0, 2.0 / 10) * 0.5  # PerfTest.cpp:62
    return snr, math.sqrt(1 / snr), dict(info_index=kw["info_idx"], info_bits=kw["info_bits"], codeword=kw["cw"])


@pytest.mark.parametrize("ndec,coll", [(1, 1), (1, 2), (3, 2), (3, 0)], ids=["1-rccl", "1-host", "3-host", "3-auto"])
def test_kat_w_native_multi(F, ndec, coll):
    """KAT-W (2732 / 100 / 393214) through fpldpc_ber_sim_multi: one RCCL communicator on the box's
    GPU (ncclCommInitAll in-process), and three decoders sharing it (one host thread each, host
    exchange -- AUTO picks it because the devices repeat); device channel, small chunks so the stop
    frame lands inside a later rank's chunk of a round."""
    kj = json.load(open(os.path.join(ROOT, "tests", "golden", "kat_w.json")))
    snr, sigma, ref = _kat_w_args(F)
    decs = [F.Decoder(F.Code.wifi_1944_r12()) for _ in range(ndec)]
    r = F.ber_sim_multi(decs, snr, sigma, collective=coll, max_frame_errors=100, device_channel=True, chunk=12288,
                        **ref)
    assert (r["bit_errors"], r["frame_errors"], r["frames"]) == (kj["bit_errors"], kj["frame_errors"], kj["frames"])
    assert r["collective"] == (1 if coll == 1 else 2)
    assert r["frames_decoded"] >= r["frames"]


@pytest.mark.parametrize("mode", ["bits_host_channel", "iters_on_frame"])
def test_native_multi_equals_single(F, mode):
    """Three ranks == one decoder, frame for frame: the same counters (incl. iteration sums), and the
    on_frame callbacks in frame order with the same values (ArrayLDPC_Debug_Shorten's per-frame
    print path); decode_fixpoint on the array code, frame-error stop and frame-limit stop."""
    code = F.Code.array(47, 5)
    snr, sigma = F.snr_sigma(4.0, code.rate)
    kw = dict(max_frame_errors=0, max_frames=5000, chunk=700)
    if mode == "bits_host_channel":
        ka = np.load(os.path.join(ROOT, "tests", "golden", "kat_a.npz"), allow_pickle=False)
        kw.update(info_index=ka["info_idx"], info_bits=ka["info_bits"], codeword=ka["cw"], host_threads=8,
                  max_frame_errors=40)
        seen1 = seen3 = None
    else:
        kw.update(count_mode=F._lib.FPLDPC_COUNT_ITERS, device_channel=True)
        seen1, seen3 = [], []
    single = F.Decoder(code, precheck=True)
    r1 = single.ber_sim(snr, sigma, on_frame=(None if seen1 is None else lambda *a: seen1.append(a)), **kw)
    decs = [F.Decoder(code, precheck=True) for _ in range(3)]
    r3 = F.ber_sim_multi(decs, snr, sigma, on_frame=(None if seen3 is None else lambda *a: seen3.append(a)), **kw)
    for k in ("bit_errors", "frame_errors", "frames", "iter_sum"):
        assert r1[k] == r3[k], (k, r1, r3)
    if seen1 is not None:
        assert seen1 == seen3 and len(seen1) == r1["frames"]
        assert [f for f, _, _ in seen1] == list(range(r1["frames"]))


def test_native_multi_argument_errors(F):
    """fpldpc_ber_sim_multi refuses what it cannot run: the same decoder object twice (a decoder is
    single-stream), decoders of different codes, RCCL over a repeated device."""
    snr, sigma, ref = _kat_w_args(F)
    w1, w2 = F.Decoder(F.Code.wifi_1944_r12()), F.Decoder(F.Code.wifi_1944_r12())
    a = F.Decoder(F.Code.array(47, 5))
    kw = dict(max_frames=1000, max_frame_errors=0, device_channel=True, **ref)
    for decs, coll, msg in (([w1, w1], 0, "same decoder"), ([w1, a], 0, "different codes"),
                            ([w1, w2], F.FPLDPC_COLL_RCCL, "distinct devices")):
        with pytest.raises(F.FpldpcError, match=msg):
            F.ber_sim_multi(decs, snr, sigma, collective=coll, **kw)
    r = F.ber_sim_multi([w1, w2], snr, sigma, **kw)  # AUTO on a repeated device: host exchange
    assert r["collective"] == F.FPLDPC_COLL_HOST and r["frames"] == 1000


@pytest.mark.parametrize("spec", ["1:0", "2:1", "0:1:abrupt", "1:2:abrupt"])
def test_native_multi_rank_failure_stops_all(spec):
    """A rank that fails (fpldpc_testing_sim_inject(rank, round, abrupt, 0), the test-only hook of
    include/fpldpc_testing.h standing in for a device error) ends the whole simulation with that
    rank's error -- through the round's status word, or, when it leaves without joining the exchange,
    through the abortable barrier -- and no rank is left waiting (run in a child process under a
    time limit)."""
    rank, rnd, *rest = spec.split(":")
    code = (
        "import sys; sys.path.insert(0, %r)\n"
        "import fixedpointldpc_amd as F\n"
        "F.lib().fpldpc_testing_sim_inject(%s, %s, %d, 0)\n"
        "c = F.Code.array(47, 5); snr, sigma = F.snr_sigma(4.0, c.rate)\n"
        "decs = [F.Decoder(c, precheck=True) for _ in range(3)]\n"
        "try:\n"
        "    F.ber_sim_multi(decs, snr, sigma, collective=F.FPLDPC_COLL_HOST, max_frame_errors=0, max_frames=20000,\n"
        "                    chunk=500, count_mode=F._lib.FPLDPC_COUNT_ITERS, device_channel=True)\n"
        "    print('NO ERROR')\n"
        "except F.FpldpcError as e:\n"
        "    print('RAISED', e)\n" % (ROOT, rank, rnd, int(rest == ["abrupt"])))
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    assert "RAISED" in p.stdout and f"rank {rank}: injected failure" in p.stdout, p.stdout


def test_native_rccl_init_failure(F, capfd):
    """A communicator that cannot be created: FPLDPC_COLL_RCCL fails with the ncclCommInitAll error;
    FPLDPC_COLL_AUTO falls back to the host exchange and reports HOST in collective_used, with the
    same counters (the fallback once still reported RCCL).  AUTO attempts RCCL only for
    decoders on distinct devices; the test hook's fail_comm_init = 2 makes it attempt RCCL with the
    one decoder of a 1-GPU box, so the fallback path itself runs end to end here: the
    failed init, the stderr notice, the released exchange and the host collectives."""
    snr, sigma, ref = _kat_w_args(F)
    w1 = F.Decoder(F.Code.wifi_1944_r12())
    kw = dict(max_frames=2000, max_frame_errors=0, device_channel=True, **ref)
    base = F.ber_sim_multi([w1], snr, sigma, collective=F.FPLDPC_COLL_RCCL, **kw)
    assert base["collective"] == F.FPLDPC_COLL_RCCL  # a 1-rank RCCL communicator
    F.lib().fpldpc_testing_sim_inject(-1, 0, 0, 1)
    try:
        with pytest.raises(F.FpldpcError, match="ncclCommInitAll"):
            F.ber_sim_multi([w1], snr, sigma, collective=F.FPLDPC_COLL_RCCL, **kw)
        r = F.ber_sim_multi([w1], snr, sigma, collective=F.FPLDPC_COLL_AUTO, **kw)
        assert r["collective"] == F.FPLDPC_COLL_HOST  # (fail_comm_init = 1: AUTO never tried RCCL)
        capfd.readouterr()
        F.lib().fpldpc_testing_sim_inject(-1, 0, 0, 2)
        r2 = F.ber_sim_multi([w1], snr, sigma, collective=F.FPLDPC_COLL_AUTO, **kw)
        err = capfd.readouterr().err
        assert "ncclCommInitAll: injected failure" in err and "through host memory instead" in err, err
        assert r2["collective"] == F.FPLDPC_COLL_HOST
        for k in ("bit_errors", "frame_errors", "frames", "iter_sum"):
            assert r[k] == base[k] and r2[k] == base[k], (k, r, r2, base)
    finally:
        F.lib().fpldpc_testing_sim_inject(-1, 0, 0, 0)
    r3 = F.ber_sim_multi([w1], snr, sigma, collective=F.FPLDPC_COLL_RCCL, **kw)  # reset: RCCL again
    assert r3["collective"] == F.FPLDPC_COLL_RCCL and r3["frames"] == base["frames"]
