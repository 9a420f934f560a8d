"""The reference's PerfTest.h programs (fpldpc_compat.hpp, C++) run on the GPU through the
fpldpc_perftest driver, their console lines compared with the reference's published output and
with the CPU oracle."""
import json
import math
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

pytestmark = pytest.mark.gpu
CLI = os.path.join(ROOT, "fixedpointldpc_amd", "fpldpc_perftest")
SEED = 123456789


def _run(*args, cwd=None, env=None):
    import fixedpointldpc_amd as F
    F.lib()  # builds the driver too when stale
    p = subprocess.run([CLI, *map(str, args)], capture_output=True, text=True, timeout=300, cwd=cwd,
                       env=None if env is None else {**os.environ, **env})
    assert p.returncode == 0, p.stderr
    return p.stdout


def _result(out):
    m = re.search(r"(\d+) (\d+) (\d+)\n FER: (\S+) BER: (\S+)$", out, re.M)
    assert m, out[-500:]
    return int(m.group(1)), int(m.group(2)), int(m.group(3)), m.group(4), m.group(5)


@pytest.mark.parametrize("host_channel", ["0", "1"], ids=["device_channel", "host_channel"])
def test_wifi_kat_published_line(tmp_path, host_channel):
    """Wrapper.cpp main -> ArrayLDPC_Debug_Wifi at 2 dB == wifi_results_4_4_2dB_30iter.txt."""
    kj = json.load(open(os.path.join(GOLDEN, "kat_w.json")))
    be, fe, fr, fer, ber = _result(_run("wifi", 2, cwd=tmp_path, env={"FPLDPC_HOST_CHANNEL": host_channel}))
    assert (be, fe, fr) == (kj["bit_errors"], kj["frame_errors"], kj["frames"])
    assert fer == kj["fer_text"] and ber.replace("e-0", "e-00") == kj["ber_text"]


def test_array_kat(tmp_path):
    kj = json.load(open(os.path.join(GOLDEN, "kat_a.json")))
    be, fe, fr, _, _ = _result(_run("array", cwd=tmp_path))
    assert (be, fe, fr) == (kj["bit_errors"], kj["frame_errors"], kj["frames"])


def test_timetrial_counts_iterations(O, codes, tmp_path):
    """ArrayLDPC_TimeTrial counts decode_fixpoint's return value as bit errors (PerfTest.cpp:596-600)
    and creates <file> and <file>_log.txt."""
    code, ocode = codes["A"]
    be, fe, fr, _, _ = _result(_run("timetrial", 3.0, 300, "tt.txt", cwd=tmp_path))
    assert (tmp_path / "tt.txt").exists() and (tmp_path / "tt.txt_log.txt").exists()
    snr = 2 * math.pow(10.0, 3.0 / 10) * code.rate
    llr = O.gen_llr(SEED, 0, 300, code.n, snr, math.sqrt(1 / snr), 4)
    it = O.decode_batch(ocode, llr, precheck=True, want_post=False)["iters"]
    assert (be, fe, fr) == (int(it.sum()), int((it > 0).sum()), 300)


def test_shorten_matches_oracle(O, codes, tmp_path):
    """ArrayLDPC_Debug_Shorten(122): first 122 info chars zeroed, LLR 7*16 forced at the first 122 info
    positions, rate (1978-976)/2209, decode_fixpoint; per-frame iterations printed."""
    import fixedpointldpc_amd as F
    code, ocode = codes["A"]
    out = _run("shorten", 122, cwd=tmp_path)
    be, fe, fr, _, _ = _result(out)
    its = [int(x) for x in re.findall(r"(\d+), ", out.split("\n")[1])]
    assert len(its) == fr
    ka = np.load(os.path.join(GOLDEN, "kat_a.npz"))
    stream = bytearray(248)
    enc = F.Encoder.from_code(code)
    # the harness info stream with its first 122 chars zeroed -> info bits / codeword
    bits = ka["info_bits"].copy()
    bits[:976] = 0
    cw = enc.encode(bits)[0]
    snr = 2 * math.pow(10.0, 4.5 / 10) * (1978.0 - 976.0) / 2209.0
    llr = O.gen_llr(SEED, 0, fr, code.n, snr, math.sqrt(1 / snr), 4, cw=cw)
    llr[:, ka["info_idx"][:122]] = 112
    r = O.decode_batch(ocode, llr, precheck=True, want_post=False)
    e = (r["hard"][:, ka["info_idx"]] != bits[None, :]).sum(axis=1)
    assert its == r["iters"].tolist()
    assert (be, fe) == (int(e.sum()), int((e > 0).sum())) and fe == 100 and e[-1] > 0
    del stream


@pytest.mark.parametrize("ebn0,packets", [(2.0, 20000), (4.0, 8300)])
def test_decode_trial(O, codes, tmp_path, ebn0, packets):
    """DecodeTrial (PerfTest.cpp:148-192): MaxPacket decode_fixpoint calls over 100 all-zero-codeword
    vectors tiled.  Besides the rate, the driver prints the iteration counts of vectors 0-99 (after
    checking every tile of the last launch repeats them); they must equal the oracle's decode_fixpoint
    of the same 100 vectors (the reference's harness draws them as 2*snr*(1 + Normal(0, sigma)))."""
    code, ocode = codes["A"]
    out = _run("decode_trial", ebn0, packets, cwd=tmp_path)
    bps = float(re.search(r"^(\S+) bits per second for decoder", out, re.M).group(1))
    assert bps > 1e9, out
    its = [int(x) for x in re.search(r"^decode_fixpoint iterations \(vectors 0-99\): (.*)$", out, re.M).group(1).split(", ") if x]
    snr = 2 * math.pow(10.0, ebn0 / 10) * code.rate
    llr = O.gen_llr(SEED, 0, 100, code.n, snr, math.sqrt(1 / snr), 4)
    ref = O.decode_batch(ocode, llr, precheck=True, want_post=False)["iters"]
    assert its == ref.tolist()


def test_encode_trial_runs(tmp_path):
    """EncodeTrial on the device encoder; the driver itself checks the codeword against the host
    encoder and fails otherwise."""
    out = _run("encode_trial", 200000, cwd=tmp_path)
    bps = float(re.search(r"^(\S+) bits per second for encoder", out, re.M).group(1))
    assert bps > 1e9, out


def test_wifi_float_through_compat_decode_general(tmp_path):
    """FP_Decoder::decode_general (fpldpc_compat.hpp -> fpldpc_decode_float_host) frame by frame on
    the WiFi KAT stream at 1 dB == the reference's own decode_general (tests/golden/float_w.npz f1)."""
    g = np.load(os.path.join(GOLDEN, "float_w.npz"))
    out = _run("wifi_float", 1.0, 48, cwd=tmp_path)
    its = [int(x) for x in re.findall(r"(\d+), ", out.split("\n")[0])]
    assert len(its) == 48
    differ = int((np.array(its) != g["f1_iters"]).sum())
    assert differ <= 1, (its, g["f1_iters"].tolist())  # BER-level tolerance (test_gpu_float.py); 0 measured


def test_harness_sharded_over_decoders(O, codes, tmp_path):
    """The PerfTest programs over several decoders (fpldpc_ber_sim_multi / DecodeTrial split by
    ranks): FPLDPC_SIM_DEVICES=0,0,0 puts three decoders on the box's one GPU (host exchange; on a
    multi-GPU node the default is every device, RCCL).  The published KAT-W line and the DecodeTrial
    iteration record must not change."""
    env = {"FPLDPC_SIM_DEVICES": "0,0,0"}
    kj = json.load(open(os.path.join(GOLDEN, "kat_w.json")))
    be, fe, fr, fer, ber = _result(_run("wifi", 2, cwd=tmp_path, env=env))
    assert (be, fe, fr) == (kj["bit_errors"], kj["frame_errors"], kj["frames"])
    kj = json.load(open(os.path.join(GOLDEN, "kat_a.json")))
    be, fe, fr, _, _ = _result(_run("array", cwd=tmp_path, env=env))
    assert (be, fe, fr) == (kj["bit_errors"], kj["frame_errors"], kj["frames"])
    code, ocode = codes["A"]
    out = _run("decode_trial", 4.0, 30000, cwd=tmp_path, env=env)
    its = [int(x) for x in re.search(r"^decode_fixpoint iterations \(vectors 0-99\): (.*)$", out, re.M).group(1).split(", ") if x]
    snr = 2 * math.pow(10.0, 4.0 / 10) * code.rate
    llr = O.gen_llr(SEED, 0, 100, code.n, snr, math.sqrt(1 / snr), 4)
    assert its == O.decode_batch(ocode, llr, precheck=True, want_post=False)["iters"].tolist()
