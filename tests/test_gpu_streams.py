"""Streams, graphs and concurrency of the C ABI (fpldpc_decode is asynchronous on the caller's
stream): a decode captured into a HIP graph and replayed gives the eager results; two decoder
objects driven from two host threads on their own streams give the oracle's results."""
import math
import threading

import numpy as np
import pytest

from conftest import assert_same

pytestmark = pytest.mark.gpu
SEED = 123456789


def _llr(O, code, frames, eb, f0=0):
    snr = 2 * math.pow(10.0, eb / 10) * code.rate
    return O.gen_llr(SEED, f0, frames, code.n, snr, math.sqrt(1 / snr), 4)


@pytest.mark.parametrize("cfg", ["A", "W", "R"])
def test_graph_capture_replay(F, O, codes, torch_dev, cfg):
    import torch
    code, ocode = codes[cfg]
    max_iter, mask = (50, 0x3F) if cfg == "R" else (30, 0xFF)
    dec = F.Decoder(code, max_iter=max_iter, width_mask=mask)
    llr_np = _llr(O, code, 512, 2.0 if cfg != "A" else 4.5)
    llr = torch.from_numpy(llr_np.astype(np.int16)).to(torch_dev)
    eager = {k: v.clone() for k, v in dec.decode_torch(llr).items()}  # also sizes the fallback lists
    torch.cuda.synchronize()
    out = {k: torch.empty_like(v) for k, v in eager.items()}
    totals = torch.zeros(4, dtype=torch.int64, device=torch_dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        s = torch.cuda.current_stream().cuda_stream
        dec.decode_ptrs(llr.data_ptr(), F.FPLDPC_LLR_I16, llr.shape[0], out["hard"].data_ptr(), out["iters"].data_ptr(),
                        out["syndrome_ok"].data_ptr(), 0, 0, totals.data_ptr(), s)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    for k in eager:
        assert torch.equal(out[k], eager[k]), k
    assert totals[2].item() == 3 * 512 and totals[3].item() == 3 * int(eager["iters"].sum().item())
    ref = O.decode_batch(ocode, llr_np, max_iter=max_iter, mask=mask, want_post=False)
    assert (out["iters"].cpu().numpy() == ref["iters"]).all()


def test_two_decoders_two_threads(F, O, codes, torch_dev):
    import torch
    jobs = []
    for cfg, eb in (("A", 4.0), ("W", 1.5)):
        code, ocode = codes[cfg]
        llr_np = _llr(O, code, 384, eb, f0=77)
        jobs.append((code, ocode, llr_np))
    results = [None, None]
    errors = []

    def run(i):
        try:
            code, _, llr_np = jobs[i]
            dec = F.Decoder(code)
            stream = torch.cuda.Stream(device=torch_dev)
            with torch.cuda.stream(stream):
                llr = torch.from_numpy(llr_np.astype(np.int16)).to(torch_dev, non_blocking=False)
                outs = []
                for _ in range(5):
                    outs.append(dec.decode_torch(llr, post=True, stream=stream.cuda_stream))
                stream.synchronize()
            results[i] = [{k: v.cpu().numpy() for k, v in o.items()} for o in outs]
        except Exception as e:  # surfaced below
            errors.append(e)

    th = [threading.Thread(target=run, args=(i,)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors
    for i, (code, ocode, llr_np) in enumerate(jobs):
        ref = O.decode_batch(ocode, llr_np)
        for r in results[i]:
            assert_same(r, ref, code.n, where=f"thread {i}")
