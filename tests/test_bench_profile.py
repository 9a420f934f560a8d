"""bench.py's roofline bookkeeping (CPU): committed PMC summaries are matched to a run by workload,
kernel build id, frames per launch, Eb/N0 and kernel variant (find_profile), never by key alone;
GPUs are counted from the KFD topology without touching HIP (count_gpus)."""
import importlib.util
import json
import os

from conftest import ROOT


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_find_profile_matches_the_exact_workload(tmp_path, monkeypatch):
    b = _bench()
    d = tmp_path / "profiles" / "r9"
    d.mkdir(parents=True)
    base = {"kernel_build_id": "abc", "describe": "flood_array2<P=47,W=3>", "profiled_ebn0_db": 0.0}
    entries = {
        "A": dict(base, workload="A", profiled_frames=4096, sq={"SQ_INSTS_VALU": 1}),
        "A_b8192": dict(base, workload="A", profiled_frames=8192, sq={"SQ_INSTS_VALU": 2}),
        "A_4.5dB": dict(base, workload="A", profiled_frames=4096, profiled_ebn0_db=4.5, sq={"SQ_INSTS_VALU": 3}),
        "A_float": dict(base, workload="A_float", profiled_frames=4096, describe="bp_float", sq={"SQ_INSTS_VALU": 4}),
    }
    (d / "pmc_traffic.json").write_text(json.dumps(entries))
    monkeypatch.setattr(b, "ROOT", str(tmp_path))
    f = lambda *a: (b.find_profile(*a) or {}).get("sq", {}).get("SQ_INSTS_VALU")
    assert f("A", "abc", 4096, 0.0, "flood_array2<P=47,W=3>") == 1
    assert f("A", "abc", 8192, 0.0, "flood_array2<P=47,W=3>") == 2
    assert f("A", "abc", 4096, 4.5, "flood_array2<P=47,W=3>") == 3
    assert f("A_float", "abc", 4096, 0.0, "bp_float") == 4
    assert f("A", "other-build", 4096, 0.0, "flood_array2<P=47,W=3>") is None   # another kernel build
    assert f("A", "abc", 2048, 0.0, "flood_array2<P=47,W=3>") is None           # another batch
    assert f("A", "abc", 4096, 0.0, "flood_array<P=47>") is None                # another variant
    assert b.find_profile("A", "abc", 4096, 0.0, "flood_array2<P=47,W=3>")["file"] == os.path.join("profiles", "r9",
                                                                                              "pmc_traffic.json")


def test_count_gpus_from_kfd_topology(monkeypatch, tmp_path):
    b = _bench()
    nodes = []
    for i, simds in enumerate([0, 1024, 1024, 0]):  # a CPU node, two GPU nodes, another CPU node
        p = tmp_path / f"{i}_properties"
        p.write_text(f"cpu_cores_count 0\nsimd_count {simds}\n")
        nodes.append(str(p))
    monkeypatch.setattr("glob.glob", lambda pattern: nodes)
    for v in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    assert b.count_gpus() == 2
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "1")
    assert b.count_gpus() == 1


def test_committed_profile_is_of_the_shipped_build(F):
    """The newest committed PMC summary was measured on the kernels the in-tree library carries
    (the library's own fpldpc_kernel_build_id, a host function: no GPU needed).  A kernel change
    without a new profiling pass would leave every bench line without its roofline fraction; this
    reports it on the CPU.  A freshness rule for evidence, not a correctness property: a
    kernel edit awaiting its profiling pass, or a hipcc that emits different bytes, skips with the
    ids named instead of failing the suite; one summary must still hold one build's counters."""
    import glob
    import pytest
    newest = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_traffic.json")))[-1]
    ids = {e.get("kernel_build_id") for e in json.load(open(newest)).values()}
    assert len(ids) == 1, (newest, ids)
    built = F.lib().fpldpc_kernel_build_id().decode()
    if ids != {built}:
        pytest.skip(f"{os.path.relpath(newest, ROOT)} profiles kernel build {ids.pop()}, the in-tree library is {built}: "
                    "re-run tools/gpu_round.sh PHASE=prof before quoting a roofline fraction")
