"""bench.py's host logic on CPU: config / mode resolution and the per-rank
gather over gloo (world_size 2), the pieces of the N>1 line that run without a GPU."""
import importlib.util
import os
import socket
import sys
import types

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load_bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def args(**kw):
    base = dict(config="auto", width=None, height=None, dims=None, range=None, mode="auto")
    base.update(kw)
    return types.SimpleNamespace(**base)


def test_resolve_defaults_follow_baseline_configs():
    b = load_bench()
    assert b.resolve(args(), 1) == ("c2", 640, 480, 512, 2.048, "single")
    # N>1: the metric's config on every GPU (independent streams); the Z-slab
    # stream is the `zslab` record, or the line itself with an explicit c4 / c5
    assert b.resolve(args(), 8) == ("c2", 640, 480, 512, 2.048, "replicas")
    assert b.resolve(args(config="c4"), 8) == ("c4", 640, 480, 1024, 2.048, "slab")
    assert b.resolve(args(config="c5"), 8) == ("c5", 1280, 720, 2048, 4.096, "slab")
    assert b.resolve(args(config="c3"), 1) == ("c3", 640, 480, 1024, 2.048, "single")
    assert b.resolve(args(mode="replicas"), 4)[-1] == "replicas"
    # an override that changes the geometry is no longer a named config
    assert b.resolve(args(dims=256), 1)[:4] == ("custom", 640, 480, 256)
    assert b.resolve(args(dims=512), 1)[0] == "c2"


def test_workload_text_names_sharding():
    b = load_bench()
    t = b.workload_text("c4", 640, 480, 1024, 2.048, "slab", 8, True)
    assert t.startswith("C4: synthetic 640x480") and "2.0 mm" in t and "8 GPUs" in t and "all-reduced" in t
    assert "replicated" in b.workload_text("c4", 640, 480, 1024, 2.048, "slab", 2, False)
    assert "independent" in b.workload_text("c2", 640, 480, 512, 2.048, "replicas", 2, False)


def _gather_rank(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, ROOT)
    b = load_bench()
    D = b.Dist(world, rank)
    rows = D.gather([float(rank), 10.0 + rank, 0.5])
    mx = D.max(float(rank) + 0.25)
    D.close()
    q.put((rank, rows, mx))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(120)
def test_dist_gather_over_gloo():
    world, port = 2, free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_gather_rank, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=100) for _ in range(world)]
    for p in ps:
        p.join(30)
        assert p.exitcode == 0
    for rank, rows, mx in res:
        assert rows == [[0.0, 10.0, 0.5], [1.0, 11.0, 0.5]]
        assert mx == 1.25


def test_cli_defaults_pin_the_measured_configs(monkeypatch):
    """The N>1 side record is one C5 stream (2048^3, north_star's scaling
    claim) Z-slab sharded over the ranks; at N=1 the C3 and C5 single-volume
    records run beside the C2 line (the N=1 points of their curves)."""
    b = load_bench()
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = b.parse()
    assert (a.gpus, a.config, a.mode, a.zslab, a.cuts, a.icp) == (1, "auto", "auto", "c5", "balanced", "replicated")
    assert a.c3_frames > 0 and a.c5_frames > 0 and a.cpu_frames > 0
    assert b.CONFIGS["c5"] == (1280, 720, 2048, 4.096)


def test_imbalance():
    b = load_bench()
    assert b.imbalance([1.0, 1.0]) == 1.0
    assert b.imbalance([3.0, 1.0]) == 1.5
    assert b.imbalance([1.0, float("nan")]) is None


class _FakeKF:
    """Stands in for kfx.KinectFusion in run_stream's plumbing test (no GPU)."""
    calls = []

    def __init__(self, intr, params, device=0, slab=None, cuts=None):
        self.slab, self.cuts, self.n = slab, cuts, 1
        _FakeKF.calls.append(("create", slab, cuts))

    def slice_work_at(self, bgr, dep, pose=None):
        import numpy as np
        _FakeKF.calls.append(("work", pose is not None))
        w = np.arange(64, dtype=np.int64)
        return w, w, w

    def pipeline_staged(self, i):
        self.n += 1

    @property
    def pose_record(self):
        import numpy as np
        return np.zeros((self.n, 4, 4))

    def graph_mode(self):
        return 1

    def kernel_timing(self):
        return {"samples": 0}

    def synchronize(self):
        return 0

    def __getattr__(self, name):  # comm_init, set_* , stage_frames, close
        return lambda *a, **k: None


def test_run_stream_plumbing_without_gpu(monkeypatch):
    """run_stream / balanced_cuts wiring on CPU with a stand-in kfx: frame
    tuples carry the trajectory's poses (or None), slab cuts come from the mean
    work of 4 calibration frames at their poses ('balanced'), of the first
    frame ('first', or no poses), or are equal ('equal')."""
    import numpy as np
    b = load_bench()
    fake = types.ModuleType("kfx")
    fake.KinectFusion = _FakeKF
    fake.KFX_OK = 0
    fake.comm_unique_id = lambda: b""
    fake.slab_balance = lambda work, world: [0, 32, 64]
    abi = types.ModuleType("kfx.abi")
    abi.Intrinsics = types.SimpleNamespace(from_any=lambda x: x)
    monkeypatch.setitem(sys.modules, "kfx", fake)
    monkeypatch.setitem(sys.modules, "kfx.abi", abi)

    class D:
        barrier = staticmethod(lambda: None)
        max = staticmethod(lambda x: x)
        bcast_bytes = staticmethod(lambda x: b"")

    params = types.SimpleNamespace(volu_dims=[64, 64, 64])
    a = types.SimpleNamespace(cuts="balanced", warmup=2, steps=6, no_graph=False, graph_full=False, no_overlap=False, graph="auto",
                              sample_every=0)
    n = 8
    frames = ([None] * n, [None] * n, list(range(n)) + list(range(n)), [np.eye(4)] * n)
    for cuts, gt, slab, want in (("balanced", True, (0, 2), 4), ("first", True, (0, 2), 1),
                                 ("balanced", False, (0, 2), 1), ("equal", True, (0, 2), 0),
                                 ("balanced", True, None, 0)):
        _FakeKF.calls = []
        a.cuts = cuts
        f = frames if gt else frames[:3] + (None,)
        kf, r = b.run_stream(a, None, params, f, D, 0, slab=slab)
        works = [c for c in _FakeKF.calls if c[0] == "work"]
        assert len(works) == want and all(w[1] == gt for w in works), (cuts, gt, slab, _FakeKF.calls)
        created = [c for c in _FakeKF.calls if c[0] == "create" and c[1] == slab]
        assert created[-1][2] == ([0, 32, 64] if want else None)
        assert r["tracked"] == a.steps and r["graph_mode"] == 1


def test_c5_defaults_to_the_captured_frame_graph(monkeypatch):
    """BASELINE C5 names a hipGraph-captured per-frame pipeline: every C5
    stream (the N>1 zslab record, --config c5, the N=1 c5_record) requests
    graph mode 2 (ICP + integrate + raycast (+ RCCL combine) captured) by
    default; other configs the preprocess graph; --graph / --no-graph /
    --graph-full override.  The record names the mode that ran."""
    b = load_bench()
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = b.parse()
    assert a.graph == "auto"
    assert b.graph_mode(a, "c5") == 2
    assert [b.graph_mode(a, c) for c in ("c2", "c3", "c4", "custom")] == [1, 1, 1, 1]
    for argv, want in ((["--graph", "0"], 0), (["--no-graph"], 0), (["--graph-full"], 2), (["--graph", "1"], 1)):
        monkeypatch.setattr(sys, "argv", ["bench.py"] + argv)
        assert b.graph_mode(b.parse(), "c5") == want, argv
    a.no_overlap = False
    assert b.graph_parts(a, "slab", 2, 2).endswith("graph (mode 2)") and "RCCL combine" in b.graph_parts(a, "slab", 2, 2)
    assert "fell back" in b.graph_parts(a, "slab", 1, 2)
    assert b.graph_parts(a, "single", 0, 0) == "none (eager)"


def test_pmc_record_attached_only_to_its_workload_and_library(tmp_path):
    """The C3 / C5 records carry PMC traffic only from a record of the same
    workload, step counts and libkfx.so (sha256)."""
    import json
    b = load_bench()
    rec = {"workload": [1024, 640, 480], "steps": 20, "warmup": 5, "lib_sha256": "ab" * 32,
           "hbm_bytes_per_launch": 123, "raycast_hbm_bytes_per_launch": 45, "command": "x", "regime": "y",
           "integrate_sq": {"valu_issue_frac_2cyc": 0.4}}
    p = tmp_path / "c3.json"
    p.write_text(json.dumps(rec))
    t, rt, sq, src = b.pmc_record(str(p), [1024, 640, 480], 20, 5, "ab" * 32)
    assert (t, rt) == (123, 45) and sq["integrate"]["valu_issue_frac_2cyc"] == 0.4 and "sha256" in src
    assert b.issue_figures(sq, "integrate")["valu_issue_frac_2cyc"] == 0.4
    t, _, _, src = b.pmc_record(str(p), [1024, 640, 480], 20, 5, "cd" * 32)
    assert t is None and src.startswith("none:")
    assert b.pmc_record(str(p), [2048, 1280, 720], 10, 5, "ab" * 32) == (None, None, None, None)
    assert b.pmc_record(str(tmp_path / "missing.json"), [1024, 640, 480], 20, 5, "ab" * 32)[0] is None
