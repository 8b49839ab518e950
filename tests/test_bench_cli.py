"""CPU tests of bench.py's driver contract: the one stdout line stays small enough for the driver to parse, `--gpus N`
with no launcher starts N ranks as a child process (no GPU call in the parent), and the timed step is the same at
N = 1 and N > 1: no split-range flag read inside the region, one read per rank after it (gloo, world size 2)."""
import json
import os
import socket
import sys
from pathlib import Path

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import yolosod_import  # noqa: F401
import conftest  # noqa: F401

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402


def _full_result(n_ops=40):
    """A full bench result of the shape measure() builds (many hip_ops / backbone ops, full cpu_baseline)."""
    ops = [{"op": "swin", "shape": [32, 64, 160, 160], "dtype": "f32", "launches": 10, "avg_ms": 0.47 - i * 1e-3,
            "kernels_ms": 0.47, "total_ms_per_step": 0.47, "GBps": 900.0, "TFLOPs": 150.0, "bound": "mfma",
            "peak": 838.9, "t_min_ms": 0.0863, "frac": 0.18, "frac_vs_dtype_peak": 0.98,
            "producer": "x" * 120} for i in range(n_ops)]
    roof = {"bound": "mfma", "achieved": 154.9, "peak": 838.9, "unit": "TFLOP/s", "frac": 0.1846,
            "traffic": 436898592, "kernel": "swin(32, 64, 160, 160) (one C-ABI call = its launch sequence)",
            "algorithmic_per_launch": 72419778560, "peak_basis": "p" * 80, "method": "m" * 80,
            "frac_vs_dtype_peak": 0.98, "dtype_peak": 157.3}
    path = {"t_min_ms": 0.507, "t_meas_ms": 1.76, "frac": 0.287, "definition": "d" * 400, "frac_vs_dtype_peak": 0.77}
    sub = {"value": 495.9, "unit": "images/s", "ms_per_step": 16.1, "steps": 20, "warmup": 5, "dtype": "f32",
           "data": "synthetic", "config": {"name": "n1280", "workload": "w" * 100, "imgsz": 1280, "batch_per_gpu": 8,
                                           "global_batch": 8, "parallelism": "dp1"},
           "roofline": dict(roof), "path_roofline": dict(path), "hip_ops": ops, "backbone_hip_ops": ops}
    res = {"metric": bench.METRIC, "value": 1918.0, "unit": "images/s", "n_gpus": 1, "steps": 20, "warmup": 5,
           "ms_per_step": 16.68, "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
           "data": "synthetic: torch.rand images in HBM, seed-0 random-init weights",
           "config": {"name": "n640", "workload": "yolov12n-sod (paper YAML) 640x640, 32 images per GPU",
                      "imgsz": 640, "batch_per_gpu": 32, "global_batch": 32, "parallelism": "dp1"},
           "roofline": roof, "path_roofline": path, "split_range_flagged": False, "hip_ops_ms_per_step": 1.76,
           "hip_ops": ops[:10], "backbone_hip_ms_per_step": 3.4, "backbone_hip_ops": ops,
           "nms_loaded": {str(n): {"ms_per_call": 0.18, "images": 32, "kept_per_image": 300.0}
                          for n in bench.NMS_LOADS},
           "cpu_baseline": {"value": 6.8, "unit": "images/s", "cores": 16, "kind": "port", "cpu_model": "EPYC",
                            "sample": "8 of the 640x640 images per iteration", "all_cores": {
                                "mafn_decode_nms_ms_per_image": 67.8}, "single_thread_configs0": {"value": 3.4},
                            "nms_loaded_ms_per_image": {"1000": 1.96, "10000": 14.6, "30000": 87.1}},
           "configs": {"n1280": sub, "m640": dict(sub, dtype="bf16")}}
    return res


def test_compact_line_is_small_and_complete():
    line = bench.compact_line(_full_result(), "gpurun_out/bench_detail.json")
    txt = json.dumps(line)
    assert len(txt.encode()) <= bench.LINE_LIMIT
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in line, k
    r = line["roofline"]
    assert {"bound", "achieved", "peak", "unit", "frac", "traffic"} <= set(r) and r["frac"] == 0.1846
    assert line["path_roofline"]["frac"] == 0.287 and "definition" not in line["path_roofline"]
    cb = line["cpu_baseline"]
    assert (cb["value"], cb["cores"], cb["kind"]) == (6.8, 16, "port") and cb["sample"]
    for n in ("n1280", "m640"):
        c = line["configs"][n]
        assert {"value", "ms_per_step", "roofline_frac", "path_roofline_frac"} <= set(c)
    assert json.loads(txt) == line


def test_compact_line_of_the_round4_result_fits():
    """Round 4's 20 KB line (profiles/r04_bench_final_default.json) compacts below the limit."""
    p = ROOT / "profiles" / "r04_bench_final_default.json"
    if not p.exists():
        pytest.skip("round-4 line not present")
    full = json.loads(p.read_text().strip().splitlines()[-1])
    full.setdefault("split_range_flagged", False)
    line = bench.compact_line(full)
    assert len(json.dumps(line).encode()) < 4000
    assert line["value"] == full["value"] and line["roofline"]["traffic"] == full["roofline"]["traffic"]


def test_launcher_starts_ranks_as_a_child(monkeypatch):
    """--gpus 2 without WORLD_SIZE: one child `torch.distributed.run --nproc-per-node=2 ... bench.py --gpus 2 ...`,
    the parent exits with the child's code and never touches the GPU."""
    import subprocess
    seen = {}

    class R:
        returncode = 7

    def fake_run(cmd, env=None, **k):
        seen["cmd"], seen["env"] = cmd, env
        return R()

    def no_gpu(*a, **k):
        raise AssertionError("parent made a GPU call")

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(subprocess, "run", fake_run)
    monkeypatch.setattr(torch.cuda, "set_device", no_gpu)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "3", "--warmup", "1"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 7
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=2" in cmd and "--master-addr=127.0.0.1" in cmd and "--nnodes=1" in cmd
    assert cmd[-6:] == ["--gpus", "2", "--steps", "3", "--warmup", "1"]
    assert Path(cmd[cmd.index("--nnodes=1") + 4]).name == "bench.py"
    assert seen["env"]["MASTER_ADDR"] == "127.0.0.1"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Timer:
    def __init__(self, select=None):
        self.select = select

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False

    def durations_ms(self):
        return [(("nms", (2, 10, 34000), None), 0.03)]


def _measure_worker(rank, world, port, q):
    """bench.measure at world size 2 on CPU with the GPU parts stubbed: counts flag reads and split_guard use."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench as b
        reads, guards, steps = [], [], []

        class Pred:
            dtype = torch.float32

            def __init__(self, *a, **k):
                pass

            def predict_padded(self, x):
                steps.append(len(reads))  # flag reads seen when this step ran
                n = x.shape[0]
                return (torch.zeros(n, 300, 6), torch.zeros(n, dtype=torch.int32),
                        torch.full((n, 300), -1, dtype=torch.int32))

        orig_sharded = b.sharded_predict

        def sharded(*a, **k):
            guards.append(k.get("split_guard", True))
            return orig_sharded(*a, **k)

        b.CONFIGS["tiny"] = ("yolov12-sod-fusion-v5-simple.yaml", 16, 2, "tiny", torch.float32)
        b.build_model = lambda *a, **k: None
        b.DetectionPredictor = Pred
        b.sharded_predict = sharded
        b._hip.op_timer = _Timer
        b._hip.split_range_flag = lambda reset=False, device=None: reads.append(1) or (rank == 1)
        exact = []

        class Exact:
            def __enter__(self):
                exact.append(len(steps))

            def __exit__(self, *a):
                return False

        b._hip.exact_fp32_matrix = Exact
        torch.cuda.synchronize = lambda *a, **k: None
        res, _, _, _ = b.measure("tiny", world, rank, torch.device("cpu"), steps=4, warmup=2, conf=0.25)
        # warmup 2 + 4 timed steps with no flag read inside; the flag (max over ranks: rank 1 flagged) is read once
        # after the region, and the flagged region is timed again on the exact kernels (4 more steps, one more read)
        ok = (len(reads) == 2 and steps == [0] * 6 + [1] * 4 and guards == [False] * 10 and exact == [6]
              and res["split_range_flagged"] is True and res["split_range_redone_exact"] is True
              and res["config"]["global_batch"] == 4 and res["value"] > 0)
        q.put((rank, bool(ok), (len(reads), steps, guards, exact, res.get("split_range_flagged"))))
    finally:
        dist.destroy_process_group()


def test_timed_step_symmetric_and_one_flag_read_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_measure_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert sorted(r[:2] for r in res) == [(0, True), (1, True)], res
