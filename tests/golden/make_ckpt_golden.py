"""Generate the checkpoint-ingest fixture by running the REFERENCE (build container only, like make_golden.py).

    python tests/golden/make_ckpt_golden.py

A reduced-width copy of the paper graph (``width_multiple`` 0.125, so the file stays small) is built by the
reference's ``DetectionModel``, given perturbed weights / BatchNorm statistics (so detections pass conf 0.25), and
saved exactly as the reference trainer saves a checkpoint (``engine/trainer.py:513-536``: ``{"ema":
deepcopy(model).half(), "model": None, "train_args": ..., ...}``). The expected outputs come from the reference's
own load path (``nn/tasks.py:941-975`` attempt_load_one_weight semantics: ``ema`` -> ``.float()`` -> ``fuse()`` ->
``eval()``) and its ``non_max_suppression``.

Outputs: tests/golden/ckpt_tiny.pt (the checkpoint, data written by this script) and tests/golden/ckpt_tiny.npz
(input seed, fused fp32 forward, NMS rows of the reloaded reference model).
"""
from __future__ import annotations

import copy
import sys
from datetime import datetime
from pathlib import Path

import numpy as np
import torch
import yaml

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
from make_golden import REF, import_reference  # noqa: E402

import recipes  # noqa: E402

WIDTH = 0.125
IMGSZ = 128


def main():
    mods, tasks, ops = import_reference()
    d = yaml.safe_load((REF / "ultralytics/cfg/models/new/yolov12-sod-fusion-v5-simple.yaml").read_text())
    d["width_multiple"] = WIDTH
    d["yaml_file"] = "yolov12-sod-fusion-v5-simple.yaml"
    torch.manual_seed(0)
    m = tasks.DetectionModel(d, verbose=False)
    dfl = {k: v.clone() for k, v in m.state_dict().items() if ".dfl." in k}
    recipes.perturb_(m, 7)
    with torch.no_grad():
        for k, v in m.state_dict().items():
            if k in dfl:
                v.copy_(dfl[k])  # DFL integral weights stay arange(16) (block.py:73-76)
    ckpt = {
        "epoch": 99,
        "best_fitness": 0.5,
        "model": None,
        "ema": copy.deepcopy(m).half(),
        "updates": 1234,
        "optimizer": None,
        "train_args": {"model": "yolov12-sod-fusion-v5-simple.yaml", "imgsz": 640, "batch": 16, "epochs": 100},
        "train_metrics": {"metrics/mAP50-95(B)": 0.25, "fitness": 0.5},
        "train_results": {"epoch": [1, 2], "metrics/mAP50(B)": [0.1, 0.2]},
        "date": datetime(2025, 1, 1).isoformat(),
        "version": "8.3.63",
        "license": "AGPL-3.0 (https://ultralytics.com/license)",
        "docs": "https://docs.ultralytics.com",
    }
    path = HERE / "ckpt_tiny.pt"
    torch.save(ckpt, path)

    # reference load path: ema -> float -> fuse -> eval (attempt_load_one_weight, autobackend fuse=True)
    ck = torch.load(path, map_location="cpu", weights_only=False)  # this script's own file, reference classes
    sd = {k: v.float().numpy() for k, v in ck["ema"].state_dict().items()}  # as saved (unfused, fp16 -> fp32)
    r = ck["ema"].float()
    r.fuse(verbose=False)
    r.eval()
    g = torch.Generator().manual_seed(3)
    x = torch.rand(2, 3, IMGSZ, IMGSZ, generator=g)
    with torch.inference_mode():
        y = r(x)[0]
    det = ops.non_max_suppression(y.clone(), 0.25, 0.7, max_det=300)
    rows = [dd.numpy() for dd in det]
    np.savez_compressed(HERE / "ckpt_tiny.npz", x_seed=np.array(3), imgsz=np.array(IMGSZ), width=np.array(WIDTH),
                        y=y.numpy(), det0=rows[0], det1=rows[1],
                        sd_keys=np.array(sorted(sd)), sd_sum=np.array([float(np.float64(sd[k]).sum()) for k in sorted(sd)]))
    print(path, path.stat().st_size, "bytes;", "y", tuple(y.shape), "detections", [len(rr) for rr in rows])


if __name__ == "__main__":
    main()
