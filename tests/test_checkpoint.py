"""Checkpoint ingest: the reference trainer's .pt layout loaded without executing the file.

Pinned to a checkpoint written by the reference itself (tests/golden/make_ckpt_golden.py: reduced-width paper
graph, perturbed weights, engine/trainer.py:513-536 layout) and to the reference's own reload + fused forward +
non_max_suppression of it. CPU only: the oracle operators run the model."""
import os
import pickle

import numpy as np
import pytest
import torch

from conftest import GOLDEN, golden

CKPT = GOLDEN / "ckpt_tiny.pt"


def test_load_checkpoint_stubs_reference_classes():
    from yolosod_amd.nn.checkpoint import load_checkpoint
    ck = load_checkpoint(CKPT)
    ema = ck["ema"]
    assert type(ema).__module__ == "ultralytics.nn.tasks" and type(ema).__name__ == "DetectionModel"
    assert ck["epoch"] == 99 and ck["train_args"]["imgsz"] == 640 and ck["model"] is None
    assert isinstance(ema.yaml, dict) and ema.yaml["width_multiple"] == 0.125
    # library modules come back as themselves
    assert isinstance(ema.model[9].window_attn.attn, torch.nn.MultiheadAttention)


def test_checkpoint_state_matches_reference_state():
    from yolosod_amd.nn.checkpoint import checkpoint_model_state, load_checkpoint
    z = golden("ckpt_tiny")
    _, sd, _ = checkpoint_model_state(load_checkpoint(CKPT))
    keys = sorted(sd)
    assert keys == list(z["sd_keys"])
    sums = np.array([float(sd[k].double().sum()) for k in keys])
    assert np.array_equal(sums, z["sd_sum"])  # fp16 -> fp32 is exact


def test_loaded_model_matches_reference_forward_and_nms():
    from oracle.model_ref import REGISTRY
    from oracle.nms import non_max_suppression_ref
    from yolosod_amd.nn.checkpoint import attempt_load_one_weight
    z = golden("ckpt_tiny")
    m, _ = attempt_load_one_weight(CKPT, device="cpu", registry=REGISTRY)
    g = torch.Generator().manual_seed(int(z["x_seed"]))
    x = torch.rand(2, 3, int(z["imgsz"]), int(z["imgsz"]), generator=g)
    with torch.inference_mode():
        y = m(x)[0]
    ref = torch.from_numpy(z["y"])
    err = (y - ref).abs()
    assert bool((err <= 1e-3 + 1e-5 * ref.abs()).all()), float(err.max())  # north-star 1e-3 abs (+ rel for |y|~1e3)
    rows, _ = non_max_suppression_ref(y.numpy().copy(), 0.25, 0.7, max_det=300)
    for i in range(2):
        d, r = np.asarray(rows[i]), z[f"det{i}"]
        assert d.shape == r.shape and len(r) > 0
        assert np.abs(d - r).max() < 1e-3


def test_save_checkpoint_round_trip(tmp_path):
    from yolosod_amd.nn.checkpoint import attempt_load_one_weight, load_checkpoint, save_checkpoint
    from yolosod_amd.nn.tasks import DetectionModel
    d = dict(load_checkpoint(CKPT)["ema"].yaml)
    torch.manual_seed(0)
    m = DetectionModel(d, probe_stats=False)
    p = save_checkpoint(m, tmp_path / "x.pt", epoch=3)
    names = torch.serialization.get_unsafe_globals_in_checkpoint(str(p))
    assert "ultralytics.nn.modules.blocks_transformer.SwinBlock" in names
    assert "ultralytics.nn.tasks.DetectionModel" in names
    assert not any(n.startswith("yolosod_amd") for n in names)
    m2, ck = attempt_load_one_weight(p, device="cpu", fuse=False)
    assert ck["epoch"] == 3
    sd, sd2 = m.state_dict(), m2.state_dict()
    assert sorted(sd) == sorted(sd2)
    for k in sd:
        if sd[k].is_floating_point():
            assert torch.equal(sd[k].half().float(), sd2[k]), k


class _Evil:
    def __init__(self, marker):
        self.marker = marker

    def __reduce__(self):
        return (os.system, (f"touch {self.marker}",))


def test_loader_executes_nothing_from_the_file(tmp_path):
    from yolosod_amd.nn.checkpoint import load_checkpoint
    marker = tmp_path / "pwned"
    p = tmp_path / "evil.pt"
    torch.save({"model": _Evil(str(marker))}, str(p))
    try:  # torch's weights_only unpickler refuses blocked modules (os/posix) outright; others would be inert stubs
        ck = load_checkpoint(p)
        assert isinstance(ck["model"], torch.nn.Module)
    except pickle.UnpicklingError:
        pass
    assert not marker.exists()


def test_save_checkpoint_restores_preexisting_reference_classes(tmp_path):
    """saving registers stub classes under the reference class paths for pickle; a module already
    imported at such a path keeps its own classes afterwards."""
    import sys
    import types
    from yolosod_amd.nn.checkpoint import save_checkpoint
    from yolosod_amd.nn.tasks import DetectionModel
    names = ["ultralytics", "ultralytics.nn", "ultralytics.nn.modules", "ultralytics.nn.modules.conv"]
    saved = {n: sys.modules.get(n) for n in names}
    fake = {n: types.ModuleType(n) for n in names}

    class Conv:  # stands in for the real reference class
        pass

    fake["ultralytics.nn.modules.conv"].Conv = Conv
    sys.modules.update(fake)
    try:
        torch.manual_seed(0)
        save_checkpoint(DetectionModel("yolov12-sod-fusion-v5-simple.yaml"), tmp_path / "m.pt")
        assert sys.modules["ultralytics.nn.modules.conv"].Conv is Conv
        assert not hasattr(sys.modules["ultralytics.nn.modules.conv"], "Concat")
    finally:
        for n, m in saved.items():
            if m is None:
                sys.modules.pop(n, None)
            else:
                sys.modules[n] = m
