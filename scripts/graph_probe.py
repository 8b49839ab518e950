"""Probe: capture the n640 predictor step (forward + decode + NMS, 3 side streams) in a torch.cuda.CUDAGraph, check
the replay against the eager step bit for bit (deterministic convs) and time both."""
import os
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
os.environ.setdefault("MIOPEN_USER_DB_PATH", str(ROOT / "yolo-sod_amd" / "miopen_db"))
import yolosod_import  # noqa: E402,F401
from yolosod_amd.engine.predictor import DetectionPredictor, seeded_images  # noqa: E402
from yolosod_amd.nn.tasks import build_model  # noqa: E402

dev = torch.device("cuda", 0)
det = "--det" in sys.argv
torch.backends.cudnn.deterministic = det
model = build_model("yolov12-sod-fusion-v5-simple.yaml", seed=0, device=dev)
pred = DetectionPredictor(model, conf=0.25, iou=0.7, max_det=300)
x = seeded_images(0, 32, 640, device=dev)
for _ in range(3):
    out_e, cnt_e, idx_e = pred.predict_padded(x)
torch.cuda.synchronize()
print("eager warm", flush=True)
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(2):
        pred.predict_padded(x)
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
t0 = time.perf_counter()
with torch.cuda.graph(g):
    out_g, cnt_g, idx_g = pred.predict_padded(x)
torch.cuda.synchronize()
print(f"captured in {time.perf_counter() - t0:.2f}s", flush=True)
g.replay()
torch.cuda.synchronize()
out_e, cnt_e, idx_e = pred.predict_padded(x)
torch.cuda.synchronize()
print("replay == eager:", torch.equal(out_g, out_e), torch.equal(cnt_g, cnt_e), torch.equal(idx_g, idx_e),
      float((out_g - out_e).abs().max()), flush=True)
for mode in ("eager", "graph", "eager", "graph"):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        if mode == "graph":
            g.replay()
        else:
            pred.predict_padded(x)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 20
    print(f"{mode}: {dt * 1e3:.3f} ms/step = {32 / dt:.1f} img/s", flush=True)
