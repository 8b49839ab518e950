"""Run-to-run determinism of the GPU forward (same input, same path twice) and equality across executor modes
(two streams / one stream / plain torch.cat executor). DET=1 sets torch.backends.cudnn.deterministic."""
import os
import sys
import torch
sys.path.insert(0, '.')
if os.environ.get("DET") == "1":
    torch.backends.cudnn.deterministic = True
import yolosod_import  # noqa
from yolosod_amd.nn.tasks import build_model
from yolosod_amd.nn import tasks
cuda = torch.device('cuda:0')
m = build_model("yolov12-sod-fusion-v5-simple.yaml", seed=0, device=cuda)
x = torch.rand(4, 3, 320, 320, generator=torch.Generator().manual_seed(5)).to(cuda)
res = {}
with torch.inference_mode():
    for name, st, fused in [("s1a", 1, True), ("s1b", 1, True), ("s0a", 0, True), ("s0b", 0, True), ("pa", 0, False), ("pb", 0, False)]:
        tasks.STREAMS = st
        m._fused = fused
        res[name] = m(x)[0].clone()
    m._fused = True
torch.cuda.synchronize()
for a, b in [("s1a", "s1b"), ("s0a", "s0b"), ("pa", "pb"), ("s1a", "s0a"), ("s0a", "pa")]:
    print(a, b, torch.equal(res[a], res[b]), float((res[a] - res[b]).abs().max()))
