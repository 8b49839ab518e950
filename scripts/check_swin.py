"""Quick GPU check of the Swin operator at one real shape: max |err| vs the fp64 oracle and run-to-run
determinism. usage: [YOLOSOD_LIB_AB=lib] python scripts/check_swin.py [swin_L28|swin_L9]"""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT / "tests" / "golden"))
import yolosod_import  # noqa: E402,F401
import recipes  # noqa: E402
from oplib import build_fixture_module  # noqa: E402
from oracle.model_ref import OP_CLASSES  # noqa: E402

CASES = {"swin_L28": ("SwinBlock", (64, 2, 7), (1, 64, 160, 160)), "swin_L9": ("SwinBlock", (256, 4, 7), (1, 256, 40, 40))}
for name in (sys.argv[1:] or ["swin_L28"]):
    recipes.OPS[name] = CASES[name]
    m, _ = build_fixture_module(name)
    ref_m, _ = build_fixture_module(name, OP_CLASSES)
    x = recipes.make_input(name, CASES[name][2])
    with torch.inference_mode():
        ref = ref_m.double()(x.double())
        md = m.cuda()
        y1 = md(x.cuda()).cpu()
        y2 = md(x.cuda()).cpu()
    err = float((y1.double() - ref).abs().max())
    print(f"{name}: max|err| {err:.3g}  deterministic {torch.equal(y1, y2)}  max|y1-y2| {float((y1 - y2).abs().max()):.3g}",
          flush=True)
    from yolosod_amd import _hip
    wa = md.window_attn
    with torch.inference_mode():
        args = (x.cuda(), wa.attn.num_heads, wa.window_size, md.dw.weight, wa.norm1.weight, wa.norm1.bias, wa.norm1.eps,
                wa.attn.in_proj_weight, wa.attn.in_proj_bias, wa.attn.out_proj.weight, wa.attn.out_proj.bias,
                wa.norm2.weight, wa.norm2.bias, wa.norm2.eps, wa.mlp[0].weight, wa.mlp[0].bias, wa.mlp[2].weight,
                wa.mlp[2].bias, md.pw.weight, md.bn.weight, md.bn.bias, md.bn.running_mean, md.bn.running_var,
                md.bn.eps)
        u1 = _hip.swin_forward(*args).cpu()
        u2 = _hip.swin_forward(*args).cpu()
    print(f"   unprepared ABI: max|err| {float((u1.double() - ref).abs().max()):.3g} deterministic {torch.equal(u1, u2)}",
          flush=True)
