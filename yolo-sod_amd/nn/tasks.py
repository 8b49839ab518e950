"""Graph builder / executor for the reference's model YAMLs (``ultralytics/nn/tasks.py`` semantics).

* :func:`parse_model` - ``tasks.py:967-1169``: YAML rows ``[from, n, module, args]`` -> ``nn.Sequential``, with the
  reference's depth/width scaling (``make_divisible(min(c2, max_channels) * width, 8)``), ``scales`` support and
  the channel-injection rules of the MAFN operators (``tasks.py:1122-1146``). Modules are resolved **by name**
  through a registry, so a caller (e.g. the CPU oracle in ``oracle/``) can substitute implementations while
  keeping parameter layout and RNG order.
* :class:`DetectionModel` - ``tasks.py:336-379``: builds the graph, materialises the lazy SE weights in layer
  order, probes strides (shape-only, on the ``meta`` device), applies ``Detect.bias_init`` and
  ``initialize_weights`` (every BatchNorm2d: eps=1e-3, momentum=0.03) and loads the BatchNorm running statistics
  that the reference's *train-mode* 256x256 stride probe leaves behind (shipped per config as
  ``cfg/<name>.probe.npz``, recorded from the reference by ``tests/golden/make_golden.py``).
* :meth:`BaseModel.fuse` - ``tasks.py:227-255``: folds BN into ``Conv``/``DWConv`` (SwinBlock.bn and CA.bn1 stay
  unfused, as in the reference).
"""
from __future__ import annotations

import ast
import contextlib
import copy
import hashlib
import math
import os
import re
from pathlib import Path

import numpy as np
import torch
import torch.nn as nn
import yaml

from .. import _hip
from . import modules as M

CFG_DIR = Path(__file__).resolve().parent.parent / "cfg"

# GPU executor: run the Detect towers of each level on a side stream as soon as that level's feature map exists
# (overlapping the rest of the neck); YOLOSOD_STREAMS=0 keeps everything on one stream (A/B)
# (2: start them only after the last MAFN operator has been enqueued, so no hot-path op shares the GPU)
# Unset: 1 for fp32 models, 2 for the bf16 config (its P2 towers are large enough that overlapping them with CA only
# moved time between the two streams: m640 1636 vs 1634 img/s same-box, CA 0.33 vs 0.12 ms on the main stream)
_STREAMS_ENV = os.environ.get("YOLOSOD_STREAMS")
STREAMS = int(_STREAMS_ENV) if _STREAMS_ENV is not None else 1
# side streams the towers are dealt to, one tower (box or class, per level) at a time, round robin. With one side
# stream every level's towers queued behind P2's (3.4 ms of 160x160 convs at n640): the P4 / P5 towers ran after the
# neck had finished, one small conv at a time, and the main stream idled ~0.65 ms per step before the head. Three
# side streams + main = the box's 4 hardware queues (GPU_MAX_HW_QUEUES); more would share queues. With the tower
# convs on the persistent fp16-split kernel two side streams are as fast (same box 3285 -> 3300 img/s, 2 x 2 runs,
# profiles/r05/streams/): the default is 2.
SIDE_STREAMS = max(1, int(os.environ.get("YOLOSOD_SIDE_STREAMS", "2")))
# SE / CBAM whose only reader is the next layer, a fused 3x3 / stride-2 Conv (SE L1 -> L2, CBAM L4 -> L5 in the paper
# YAML): the gate only, then the Conv applies it while staging its input (csrc/conv3x3s2.hip) - the gate's apply pass
# and the conv's re-read of its output disappear. YOLOSOD_GATE_FUSE=0: the operator's own apply + MIOpen (A/B)
GATE_FUSE = os.environ.get("YOLOSOD_GATE_FUSE", "1") != "0"
# the neck's nearest 2x upsample into its Concat slice as one HIP pass (YOLOSOD_UPSAMPLE_HIP=0: PyTorch's strided
# copy, for A/B)
UPSAMPLE_HIP = os.environ.get("YOLOSOD_UPSAMPLE_HIP", "1") != "0"
# a neck Concat read only by the next C2f's cv1 (a 1x1 conv whose kernel reads both parts in place) is handed over as
# a _hip.CatView instead of a buffer: the skip input (an earlier layer's saved output) is not copied at all, the -1
# producer writes its own tensor (YOLOSOD_CATVIEW=0: the concat buffer with the producer's slice written in place)
CATVIEW = os.environ.get("YOLOSOD_CATVIEW", "1") != "0"

# name -> class; the YAML resolves module strings through this (tasks.py:995-1002)
DEFAULT_REGISTRY = {
    "Conv": M.Conv, "DWConv": M.DWConv, "Concat": M.Concat, "Bottleneck": M.Bottleneck, "C2f": M.C2f,
    "SPPF": M.SPPF, "DFL": M.DFL, "SE": M.SE, "SE_Block": M.SE_Block, "CBAM_Block": M.CBAM_Block,
    "CA_Block": M.CA_Block, "A2_Attn": M.A2_Attn, "SwinBlock": M.SwinBlock, "MambaBlock": M.MambaBlock,
    "Detect": M.Detect,
}

# channel-injection classes of the reference parse_model (by name)
_SCALED_C1C2 = {"Conv", "DWConv", "Bottleneck", "C2f", "SPPF"}
_REPEAT_INSERT = {"C2f"}
_KEEP_CH = {"SE", "SE_Block", "SwinBlock", "CA_Block", "A2_Attn", "CBAM_Block", "MambaBlock"}
_DETECT = {"Detect"}


def make_divisible(x, divisor):
    """ops.py:130-143."""
    if isinstance(divisor, torch.Tensor):
        divisor = int(divisor.max())
    return math.ceil(x / divisor) * divisor


def guess_model_scale(model_path) -> str:
    """tasks.py guess_model_scale: the n/s/m/l/x letter after 'yolov<digits>' in the file stem, else ''."""
    m = re.search(r"yolov\d+([nslmx])", Path(model_path).stem)
    return m.group(1) if m else ""


def yaml_model_load(path) -> dict:
    """Load a model YAML (tasks.py:1172-1185 minus the unified-name lookup; ``scale`` from the YAML wins)."""
    path = Path(path)
    if not path.exists() and (CFG_DIR / path.name).exists():
        path = CFG_DIR / path.name
    d = yaml.safe_load(path.read_text())
    d.setdefault("scale", guess_model_scale(path))
    d["yaml_file"] = str(path)
    return d


def parse_model(d: dict, ch: int, verbose: bool = False, registry: dict | None = None):
    """YAML dict -> (nn.Sequential, sorted save list). Mirrors tasks.py:967-1169 for the operators of this path."""
    reg = dict(DEFAULT_REGISTRY)
    if registry:
        reg.update(registry)
    legacy = True
    max_channels = float("inf")
    nc, act, scales = (d.get(x) for x in ("nc", "activation", "scales"))
    depth, width, kpt_shape = (d.get(x, 1.0) for x in ("depth_multiple", "width_multiple", "kpt_shape"))
    if scales:
        scale = d.get("scale")
        if not scale:
            scale = tuple(scales.keys())[0]
        depth, width, max_channels = scales[scale]
    if act:
        raise NotImplementedError("custom 'activation' is not supported on this path")

    ch = [ch]
    layers, save, c2 = [], [], ch[-1]
    for i, (f, n, m, args) in enumerate(d.get("backbone", []) + d.get("neck", []) + d.get("head", [])):
        name = m
        if m.startswith("nn."):
            cls = getattr(torch.nn, m[3:])
        else:
            if m not in reg:
                raise KeyError(f"module '{m}' (layer {i}) is not provided by yolosod_amd")
            cls = reg[m]
        args = list(args)
        for j, a in enumerate(args):
            if isinstance(a, str):
                with contextlib.suppress(ValueError):
                    args[j] = locals()[a] if a in locals() else ast.literal_eval(a)
        n = n_ = max(round(n * depth), 1) if n > 1 else n
        if name in _SCALED_C1C2:
            c1, c2 = ch[f], args[0]
            if c2 != nc:
                c2 = make_divisible(min(c2, max_channels) * width, 8)
            args = [c1, c2, *args[1:]]
            if name in _REPEAT_INSERT:
                args.insert(2, n)
                n = 1
        elif name == "Concat":
            c2 = sum(ch[x] for x in f)
        elif name in _KEEP_CH:
            c2 = ch[f]
            if name in {"SwinBlock", "MambaBlock", "CA_Block", "CBAM_Block"}:
                args = [ch[f], *args]
            elif name == "A2_Attn":
                args = [ch[f], None, *args]
        elif name in _DETECT:
            f_list = f if isinstance(f, (list, tuple)) else [f]
            args.append([ch[x] for x in f_list])
            cls.legacy = legacy
        else:
            c2 = ch[f]

        m_ = nn.Sequential(*(cls(*args) for _ in range(n))) if n > 1 else cls(*args)
        t = name if not name.startswith("nn.") else f"torch.nn.modules.{name[3:]}"
        m_.np = sum(x.numel() for x in m_.parameters())
        m_.i, m_.f, m_.type = i, f, t
        m_.c_in = ch[f] if isinstance(f, int) else [ch[x] for x in f]
        if verbose:
            print(f"{i:>3}{str(f):>20}{n_:>3}{m_.np:10.0f}  {t:<45}{str(args):<30}")
        save.extend(x % i for x in ([f] if isinstance(f, int) else f) if x != -1)
        layers.append(m_)
        if i == 0:
            ch = []
        ch.append(c2)
    return nn.Sequential(*layers), sorted(save)


def initialize_weights(model: nn.Module) -> None:
    """torch_utils.py:410-420."""
    for m in model.modules():
        t = type(m)
        if t is nn.BatchNorm2d:
            m.eps = 1e-3
            m.momentum = 0.03
        elif t in {nn.Hardswish, nn.LeakyReLU, nn.ReLU, nn.ReLU6, nn.SiLU}:
            m.inplace = True


def state_dict_sha256(model: nn.Module) -> str:
    """Hash over (key, float tensor bytes) in state_dict order - the manifest identity of seeded weights."""
    h = hashlib.sha256()
    for k, v in model.state_dict().items():
        h.update(k.encode())
        h.update(v.detach().cpu().contiguous().numpy().tobytes())
    return h.hexdigest()


class BaseModel(nn.Module):
    def forward(self, x, *args, **kwargs):
        return self.predict(x, *args, **kwargs)

    def predict(self, x, profile=False, visualize=False, augment=False, embed=None):
        return self._predict_once(x)

    def _predict_once(self, x):
        """tasks.py:165-192: run layers in YAML order, keeping the outputs other layers read."""
        if x.device.type == "cuda" and getattr(self, "_fused", False):
            return self._predict_once_planned(x)
        y = []
        for m in self.model:
            if m.f != -1:
                x = y[m.f] if isinstance(m.f, int) else [x if j == -1 else y[j] for j in m.f]
            x = m(x)
            y.append(x if m.i in self.save else None)
        return x

    def _concat_producers(self):
        """Concat layers whose ``-1`` input is a layer that can write its output straight into the Concat's
        channel slice: a fused Conv (the HIP epilogue takes a batch-strided ``out``) or a nearest 2x Upsample
        (one strided copy), read by nothing else. Returns {producer index: concat index}."""
        plan = getattr(self, "_cplan", None)
        if plan is not None:
            return plan
        plan = {}
        for c, m in enumerate(self.model):
            if not isinstance(m, M.Concat) or m.d != 1 or not isinstance(m.f, (list, tuple)) or -1 not in m.f:
                continue
            p = c - 1
            prod = self.model[p]
            if p in self.save or sum(1 for j in m.f if j in (-1, p)) != 1:
                continue
            if (isinstance(prod, M.Conv) and prod.is_fused() and prod.emit_stats is None) or (
                    isinstance(prod, nn.Upsample) and prod.mode == "nearest" and prod.size is None
                    and prod.scale_factor in (2, 2.0, (2, 2), (2.0, 2.0))):
                plan[p] = c
        self._cplan = plan
        return plan

    def _gate_consumers(self):
        """{gate layer index: consumer Conv} for SE / CBAM layers read only by the next layer, a fused 3x3 / stride-2
        Conv with 64 or 128 outputs (the shapes are checked again per call: Conv.gated_ok)."""
        plan = getattr(self, "_gplan", None)
        if plan is not None:
            return plan
        plan = {}
        # a consumer that writes into a planned Concat slice or feeds a Detect level keeps its own path: the gated
        # form returns early, before the concat-plan and tower bookkeeping of the executor
        det = self.model[-1]
        busy = set(self._concat_producers()) | (set(det.f) if isinstance(det, M.Detect) and isinstance(
            det.f, (list, tuple)) else set())
        for k in range(len(self.model) - 1):
            m, nxt = self.model[k], self.model[k + 1]
            if (isinstance(m, (M.SE, M.CBAM_Block)) and k not in self.save and k + 1 not in busy
                    and isinstance(nxt, M.Conv)
                    and not isinstance(nxt, M.DWConv) and nxt.f == -1 and nxt.conv.kernel_size == (3, 3)
                    and nxt.conv.stride == (2, 2) and nxt.conv.groups == 1 and nxt.conv.out_channels in (64, 128)):
                plan[k] = nxt
        self._gplan = plan
        return plan

    def _predict_once_planned(self, x):
        """GPU fused forward with concat elision: for a planned Concat, the buffer is allocated when its ``-1``
        producer runs (every other input is an earlier layer's saved output, so all shapes are known), the
        producer writes its channel slice in place, and the Concat copies only the other inputs. Same values as
        torch.cat (pure copies), one HBM round trip less for the producer's part."""
        plan = self._concat_producers()
        det = self.model[-1]
        towers = lvl = main = side = None
        streams = STREAMS
        if _STREAMS_ENV is None and x.dtype == torch.bfloat16:
            streams = 2
        if (streams > 0 and isinstance(det, M.Detect) and isinstance(det.f, (list, tuple)) and len(set(det.f)) == len(det.f)
                and det._fused_ok([x])):
            lvl = {j: k for k, j in enumerate(det.f)}
            towers = {}
            ready = []  # levels whose feature map exists but whose towers wait for the last MAFN op (STREAMS == 2)
            last_mafn = max((k for k, mm in enumerate(self.model)
                             if isinstance(mm, (M.SE, M.CBAM_Block, M.CA_Block, M.A2_Attn, M.SwinBlock))), default=-1)
            main = torch.cuda.current_stream(x.device)
            side = getattr(self, "_side_streams", None)
            if side is None or len(side) != SIDE_STREAMS or side[0].device != x.device:
                side = self._side_streams = [torch.cuda.Stream(device=x.device) for _ in range(SIDE_STREAMS)]
            rr = 0  # next side stream (round robin over towers)
        y = []
        pend = {}  # concat index -> (buffer, channel offset of each input)
        cvpend = {}  # concat index -> True: handed to the next C2f as a CatView
        elided = 0
        gplan = self._gate_consumers() if GATE_FUSE else {}
        gated = None  # (gate input, channel gate, spatial gate, fused-op key) for the next layer
        for m in self.model:
            if gated is not None:  # the consumer Conv of the previous layer's gate
                xg, gc, gp, key = gated
                gated = None
                x = m.forward_gated(xg, gc, gp, key)
                y.append(x if m.i in self.save else None)
                continue
            inp = x
            if m.f != -1:
                inp = y[m.f] if isinstance(m.f, int) else [x if j == -1 else y[j] for j in m.f]
            cons = gplan.get(m.i)
            if cons is not None and isinstance(inp, torch.Tensor) and cons.gated_ok(inp):
                if isinstance(m, M.SE):
                    gc, gp = m.gate(inp), None
                    key = ("se_conv", tuple(inp.shape), (cons.conv.out_channels, m.fc1.out_channels))
                else:
                    gc, gp = m.gates(inp)
                    key = ("cbam_conv", tuple(inp.shape),
                           (cons.conv.out_channels, m.channel_attention.fc[0].out_channels))
                gated = (inp, gc, gp, key)
                x = None
                y.append(None)
                continue
            c = plan.get(m.i)
            if c is not None and isinstance(inp, torch.Tensor) and inp.dim() == 4:
                cat = self.model[c]
                B, _, H, W = inp.shape
                if isinstance(m, nn.Upsample):
                    H, W = 2 * H, 2 * W
                    cp = inp.shape[1]
                else:
                    cv = m.conv
                    cp = cv.out_channels
                    H, W = ((n + 2 * p - d * (k - 1) - 1) // s + 1 for n, p, d, k, s in
                            zip((H, W), cv.padding, cv.dilation, cv.kernel_size, cv.stride))
                srcs = [None if j == -1 else y[j] for j in cat.f]
                chans = [cp if s is None else s.shape[1] for s in srcs]
                nxt = self.model[c + 1] if c + 1 < len(self.model) else None
                if (CATVIEW and len(srcs) == 2 and c not in self.save and isinstance(nxt, M.C2f) and nxt.f == -1
                        and all(s is None or (s.shape[0], s.shape[2], s.shape[3]) == (B, H, W) for s in srcs)
                        and M.catview_route(nxt.cv1, chans[0], chans[1], H, W, inp.dtype)):
                    # the Concat becomes a CatView of its inputs: the producer writes its own tensor
                    if isinstance(m, nn.Upsample):
                        x = torch.empty((B, cp, H, W), dtype=inp.dtype, device=inp.device)
                        if not (UPSAMPLE_HIP and _hip.upsample2x_into(inp, x)):
                            x = m(inp)
                    else:
                        x = m(inp)
                    cvpend[c] = True
                    y.append(None)
                    continue
                if all(s is None or (s.shape[0], s.shape[2], s.shape[3]) == (B, H, W) for s in srcs):
                    buf = torch.empty((B, sum(chans), H, W), dtype=inp.dtype, device=inp.device)
                    offs = [sum(chans[:i]) for i in range(len(chans))]
                    k = [j for j in cat.f].index(-1)
                    out = buf[:, offs[k]:offs[k] + cp]
                    if isinstance(m, nn.Upsample):
                        h, w = inp.shape[2], inp.shape[3]
                        if not (UPSAMPLE_HIP and _hip.upsample2x_into(inp, out)):
                            out.view(B, cp, h, 2, w, 2).copy_(inp[:, :, :, None, :, None].expand(B, cp, h, 2, w, 2))
                    else:
                        m.forward_fuse(inp, out=out)
                    pend[c] = (buf, offs, chans)
                    x = out
                    y.append(None)
                    continue
            if cvpend.pop(m.i, False):
                x = _hip.CatView([x if j == -1 else y[j] for j in m.f])
                elided += 1
            elif m.i in pend:
                buf, offs, chans = pend.pop(m.i)
                elided += 1
                for j, o, n in zip(m.f, offs, chans):
                    if j != -1:
                        buf[:, o:o + n].copy_(y[j])
                x = buf
            elif m is det and towers is not None and len(towers) == det.nl:
                feats = [towers[k] for k in range(det.nl)]
                for sd in side:  # every level's tower features are ready (and owned by main from here)
                    main.wait_stream(sd)
                x = det.forward_towers(feats)
            else:
                x = m(inp)
            if towers is not None and m is not det:
                # Detect towers (PyTorch-ROCm convs + HIP epilogues) of each level on the side stream, overlapping
                # the rest of the neck; inputs / outputs cross streams via record_stream
                if m.i in lvl:
                    ready.append((lvl[m.i], x))
                if ready and (streams != 2 or m.i >= last_mafn):
                    for k, xk in ready:
                        feats = []
                        for tower in (det.cv2[k], det.cv3[k]):  # box, class tower (Detect.tower_features)
                            sd = side[rr % len(side)]
                            rr += 1
                            sd.wait_stream(main)
                            xk.record_stream(sd)
                            with torch.cuda.stream(sd):
                                f = tower[:-1](xk).contiguous()
                            f.record_stream(main)
                            feats.append(f)
                        towers[k] = tuple(feats)
                    ready = []
            y.append(x if m.i in self.save else None)
        self._last_elided = elided
        return x

    def is_fused(self, thresh=10):
        bn = tuple(v for k, v in nn.__dict__.items() if "Norm" in k)
        return sum(isinstance(v, bn) for v in self.modules()) < thresh

    def fuse(self, verbose=False):
        """Fold BN into Conv/DWConv (tasks.py:227-255 + torch_utils.fuse_conv_and_bn :238-265)."""
        if not self.is_fused():
            for m in self.model.modules():
                if isinstance(m, M.Conv) and hasattr(m, "bn"):
                    m.conv = _fuse_conv_and_bn(m.conv, m.bn)
                    delattr(m, "bn")
                    m.forward = m.forward_fuse
        self._fused = True
        self._cplan = None
        return self


def _fuse_conv_and_bn(conv: nn.Conv2d, bn: nn.BatchNorm2d) -> nn.Conv2d:
    fused = nn.Conv2d(conv.in_channels, conv.out_channels, kernel_size=conv.kernel_size, stride=conv.stride,
                      padding=conv.padding, dilation=conv.dilation, groups=conv.groups,
                      bias=True).requires_grad_(False).to(conv.weight.device)
    with torch.no_grad():
        w, b = M.fold_conv_bn(conv, bn)
        fused.weight.copy_(w)
        fused.bias.copy_(b)
    return fused


def probe_manifest_path(yaml_file) -> Path:
    return CFG_DIR / (Path(yaml_file).stem + ".probe.npz")


class DetectionModel(BaseModel):
    """Detection model (tasks.py:336-379) for the YOLO-SOD YAMLs."""

    def __init__(self, cfg="yolov12-sod-fusion-v5-simple.yaml", ch=3, nc=None, verbose=False, registry=None,
                 probe_stats: bool = True):
        super().__init__()
        self.yaml = cfg if isinstance(cfg, dict) else yaml_model_load(cfg)
        ch = self.yaml["ch"] = self.yaml.get("ch", ch)
        if nc and nc != self.yaml["nc"]:
            self.yaml["nc"] = nc
        self.model, self.save = parse_model(copy.deepcopy(self.yaml), ch=ch, verbose=verbose, registry=registry)
        self.names = {i: f"{i}" for i in range(self.yaml["nc"])}
        self.inplace = self.yaml.get("inplace", True)

        # SE / CBAM / CA whose input is the previous layer's conv output: that conv's epilogue emits the gate's
        # plane statistics (CA: row / column means) in the same pass (no statistics re-read; HIP path only)
        for i, m in enumerate(self.model):
            if i and m.f == -1 and isinstance(m, (M.SE, M.CBAM_Block, M.CA_Block)):
                prod = self.model[i - 1]
                conv = prod if isinstance(prod, M.Conv) else getattr(prod, "cv2", None)
                if isinstance(conv, M.Conv):
                    conv.emit_stats = ("summax" if isinstance(m, M.CBAM_Block) else
                                       "capool" if isinstance(m, M.CA_Block) else "sum")

        # the neck's 3x3 / stride-2 convs run on the stride-2 fp16-split kernel (modules.S2_NECK); the backbone's
        # convs stay on PyTorch-ROCm (north_star), except SE L1's / CBAM L4's consumers, which apply those gates
        n_backbone = len(self.yaml.get("backbone", []))
        for i, m in enumerate(self.model):
            if (i >= n_backbone and isinstance(m, M.Conv) and not isinstance(m, M.DWConv)
                    and m.conv.kernel_size == (3, 3) and m.conv.stride == (2, 2) and m.conv.groups == 1):
                m.s2 = True
            if i >= n_backbone and isinstance(m, M.C2f):  # the neck C2fs' Bottleneck 3x3 convs (S1_NECK)
                for bt in m.m:
                    for cv in (bt.cv1, bt.cv2):
                        if cv.conv.kernel_size == (3, 3) and cv.conv.stride == (1, 1) and cv.conv.groups == 1:
                            cv.s1 = True
            # the neck's wide 1x1 convs (N1_NECK): lateral Convs and the C2fs' cv1 / cv2
            if i >= n_backbone:
                for cv in ([m] if isinstance(m, M.Conv) and not isinstance(m, M.DWConv) else
                           [m.cv1, m.cv2] if isinstance(m, M.C2f) else []):
                    if cv.conv.kernel_size == (1, 1) and cv.conv.groups == 1 and cv.conv.out_channels % 128 == 0:
                        cv.n1 = True

        # lazy SE weights: the reference creates them during the stride probe, in forward (= layer) order,
        # after every eager module -> same RNG stream position here.
        for m in self.model:
            if isinstance(m, M.SE):
                m._maybe_build(m.c_in, None)

        det = self.model[-1]
        if not isinstance(det, M.Detect):
            raise NotImplementedError("only Detect-headed models are supported")
        det.stride = self._probe_strides(ch)
        self.stride = det.stride
        det.bias_init()
        initialize_weights(self)
        if probe_stats:
            self._load_probe_stats()

    def _probe_strides(self, ch: int, s: int = 256) -> torch.Tensor:
        """Shape-only replica of the reference's 256x256 stride probe (tasks.py:369), on the meta device."""
        meta = copy.deepcopy(self).to("meta")
        meta.train()
        with torch.no_grad():
            out = meta._predict_once(torch.zeros(1, ch, s, s, device="meta"))
        return torch.tensor([s / x.shape[-2] for x in out])

    def _load_probe_stats(self) -> None:
        """BatchNorm running stats produced by the reference's train-mode stride probe (not re-derivable from the
        seed alone: they depend on that forward's arithmetic). Recorded from the reference, see module doc."""
        p = probe_manifest_path(self.yaml.get("yaml_file", ""))
        if not p.exists():
            import warnings
            warnings.warn(f"no stride-probe BatchNorm manifest {p.name}; running stats keep their init values")
            return
        z = np.load(p, allow_pickle=False)
        sd = self.state_dict()
        with torch.no_grad():
            for k in z.files:
                if k not in sd:
                    raise KeyError(f"probe manifest key {k} not in model")
                sd[k].copy_(torch.from_numpy(z[k]).to(sd[k].dtype))


def build_model(cfg="yolov12-sod-fusion-v5-simple.yaml", seed: int = 0, device="cuda", fuse: bool = True,
                registry=None, dtype=torch.float32) -> DetectionModel:
    """Seeded construction -> (fused) eval model on ``device`` (autobackend.py:145-156 semantics).

    ``dtype=torch.bfloat16`` is the bf16 config: fuse in fp32, then store every parameter / buffer and every
    activation as bf16 - AutoBackend's ``fp16`` path (``model.half()`` after ``fuse()``, autobackend.py:145-156, and
    the predictor's ``im.half()``) with bfloat16. The HIP operators accumulate in fp32; Detect's decode and NMS stay
    fp32."""
    torch.manual_seed(seed)
    m = DetectionModel(cfg, registry=registry)
    if fuse:
        m.fuse()
    m = m.to(device)
    if dtype != torch.float32:
        m = m.to(dtype)
    return m.eval()
