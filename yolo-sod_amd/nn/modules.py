"""Operator library resolved by YAML name (the reference's ``ultralytics.nn.modules`` API surface for this path).

Classes keep the reference's names, constructor signatures, attribute names (hence ``state_dict`` keys) and the
order in which they create parameters (hence seed-for-seed identical random init).

* Backbone / neck building blocks (``Conv``, ``C2f``, ``Bottleneck``, ``SPPF``, ``Concat``) are ordinary PyTorch
  modules: their convolutions run on PyTorch-ROCm (MIOpen). Reference: ``ultralytics/nn/modules/conv.py:37-55,
  102-107, 323-333`` and ``block.py:178-197, 233-255, 343-356``.
* The hot-path operators - ``SE``/``SE_Block``, ``CBAM_Block``, ``CA_Block``, ``A2_Attn``, ``SwinBlock`` and the
  decode of ``Detect`` - run exclusively through the gfx950 HIP library (``yolosod_amd._hip``). They have no CPU
  compute path: a CPU tensor raises. On the ``meta`` device they only propagate shapes (used for the stride probe
  of :class:`~yolosod_amd.nn.tasks.DetectionModel`).
"""
from __future__ import annotations

import contextlib
import math
import os
from collections.abc import Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _hip

__all__ = (
    "Conv", "DWConv", "Concat", "Bottleneck", "C2f", "SPPF", "DFL", "SE", "SE_Block", "CBAM_Block",
    "ChannelAttention", "SpatialAttention", "CA_Block", "h_sigmoid", "A2_Attn", "WindowAttention", "SwinBlock",
    "Conv1x1BN", "GLUBlock", "MambaBlock", "Detect",
)


def autopad(k, p=None, d=1):
    """'same' padding (conv.py:28-34)."""
    if d > 1:
        k = d * (k - 1) + 1 if isinstance(k, int) else [d * (x - 1) + 1 for x in k]
    if p is None:
        p = k // 2 if isinstance(k, int) else [x // 2 for x in k]
    return p


def _is_meta(x: torch.Tensor) -> bool:
    return x.device.type == "meta"


def _cached(mod: nn.Module, tag: str, srcs, make):
    """``make()`` cached on ``mod`` against the identity / version / dtype of the source tensors (parameter
    conversions for the HIP operators: recomputed only when a parameter is replaced or modified in place)."""
    # inference tensors (made under torch.inference_mode, e.g. A2's folded weights) have no version counter: they
    # are never modified in place outside inference mode, their identity is the key
    # id(t) too: a replaced parameter can land at the freed address with version 0 (load_state_dict(assign=True),
    # new Parameters), which (data_ptr, version) alone would take for the old one
    # A cached device tensor is allocated on the stream that first made it (main or a Detect tower's side stream) and
    # may later be read on another: each use from a different stream records that stream on it, so that the caching
    # allocator does not hand the block out again (after a parameter replacement) while such a launch still reads it.
    key = tuple((id(t), t.data_ptr(), -1 if t.is_inference() else t._version, t.dtype, t.device) for t in srcs)
    cache = mod.__dict__.setdefault("_ys_cache", {})
    ent = cache.get(tag)
    if ent is None or ent[0] != key:
        val = make()
        dev = _cuda_device(val)
        ent = cache[tag] = (key, val, torch.cuda.current_stream(dev) if dev is not None else None)
    elif ent[2] is not None:
        cur = torch.cuda.current_stream(ent[2].device)
        if cur != ent[2]:
            _record_stream(ent[1], cur)
    return ent[1]


def _cuda_device(v):
    if isinstance(v, torch.Tensor):
        return v.device if v.is_cuda else None
    if isinstance(v, (tuple, list)):
        for t in v:
            d = _cuda_device(t)
            if d is not None:
                return d
    return None


def _record_stream(v, stream):
    if isinstance(v, torch.Tensor):
        if v.is_cuda:
            v.record_stream(stream)
    elif isinstance(v, (tuple, list)):
        for t in v:
            _record_stream(t, stream)


def _f32(mod: nn.Module, tag: str, *ts):
    """fp32 contiguous views of parameters (the HIP operators' small parameters are fp32 in either config); in
    the bf16 model these are cached widened copies (exact)."""
    if all(t.dtype == torch.float32 and t.is_contiguous() for t in ts):
        return tuple(t.detach() for t in ts)
    return _cached(mod, tag, ts, lambda: tuple(t.detach().float().contiguous() for t in ts))


def _as(mod: nn.Module, tag: str, dtype, *ts):
    """Parameters as contiguous ``dtype`` tensors (GEMM weights follow the activation dtype)."""
    if all(t.dtype == dtype and t.is_contiguous() for t in ts):
        return tuple(t.detach() for t in ts)
    return _cached(mod, tag, ts, lambda: tuple(t.detach().to(dtype).contiguous() for t in ts))


# ---------------------------------------------------------------------------------------------------------------
# host PyTorch blocks
# ---------------------------------------------------------------------------------------------------------------
def _act_code(act):
    if isinstance(act, nn.SiLU):
        return 1
    if isinstance(act, nn.Identity):
        return 0
    return None


# thin 1x1 convs (Cout 64, Cin <= 256, H*W % 64 == 0) as one fused HIP kernel instead of MIOpen + epilogue
# (scripts/bench_conv1x1.py: 96->64 at 160^2 0.16 vs 0.38 ms; at Cout 128 the MIOpen path stays faster)
THIN1X1 = os.environ.get("YOLOSOD_THIN1X1", "1") == "1"
# the Detect head's 3x3 tower convs (64 outputs) as the library's fp16-split implicit-GEMM kernel (csrc/conv3x3.hip)
# instead of MIOpen + the epilogue pass (faster at every tower shape, P5's 20 x 20 maps included:
# scripts/bench_conv3x3.py). YOLOSOD_CONV3X3=0 restores MIOpen (A/B), =all also takes every other eligible 3x3 conv of
# the model (the backbone stays on MIOpen by default, as north_star asks)
CONV3X3 = os.environ.get("YOLOSOD_CONV3X3", "1")
# the PAN neck's 3x3 / stride-2 convs (layers 29 / 33 / 36 of the paper YAML: the consumers of Swin L28 and CA L32,
# and P4 -> P5) on the stride-2 fp16-split kernel (csrc/conv3x3s2.hip), writing straight into their Concat slice,
# instead of MIOpen's NHWC implicit GEMM with its layout transposes + the bias / SiLU pass; YOLOSOD_S2_NECK=0: MIOpen
S2_NECK = os.environ.get("YOLOSOD_S2_NECK", "1") != "0"
# the PAN neck's C2f Bottleneck 3x3 convs (layers 17 / 22 / 27 / 31 / 35 / 38) on the fp16-split stride-1 kernel, the
# shortcut added and the output written into the C2f concat slice in its epilogue; YOLOSOD_S1_NECK=0: MIOpen
S1_NECK = os.environ.get("YOLOSOD_S1_NECK", "1") != "0"
# the PAN neck's wide 1x1 convs (Cout a multiple of 128: C2f cv1 / cv2, lateral convs) on the fp16-split 1x1 kernel
# (csrc/conv1x1x2.hip) with bias / SiLU / concat slice / C2f's dual store in its epilogue; YOLOSOD_N1_NECK=0: MIOpen
N1_NECK = os.environ.get("YOLOSOD_N1_NECK", "1") != "0"
# the neck C2fs' Bottlenecks (stride-1 fp16-split kernel) read their inputs as slices of the C2f buffer instead of
# packed copies written by a second store (YOLOSOD_C2F_SLICES=0: the dual-store form)
C2F_SLICES = os.environ.get("YOLOSOD_C2F_SLICES", "1") != "0"
# SPPF's three chained max pools + concat as one HIP pass into the buffer cv1 writes (csrc/sppf.hip); 0: PyTorch
SPPF_HIP = os.environ.get("YOLOSOD_SPPF_HIP", "1") != "0"


def conv_epilogue(conv: nn.Conv2d, act_code, x, out=None, res=None, stats=None, out2=None, c2lo=0, tower=False,
                  s2=False, s1=False, n1=False):
    """GPU fast path of ``act(conv(x)) (+ res)``: MIOpen conv without bias, then one HIP pass for bias +
    activation (+ shortcut), optionally written straight into a channel slice ``out`` of a concat buffer.
    ``stats`` ("sum" / "summax"): the same pass emits the output's per-plane partial statistics for a following
    SE / CBAM gate (``_hip.PlaneStats`` on the returned tensor).
    ``out2``: also store channels [c2lo, C) packed there (the next conv's input; C2f's Bottleneck chain).
    ``tower``: the conv is one of the Detect head's 3x3 tower convs (the fp16-split conv kernel takes it).
    ``s2``: the conv is one of the neck's 3x3 / stride-2 convs (the stride-2 fp16-split kernel takes it).
    ``s1``: one of the neck's C2f Bottleneck 3x3 convs (the stride-1 fp16-split kernel, with out / res).
    ``n1``: one of the neck's wide 1x1 convs (the fp16-split 1x1 kernel, with out / out2).
    Returns None when the fast path does not apply (CPU tensor, no bias, unsupported activation / shape)."""
    if x.device.type != "cuda" or conv.bias is None or act_code is None or x.dtype not in (torch.float32,
                                                                                           torch.bfloat16):
        return None
    split = _hip.split_convs_enabled()  # false inside _hip.exact_fp32_matrix(): no fp16-split conv kernel
    if isinstance(x, _hip.CatView):  # a virtual concat: a 1x1 kernel reads both parts in place, else materialise
        if act_code == 1 and res is None and stats is None and conv.kernel_size == (1, 1):
            if split and n1 and N1_NECK and _hip.conv1x1x2_ok(x, conv) and (out is None or _hip._imgs_contig(out)) and (
                    out2 is None or _hip._imgs_contig(out2)):
                prep = lambda: _cached(conv, "c1prep", (conv.weight,), lambda: _hip.conv1x1x2_prepare(conv.weight))  # noqa: E731
                return _hip.conv1x1x2_silu(x, conv.bias, prep, conv.out_channels, out=out, out2=out2, c2lo=c2lo)
            if (THIN1X1 and conv.out_channels == 64 and conv.stride == (1, 1) and conv.groups == 1
                    and conv.padding == (0, 0) and _hip.conv1x1_thin_ok(x, conv.out_channels)
                    and (out is None or out.data_ptr() % 16 == 0)):
                return _hip.conv1x1_thin(x, conv.weight.detach().reshape(conv.out_channels, -1), conv.bias.detach(),
                                         out=out, out2=out2, c2lo=c2lo)
        x = x.materialize()
    if (split and act_code == 1 and out is None and res is None and stats is None and out2 is None and CONV3X3 != "0"
            and (CONV3X3 == "all" or tower) and _hip.conv3x3_ok(x, conv)):
        prep = lambda: _cached(conv, "c3prep", (conv.weight,), lambda: _hip.conv3x3_prepare(conv.weight))  # noqa: E731
        return _hip.conv3x3_silu(x, conv.bias, prep, conv.out_channels)
    if (split and n1 and N1_NECK and act_code == 1 and res is None and stats is None and _hip.conv1x1x2_ok(x, conv)
            and (out is None or _hip._imgs_contig(out)) and (out2 is None or _hip._imgs_contig(out2))):
        prep = lambda: _cached(conv, "c1prep", (conv.weight,), lambda: _hip.conv1x1x2_prepare(conv.weight))  # noqa: E731
        return _hip.conv1x1x2_silu(x, conv.bias, prep, conv.out_channels, out=out, out2=out2, c2lo=c2lo)
    if (split and s1 and S1_NECK and act_code == 1 and stats is None and out2 is None and _hip.conv3x3_ok(x, conv)
            and x.shape[3] % 4 == 0 and (res is None or _hip._imgs_contig(res))):
        prep = lambda: _cached(conv, "c3prep", (conv.weight,), lambda: _hip.conv3x3_prepare(conv.weight))  # noqa: E731
        return _hip.conv3x3_silu(x, conv.bias, prep, conv.out_channels, out=out, res=res)
    if (split and s2 and S2_NECK and act_code == 1 and res is None and stats is None and out2 is None
            and _hip.conv3x3s2_ok(x, conv)):
        prep = lambda: _cached(conv, "c3s2prep", (conv.weight,), lambda: _hip.conv3x3s2_prepare(conv.weight))  # noqa: E731
        return _hip.conv3x3s2_silu(x, conv.bias, prep, conv.out_channels, out=out)
    if (THIN1X1 and act_code == 1 and (stats is None or (stats in ("sum", "summax") and res is None and out2 is None))
            and conv.out_channels == 64 and conv.kernel_size == (1, 1) and conv.stride == (1, 1)
            and conv.groups == 1 and conv.padding == (0, 0) and _hip.conv1x1_thin_ok(x, conv.out_channels)
            and (out is None or out.data_ptr() % 16 == 0) and (res is None or res.data_ptr() % 16 == 0)):
        return _hip.conv1x1_thin(x, conv.weight.detach().reshape(conv.out_channels, -1), conv.bias.detach(),
                                 out=out, res=res, out2=out2, c2lo=c2lo, stats=stats)
    y = F.conv2d(x, conv.weight, None, conv.stride, conv.padding, conv.dilation, conv.groups)
    if (y.shape[2] * y.shape[3]) % 4 or y.dtype != x.dtype:
        y = y + conv.bias.view(1, -1, 1, 1)
        y = F.silu(y) if act_code == 1 else y
        if res is not None:
            y = y + res
        if out2 is not None:
            out2.copy_(y[:, c2lo:])
        if out is not None:
            out.copy_(y)
            return out
        return y
    (bias,) = _f32(conv, "bias", conv.bias)
    return _hip.bias_act(y, bias, act_code, out=out, res=res, stats=stats, out2=out2, c2lo=c2lo)


def catview_route(cv, c0, c1, H, W, dtype) -> bool:
    """Whether the fused Conv ``cv`` (a C2f cv1 after a two-input Concat of c0 + c1 channels) reads the concat as a
    ``_hip.CatView`` in place: the wide 1x1 kernel (n1 convs, the split on a 128-channel stage) or the thin 1x1 kernel
    (64 outputs). The executor decides with this before the Concat's producers run (YOLOSOD_CATVIEW)."""
    conv = cv.conv
    if (dtype != torch.float32 or not cv.is_fused() or conv.bias is None or _act_code(cv.act) != 1
            or cv.emit_stats is not None or conv.kernel_size != (1, 1) or conv.stride != (1, 1) or conv.groups != 1
            or conv.padding != (0, 0) or conv.in_channels != c0 + c1):
        return False
    if cv.n1 and N1_NECK and _hip.split_convs_enabled() and c0 % 128 == 0 and c1 % 32 == 0 and (H * W) % 4 == 0 and int(
            _hip.load_library().yolosod_conv1x1x2_prep_bytes(c0 + c1, conv.out_channels)) > 0:
        return True
    return (THIN1X1 and conv.out_channels == 64 and c0 + c1 in _hip.THIN1X1_CIN and (H * W) % 64 == 0
            and c0 % 4 == 0 and c1 % 4 == 0)


class Conv(nn.Module):
    """Conv2d(no bias) + BatchNorm2d + SiLU; after ``fuse()`` the BN is folded into the conv (conv.py:37-55).

    Fused form on GPU: MIOpen conv + one HIP epilogue pass (bias + SiLU, optional shortcut / concat slice)."""

    default_act = nn.SiLU()
    # set by DetectionModel when this conv's output feeds an SE ("sum") / CBAM ("summax") / CA ("capool") directly
    emit_stats = None
    # set by Detect on its 3x3 tower convs (head.py:43-57): the fp16-split conv kernel runs them (CONV3X3)
    tower = False
    # set by DetectionModel on the neck's 3x3 / stride-2 convs: the stride-2 fp16-split kernel runs them (S2_NECK)
    s2 = False
    # set by DetectionModel on the neck's C2f Bottleneck 3x3 convs: the stride-1 fp16-split kernel runs them (S1_NECK)
    s1 = False
    # set by DetectionModel on the neck's wide 1x1 convs: the fp16-split 1x1 kernel runs them (N1_NECK)
    n1 = False

    def __init__(self, c1, c2, k=1, s=1, p=None, g=1, d=1, act=True):
        super().__init__()
        self.conv = nn.Conv2d(c1, c2, k, s, autopad(k, p, d), groups=g, dilation=d, bias=False)
        self.bn = nn.BatchNorm2d(c2)
        self.act = self.default_act if act is True else act if isinstance(act, nn.Module) else nn.Identity()

    def forward(self, x):
        return self.act(self.bn(self.conv(x)))

    def gated_ok(self, x) -> bool:
        """This (fused, SiLU) Conv can run as the stride-2 kernel with its producer's gate applied at staging."""
        return (not hasattr(self, "bn") and self.conv.bias is not None and isinstance(self.act, nn.SiLU)
                and _hip.split_convs_enabled() and _hip.conv3x3s2_ok(x, self.conv))

    def forward_gated(self, x, gate_c, gate_p, key):
        """SiLU(conv((x * gate_c) * gate_p) + b): the consumer of an SE (gate_c) / CBAM (gate_c = ca, gate_p = sa)
        whose output is never materialised (csrc/conv3x3s2.hip); ``key``: the op_timer key of the fused operator."""
        cv = self.conv
        prep = lambda: _cached(cv, "c3s2prep", (cv.weight,), lambda: _hip.conv3x3s2_prepare(cv.weight))  # noqa: E731
        return _hip.conv3x3s2_silu(x, cv.bias, prep, cv.out_channels, gate_c, gate_p, key=key)

    def forward_fuse(self, x, out=None, res=None, out2=None, c2lo=0):
        y = conv_epilogue(self.conv, _act_code(self.act), x, out, res, self.emit_stats, out2, c2lo, self.tower,
                          self.s2, self.s1, self.n1)
        if y is not None:
            return y
        if isinstance(x, _hip.CatView):
            x = x.materialize()
        y = self.act(self.conv(x))
        if res is not None:
            y = y + res
        if out2 is not None:
            out2.copy_(y[:, c2lo:])
        if out is not None:
            out.copy_(y)
            return out
        return y

    def is_fused(self):
        return not hasattr(self, "bn")


class DWConv(Conv):
    """Depth-wise Conv (conv.py:102-107)."""

    def __init__(self, c1, c2, k=1, s=1, d=1, act=True):
        super().__init__(c1, c2, k, s, g=math.gcd(c1, c2), d=d, act=act)


class Concat(nn.Module):
    def __init__(self, dimension=1):
        super().__init__()
        self.d = dimension

    def forward(self, x):
        return torch.cat(x, self.d)


class Bottleneck(nn.Module):
    def __init__(self, c1, c2, shortcut=True, g=1, k=(3, 3), e=0.5):
        super().__init__()
        c_ = int(c2 * e)
        self.cv1 = Conv(c1, c_, k[0], 1)
        self.cv2 = Conv(c_, c2, k[1], 1, g=g)
        self.add = shortcut and c1 == c2

    def forward(self, x, out=None, out2=None):
        if self.cv2.is_fused():  # shortcut fused into cv2's epilogue, output optionally into a concat slice
            return self.cv2.forward_fuse(self.cv1(x), out=out, res=x if self.add else None, out2=out2)
        y = x + self.cv2(self.cv1(x)) if self.add else self.cv2(self.cv1(x))
        if out2 is not None:
            out2.copy_(y)
        if out is not None:
            out.copy_(y)
            return out
        return y


class C2f(nn.Module):
    def __init__(self, c1, c2, n=1, shortcut=False, g=1, e=0.5):
        super().__init__()
        self.c = int(c2 * e)
        self.cv1 = Conv(c1, 2 * self.c, 1, 1)
        self.cv2 = Conv((2 + n) * self.c, c2, 1)
        self.m = nn.ModuleList(Bottleneck(self.c, self.c, shortcut, g, k=((3, 3), (3, 3)), e=1.0) for _ in range(n))

    def forward(self, x):
        if isinstance(x, _hip.CatView) and not (x.device.type == "cuda" and self.cv1.is_fused()):
            x = x.materialize()
        if x.device.type == "cuda" and self.cv1.is_fused():
            # every branch writes its channel slice of one buffer: no torch.cat copy (block.py:249-253 semantics)
            B, _, H, W = x.shape
            n, c = len(self.m), self.c
            # each Bottleneck's input also lands packed in `t` (dual-store epilogue): MIOpen reads packed tensors,
            # so a channel slice of z would cost a copy pass per Bottleneck
            z = torch.empty((B, (2 + n) * c, H, W), dtype=x.dtype, device=x.device)
            if (n and S1_NECK and C2F_SLICES and _hip.split_convs_enabled() and x.dtype == torch.float32 and W % 4 == 0
                    and all(m.cv1.s1 and m.cv2.s1 and m.cv1.conv.kernel_size == (3, 3) for m in self.m)):
                # the Bottlenecks run on the stride-1 fp16-split kernel, which reads channel slices: each one reads
                # its input in place from z (no packed second store)
                self.cv1.forward_fuse(x, out=z[:, : 2 * c])
                for i, m in enumerate(self.m):
                    m(z[:, (1 + i) * c:(2 + i) * c], out=z[:, (2 + i) * c:(3 + i) * c])
                return self.cv2(z)
            t = torch.empty((B, c, H, W), dtype=x.dtype, device=x.device) if n else None
            self.cv1.forward_fuse(x, out=z[:, : 2 * c], out2=t, c2lo=c)
            for i, m in enumerate(self.m):
                nxt = torch.empty_like(t) if i + 1 < n else None
                m(t, out=z[:, (2 + i) * c:(3 + i) * c], out2=nxt)
                t = nxt
            return self.cv2(z)
        y = list(self.cv1(x).chunk(2, 1))
        y.extend(m(y[-1]) for m in self.m)
        return self.cv2(torch.cat(y, 1))


class SPPF(nn.Module):
    def __init__(self, c1, c2, k=5):
        super().__init__()
        c_ = c1 // 2
        self.cv1 = Conv(c1, c_, 1, 1)
        self.cv2 = Conv(c_ * 4, c2, 1, 1)
        self.m = nn.MaxPool2d(kernel_size=k, stride=1, padding=k // 2)

    def forward(self, x):
        mp = self.m
        if (SPPF_HIP and x.device.type == "cuda" and x.dtype == torch.float32 and self.cv1.is_fused()
                and mp.kernel_size == 5 and mp.stride in (1, (1, 1)) and mp.padding == 2 and mp.dilation == 1
                and not mp.ceil_mode and x.shape[2] * x.shape[3] <= 4096):
            # cv1 writes channels [0, c) of the concat buffer, one HIP pass writes the three pools (csrc/sppf.hip)
            B, _, H, W = x.shape
            c = self.cv1.conv.out_channels
            z = torch.empty((B, 4 * c, H, W), dtype=x.dtype, device=x.device)
            self.cv1.forward_fuse(x, out=z[:, :c])
            _hip.sppf_pool(z, c)
            return self.cv2(z)
        y = [self.cv1(x)]
        y.extend(self.m(y[-1]) for _ in range(3))
        return self.cv2(torch.cat(y, 1))


class DFL(nn.Module):
    """Distribution Focal Loss integral (block.py:64-83): fixed 1x1 conv with weights 0..c1-1.

    Kept for the state_dict (``dfl.conv.weight``); the decode itself runs in ``yolosod_detect_decode``."""

    def __init__(self, c1=16):
        super().__init__()
        self.conv = nn.Conv2d(c1, 1, 1, bias=False).requires_grad_(False)
        x = torch.arange(c1, dtype=torch.float)
        self.conv.weight.data[:] = nn.Parameter(x.view(1, c1, 1, 1))
        self.c1 = c1


def fold_conv_bn(conv: nn.Conv2d, bn: nn.BatchNorm2d):
    """(weight, bias) of conv followed by eval-mode BN, with the reference's arithmetic (torch_utils.py:238-265)."""
    w_conv = conv.weight.view(conv.out_channels, -1)
    w_bn = torch.diag(bn.weight.div(torch.sqrt(bn.eps + bn.running_var)))
    w = torch.mm(w_bn, w_conv).view(conv.weight.shape)
    b_conv = torch.zeros(conv.weight.shape[0], device=conv.weight.device) if conv.bias is None else conv.bias
    b_bn = bn.bias - bn.weight.mul(bn.running_mean).div(torch.sqrt(bn.running_var + bn.eps))
    b = torch.mm(w_bn, b_conv.reshape(-1, 1)).reshape(-1) + b_bn
    return w, b


def conv_weight_bias(m: Conv):
    """Folded (weight [c2, c1*k*k], bias [c2]) of a Conv whether or not ``fuse()`` has run."""
    if hasattr(m, "bn"):
        w, b = fold_conv_bn(m.conv, m.bn)
    else:
        w, b = m.conv.weight, m.conv.bias
    return w.detach().reshape(w.shape[0], -1).contiguous(), b.detach().contiguous()


# ---------------------------------------------------------------------------------------------------------------
# MAFN operators (HIP)
# ---------------------------------------------------------------------------------------------------------------
class SE(nn.Module):
    """Squeeze-Excitation with lazily created fc1/fc2 (smallobj_modules.py:57-92).

    The YAML argument is the *reduction*: hidden = max(C // reduction, 4). fc1/fc2 are created on first use for
    the observed channel count; ``DetectionModel`` materialises them right after graph construction in layer order,
    which reproduces the reference's RNG order (they are built during its stride probe)."""

    def __init__(self, reduction: int = 16) -> None:
        super().__init__()
        self.reduction = reduction
        self.fc1: nn.Conv2d | None = None
        self.fc2: nn.Conv2d | None = None
        self.in_channels: int | None = None

    def _maybe_build(self, c: int, device):
        hidden = max(c // self.reduction, 4)
        if (self.fc1 is None) or (self.in_channels != c):
            self.fc1 = nn.Conv2d(c, hidden, 1, bias=True)
            self.fc2 = nn.Conv2d(hidden, c, 1, bias=True)
            self.in_channels = c
        if device is not None and torch.device(device).type != "meta":
            self.fc1.to(device=device)
            self.fc2.to(device=device)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        b, c, h, w = x.shape
        if _is_meta(x):
            if self.fc1 is None or self.in_channels != c:
                raise RuntimeError("SE: lazy weights must be materialised before a meta shape probe")
            return torch.empty_like(x)
        self._maybe_build(c, x.device)
        return _hip.se_forward(x, *_f32(self, "fc", self.fc1.weight, self.fc1.bias, self.fc2.weight, self.fc2.bias))

    def gate(self, x: torch.Tensor) -> torch.Tensor:
        """The gate a [B, C] only (smallobj_modules.py:87-90), for a consumer that applies x * a itself (the
        executor's gate fusion: Conv.forward_gated)."""
        self._maybe_build(x.shape[1], x.device)
        return _hip.se_gate(x, *_f32(self, "fc", self.fc1.weight, self.fc1.bias, self.fc2.weight, self.fc2.bias))


SE_Block = SE


class ChannelAttention(nn.Module):
    """CBAM channel branch parameters (cbam_block.py:8-23)."""

    def __init__(self, in_planes, ratio=16):
        super().__init__()
        self.avg_pool = nn.AdaptiveAvgPool2d(1)
        self.max_pool = nn.AdaptiveMaxPool2d(1)
        self.fc = nn.Sequential(nn.Conv2d(in_planes, in_planes // ratio, 1, bias=False), nn.ReLU(),
                                nn.Conv2d(in_planes // ratio, in_planes, 1, bias=False))
        self.sigmoid = nn.Sigmoid()


class SpatialAttention(nn.Module):
    """CBAM spatial branch parameters (cbam_block.py:25-37)."""

    def __init__(self, kernel_size=7):
        super().__init__()
        self.conv1 = nn.Conv2d(2, 1, kernel_size, padding=kernel_size // 2, bias=False)
        self.sigmoid = nn.Sigmoid()


class CBAM_Block(nn.Module):
    """CBAM (cbam_block.py:39-55): y = (x * ca) * sa."""

    def __init__(self, c1, c2=None, reduction=16):
        super().__init__()
        self.channel_attention = ChannelAttention(c1, reduction)
        self.spatial_attention = SpatialAttention()

    def forward(self, x):
        if _is_meta(x):
            return torch.empty_like(x)
        fc = self.channel_attention.fc
        if self.spatial_attention.conv1.kernel_size != (7, 7):
            raise RuntimeError("CBAM_Block: only the 7x7 spatial kernel is implemented")
        return _hip.cbam_forward(x, *_f32(self, "p", fc[0].weight, fc[2].weight,
                                          self.spatial_attention.conv1.weight))

    def gates(self, x):
        """(ca [B, C], sa [B, H, W]) only (cbam_block.py:14-23,33-37), for a consumer that applies (x * ca) * sa
        itself (Conv.forward_gated)."""
        fc = self.channel_attention.fc
        if self.spatial_attention.conv1.kernel_size != (7, 7):
            raise RuntimeError("CBAM_Block: only the 7x7 spatial kernel is implemented")
        return _hip.cbam_gates(x, *_f32(self, "p", fc[0].weight, fc[2].weight, self.spatial_attention.conv1.weight))


class h_sigmoid(nn.Module):
    def __init__(self, inplace=True):
        super().__init__()
        self.relu = nn.ReLU6(inplace=inplace)

    def forward(self, x):
        return self.relu(x + 3) / 6


class CA_Block(nn.Module):
    """Coordinate attention (ca_block.py:16-59): y = (x * a_w) * a_h."""

    def __init__(self, c1, c2=None, reduction=32):
        super().__init__()
        self.pool_h = nn.AdaptiveAvgPool2d((None, 1))
        self.pool_w = nn.AdaptiveAvgPool2d((1, None))
        mip = max(8, c1 // reduction)
        self.conv1 = nn.Conv2d(c1, mip, kernel_size=1, stride=1, padding=0)
        self.bn1 = nn.BatchNorm2d(mip)
        self.act = h_sigmoid()
        self.conv_h = nn.Conv2d(mip, c1, kernel_size=1, stride=1, padding=0)
        self.conv_w = nn.Conv2d(mip, c1, kernel_size=1, stride=1, padding=0)

    def forward(self, x):
        if _is_meta(x):
            return torch.empty_like(x)
        if self.training:
            raise RuntimeError("CA_Block: HIP path is inference-only (eval-mode BatchNorm)")
        p = _f32(self, "p", self.conv1.weight, self.conv1.bias, self.bn1.weight, self.bn1.bias,
                 self.bn1.running_mean, self.bn1.running_var, self.conv_h.weight, self.conv_h.bias,
                 self.conv_w.weight, self.conv_w.bias)
        return _hip.ca_forward(x, *p[:6], self.bn1.eps, *p[6:])


class A2_Attn(nn.Module):
    """Area attention (a2_attn.py:9-69): proj -> pool to areas -> LN -> MHA -> bilinear up -> out_proj -> +x."""

    def __init__(self, c1, c2=None, num_areas=4, num_heads=4):
        super().__init__()
        if c2 is None:
            c2 = c1
        self.num_areas = num_areas
        self.num_heads = num_heads
        assert c1 % num_heads == 0, f"Input channels {c1} must be divisible by num_heads {num_heads}"
        self.proj = Conv(c1, c1, 1)
        self.attention = nn.MultiheadAttention(embed_dim=c1, num_heads=num_heads, batch_first=True)
        self.out_proj = Conv(c1, c2, 1)
        self.layer_norm = nn.LayerNorm(c1)

    def forward(self, x):
        if _is_meta(x):
            return torch.empty((x.shape[0], self.out_proj.conv.out_channels, *x.shape[2:]), device="meta")
        if self.training:
            raise RuntimeError("A2_Attn: HIP path is inference-only")
        if self.out_proj.conv.out_channels != x.shape[1]:
            raise RuntimeError("A2_Attn: HIP path implements the residual (c2 == c1) form only")
        pw, pb = conv_weight_bias(self.proj)
        at = self.attention
        fw, fb = self._fused_out()
        dt = x.dtype
        pw, at_w, fw = _as(self, "w", dt, pw, at.in_proj_weight, fw)
        pb, lw, lb, at_b, fb = _f32(self, "b", pb, self.layer_norm.weight, self.layer_norm.bias, at.in_proj_bias, fb)
        pr = self.proj
        srcs = (self.layer_norm.weight, self.layer_norm.bias, at.in_proj_weight, at.in_proj_bias, pr.conv.weight)
        srcs += ((pr.bn.weight, pr.bn.bias, pr.bn.running_mean, pr.bn.running_var) if hasattr(pr, "bn")
                 else (pr.conv.bias,))
        # the fused kernels' weight split (proj conv; in_proj with the LN affine folded), once per parameter version
        prep = lambda: _cached(self, "a2prep", srcs, lambda: _hip.a2_prepare(  # noqa: E731
            x, self.num_areas, self.num_heads, pw, lw, lb, at_w, at_b))
        return _hip.a2_forward(x, self.num_areas, self.num_heads, pw, pb, lw, lb, self.layer_norm.eps, at_w, at_b,
                               None, None, fw, fb, prep=prep)

    def _fused_out(self):
        """MHA out-projection (a2_attn.py:53) and the output 1x1 conv (a2_attn.py:63) are consecutive linear maps
        (the bilinear upsample between them commutes with the conv): folded once into Wf = Wconv @ Wmha,
        bf = Wconv @ bmha + bconv (float64 product, like the BN fold), cached against the parameters' versions, so
        the per-call path runs one token GEMM instead of two."""
        at, op = self.attention, self.out_proj
        src = [at.out_proj.weight, at.out_proj.bias, op.conv.weight]
        src += [op.bn.weight, op.bn.bias, op.bn.running_mean, op.bn.running_var] if hasattr(op, "bn") else [op.conv.bias]
        key = tuple((t.data_ptr(), t._version, t.device) for t in src)
        cache = getattr(self, "_fused_cache", None)
        if cache is None or cache[0] != key:
            ow, ob = conv_weight_bias(op)
            mw, mb = at.out_proj.weight.detach(), at.out_proj.bias.detach()
            fw = (ow.double() @ mw.double()).to(ow.dtype).contiguous()
            fb = (ow.double() @ mb.double() + ob.double()).to(ow.dtype).contiguous()
            cache = (key, fw, fb)
            self._fused_cache = cache
        return cache[1], cache[2]


class WindowAttention(nn.Module):
    """Parameters of the window attention (blocks_transformer.py:81-131)."""

    def __init__(self, dim: int, num_heads: int = 4, window_size: int = 7, mlp_ratio: float = 2.0):
        super().__init__()
        self.window_size = window_size
        self.dim = dim
        self.norm1 = nn.LayerNorm(dim)
        self.attn = nn.MultiheadAttention(dim, num_heads, batch_first=True)
        self.norm2 = nn.LayerNorm(dim)
        self.mlp = nn.Sequential(nn.Linear(dim, int(dim * mlp_ratio)), nn.GELU(), nn.Linear(int(dim * mlp_ratio), dim))


class SwinBlock(nn.Module):
    """dw3x3 -> window attention (pad, LN, MHA, MLP) -> pw1x1 -> BN -> SiLU -> +x (blocks_transformer.py:133-171)."""

    def __init__(self, c: int, num_heads: int = 4, window_size: int = 7):
        super().__init__()
        self.dw = nn.Conv2d(c, c, 3, padding=1, groups=c, bias=False)
        self.window_attn = WindowAttention(c, num_heads=num_heads, window_size=window_size)
        self.pw = nn.Conv2d(c, c, 1, bias=False)
        self.bn = nn.BatchNorm2d(c)
        self.act = nn.SiLU(inplace=True)

    def forward(self, x):
        if _is_meta(x):
            return torch.empty_like(x)
        if self.training:
            raise RuntimeError("SwinBlock: HIP path is inference-only (eval-mode BatchNorm)")
        wa = self.window_attn
        at = wa.attn
        in_w, out_w, m1_w, m2_w, pw_w = _as(self, "w", x.dtype, at.in_proj_weight, at.out_proj.weight,
                                            wa.mlp[0].weight, wa.mlp[2].weight, self.pw.weight)
        (dw, n1w, n1b, in_b, out_b, n2w, n2b, m1_b, m2_b, bnw, bnb, bnm, bnv) = _f32(
            self, "p", self.dw.weight, wa.norm1.weight, wa.norm1.bias, at.in_proj_bias, at.out_proj.bias,
            wa.norm2.weight, wa.norm2.bias, wa.mlp[0].bias, wa.mlp[2].bias, self.bn.weight, self.bn.bias,
            self.bn.running_mean, self.bn.running_var)
        srcs = (wa.norm1.weight, wa.norm1.bias, at.in_proj_weight, at.in_proj_bias, at.out_proj.weight,
                wa.norm2.weight, wa.norm2.bias, wa.mlp[0].weight, wa.mlp[0].bias, wa.mlp[2].weight, self.pw.weight,
                self.bn.weight, self.bn.bias, self.bn.running_mean, self.bn.running_var)
        # the fp16-split kernels' weight split / folds, made once per parameter version (not per call)
        prep = lambda: _cached(self, "x3prep", srcs, lambda: _hip.swin_prepare(  # noqa: E731
            x, at.num_heads, n1w, n1b, in_w, in_b, out_w, n2w, n2b, m1_w, m1_b, m2_w, pw_w, bnw, bnb, bnm, bnv,
            self.bn.eps))
        return _hip.swin_forward(
            x, at.num_heads, wa.window_size, dw, n1w, n1b, wa.norm1.eps, in_w, in_b, out_w, out_b, n2w, n2b,
            wa.norm2.eps, m1_w, m1_b, m2_w, m2_b, pw_w, bnw, bnb, bnm, bnv, self.bn.eps, prep=prep)


class Conv1x1BN(nn.Sequential):
    """1x1 conv (no bias) + BatchNorm + SiLU (blocks_mamba.py:84-92); not folded by fuse(), as in the reference."""

    def __init__(self, c_in: int, c_out: int):
        super().__init__(nn.Conv2d(c_in, c_out, 1, bias=False), nn.BatchNorm2d(c_out), nn.SiLU(inplace=True))


class GLUBlock(nn.Module):
    """GLU gated conv block, MambaBlock's fallback (blocks_mamba.py:94-113):
    pw1 -> split (a, g) -> sigmoid(g) * a -> dw3x3 -> BN -> SiLU -> pw2."""

    def __init__(self, c: int, expansion: int = 2):
        super().__init__()
        hidden = c * expansion
        self.pw1 = nn.Conv2d(c, hidden * 2, 1, bias=False)
        self.dw = nn.Conv2d(hidden, hidden, 3, padding=1, groups=hidden, bias=False)
        self.bn = nn.BatchNorm2d(hidden)
        self.pw2 = nn.Conv2d(hidden, c, 1, bias=False)
        self.act = nn.SiLU(inplace=True)


class MambaBlock(nn.Module):
    """MambaBlock as the reference runs it without ``mamba_ssm`` (blocks_mamba.py:115-236): the GLU fallback.

    y = x + out_proj(up_nearest(GLU(avg_pool_r(in_proj(x))))), in_proj / out_proj = Conv1x1BN, r = seq_reduction.
    ``mamba_ssm`` is not part of this image (nor a dependency the reference vendors), so ``use_mamba`` is False as
    in the reference's own fallback; parameters are created in the reference's order (in_proj, out_proj,
    fallback). One HIP launch sequence: ``yolosod_mamba_glu_forward``."""

    def __init__(self, c: int, c_hidden: int = 256, seq_reduction: int = 2):
        super().__init__()
        self.in_proj = Conv1x1BN(c, c_hidden)
        self.out_proj = Conv1x1BN(c_hidden, c)
        self.reduction = seq_reduction
        self.use_mamba = False
        self.fallback = GLUBlock(c_hidden, expansion=2)

    def forward(self, x):
        if _is_meta(x):
            return torch.empty_like(x)
        if self.training:
            raise RuntimeError("MambaBlock: HIP path is inference-only (eval-mode BatchNorm)")
        d = lambda t: t.detach()  # noqa: E731
        ip, op, fb = self.in_proj, self.out_proj, self.fallback
        bn = lambda b: (d(b.weight), d(b.bias), d(b.running_mean), d(b.running_var), b.eps)  # noqa: E731
        return _hip.mamba_glu_forward(x, self.reduction, d(ip[0].weight), *bn(ip[1]), d(fb.pw1.weight),
                                      d(fb.dw.weight), *bn(fb.bn), d(fb.pw2.weight), d(op[0].weight), *bn(op[1]))


class Detect(nn.Module):
    """YOLO Detect head (head.py:21-172). Towers stay PyTorch; ``_inference`` (DFL decode, anchors, stride,
    class sigmoid) is one HIP kernel."""

    dynamic = False
    export = False
    format = None
    end2end = False
    max_det = 300
    shape = None
    anchors = torch.empty(0)
    strides = torch.empty(0)
    legacy = False

    def __init__(self, nc=80, ch=()):
        super().__init__()
        self.nc = nc
        self.nl = len(ch)
        self.reg_max = 16
        self.no = nc + self.reg_max * 4
        self.stride = torch.zeros(self.nl)
        c2, c3 = max((16, ch[0] // 4, self.reg_max * 4)), max(ch[0], min(self.nc, 100))
        self.cv2 = nn.ModuleList(
            nn.Sequential(Conv(x, c2, 3), Conv(c2, c2, 3), nn.Conv2d(c2, 4 * self.reg_max, 1)) for x in ch)
        self.cv3 = (
            nn.ModuleList(nn.Sequential(Conv(x, c3, 3), Conv(c3, c3, 3), nn.Conv2d(c3, self.nc, 1)) for x in ch)
            if self.legacy
            else nn.ModuleList(
                nn.Sequential(nn.Sequential(DWConv(x, x, 3), Conv(x, c3, 1)),
                              nn.Sequential(DWConv(c3, c3, 3), Conv(c3, c3, 1)), nn.Conv2d(c3, self.nc, 1))
                for x in ch))
        self.dfl = DFL(self.reg_max) if self.reg_max > 1 else nn.Identity()
        for seq in (*self.cv2, *self.cv3):
            for m in seq:
                if isinstance(m, Conv) and m.conv.kernel_size == (3, 3) and not isinstance(m, DWConv):
                    m.tower = True

    # GPU inference runs the fused head tail + decode (one HIP kernel; the [B, 64+nc, Hi, Wi] raw maps are never
    # written). The second output keeps the reference's meaning (head.py:70-74: the raw maps) as a RawMaps
    # sequence that computes them from the kept tower features on first access. keep_raw = True runs the
    # unfused reference-shaped path instead (raw maps materialised, second output a plain list).
    keep_raw = False

    def forward(self, x):
        if self._fused_ok(x):
            return self._fused_forward(x)
        for i in range(self.nl):
            x[i] = self._tower(i, x[i])
        if self.training:
            return x
        y = self._inference(x)
        return y if self.export else (y, x)

    def _fused_ok(self, x):
        if self.training or self.keep_raw or self.export or x[0].device.type != "cuda":
            return False
        b2, b3 = self.cv2[0][-1], self.cv3[0][-1]
        return (self.reg_max == 16 and 1 <= self.nc <= 16 and b2.in_channels == 64 and b3.in_channels in (64, 128)
                and b2.bias is not None and b3.bias is not None and x[0].dtype in (torch.float32, torch.bfloat16))

    def tower_features(self, i, xi):
        """Level i's box / class tower features (cv2[i][:-1], cv3[i][:-1]): the inputs of the fused head kernel."""
        return self.cv2[i][:-1](xi).contiguous(), self.cv3[i][:-1](xi).contiguous()

    def forward_towers(self, feats, wait_last=None):
        """The fused head on tower features computed elsewhere (the executor's side streams): [(fb_i, fc_i)].
        ``wait_last``: the levels before the last are decoded first, then ``wait_last()`` (the caller's stream
        waits for the last level's towers) and the last level - its towers start only when the neck's last feature
        map exists, so the other levels' decode overlaps them."""
        return self._head([f[0] for f in feats], [f[1] for f in feats], wait_last)

    def _fused_forward(self, x):
        """cv2[i][:-1] / cv3[i][:-1] towers (PyTorch-ROCm convs + HIP epilogues), then the last 1x1 convs of both
        towers fused with DFL / dist2bbox / sigmoid in one HIP kernel (head.py:70 + _inference :100-131)."""
        fb, fc = [], []
        for i in range(self.nl):
            b, c = self.tower_features(i, x[i])
            fb.append(b)
            fc.append(c)
        return self._head(fb, fc)

    def _head(self, fb, fc, wait_last=None):
        nl = self.nl
        p = _f32(self, "head", *[c[-1].weight for c in self.cv2], *[c[-1].bias for c in self.cv2],
                 *[c[-1].weight for c in self.cv3], *[c[-1].bias for c in self.cv3])
        w = lambda t: t.reshape(t.shape[0], -1)  # noqa: E731
        args = (fb, fc, [w(t) for t in p[:nl]], list(p[nl:2 * nl]), [w(t) for t in p[2 * nl:3 * nl]],
                list(p[3 * nl:]), [float(s) for s in self.stride], self.nc, self.reg_max)
        if wait_last is None or nl < 2:
            if wait_last is not None:
                wait_last()
            return _hip.detect_head(*args), RawMaps(self, fb, fc)
        A = sum(t.shape[2] * t.shape[3] for t in fb)
        y = torch.empty((fb[0].shape[0], 4 + self.nc, A), dtype=torch.float32, device=fb[0].device)
        _hip.detect_head_into(y, 0, nl - 1, *args)
        wait_last()
        _hip.detect_head_into(y, nl - 1, nl, *args)
        return y, RawMaps(self, fb, fc)

    def raw_from_features(self, i, h2, h3):
        """Level i's raw map torch.cat((cv2[i](x), cv3[i](x)), 1) (head.py:70) from its tower features: on GPU the
        two final 1x1 convs write their slices of the [B, 4*reg_max+nc, H, W] map directly (bias in the HIP
        epilogue)."""
        b2, b3 = self.cv2[i], self.cv3[i]
        B, _, H, W = h2.shape
        if h2.device.type == "cuda" and (H * W) % 4 == 0 and b2[-1].bias is not None and b3[-1].bias is not None:
            z = torch.empty((B, self.no, H, W), dtype=h2.dtype, device=h2.device)
            conv_epilogue(b2[-1], 0, h2, out=z[:, : 4 * self.reg_max])
            conv_epilogue(b3[-1], 0, h3, out=z[:, 4 * self.reg_max:])
            return z
        return torch.cat((b2[-1](h2), b3[-1](h3)), 1)

    def _tower(self, i, xi):
        """torch.cat((cv2[i](x), cv3[i](x)), 1) (head.py:70)."""
        b2, b3 = self.cv2[i], self.cv3[i]
        if xi.device.type == "cuda" and not self.training:
            return self.raw_from_features(i, b2[:-1](xi), b3[:-1](xi))
        return torch.cat((b2(xi), b3(xi)), 1)

    def _inference(self, x):
        if x[0].device.type == "meta":
            a = sum(t.shape[2] * t.shape[3] for t in x)
            return torch.empty((x[0].shape[0], 4 + self.nc, a), device="meta")
        # the decode runs in fp32 in either config (fp32 anchors / decode in the bf16 model)
        return _hip.detect_decode([t.float().contiguous() for t in x], [float(s) for s in self.stride], self.nc,
                                  self.reg_max)

    def bias_init(self):
        """Detect biases (head.py:133-144)."""
        for a, b, s in zip(self.cv2, self.cv3, self.stride):
            a[-1].bias.data[:] = 1.0
            b[-1].bias.data[: self.nc] = math.log(5 / self.nc / (640 / s) ** 2)


class RawMaps(Sequence):
    """Second output of the fused Detect forward: the reference's list of raw [B, 4*reg_max+nc, Hi, Wi] maps
    (head.py:70-74), computed from the kept tower features on first access (``raw_from_features``) - the fused
    kernel never writes them, and callers that only read ``preds[0]`` (NMS, ops.py:219-220) never pay for them.
    Indexing / iteration / ``len`` / ``list(...)`` give the reference's tensors; ``features`` holds the
    (box, class) tower features per level; ``materialize()`` returns the plain list."""

    __slots__ = ("_det", "features", "_maps")

    def __init__(self, det, fb, fc):
        self._det = det
        self.features = list(zip(fb, fc))
        self._maps = None

    def materialize(self) -> list:
        if self._maps is None:
            # features made under inference_mode are inference tensors: read outside that mode, an autograd-
            # recording conv on them would fail ("Inference tensors cannot be saved for backward"), so the maps are
            # computed under inference_mode whenever the features are inference tensors
            inf = any(t.is_inference() for pair in self.features for t in pair)
            with torch.inference_mode(inf) if inf else contextlib.nullcontext():
                self._maps = [self._det.raw_from_features(i, b, c) for i, (b, c) in enumerate(self.features)]
        return self._maps

    def __getitem__(self, i):
        return self.materialize()[i]

    def __len__(self):
        return len(self.features)

    def __iter__(self):
        return iter(self.materialize())

    def __repr__(self):
        state = "materialised" if self._maps is not None else "lazy"
        return f"RawMaps({len(self)} levels, {state})"
