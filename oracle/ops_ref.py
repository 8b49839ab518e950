"""ORACLE - TEST INFRASTRUCTURE ONLY.

CPU restatement (PyTorch-CPU tensor math, any float dtype) of the reference's hot-path operators, written from the
reference's algorithm, each function citing the quitedob/yolo-sod file:line it follows. Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this package, and only as the
checker / the timed CPU baseline - never as the product path (``yolo-sod_amd/`` has no CPU compute fallback).

Pinned against the reference itself: ``tests/golden/*.npz`` were produced by importing the reference's modules in
this container (``tests/golden/make_golden.py``); ``tests/test_oracle_golden.py`` checks every function here
against them.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def _conv1x1(x, w, b=None):
    return F.conv2d(x, w.reshape(w.shape[0], -1, 1, 1).to(x.dtype), None if b is None else b.to(x.dtype))


def se_ref(x, fc1_w, fc1_b, fc2_w, fc2_b):
    """SE forward - smallobj_modules.py:84-92: x * sigmoid(fc2(relu(fc1(avgpool(x)))))."""
    m = F.adaptive_avg_pool2d(x, 1)
    a = F.relu(_conv1x1(m, fc1_w, fc1_b))
    a = torch.sigmoid(_conv1x1(a, fc2_w, fc2_b))
    return x * a


def cbam_ref(x, fc0_w, fc2_w, sa_w):
    """CBAM_Block forward - cbam_block.py:19-23 (channel), :32-37 (spatial), :52-55 ((x*ca)*sa)."""
    def fc(v):
        return _conv1x1(F.relu(_conv1x1(v, fc0_w)), fc2_w)

    ca = torch.sigmoid(fc(F.adaptive_avg_pool2d(x, 1)) + fc(F.adaptive_max_pool2d(x, 1)))
    out = ca * x
    s = torch.cat([torch.mean(out, dim=1, keepdim=True), torch.max(out, dim=1, keepdim=True)[0]], dim=1)
    sa = torch.sigmoid(F.conv2d(s, sa_w.to(x.dtype), padding=sa_w.shape[-1] // 2))
    return sa * out


def _bn_eval(y, w, b, mean, var, eps):
    return F.batch_norm(y, mean.to(y.dtype), var.to(y.dtype), w.to(y.dtype), b.to(y.dtype), False, 0.0, eps)


def ca_ref(x, conv1_w, conv1_b, bn_w, bn_b, bn_mean, bn_var, bn_eps, convh_w, convh_b, convw_w, convw_b):
    """CA_Block forward - ca_block.py:38-59 (h_sigmoid :8-14): (x * a_w) * a_h."""
    n, c, h, w = x.shape
    x_h = F.adaptive_avg_pool2d(x, (None, 1))
    x_w = F.adaptive_avg_pool2d(x, (1, None)).permute(0, 1, 3, 2)
    y = torch.cat([x_h, x_w], dim=2)
    y = _conv1x1(y, conv1_w, conv1_b)
    y = _bn_eval(y, bn_w, bn_b, bn_mean, bn_var, bn_eps)
    y = F.relu6(y + 3) / 6
    y_h, y_w = torch.split(y, [h, w], dim=2)
    y_w = y_w.permute(0, 1, 3, 2)
    a_h = torch.sigmoid(_conv1x1(y_h, convh_w, convh_b))
    a_w = torch.sigmoid(_conv1x1(y_w, convw_w, convw_b))
    return x * a_w * a_h


def mha_ref(q_in, in_w, in_b, out_w, out_b, num_heads):
    """nn.MultiheadAttention self-attention (batch_first, no mask, eval): packed in_proj [q;k;v], per-head
    softmax(q*s . k^T) v with s = 1/sqrt(head_dim), out_proj. Used by a2_attn.py:53 and blocks_transformer.py:116."""
    B, L, C = q_in.shape
    hd = C // num_heads
    qkv = q_in @ in_w.to(q_in.dtype).t() + in_b.to(q_in.dtype)
    q, k, v = qkv.split(C, dim=-1)
    q = q.reshape(B, L, num_heads, hd).transpose(1, 2) * (1.0 / math.sqrt(hd))
    k = k.reshape(B, L, num_heads, hd).transpose(1, 2)
    v = v.reshape(B, L, num_heads, hd).transpose(1, 2)
    p = torch.softmax(q @ k.transpose(-1, -2), dim=-1)
    o = (p @ v).transpose(1, 2).reshape(B, L, C)
    return o @ out_w.to(q_in.dtype).t() + out_b.to(q_in.dtype)


def a2_ref(x, num_areas, num_heads, proj_w, proj_b, ln_w, ln_b, ln_eps, in_w, in_b, mo_w, mo_b, op_w, op_b):
    """A2_Attn forward with fused Conv weights - a2_attn.py:35-69 (Conv.forward_fuse = SiLU(conv + b))."""
    b, c, h, w = x.shape
    xp = F.silu(_conv1x1(x, proj_w, proj_b))
    pooled = F.adaptive_avg_pool2d(xp, (num_areas, w))
    seq = pooled.flatten(2).transpose(1, 2)
    s = F.layer_norm(seq, (c,), ln_w.to(x.dtype), ln_b.to(x.dtype), ln_eps)
    a = mha_ref(s, in_w, in_b, mo_w, mo_b, num_heads)
    a = a.transpose(1, 2).reshape(b, c, num_areas, w)
    up = F.interpolate(a, size=(h, w), mode="bilinear", align_corners=False)
    out = F.silu(_conv1x1(up, op_w, op_b))
    return out + x


def window_partition_ref(x, ws):
    """blocks_transformer.py:8-47 (zero pad bottom/right, windows ordered (b, wy, wx), tokens (iy, ix))."""
    B, C, H, W = x.shape
    if H <= ws and W <= ws:
        return x.permute(0, 2, 3, 1).reshape(B, H * W, C), (H, W), (H, W)
    wh, ww = min(ws, H), min(ws, W)
    ph, pw = (wh - H % wh) % wh, (ww - W % ww) % ww
    if ph or pw:
        x = F.pad(x, (0, pw, 0, ph))
    Hp, Wp = H + ph, W + pw
    x = x.view(B, C, Hp // wh, wh, Wp // ww, ww).permute(0, 2, 4, 3, 5, 1).reshape(-1, wh * ww, C)
    return x, (Hp, Wp), (wh, ww)


def window_reverse_ref(windows, size, win):
    """blocks_transformer.py:49-79."""
    Hp, Wp = size
    wh, ww = win
    nwh, nww = Hp // wh, Wp // ww
    B = windows.shape[0] // (nwh * nww)
    x = windows.view(B, nwh, nww, wh, ww, -1).permute(0, 5, 1, 3, 2, 4)
    return x.reshape(B, -1, Hp, Wp)


def swin_ref(x, num_heads, window, dw_w, ln1_w, ln1_b, ln1_eps, in_w, in_b, out_w, out_b, ln2_w, ln2_b, ln2_eps,
             m1_w, m1_b, m2_w, m2_b, pw_w, bn_w, bn_b, bn_mean, bn_var, bn_eps):
    """SwinBlock forward - blocks_transformer.py:150-171 with WindowAttention.forward :100-131."""
    B, C, H, W = x.shape
    dt = x.dtype
    t = F.conv2d(x, dw_w.to(dt), padding=1, groups=C)
    win, size, wsz = window_partition_ref(t, window)
    u = F.layer_norm(win, (C,), ln1_w.to(dt), ln1_b.to(dt), ln1_eps)
    win = win + mha_ref(u, in_w, in_b, out_w, out_b, num_heads)
    u = F.layer_norm(win, (C,), ln2_w.to(dt), ln2_b.to(dt), ln2_eps)
    hmid = F.gelu(u @ m1_w.to(dt).t() + m1_b.to(dt))
    win = win + (hmid @ m2_w.to(dt).t() + m2_b.to(dt))
    y = window_reverse_ref(win, size, wsz)[:, :, :H, :W]
    y = F.conv2d(y, pw_w.to(dt))
    y = _bn_eval(y, bn_w, bn_b, bn_mean, bn_var, bn_eps)
    return x + F.silu(y)


def mamba_glu_ref(x, reduction, in_w, in_bn, pw1_w, dw_w, bn, pw2_w, out_w, out_bn):
    """MambaBlock without mamba_ssm = GLU fallback (blocks_mamba.py:198-236, GLUBlock :94-113, Conv1x1BN :84-92).
    *_bn = (weight, bias, running_mean, running_var, eps), eval-mode BatchNorm."""
    B, C, H, W = x.shape
    y = F.silu(_bn_eval(F.conv2d(x, in_w), *in_bn))                      # in_proj (:201)
    if reduction > 1:
        y = F.avg_pool2d(y, reduction, reduction)                         # (:204-205)
    hid = pw1_w.shape[0] // 2
    a, g = F.conv2d(y, pw1_w).chunk(2, dim=1)                             # GLUBlock.pw1 + split (:107)
    z = torch.sigmoid(g) * a                                              # (:108)
    z = F.conv2d(z, dw_w, padding=1, groups=hid)                          # dw (:109)
    z = F.silu(_bn_eval(z, *bn))                                          # bn, act (:110-111)
    y = F.conv2d(z, pw2_w)                                                # pw2 (:112)
    if reduction > 1:
        y = F.interpolate(y, size=(H, W), mode="nearest")                 # (:231-232)
    y = F.silu(_bn_eval(F.conv2d(y, out_w), *out_bn))                     # out_proj (:235)
    return x + y                                                          # (:236)


def make_anchors_ref(shapes, strides, dtype=torch.float32, offset=0.5):
    """utils/tal.py:333-345: anchor (ix+0.5, iy+0.5), row-major per level, levels concatenated."""
    pts, st = [], []
    for (h, w), s in zip(shapes, strides):
        sx = torch.arange(w, dtype=dtype) + offset
        sy = torch.arange(h, dtype=dtype) + offset
        sy, sx = torch.meshgrid(sy, sx, indexing="ij")
        pts.append(torch.stack((sx, sy), -1).view(-1, 2))
        st.append(torch.full((h * w, 1), float(s), dtype=dtype))
    return torch.cat(pts), torch.cat(st)


def decode_ref(maps, strides, nc, reg_max=16):
    """Detect._inference - head.py:100-131; DFL block.py:79-82; dist2bbox(xywh) tal.py:348-357."""
    b = maps[0].shape[0]
    no = nc + 4 * reg_max
    dt = maps[0].dtype
    x_cat = torch.cat([m.reshape(b, no, -1) for m in maps], 2)
    anchors, st = make_anchors_ref([m.shape[2:] for m in maps], strides, dt)
    anchors, st = anchors.transpose(0, 1), st.transpose(0, 1)
    box, cls = x_cat.split((reg_max * 4, nc), 1)
    a = box.shape[-1]
    p = box.view(b, 4, reg_max, a).transpose(2, 1).softmax(1)
    dist = (p * torch.arange(reg_max, dtype=dt).view(1, reg_max, 1, 1)).sum(1)
    lt, rb = dist.chunk(2, 1)
    x1y1 = anchors.unsqueeze(0) - lt
    x2y2 = anchors.unsqueeze(0) + rb
    dbox = torch.cat(((x1y1 + x2y2) / 2, x2y2 - x1y1), 1) * st
    return torch.cat((dbox, cls.sigmoid()), 1)
