"""ctypes binding of the C ABI in ``include/yolosod_hip.h`` (``lib/libyolosod_hip.so``).

PyTorch is only plumbing here: it owns device memory (caching allocator) and the current HIP stream. Every
wrapper checks device / dtype / contiguity / shapes on the host before launching (a kernel never sees a shape it
was not written for) and raises ``RuntimeError`` with the library's message on failure. There is no CPU
fallback: calling an op on a CPU tensor, or without the built library, raises.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import torch

LIB_PATH = Path(__file__).resolve().parent / "lib" / "libyolosod_hip.so"

_c_float_p = ctypes.c_void_p
_vp = ctypes.c_void_p
_i = ctypes.c_int
_l = ctypes.c_long
_f = ctypes.c_float
_d = ctypes.c_double
_sz = ctypes.c_size_t

# name -> (restype, argtypes)
SIGNATURES = {
    "yolosod_abi_version": (_i, []),
    "yolosod_last_error": (ctypes.c_char_p, []),
    "yolosod_se_workspace": (_sz, [_i, _i, _i, _i]),
    "yolosod_se_forward": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _i, _vp, _sz, _vp]),
    "yolosod_cbam_workspace": (_sz, [_i, _i, _i, _i]),
    "yolosod_cbam_forward": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _vp, _i, _vp, _vp, _sz, _vp]),
    "yolosod_ca_workspace": (_sz, [_i, _i, _i, _i]),
    "yolosod_ca_forward": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _vp, _i, _vp, _vp, _vp, _vp, _f, _vp, _vp, _vp,
                                _vp, _vp, _sz, _vp]),
    "yolosod_a2_workspace": (_sz, [_i, _i, _i, _i, _i]),
    "yolosod_a2_forward": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _f, _vp, _vp, _vp, _vp, _vp,
                                _vp, _vp, _sz, _vp]),
    "yolosod_swin_workspace": (_sz, [_i, _i, _i, _i, _i, _i]),
    "yolosod_swin_workspace_v2": (_sz, [_i, _i, _i, _i, _i, _i, _i]),
    "yolosod_swin_forward": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _i, _vp, _vp, _vp, _f, _vp, _vp, _vp, _vp, _vp, _vp,
                                  _f, _vp, _vp, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _f, _vp, _sz, _vp]),
    "yolosod_detect_decode": (_i, [_i, _vp, _vp, _vp, _vp, _i, _i, _i, _vp, _vp]),
    "yolosod_detect_head": (_i, [_i, _vp, _vp, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _vp, _vp]),
    "yolosod_nms_workspace": (_sz, [_i, _i, _i, _i]),
    "yolosod_nms_workspace_v2": (_sz, [_i, _i, _i, _i, _i]),
    "yolosod_nms": (_i, [_vp, _i, _i, _i, _f, _d, _vp, _i, _i, _i, _i, _i, _f, _i, _vp, _vp, _vp, _vp, _sz, _vp]),
    "yolosod_gemm_f32": (_i, [_vp, _l, _i, _vp, _l, _i, _i, _vp, _l, _i, _i, _i, _i, _i, _vp, _i, _i, _vp, _vp]),
    "yolosod_layernorm": (_i, [_vp, _vp, _l, _i, _vp, _vp, _f, _vp]),
    "yolosod_attention": (_i, [_vp, _vp, _l, _i, _i, _i, _vp]),
    "yolosod_bias_act": (_i, [_vp, _l, _vp, _l, _vp, _vp, _l, _i, _i, _l, _i, _vp]),
    "yolosod_upsample2x": (_i, [_vp, _vp, _l, _i, _i, _i, _i, _i, _vp]),
    "yolosod_conv1x1_thin_stats": (_i, [_vp, _l, _vp, _vp, _vp, _l, _i, _i, _i, _l, _i, _vp, _vp, _vp, _vp]),
    "yolosod_conv1x1_thin": (_i, [_vp, _l, _vp, _vp, _vp, _l, _vp, _l, _vp, _l, _i, _i, _i, _i, _l, _vp]),
    "yolosod_bias_act_dual": (_i, [_vp, _l, _vp, _l, _vp, _vp, _l, _vp, _l, _i, _i, _i, _l, _i, _vp]),
    "yolosod_bias_act_capool": (_i, [_vp, ctypes.c_long, _vp, ctypes.c_long, _vp, _vp, ctypes.c_long, _i, _i, _i, _i,
                                     _i, _vp, _vp]),
    "yolosod_ca_forward_pre": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _vp, _i, _vp, _vp, _vp, _vp, _f, _vp, _vp, _vp, _vp,
                                    _vp, _vp, ctypes.c_size_t, _vp]),
    "yolosod_bias_act_stats": (_i, [_vp, _l, _vp, _l, _vp, _vp, _l, _i, _i, _l, _i, _i, _l, _vp, _vp, _vp]),
    "yolosod_plane_parts": (_i, [_l, ctypes.POINTER(ctypes.c_long)]),
    "yolosod_se_forward_pre": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _i, _vp, _vp, _sz, _vp]),
    "yolosod_cbam_forward_pre": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _vp, _i, _vp, _vp, _vp, _vp, _sz, _vp]),
    "yolosod_conv1x1": (_i, [_vp, _l, _vp, _vp, _vp, _l, _vp, _l, _i, _i, _i, _l, _i, _vp]),
    "yolosod_conv3x3_prep_bytes": (_sz, [_i]),
    "yolosod_conv3x3_prepare": (_i, [_vp, _i, _vp, _sz, _vp]),
    "yolosod_conv3x3_silu": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _vp, _sz, _vp]),
    "yolosod_conv1x1x2_prep_bytes": (_sz, [_i, _i]),
    "yolosod_conv1x1x2_prepare": (_i, [_vp, _i, _i, _vp, _sz, _vp]),
    "yolosod_conv1x1x2_silu": (_i, [_vp, _l, _vp, _l, _vp, _l, _i, _i, _i, _i, _i, _vp, _vp, _sz, _vp]),
    "yolosod_conv1x1x2_silu_cat": (_i, [_vp, _l, _vp, _l, _i, _vp, _l, _vp, _l, _i, _i, _i, _i, _i, _vp, _vp, _sz,
                                        _vp]),
    "yolosod_sppf_pool": (_i, [_vp, _l, _i, _i, _i, _i, _vp]),
    "yolosod_conv1x1_thin_cat": (_i, [_vp, _l, _vp, _l, _i, _vp, _vp, _vp, _l, _vp, _l, _i, _i, _i, _i, _l, _vp]),
    "yolosod_conv3x3_prep_bytes_ex": (_sz, [_i, _i]),
    "yolosod_conv3x3_prepare_ex": (_i, [_vp, _i, _i, _vp, _sz, _vp]),
    "yolosod_conv3x3_silu_ex": (_i, [_vp, _vp, _l, _vp, _l, _i, _i, _i, _i, _i, _vp, _vp, _sz, _vp]),
    "yolosod_conv3x3_silu_xs": (_i, [_vp, _l, _vp, _l, _vp, _l, _i, _i, _i, _i, _i, _vp, _vp, _sz, _vp]),
    "yolosod_debug_set_swin_fused": (None, [_i]),
    "yolosod_debug_set_swin_x3": (_i, [_i]),
    "yolosod_debug_set_head_x2": (_i, [_i]),
    "yolosod_debug_set_a2_x2": (_i, [_i]),
    "yolosod_debug_set_gemm_x2": (None, [_i]),
    "yolosod_debug_split_f16": (_i, [_vp, _vp, _vp, _l, _vp]),
    "yolosod_swin_prep_bytes": (_sz, [_i, _i, _i]),
    "yolosod_split_range_flag": (_i, [_i, _vp]),
    "yolosod_swin_prepare": (_i, [_i, _i, _i] + [_vp] * 15 + [_f, _vp, _sz, _vp]),
    "yolosod_swin_forward_prepared": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _i, _vp, _f, _vp, _f, _i, _vp, _vp, _sz,
                                           _vp, _sz, _vp]),
    "yolosod_swin_prepared_workspace": (_sz, [_i, _i, _i, _i, _i, _i, _i]),
    "yolosod_a2_prep_bytes": (_sz, [_i, _i, _i, _i]),
    "yolosod_a2_prepare": (_i, [_i, _vp, _vp, _vp, _vp, _vp, _vp, _sz, _vp]),
    "yolosod_a2_forward_prepared": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _f, _vp, _vp, _vp,
                                         _vp, _vp, _sz, _vp, _sz, _vp]),
    "yolosod_init": (_i, [_i]),
    "yolosod_debug_set_a2_fused": (_i, [_i]),
    "yolosod_debug_set_a2_pool_wide": (_i, [_i]),
    "yolosod_debug_set_conv3x3_abl": (_i, [_i]),
    "yolosod_debug_set_conv3x3s2_abl": (_i, [_i]),
    "yolosod_se_gate": (_i, [_vp, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _i, _vp, _vp, _vp, _sz, _vp]),
    "yolosod_cbam_gates": (_i, [_vp, _i, _i, _i, _i, _vp, _vp, _i, _vp, _vp, _vp, _vp, _vp, _vp, _sz, _vp]),
    "yolosod_conv3x3s2_prep_bytes": (_sz, [_i, _i]),
    "yolosod_conv3x3s2_prepare": (_i, [_vp, _i, _i, _vp, _sz, _vp]),
    "yolosod_conv3x3s2_silu": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _sz, _vp]),
    "yolosod_conv3x3s2_silu_out": (_i, [_vp, _vp, _l, _i, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _sz, _vp]),
    "yolosod_debug_set_swin_tokln": (_i, [_i]),
    "yolosod_debug_set_a2_pool_px": (_i, [_i]),
    "yolosod_mamba_glu_workspace": (_sz, [_i, _i, _i, _i, _i, _i]),
    "yolosod_mamba_glu_forward": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _f, _vp, _vp,
                                       _vp, _vp, _vp, _vp, _f, _vp, _vp, _vp, _vp, _vp, _vp, _f, _vp, _sz, _vp]),
    # bf16 storage (the bf16 model config): activations / GEMM weights bf16, other parameters fp32
    "yolosod_se_forward_bf16": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _i, _vp, _vp, _sz, _vp]),
    "yolosod_cbam_forward_bf16": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _vp, _i, _vp, _vp, _vp, _vp, _sz, _vp]),
    "yolosod_ca_forward_bf16": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _vp, _i, _vp, _vp, _vp, _vp, _f, _vp, _vp, _vp,
                                     _vp, _vp, _vp, _sz, _vp]),
    "yolosod_bias_act_bf16": (_i, [_vp, _l, _vp, _l, _vp, _vp, _l, _vp, _l, _i, _i, _i, _l, _i, _vp]),
    "yolosod_bias_act_stats_bf16": (_i, [_vp, _l, _vp, _l, _vp, _vp, _l, _i, _i, _l, _i, _i, _l, _vp, _vp, _vp]),
    "yolosod_bias_act_capool_bf16": (_i, [_vp, _l, _vp, _l, _vp, _vp, _l, _i, _i, _i, _i, _i, _vp, _vp]),
    "yolosod_swin_workspace_bf16": (_sz, [_i, _i, _i, _i, _i, _i, _i]),
    "yolosod_swin_forward_bf16": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _i, _vp, _vp, _vp, _f, _vp, _vp, _vp, _vp, _vp,
                                       _vp, _f, _vp, _vp, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _f, _vp, _sz, _vp]),
    "yolosod_a2_workspace_bf16": (_sz, [_i, _i, _i, _i, _i]),
    "yolosod_a2_forward_bf16": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _f, _vp, _vp, _vp, _vp,
                                     _vp, _sz, _vp]),
    "yolosod_detect_head_bf16": (_i, [_i, _vp, _vp, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _vp,
                                      _vp]),
    "yolosod_detect_head_levels": (_i, [_i, _i, _i, _vp, _vp, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i,
                                        _i, _vp, _i, _vp]),
    "yolosod_gemm_bf16": (_i, [_vp, _l, _i, _vp, _l, _i, _i, _vp, _l, _i, _i, _i, _i, _i, _vp, _i, _i, _vp, _vp]),
    "yolosod_attention_bf16": (_i, [_vp, _vp, _l, _i, _i, _i, _vp]),
}

_LIB = None


def load_library() -> ctypes.CDLL:
    """Load (once) the in-tree HIP library; raises if it has not been built."""
    global _LIB
    if _LIB is None:
        if not LIB_PATH.exists():
            raise RuntimeError(
                f"yolosod_amd: HIP library {LIB_PATH} is missing - run __graft_entry__.build() "
                "(or python yolo-sod_amd/build.py). There is no CPU fallback.")
        path = os.environ.get("YOLOSOD_LIB_AB") or str(LIB_PATH)  # diagnostic A/B builds only
        lib = ctypes.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            if path != str(LIB_PATH) and name.startswith("yolosod_debug_") and not hasattr(lib, name):
                continue  # an older A/B build may predate a test hook
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = lib
    return _LIB


OPS_LIB_PATH = LIB_PATH.parent / "yolosod_torch_ops.so"
_OPS = None


def ops():
    """torch.ops.yolosod (csrc/torch_ops.cpp over the C ABI): the op-registered form every hot-path wrapper below
    dispatches through (TORCH_CHECK errors, outputs and workspaces from the caching allocator on the current
    stream, Meta kernels for shape propagation). Raises if the extension has not been built - no fallback."""
    global _OPS
    if _OPS is None:
        load_library()  # the ops library links it (RUNPATH $ORIGIN); loaded first so both share one handle
        if not OPS_LIB_PATH.exists():
            raise RuntimeError(f"yolosod_amd: torch-op library {OPS_LIB_PATH} is missing - run "
                               "__graft_entry__.build() (or python yolo-sod_amd/build.py). There is no CPU fallback.")
        if not hasattr(torch.ops.yolosod, "se_fwd"):
            torch.ops.load_library(str(OPS_LIB_PATH))
        _OPS = torch.ops.yolosod
    return _OPS


class _OpTimer:
    """Records HIP events around every C-ABI launch sequence (on the launch stream) while active; with ``select``,
    only around the launches whose key it accepts (an event pair is a timestamped barrier on the stream: timing every
    launch of a step costs the step a few per cent)."""

    def __init__(self, select=None):
        self.records = []
        self.select = select

    def durations_ms(self):
        torch.cuda.synchronize()
        out = []
        for key, e0, e1 in self.records:
            out.append((key, e0.elapsed_time(e1)))
        return out


_TIMER: _OpTimer | None = None


class op_timer:
    """``with op_timer() as t: ...`` -> ``t.durations_ms()`` = [((op, shape, extra), ms), ...] per launch;
    ``op_timer(select)``: only the launches whose key ``select(key)`` accepts are timed."""

    def __init__(self, select=None):
        self.select = select

    def __enter__(self):
        global _TIMER
        self.t = _OpTimer(self.select)
        _TIMER = self.t
        return self.t

    def __exit__(self, *exc):
        global _TIMER
        _TIMER = None
        return False


_INIT_DEVS = set()


def _init_device(dev) -> None:
    """yolosod_init once per device: the library's device state (the split-range flag word) is allocated and zeroed
    before the first launch there, never lazily inside a stream capture."""
    idx = torch.device(dev).index
    idx = torch.cuda.current_device() if idx is None else idx
    if idx not in _INIT_DEVS:
        _check(load_library().yolosod_init(int(idx)), "init")
        _INIT_DEVS.add(idx)


def _launch(key, dev, fn, *args):
    """Run one C-ABI launch sequence with ``dev`` (the operands' device) as the current HIP device; the stream
    argument inside ``args`` is that device's current stream (``_stream(dev)``). While an :class:`op_timer` is
    active, HIP events bracket the sequence on that stream."""
    _init_device(dev)
    with torch.cuda.device(dev):
        t = _TIMER
        if t is None or (t.select is not None and not t.select(key)):
            return fn(*args)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = fn(*args)
        e1.record()
        t.records.append((key, e0, e1))
        return rc


def _check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load_library().yolosod_last_error().decode(errors="replace")
        raise RuntimeError(f"yolosod_amd.{what} failed (rc={rc}): {msg}")


def _dev(t: torch.Tensor, name: str, dtype=torch.float32) -> int:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name}: expected a tensor")
    if t.device.type != "cuda":
        raise RuntimeError(f"{name}: HIP kernel requires a GPU tensor (got device {t.device}); no CPU fallback")
    if t.dtype != dtype:
        raise RuntimeError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise RuntimeError(f"{name}: expected a contiguous tensor")
    return t.data_ptr()


def _p(t: torch.Tensor, name: str, numel: int | None = None, dtype=torch.float32) -> int:
    """Pointer of a (parameter) tensor after checking its element count (and, via ``_dev``, that it is a
    contiguous GPU tensor of ``dtype``: this only validates - callers pass prepared parameters, e.g. the modules'
    cached fp32 / bf16 copies)."""
    if numel is not None and t.numel() != numel:
        raise RuntimeError(f"{name}: expected {numel} elements, got {t.numel()}")
    return _dev(t, name, dtype)


_BF16 = torch.bfloat16


def _act_dtype(x: torch.Tensor) -> bool:
    """True for bf16 activations (the bf16 model config), False for fp32; anything else raises."""
    if x.dtype == torch.float32:
        return False
    if x.dtype == _BF16:
        return True
    raise RuntimeError(f"yolosod_amd: activations must be float32 or bfloat16, got {x.dtype}")


def _stream(dev) -> int:
    """The current stream of ``dev`` (the operands' device, not the current device: ADVICE r1)."""
    return torch.cuda.current_stream(dev).cuda_stream


def _workspace(nbytes: int, device) -> torch.Tensor:
    return torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)


def _c(t: torch.Tensor) -> torch.Tensor:
    return t.detach().float().contiguous()


# ---------------------------------------------------------------------------------------------------------------
# operator wrappers (parameters are passed as tensors already on the input's device)
# ---------------------------------------------------------------------------------------------------------------
class PlaneStats:
    """Per-plane partial sums (+ maxes) of a tensor, emitted by its producer's epilogue (bias_act(stats=...)) in
    the segmentation yolosod_plane_parts gives for its H*W; SE / CBAM consume them instead of re-reading it."""

    __slots__ = ("psum", "pmax", "parts", "shape")

    def __init__(self, psum, pmax, parts, shape):
        self.psum, self.pmax, self.parts, self.shape = psum, pmax, parts, tuple(shape)


_PARTS = {}


def plane_parts(HW: int):
    """(parts, seg) of the channel-attention statistics plan for planes of HW floats."""
    if HW not in _PARTS:
        seg = ctypes.c_long(0)
        parts = load_library().yolosod_plane_parts(int(HW), ctypes.byref(seg))
        _PARTS[HW] = (int(parts), int(seg.value))
    return _PARTS[HW]


def _pre_stats(x, need_max):
    st = getattr(x, "_ys_plane_stats", None)
    if st is None or st.shape != tuple(x.shape) or (need_max and st.pmax is None):
        return None
    return st


def _t(t, name):
    """A GPU tensor argument (device / dtype / shape checks are the op's TORCH_CHECKs)."""
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name}: expected a tensor")
    if t.device.type != "cuda":
        raise RuntimeError(f"{name}: HIP kernel requires a GPU tensor (got device {t.device}); no CPU fallback")
    return t


def se_forward(x, fc1_w, fc1_b, fc2_w, fc2_b):
    """SE on fp32 or bf16 activations (parameters fp32) -> torch.ops.yolosod.se_fwd."""
    bf = _act_dtype(_t(x, "x"))
    hid = fc1_w.shape[0]
    pre = _pre_stats(x, False)  # plane sums that came with x from its producer's epilogue
    return _launch(("se", tuple(x.shape), hid) + ((2,) if bf else ()), x.device, ops().se_fwd, x, fc1_w, fc1_b,
                   fc2_w, fc2_b, None if pre is None else pre.psum)


def cbam_forward(x, fc0_w, fc2_w, sa_w):
    """CBAM on fp32 or bf16 activations (parameters fp32) -> torch.ops.yolosod.cbam_fwd."""
    bf = _act_dtype(_t(x, "x"))
    hid = fc0_w.shape[0]
    pre = _pre_stats(x, True)
    return _launch(("cbam", tuple(x.shape), hid) + ((2,) if bf else ()), x.device, ops().cbam_fwd, x, fc0_w, fc2_w,
                   sa_w, None if pre is None else pre.psum, None if pre is None else pre.pmax)


def se_gate(x, fc1_w, fc1_b, fc2_w, fc2_b):
    """The SE gate only (yolosod_se_gate): [B, C] fp32, for a consumer that applies x * gate itself (the fused
    stride-2 conv, conv3x3s2_silu). fp32 activations; x's producer statistics are used when they came with it."""
    lib = load_library()
    B, C, H, W = x.shape
    hid = int(fc1_w.shape[0])
    pre = _pre_stats(x, False)
    gate = torch.empty((B, C), dtype=torch.float32, device=x.device)
    ws = torch.empty(int(lib.yolosod_se_workspace(B, C, H, W)), dtype=torch.uint8, device=x.device)
    _check(_launch(("se_gate", tuple(x.shape), hid), x.device, lib.yolosod_se_gate, _dev(x, "x"), B, C, H, W,
                   _dev(fc1_w, "fc1_w"), _dev(fc1_b, "fc1_b"), _dev(fc2_w, "fc2_w"), _dev(fc2_b, "fc2_b"), hid,
                   None if pre is None else _dev(pre.psum, "psum"), gate.data_ptr(), ws.data_ptr(), ws.numel(),
                   _stream(x.device)), "se_gate")
    return gate


def cbam_gates(x, fc0_w, fc2_w, sa_w):
    """The CBAM gates only (yolosod_cbam_gates): (ca [B, C], sa [B, H, W]) fp32, for a consumer that applies
    (x * ca) * sa itself (conv3x3s2_silu). fp32 activations; x's producer statistics are used when they came with it."""
    lib = load_library()
    B, C, H, W = x.shape
    hid = int(fc0_w.shape[0])
    pre = _pre_stats(x, True)
    ca = torch.empty((B, C), dtype=torch.float32, device=x.device)
    sa = torch.empty((B, H, W), dtype=torch.float32, device=x.device)
    ws = torch.empty(int(lib.yolosod_cbam_workspace(B, C, H, W)), dtype=torch.uint8, device=x.device)
    _check(_launch(("cbam_gate", tuple(x.shape), hid), x.device, lib.yolosod_cbam_gates, _dev(x, "x"), B, C, H, W,
                   _dev(fc0_w, "fc0_w"), _dev(fc2_w, "fc2_w"), hid, _dev(sa_w, "sa_w"),
                   None if pre is None else _dev(pre.psum, "psum"), None if pre is None else _dev(pre.pmax, "pmax"),
                   ca.data_ptr(), sa.data_ptr(), ws.data_ptr(), ws.numel(), _stream(x.device)), "cbam_gates")
    return ca, sa


def ca_forward(x, conv1_w, conv1_b, bn_w, bn_b, bn_mean, bn_var, bn_eps, convh_w, convh_b, convw_w, convw_b):
    """CA on fp32 or bf16 activations (parameters fp32) -> torch.ops.yolosod.ca_fwd."""
    bf = _act_dtype(_t(x, "x"))
    mip = conv1_w.shape[0]
    pre = getattr(x, "_ys_ca_pool", None)  # row / column means that came with x from its producer
    yin = pre[0] if pre is not None and pre[1] == tuple(x.shape) else None
    return _launch(("ca", tuple(x.shape), mip) + ((2,) if bf else ()), x.device, ops().ca_fwd, x, conv1_w, conv1_b,
                   bn_w, bn_b, bn_mean, bn_var, float(bn_eps), convh_w, convh_b, convw_w, convw_b, yin)


def a2_prep_bytes(C, num_heads, num_areas, W) -> int:
    """Size of the fused LN / QKV / attention kernel's prepared block (0: the shape does not take that kernel)."""
    return int(load_library().yolosod_a2_prep_bytes(int(C), int(num_heads), int(num_areas), int(W)))


def a2_prepare(x, num_areas, num_heads, proj_w, ln_w, ln_b, in_w, in_b):
    """The prepared block (proj and in_proj fp16 planes, uint8 tensor on x's device) for a2_forward(..., prep=...)."""
    return ops().a2_prep(x, int(num_areas), int(num_heads), proj_w, ln_w, ln_b, in_w, in_b)


def a2_forward(x, num_areas, num_heads, proj_w, proj_b, ln_w, ln_b, ln_eps, in_w, in_b, mo_w, mo_b, op_w, op_b,
               prep=None):
    """A2_Attn -> torch.ops.yolosod.a2_fwd. mo_w = mo_b = None: op_w / op_b are the pre-multiplied MHA-out x
    output-conv weights (A2_Attn._fused_out). bf16 activations: proj_w / in_w / op_w bf16 (pre-multiplied form
    only), biases and LN fp32. ``prep``: a callable returning the cached prepared block (a2_prepare) - used when the
    shape takes the fused LN / QKV / attention kernel (fp32)."""
    bf = _act_dtype(_t(x, "x"))
    B, C, H, W = x.shape
    if num_areas * W > 320:
        raise RuntimeError(f"A2_Attn: sequence length {num_areas * W} > 320 unsupported")
    if bf and (C // num_heads not in (32, 64, 128) or C % 64):
        raise RuntimeError(f"A2_Attn (bf16): C={C} with head dim {C // num_heads} unsupported")
    use_prep = prep is not None and not bf and mo_w is None and a2_prep_bytes(C, num_heads, num_areas, W) > 0

    def run():
        # the preparation (a launch on first use of a parameter version) runs inside _launch: after the device's
        # yolosod_init, under its device guard, and timed as part of this operator
        return ops().a2_fwd(x, int(num_areas), int(num_heads), proj_w, proj_b, ln_w, ln_b, float(ln_eps), in_w, in_b,
                            mo_w, mo_b, op_w, op_b, prep() if use_prep else None)

    return _launch(("a2", tuple(x.shape), (num_areas, num_heads)) + ((2,) if bf else ()), x.device, run)


def swin_forward(x, num_heads, window, dw_w, ln1_w, ln1_b, ln1_eps, in_w, in_b, out_w, out_b, ln2_w, ln2_b,
                 ln2_eps, m1_w, m1_b, m2_w, m2_b, pw_w, bn_w, bn_b, bn_mean, bn_var, bn_eps, prep=None):
    """SwinBlock -> torch.ops.yolosod.swin_fwd on fp32 or bf16 activations. bf16: the projection / MLP / pw weights
    (in_w, out_w, m1_w, m2_w, pw_w) are bf16, every other parameter fp32. ``prep``: a callable returning the cached
    prepared-parameter block (swin_prepare) - used when the shape takes the fp16-split kernels
    (torch.ops.yolosod.swin_fwd_prepared: the weight split is not redone per call)."""
    bf = _act_dtype(_t(x, "x"))
    B, C, H, W = x.shape
    hid = m1_w.shape[0]
    wh = H if (H <= window and W <= window) else min(window, H)
    ww = W if (H <= window and W <= window) else min(window, W)
    if wh * ww > 320:
        raise RuntimeError(f"SwinBlock: window of {wh}x{ww} tokens unsupported")
    if C % num_heads or (C // num_heads) not in ((32, 64, 128) if bf else (8, 16, 32, 64, 128)):
        raise RuntimeError(f"SwinBlock: head dim {C}/{num_heads} unsupported")
    key = ("swin", tuple(x.shape), (num_heads, window, hid)) + ((2,) if bf else ())
    if (prep is not None and not bf and wh == 7 and ww == 7 and C * H * W < (1 << 30)
            and swin_prep_bytes(C, num_heads, hid) > 0):
        # the weight split / folds were made once (``prep`` = swin_prepare of these parameters): one kernel launch;
        # prep() runs inside _launch (device initialised, timed with the operator), as in a2_forward
        return _launch(key, x.device, lambda: ops().swin_fwd_prepared(x, prep(), int(num_heads), int(window), dw_w,
                                                                      float(ln1_eps), out_b, float(ln2_eps), int(hid),
                                                                      m2_b))
    return _launch(key, x.device, ops().swin_fwd, x, int(num_heads), int(window), dw_w, ln1_w, ln1_b, float(ln1_eps),
                   in_w, in_b, out_w, out_b, ln2_w, ln2_b, float(ln2_eps), m1_w, m1_b, m2_w, m2_b, pw_w, bn_w, bn_b,
                   bn_mean, bn_var, float(bn_eps))


def split_range_flag(reset: bool = True, device=None) -> bool:
    """True if a fp16-split kernel on ``device`` (default: current) saw an operand beyond fp16's range since the last
    reset (the C-ABI's split-range guard); synchronises the device's current stream."""
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    with torch.cuda.device(dev):
        rc = load_library().yolosod_split_range_flag(int(bool(reset)), _stream(dev))
    if rc < 0:
        _check(rc, "split_range_flag")
    return rc == 1


_split_convs_off = 0  # > 0 inside exact_fp32_matrix(): the fp16-split convolution kernels are bypassed


def split_convs_enabled() -> bool:
    """Whether the executor may route convolutions to the fp16-split conv kernels (conv3x3 / conv3x3s2 / conv1x1x2:
    Detect towers, the gate-fused SE / CBAM consumers, the neck); false inside exact_fp32_matrix(), where they run on
    MIOpen (+ the exact-fp32 epilogue / thin 1x1 kernels) instead."""
    return _split_convs_off == 0


class exact_fp32_matrix:
    """``with exact_fp32_matrix(): ...`` runs the fp32 model's matrix products on the exact fp32 MFMA kernels
    (Swin swin_fused / swin_wide, Detect head LDS kernel, A2 fp32 GEMMs) instead of the fp16 two-term splits, and its
    convolutions on MIOpen instead of the fp16-split conv kernels (split_convs_enabled) - the fallback when
    split_range_flag() reports an operand outside fp16's range."""

    _SWITCHES = ("yolosod_debug_set_swin_x3", "yolosod_debug_set_head_x2", "yolosod_debug_set_a2_x2")

    def __enter__(self):
        global _split_convs_off
        lib = load_library()
        # each switch returns its previous state, restored on exit (a user's YOLOSOD_*=0 or an outer setting stays)
        self._prev = [int(getattr(lib, f)(0)) for f in self._SWITCHES]
        _split_convs_off += 1
        return self

    def __exit__(self, *exc):
        global _split_convs_off
        lib = load_library()
        for f, v in zip(self._SWITCHES, self._prev):
            getattr(lib, f)(v)
        _split_convs_off -= 1
        return False


def swin_prep_bytes(C, num_heads, hid) -> int:
    """Size of the fp16-split Swin kernels' prepared-parameter block (0: no prepared path for this shape, or the
    split kernels are switched off - yolosod_debug_set_swin_x3 / YOLOSOD_SWIN_X3=0)."""
    return int(load_library().yolosod_swin_prep_bytes(int(C), int(num_heads), int(hid)))


def swin_prepare(x, num_heads, ln1_w, ln1_b, in_w, in_b, out_w, ln2_w, ln2_b, m1_w, m1_b, m2_w, pw_w, bn_w, bn_b,
                 bn_mean, bn_var, bn_eps):
    """The prepared-parameter block (uint8 tensor on x's device) for swin_forward(..., prep=...)."""
    return ops().swin_prep(x, int(num_heads), ln1_w, ln1_b, in_w, in_b, out_w, ln2_w, ln2_b, m1_w, m1_b, m2_w, pw_w,
                           bn_w, bn_b, bn_mean, bn_var, float(bn_eps))


def mamba_glu_forward(x, reduction, in_w, in_bn_w, in_bn_b, in_bn_m, in_bn_v, in_eps, pw1_w, dw_w, bn_w, bn_b, bn_m,
                      bn_v, bn_eps, pw2_w, out_w, out_bn_w, out_bn_b, out_bn_m, out_bn_v, out_eps):
    """MambaBlock GLU fallback (blocks_mamba.py:94-113,198-236): x [B,C,H,W] -> x + out_proj(up(GLU(pool(in_proj x))))."""
    lib = load_library()
    B, C, H, W = x.shape
    ch = in_w.shape[0]
    hd = 2 * ch
    r = int(reduction)
    if r < 1 or H // r < 1 or W // r < 1:
        raise RuntimeError(f"MambaBlock: seq_reduction {r} too large for {H}x{W}")
    if C % 32 or ch % 32:
        raise RuntimeError(f"MambaBlock: channels {C} / hidden {ch} must be multiples of 32 (MFMA GEMM K tiles)")
    y = torch.empty_like(x)
    ws = _workspace(lib.yolosod_mamba_glu_workspace(B, C, H, W, ch, r), x.device)
    _check(_launch(("mamba", tuple(x.shape), (ch, r)), x.device, lib.yolosod_mamba_glu_forward,
        _dev(x, "x"), _dev(y, "y"), B, C, H, W, ch, r, _p(in_w, "in_proj.0.weight", ch * C),
        _p(in_bn_w, "in_proj.1.weight", ch), _p(in_bn_b, "in_proj.1.bias", ch), _p(in_bn_m, "in_proj.1.running_mean", ch),
        _p(in_bn_v, "in_proj.1.running_var", ch), float(in_eps), _p(pw1_w, "fallback.pw1.weight", 2 * hd * ch),
        _p(dw_w, "fallback.dw.weight", hd * 9), _p(bn_w, "fallback.bn.weight", hd), _p(bn_b, "fallback.bn.bias", hd),
        _p(bn_m, "fallback.bn.running_mean", hd), _p(bn_v, "fallback.bn.running_var", hd), float(bn_eps),
        _p(pw2_w, "fallback.pw2.weight", ch * hd), _p(out_w, "out_proj.0.weight", C * ch),
        _p(out_bn_w, "out_proj.1.weight", C), _p(out_bn_b, "out_proj.1.bias", C),
        _p(out_bn_m, "out_proj.1.running_mean", C), _p(out_bn_v, "out_proj.1.running_var", C), float(out_eps),
        ws.data_ptr(), ws.numel(), _stream(x.device)), "mamba_glu_forward")
    return y


def detect_decode(maps, strides, nc, reg_max=16):
    """maps: list of [B, 4*reg_max+nc, Hi, Wi] fp32 -> y [B, 4+nc, A] (torch.ops.yolosod.detect_decode_fwd)."""
    no = 4 * reg_max + nc
    B = maps[0].shape[0]
    for i, m in enumerate(maps):
        _t(m, f"maps[{i}]")
        if m.dim() != 4 or m.shape[0] != B or m.shape[1] != no:
            raise RuntimeError(f"detect_decode: map {i} has shape {tuple(m.shape)}, expected [B,{no},H,W]")
    A = sum(m.shape[2] * m.shape[3] for m in maps)
    return _launch(("decode", (B, A), nc), maps[0].device, ops().detect_decode_fwd, list(maps),
                   [float(s) for s in strides], int(nc), int(reg_max))


def detect_head(box_feats, cls_feats, box_w, box_b, cls_w, cls_b, strides, nc, reg_max=16):
    """Fused last 1x1 convs of both Detect towers + decode (torch.ops.yolosod.detect_head_fwd). box_feats[i]
    [B, c2, Hi, Wi], cls_feats[i] [B, c3, Hi, Wi] contiguous fp32 or bf16 (all levels alike); box_w[i] [64, c2],
    cls_w[i] [nc, c3] and biases fp32 -> y [B, 4+nc, A] fp32 (the decode stays fp32 in the bf16 config)."""
    bf = _act_dtype(_t(box_feats[0], "box_feats[0]"))
    B, c2 = box_feats[0].shape[:2]
    c3 = cls_feats[0].shape[1]
    A = sum(t.shape[2] * t.shape[3] for t in box_feats)
    return _launch(("head", (B, A), (nc, c2, c3)) + ((2,) if bf else ()), box_feats[0].device, ops().detect_head_fwd,
                   list(box_feats), list(cls_feats), list(box_w), list(box_b), list(cls_w), list(cls_b),
                   [float(s) for s in strides], int(nc), int(reg_max))


def detect_head_into(y, l0, l1, box_feats, cls_feats, box_w, box_b, cls_w, cls_b, strides, nc, reg_max=16):
    """``detect_head`` for levels [l0, l1) only, into y [B, 4+nc, A] laid out for all levels (torch.ops.yolosod.
    detect_head_into): the executor decodes the levels whose towers are done while the last level's still run."""
    bf = _act_dtype(_t(box_feats[0], "box_feats[0]"))
    B, c2 = box_feats[0].shape[:2]
    c3 = cls_feats[0].shape[1]
    A = sum(t.shape[2] * t.shape[3] for t in box_feats[l0:l1])
    _launch(("head", (B, A), (nc, c2, c3)) + ((2,) if bf else ()), box_feats[0].device, ops().detect_head_into, y,
            int(l0), int(l1), list(box_feats), list(cls_feats), list(box_w), list(box_b), list(cls_w), list(cls_b),
            [float(s) for s in strides], int(nc), int(reg_max))
    return y


def nms(pred, conf_thres, iou_thres, classes, agnostic, multi_label, max_det, max_nms, max_wh, in_place):
    """Batched NMS on pred [B, 4+nc, A] (GPU; torch.ops.yolosod.nms_batched). Returns (out [B,max_det,6],
    counts [B] int32, index [B,max_det] int32). in_place: pred[:, :4] is rewritten to xyxy (the reference's
    non_max_suppression(in_place=True)); otherwise pred is left untouched (no copy is made)."""
    B, no, A = _t(pred, "prediction").shape
    cls = None
    if classes is not None:
        cls = torch.as_tensor(classes, dtype=torch.int32, device=pred.device).reshape(-1).contiguous()
    return _launch(("nms", (B, no - 4, A), int(multi_label)), pred.device, ops().nms_batched, pred, float(conf_thres),
                   float(iou_thres), cls, bool(agnostic), bool(multi_label), int(max_det), int(max_nms), float(max_wh),
                   bool(in_place))


def bias_act(y, bias, act, out=None, res=None, stats=None, out2=None, c2lo=0):
    """Backbone conv epilogue: out = act(y + bias[c]) (+ res). ``out`` may be a channel slice [B, C, H, W] of a
    larger contiguous concat buffer (batch stride > C*H*W); ``res`` likewise. In place when out is None.
    ``stats`` ("sum" / "summax"): also emit out's per-plane partial sums (+ maxes) for a following SE / CBAM,
    attached to the returned tensor as ``_ys_plane_stats`` (PlaneStats); "capool": the row / column means a
    following CA_Block pools, attached as ``_ys_ca_pool`` ([B, C, H + W], shape). y / out / res / out2 are fp32
    or bf16 (all alike; bias fp32); the statistics are fp32 of the stored values."""
    lib = load_library()
    bf = _act_dtype(y)
    dt = y.dtype
    B, C, H, W = y.shape
    HW = H * W
    if out is None:
        out = y
    if out2 is not None and stats is not None:  # statistics variants have no dual store: copy afterwards
        out = bias_act(y, bias, act, out=out, res=res, stats=stats)
        out2.copy_(out[:, c2lo:])
        return out

    def bstride(t, name):
        if t.device.type != "cuda" or t.dtype != dt:
            raise RuntimeError(f"bias_act: {name} must be a {dt} GPU tensor")
        if t.shape != y.shape or t.stride(3) != 1 or t.stride(2) != W or t.stride(1) != HW:
            raise RuntimeError(f"bias_act: {name} must be [B,C,H,W] with contiguous channels (got {t.stride()})")
        return t.stride(0)

    yb = bstride(y, "y")
    ob = bstride(out, "out")
    rb = bstride(res, "res") if res is not None else 0
    rp = None if res is None else res.data_ptr()
    bp = _dev(bias, "bias")
    # op_timer key: extra = variant (+ "+res" with a shortcut input); bf16 launches carry the element size 2
    tail = (2,) if bf else ()
    rs = "" if res is None else "+res"

    def key(variant):
        return ("bias_act", tuple(y.shape), (variant + rs) if variant else (rs[1:] or None)) + tail

    if out2 is not None and stats is None:  # ``out2`` = packed copy of channels [c2lo, C) (next conv's input)
        if (out2.device.type != "cuda" or out2.dtype != dt or tuple(out2.shape) != (B, C - c2lo, H, W)
                or out2.stride(3) != 1 or out2.stride(2) != W or out2.stride(1) != HW):
            raise RuntimeError(f"bias_act: out2 must be a {dt} GPU tensor [B, C - c2lo, H, W] with contiguous channels")
        if bf:
            _check(_launch(key("dual"), y.device, lib.yolosod_bias_act_bf16, y.data_ptr(), yb,
                           out.data_ptr(), ob, bp, rp, rb, out2.data_ptr(), out2.stride(0), int(c2lo), B, C, HW,
                           int(act), _stream(y.device)), "bias_act_bf16")
        else:
            _check(_launch(key("dual"), y.device, lib.yolosod_bias_act_dual, y.data_ptr(), yb,
                           out.data_ptr(), ob, bp, rp, rb, out2.data_ptr(), out2.stride(0), int(c2lo), B, C, HW,
                           int(act), _stream(y.device)), "bias_act_dual")
        return out
    if stats == "capool":  # CA_Block input: pooled row / column means of out, [B, C, H + W]
        if W % 4 or W > 1024:
            stats = None
        else:
            yin = torch.empty((B, C, H + W), dtype=torch.float32, device=y.device)
            fn = lib.yolosod_bias_act_capool_bf16 if bf else lib.yolosod_bias_act_capool
            _check(_launch(key("capool"), y.device, fn, y.data_ptr(), yb, out.data_ptr(), ob,
                           bp, rp, rb, B, C, H, W, int(act), yin.data_ptr(), _stream(y.device)), "bias_act_capool")
            out._ys_ca_pool = (yin, tuple(out.shape))
            return out
    if stats is not None:
        parts, seg = plane_parts(HW)
        psum = torch.empty(B * C * parts, dtype=torch.float32, device=y.device)
        pmax = torch.empty_like(psum) if stats == "summax" else None
        fn = lib.yolosod_bias_act_stats_bf16 if bf else lib.yolosod_bias_act_stats
        _check(_launch(key(stats), y.device, fn, y.data_ptr(), yb, out.data_ptr(), ob, bp,
                       rp, rb, B, C, HW, int(act), parts, seg, psum.data_ptr(),
                       None if pmax is None else pmax.data_ptr(), _stream(y.device)), "bias_act_stats")
        out._ys_plane_stats = PlaneStats(psum, pmax, parts, out.shape)
        return out
    if bf:
        _check(_launch(key(None), y.device, lib.yolosod_bias_act_bf16, y.data_ptr(), yb,
                       out.data_ptr(), ob, bp, rp, rb, None, 0, 0, B, C, HW, int(act), _stream(y.device)),
               "bias_act_bf16")
        return out
    _check(_launch(key(None), y.device, lib.yolosod_bias_act, y.data_ptr(), yb, out.data_ptr(),
                   ob, bp, rp, rb, B, C, HW, int(act), _stream(y.device)), "bias_act")
    return out


def upsample2x_into(x, out) -> bool:
    """Nearest 2x upsample of x [B, C, h, w] (contiguous, fp32 / bf16) into ``out`` [B, C, 2h, 2w], a channel slice
    of a Concat buffer (contiguous channels, any batch stride): the neck's ``nn.Upsample`` + ``Concat`` glue
    (tasks._predict_once_planned). Returns False, launching nothing, when the HIP kernel's shape / alignment
    conditions (w % 4 == 0, 16-byte aligned operands and strides) do not hold."""
    B, C, h, w = x.shape
    if (x.device.type != "cuda" or out.device != x.device or out.dtype != x.dtype or x.dtype not in (torch.float32, _BF16)
            or not x.is_contiguous() or tuple(out.shape) != (B, C, 2 * h, 2 * w) or out.stride(3) != 1
            or out.stride(2) != 2 * w or out.stride(1) != 4 * h * w):
        return False
    eb = x.element_size()
    if (w % 4 or x.data_ptr() % 16 or out.data_ptr() % 16 or (out.stride(0) * eb) % 16 or (4 * h * w * eb) % 16
            or B == 0):
        return False
    _check(_launch(("upsample2x", tuple(x.shape), None), x.device, load_library().yolosod_upsample2x, x.data_ptr(),
                   out.data_ptr(), out.stride(0), B, C, h, w, eb, _stream(x.device)), "upsample2x")
    return True


THIN1X1_COUT = (64, 128)
THIN1X1_CIN = (64, 96, 128, 192, 256)


def conv1x1_thin_ok(x, cout) -> bool:
    """Shapes the thin fused 1x1 conv kernel takes (yolosod_conv1x1_thin; a CatView: yolosod_conv1x1_thin_cat)."""
    if isinstance(x, CatView):  # any split; both parts fp32 on the GPU with contiguous images
        B, Cin, H, W = x.shape
        return (x.device.type == "cuda" and x.dtype == torch.float32 and cout in THIN1X1_COUT and Cin in THIN1X1_CIN
                and (H * W) % 64 == 0 and all(_imgs_contig(t) for t in x.parts))
    B, Cin, H, W = x.shape
    return (x.device.type == "cuda" and x.dtype == torch.float32 and cout in THIN1X1_COUT and Cin in THIN1X1_CIN
            and (H * W) % 64 == 0 and x.stride(3) == 1 and x.stride(2) == W and x.stride(1) == H * W
            and x.stride(0) % 4 == 0 and x.data_ptr() % 16 == 0)


def conv1x1_thin(x, w, bias, out=None, res=None, out2=None, c2lo=0, stats=None):
    """SiLU(1x1 conv(x) + bias) (+ res) for Cout 64 / 128 and Cin <= 256 in one HIP kernel (weights in registers,
    x tiles in LDS, fp32 MFMA); ``x`` / ``out`` / ``res`` may be channel slices, ``out2`` = packed channels
    [c2lo, Cout)."""
    lib = load_library()
    B, Cin, H, W = x.shape
    Cout = w.shape[0]
    HW = H * W
    if out is None:
        out = torch.empty((B, Cout, H, W), dtype=torch.float32, device=x.device)

    def bstride(t, name, C):
        if t.device.type != "cuda" or t.dtype != torch.float32:
            raise RuntimeError(f"conv1x1_thin: {name} must be a float32 GPU tensor")
        if tuple(t.shape) != (B, C, H, W) or t.stride(3) != 1 or t.stride(2) != W or t.stride(1) != HW:
            raise RuntimeError(f"conv1x1_thin: {name} must be [B,{C},H,W] with contiguous channels")
        return t.stride(0)

    if isinstance(x, CatView):  # a virtual concat: both parts read in place (no residual / statistics)
        if res is not None or stats is not None:
            raise RuntimeError("conv1x1_thin: a CatView input takes no res / stats")
        x0, x1 = x.parts
        k1 = int(x0.shape[1])
        ob = bstride(out, "out", Cout)
        o2 = bstride(out2, "out2", Cout - c2lo) if out2 is not None else 0
        _check(_launch(("conv1x1_thin", tuple(x.shape), (Cout, False, out2 is not None, "cat")), x.device,
                       lib.yolosod_conv1x1_thin_cat, x0.data_ptr(), bstride(x0, "x", k1), x1.data_ptr(),
                       bstride(x1, "x2", Cin - k1), k1, _dev(w.contiguous(), "weight"), _dev(bias, "bias"),
                       out.data_ptr(), ob, None if out2 is None else out2.data_ptr(), o2, int(c2lo), B, Cin, Cout, HW,
                       _stream(x.device)), "conv1x1_thin_cat")
        return out
    xb = bstride(x, "x", Cin)
    ob = bstride(out, "out", Cout)
    rb = bstride(res, "res", Cout) if res is not None else 0
    o2 = bstride(out2, "out2", Cout - c2lo) if out2 is not None else 0
    if stats in ("sum", "summax") and res is None and out2 is None:
        # the same pass also yields the following SE / CBAM gate's plane statistics (PlaneStats on the output)
        parts, _ = plane_parts(HW)
        psum = torch.empty(B * Cout * parts, dtype=torch.float32, device=x.device)
        pmax = torch.empty_like(psum) if stats == "summax" else None
        tws = torch.empty(2 * B * Cout * (HW // 64), dtype=torch.float32, device=x.device)
        _check(_launch(("conv1x1_thin", tuple(x.shape), (Cout, stats)), x.device, lib.yolosod_conv1x1_thin_stats, x.data_ptr(), xb, _dev(w.contiguous(), "weight"), _dev(bias, "bias"),
                                              out.data_ptr(), ob, B, Cin, Cout, HW, parts, psum.data_ptr(),
                                              None if pmax is None else pmax.data_ptr(), tws.data_ptr(), _stream(x.device)),
               "conv1x1_thin_stats")
        out._ys_plane_stats = PlaneStats(psum, pmax, parts, out.shape)
        return out
    if stats is not None:
        raise RuntimeError(f"conv1x1_thin: stats={stats!r} needs res=None and out2=None")
    _check(_launch(("conv1x1_thin", tuple(x.shape), (Cout, res is not None, out2 is not None)), x.device, lib.yolosod_conv1x1_thin, x.data_ptr(), xb, _dev(w.contiguous(), "weight"), _dev(bias, "bias"),
                                    out.data_ptr(), ob, None if res is None else res.data_ptr(), rb,
                                    None if out2 is None else out2.data_ptr(), o2, int(c2lo), B, Cin, Cout, HW,
                                    _stream(x.device)), "conv1x1_thin")
    return out


def conv1x1(x, w, bias, act, out=None, res=None):
    """1x1 conv (stride 1, groups 1) + bias + act (+ res) as one fused GEMM; ``x``/``out``/``res`` may be
    channel slices of concat buffers (contiguous channels, any batch stride)."""
    lib = load_library()
    B, Cin, H, W = x.shape
    Cout = w.shape[0]
    HW = H * W
    if out is None:
        out = torch.empty((B, Cout, H, W), dtype=torch.float32, device=x.device)

    def bstride(t, name, C):
        if t.device.type != "cuda" or t.dtype != torch.float32:
            raise RuntimeError(f"conv1x1: {name} must be a float32 GPU tensor")
        if tuple(t.shape) != (B, C, H, W) or t.stride(3) != 1 or t.stride(2) != W or t.stride(1) != HW:
            raise RuntimeError(f"conv1x1: {name} must be [B,{C},H,W] with contiguous channels")
        return t.stride(0)

    xb = bstride(x, "x", Cin)
    ob = bstride(out, "out", Cout)
    rb = bstride(res, "res", Cout) if res is not None else 0
    _check(_launch(("conv1x1", tuple(x.shape), Cout), x.device, lib.yolosod_conv1x1, x.data_ptr(), xb, _dev(w, "weight"), None if bias is None else _dev(bias, "bias"),
                               out.data_ptr(), ob, None if res is None else res.data_ptr(), rb, B, Cin, Cout, HW,
                               int(act), _stream(x.device)), "conv1x1")
    return out


def conv3x3_ok(x, conv) -> bool:
    """Shapes the fp16-split 3x3 conv kernel takes (yolosod_conv3x3_silu_xs): fp32 NCHW on a GPU with contiguous
    images (any batch stride: a channel slice), 3x3 / stride 1 / pad 1 / dilation 1 / groups 1, 32 or a multiple of
    64 (<= 512) outputs, Cin a multiple of 32."""
    return (x.device.type == "cuda" and x.dtype == torch.float32 and x.dim() == 4 and _imgs_contig(x)
            and conv.kernel_size == (3, 3) and conv.stride == (1, 1) and conv.padding == (1, 1)
            and conv.dilation == (1, 1) and conv.groups == 1 and x.shape[1] == conv.in_channels
            and int(load_library().yolosod_conv3x3_prep_bytes_ex(int(conv.in_channels), int(conv.out_channels))) > 0)


def conv3x3_prepare(w):
    """Prepared block (fragment-major fp16 split planes of 64 W, uint8 tensor) of a [Cout, Cin, 3, 3] fp32 weight."""
    lib = load_library()
    cout, cin = int(w.shape[0]), int(w.shape[1])
    nbytes = int(lib.yolosod_conv3x3_prep_bytes_ex(cin, cout))
    if nbytes == 0:
        raise RuntimeError(f"conv3x3: (Cin={cin}, Cout={cout}) unsupported")
    blk = torch.empty(nbytes, dtype=torch.uint8, device=w.device)
    wc = w.detach().float().contiguous()
    _check(_launch(("conv3x3_prep", (cout, cin), None), w.device, lib.yolosod_conv3x3_prepare_ex, _dev(wc, "weight"),
                   cin, cout, blk.data_ptr(), nbytes, _stream(w.device)), "conv3x3_prepare")
    return blk


def _img_view(t, shape, name):
    """t is a [B, C, H, W] fp32 view on the GPU whose images are contiguous (a channel slice of a concat buffer)."""
    B, C, H, W = shape
    if (tuple(t.shape) != tuple(shape) or t.dtype != torch.float32 or t.device.type != "cuda"
            or t.stride()[1:] != (H * W, W, 1) or t.data_ptr() % 16 or t.stride(0) % 4):
        raise RuntimeError(f"{name} {tuple(t.shape)} / {t.stride()} is not a [{B}, {C}, {H}, {W}] fp32 view with "
                           "contiguous 16-byte aligned images")


def conv3x3_silu(x, bias, prep, cout=64, out=None, res=None):
    """SiLU(conv3x3(x) + bias) (+ res) on the fp16 two-term split MFMA (csrc/conv3x3.hip); ``prep`` is a callable
    returning the cached prepared block of the weights (conv3x3_prepare); ``out``: a [B, Cout, H, W] view with
    contiguous images (a concat slice) to write; ``res``: the residual added after the activation (same shape)."""
    lib = load_library()
    B, Cin, H, W = x.shape
    if out is None:
        y = torch.empty((B, cout, H, W), dtype=torch.float32, device=x.device)
    else:
        _img_view(out, (B, cout, H, W), "conv3x3: out")
        y = out
    if res is not None:
        _img_view(res, (B, cout, H, W), "conv3x3: res")
    b = bias.detach().float().contiguous()

    def run():
        blk = prep()
        _img_view(x, (B, Cin, H, W), "conv3x3: x")
        return lib.yolosod_conv3x3_silu_xs(x.data_ptr(), x.stride(0), y.data_ptr(), y.stride(0),
                                           None if res is None else res.data_ptr(),
                                           0 if res is None else res.stride(0), B, Cin, cout, H, W, _dev(b, "bias"),
                                           blk.data_ptr(), blk.numel(), _stream(x.device))

    _check(_launch(("conv3x3", tuple(x.shape), cout if res is None else (cout, "res")), x.device, run), "conv3x3")
    return y


class CatView:
    """A two-part channel concat left unmaterialised: [B, C0 + C1, H, W] as its parts. A neck Concat whose only reader
    is the next C2f's cv1 (a 1x1 conv) hands this over, and the 1x1 kernels read both parts in place
    (yolosod_conv1x1x2_silu_cat / yolosod_conv1x1_thin_cat) instead of a materialised concat (block.py:249-253,
    conv.py:336-340: the conv of a concat = the sum of the convs of its parts over their channel ranges)."""

    def __init__(self, parts):
        a, b = parts
        if a.shape[0] != b.shape[0] or a.shape[2:] != b.shape[2:] or a.dtype != b.dtype or a.device != b.device:
            raise ValueError("CatView: parts must agree in batch, spatial size, dtype and device")
        self.parts = (a, b)
        self.shape = torch.Size((a.shape[0], a.shape[1] + b.shape[1], a.shape[2], a.shape[3]))
        self.device, self.dtype = a.device, a.dtype

    def dim(self):
        return 4

    def materialize(self):
        return torch.cat(self.parts, 1)


def sppf_pool(z, c):
    """SPPF's pooling pyramid in place (yolosod_sppf_pool): z [B, 4c, H, W] fp32 with contiguous images (any batch
    stride); channels [c, 4c) <- the one-, two- and three-fold 5x5 / stride-1 / pad-2 max pools of channels [0, c)."""
    B, C4, H, W = z.shape
    if (C4 != 4 * c or z.dtype != torch.float32 or z.device.type != "cuda"
            or z.stride()[1:] != (H * W, W, 1)):  # scalar accesses: no alignment needed
        raise RuntimeError("sppf_pool: z must be a [B, 4c, H, W] fp32 GPU tensor with contiguous images")
    lib = load_library()
    _check(_launch(("sppf_pool", (B, c, H, W), None), z.device, lib.yolosod_sppf_pool, z.data_ptr(), z.stride(0), B,
                   int(c), H, W, _stream(z.device)), "sppf_pool")
    return z


def _imgs_contig(t) -> bool:
    """[B, C, H, W] whose images are contiguous (any batch stride, e.g. a channel slice of a concat buffer)."""
    B, C, H, W = t.shape
    return t.stride()[1:] == (H * W, W, 1) and t.stride(0) % 4 == 0 and t.data_ptr() % 16 == 0


def conv1x1x2_ok(x, conv) -> bool:
    """Shapes the fp16-split 1x1 conv kernel takes (yolosod_conv1x1x2_silu): fp32 on a GPU with contiguous images,
    1x1 / stride 1 / groups 1, Cout a multiple of 128 (<= 1024), Cin a multiple of 32, H*W a multiple of 4."""
    if isinstance(x, CatView):  # both parts in place: the split on a 128-channel stage boundary
        if not (all(_imgs_contig(t) for t in x.parts) and x.parts[0].shape[1] % 128 == 0):
            return False
    elif not (x.dim() == 4 and _imgs_contig(x)):
        return False
    return (x.device.type == "cuda" and x.dtype == torch.float32
            and conv.kernel_size == (1, 1) and conv.stride == (1, 1) and conv.padding == (0, 0) and conv.groups == 1
            and x.shape[1] == conv.in_channels and (x.shape[2] * x.shape[3]) % 4 == 0
            and int(load_library().yolosod_conv1x1x2_prep_bytes(int(conv.in_channels), int(conv.out_channels))) > 0)


def conv1x1x2_prepare(w):
    """Prepared block (fragment-major fp16 split planes of 64 W, Cin padded to 128) of a [Cout, Cin(, 1, 1)] weight."""
    lib = load_library()
    cout, cin = int(w.shape[0]), int(w.shape[1])
    nbytes = int(lib.yolosod_conv1x1x2_prep_bytes(cin, cout))
    if nbytes == 0:
        raise RuntimeError(f"conv1x1x2: (Cin={cin}, Cout={cout}) unsupported")
    blk = torch.empty(nbytes, dtype=torch.uint8, device=w.device)
    wc = w.detach().float().reshape(cout, cin).contiguous()
    _check(_launch(("conv1x1x2_prep", (cout, cin), None), w.device, lib.yolosod_conv1x1x2_prepare, _dev(wc, "weight"),
                   cin, cout, blk.data_ptr(), nbytes, _stream(w.device)), "conv1x1x2_prepare")
    return blk


def conv1x1x2_silu(x, bias, prep, cout, out=None, out2=None, c2lo=0):
    """SiLU(W x + bias) for a 1x1 conv on the fp16 two-term split MFMA (csrc/conv1x1x2.hip). ``x``, ``out`` may be
    channel slices of concat buffers (contiguous images); ``out2``: channels [c2lo, Cout) stored again (packed)."""
    lib = load_library()
    B, Cin, H, W = x.shape
    if out is None:
        y = torch.empty((B, cout, H, W), dtype=torch.float32, device=x.device)
    else:
        _img_view(out, (B, cout, H, W), "conv1x1x2: out")
        y = out
    if out2 is not None:
        _img_view(out2, (B, cout - c2lo, H, W), "conv1x1x2: out2")
    b = bias.detach().float().contiguous()

    x0, x1 = x.parts if isinstance(x, CatView) else (x, None)

    def run():
        blk = prep()
        return lib.yolosod_conv1x1x2_silu_cat(x0.data_ptr(), x0.stride(0), None if x1 is None else x1.data_ptr(),
                                              0 if x1 is None else x1.stride(0), int(x0.shape[1]), y.data_ptr(),
                                              y.stride(0), None if out2 is None else out2.data_ptr(),
                                              0 if out2 is None else out2.stride(0), int(c2lo), B, Cin, cout, H * W,
                                              _dev(b, "bias"), blk.data_ptr(), blk.numel(), _stream(x.device))

    extra = (cout, out2 is not None) + (("cat",) if x1 is not None else ())
    _check(_launch(("conv1x1x2", tuple(x.shape), extra), x.device, run), "conv1x1x2")
    return y


def conv3x3s2_ok(x, conv) -> bool:
    """Shapes the stride-2 fused-gate conv kernel takes (yolosod_conv3x3s2_silu): fp32 contiguous NCHW on a GPU,
    3x3 / stride 2 / pad 1 / dilation 1 / groups 1, 64 or a multiple of 128 (<= 512) outputs, Cin a multiple of 32,
    output width % 4 == 0."""
    return (x.device.type == "cuda" and x.dtype == torch.float32 and x.is_contiguous() and x.dim() == 4
            and conv.kernel_size == (3, 3) and conv.stride == (2, 2) and conv.padding == (1, 1)
            and conv.dilation == (1, 1) and conv.groups == 1
            and (conv.out_channels == 64 or (conv.out_channels % 128 == 0 and conv.out_channels <= 512))
            and conv.in_channels % 32 == 0 and x.shape[1] == conv.in_channels and ((x.shape[3] + 1) // 2) % 4 == 0
            and x.numel() * 4 < 2 ** 32
            and int(load_library().yolosod_conv3x3s2_prep_bytes(int(conv.in_channels), int(conv.out_channels))) > 0)


def conv3x3s2_prepare(w):
    """Prepared block (fragment-major fp16 split planes of 64 W, uint8 tensor) of a [Cout, Cin, 3, 3] fp32 weight."""
    lib = load_library()
    cout, cin = int(w.shape[0]), int(w.shape[1])
    nbytes = int(lib.yolosod_conv3x3s2_prep_bytes(cin, cout))
    if nbytes == 0:
        raise RuntimeError(f"conv3x3s2: (Cin={cin}, Cout={cout}) unsupported")
    blk = torch.empty(nbytes, dtype=torch.uint8, device=w.device)
    wc = w.detach().float().contiguous()
    _check(_launch(("conv3x3s2_prep", (cout, cin), None), w.device, lib.yolosod_conv3x3s2_prepare, _dev(wc, "weight"),
                   cin, cout, blk.data_ptr(), nbytes, _stream(w.device)), "conv3x3s2_prepare")
    return blk


def conv3x3s2_silu(x, bias, prep, cout, gate_c=None, gate_p=None, key=None, out=None):
    """SiLU(conv3x3_stride2((x * gate_c) * gate_p) + bias) on the fp16 two-term split MFMA (csrc/conv3x3s2.hip):
    gate_c [B, Cin] (an SE / CBAM channel gate), gate_p [B, H, W] (CBAM's spatial gate), either may be None.
    ``prep``: a callable returning the cached prepared block (conv3x3s2_prepare); ``key``: the op_timer key (default
    ("conv3x3s2", shape, (Cout, gate_c given, gate_p given))); ``out``: a [B, Cout, Ho, Wo] fp32 view whose images are contiguous (e.g. a
    channel slice of a concat buffer) to write instead of a new tensor."""
    lib = load_library()
    B, Cin, H, W = x.shape
    Ho, Wo = (H + 1) // 2, (W + 1) // 2
    if out is None:
        y = torch.empty((B, cout, Ho, Wo), dtype=torch.float32, device=x.device)
    else:
        y = out
        if (tuple(y.shape) != (B, cout, Ho, Wo) or y.dtype != torch.float32 or y.device != x.device
                or y.stride()[1:] != (Ho * Wo, Wo, 1) or y.data_ptr() % 16 or y.stride(0) % 4):
            raise RuntimeError(f"conv3x3s2: out {tuple(y.shape)} / {y.stride()} is not a [{B}, {cout}, {Ho}, {Wo}] "
                               "fp32 view with contiguous 16-byte aligned images")
    b = bias.detach().float().contiguous()
    gc = None if gate_c is None else gate_c.float().contiguous()
    gp = None if gate_p is None else gate_p.float().contiguous()
    if gc is not None and (tuple(gc.shape) != (B, Cin) or gc.data_ptr() % 16):
        raise RuntimeError(f"conv3x3s2: channel gate {tuple(gc.shape)} (16-byte aligned [{B}, {Cin}] expected)")
    if gp is not None and gp.numel() != B * H * W:
        raise RuntimeError(f"conv3x3s2: spatial gate of {gp.numel()} values ({B * H * W} expected)")

    def run():
        blk = prep()
        return lib.yolosod_conv3x3s2_silu_out(_dev(x, "x"), y.data_ptr(), y.stride(0), B, Cin, cout, H, W,
                                              _dev(b, "bias"), None if gc is None else _dev(gc, "gate_c"),
                                              None if gp is None else _dev(gp, "gate_p"), blk.data_ptr(), blk.numel(),
                                              _stream(x.device))

    if key is None:
        key = ("conv3x3s2", tuple(x.shape), (cout, gc is not None, gp is not None))
    _check(_launch(key, x.device, run), "conv3x3s2")
    return y


def gemm_f32(A, B, b_kcontig, bias=None, bias_mode=0, act=0, res=None):
    """Test hook: A [M,K]; B [N,K] (b_kcontig) or [K,N]; returns C [M,N]."""
    lib = load_library()
    M, K = A.shape
    N = B.shape[0] if b_kcontig else B.shape[1]
    C = torch.empty((M, N), dtype=torch.float32, device=A.device)
    _check(_launch(("gemm", (M, N, K), None), A.device, lib.yolosod_gemm_f32, _dev(A, "A"), 0, K, _dev(B, "B"), 0, B.shape[1], int(b_kcontig), _dev(C, "C"), 0, N,
                                M, N, K, 1, None if bias is None else _dev(bias, "bias"), bias_mode, act,
                                None if res is None else _dev(res, "res"), _stream(A.device)), "gemm_f32")
    return C


def layernorm(x, w, b, eps):
    lib = load_library()
    rows, C = x.shape
    y = torch.empty_like(x)
    _check(_launch(("layernorm", (rows, C), None), x.device, lib.yolosod_layernorm, _dev(x, "x"), _dev(y, "y"), rows, C, _dev(w, "w"), _dev(b, "b"), float(eps),
                                 _stream(x.device)), "layernorm")
    return y


def attention(qkv, n_seq, L, C, heads):
    lib = load_library()
    out = torch.empty((n_seq * L, C), dtype=torch.float32, device=qkv.device)
    _check(_launch(("attention", (n_seq, L, C), heads), qkv.device, lib.yolosod_attention, _dev(qkv, "qkv"), _dev(out, "out"), n_seq, L, C, heads, _stream(qkv.device)), "attention")
    return out


def gemm_bf16(A, B, b_kcontig, bias=None, bias_mode=0, act=0, res=None):
    """Test hook: A [M,K] bf16; B [N,K] (b_kcontig) or [K,N] bf16; returns C [M,N] bf16 (fp32 accumulation)."""
    lib = load_library()
    M, K = A.shape
    N = B.shape[0] if b_kcontig else B.shape[1]
    C = torch.empty((M, N), dtype=_BF16, device=A.device)
    _check(_launch(("gemm_bf16", (M, N, K), None), A.device, lib.yolosod_gemm_bf16, _dev(A, "A", _BF16), 0, K,
                   _dev(B, "B", _BF16), 0, B.shape[1], int(b_kcontig), _dev(C, "C", _BF16), 0, N, M, N, K, 1,
                   None if bias is None else _dev(bias, "bias"), bias_mode, act,
                   None if res is None else _dev(res, "res", _BF16), _stream(A.device)), "gemm_bf16")
    return C


def attention_bf16(qkv, n_seq, L, C, heads):
    """Test hook: bf16 attention over n_seq contiguous sequences of L rows of qkv [n_seq*L, 3C] -> [n_seq*L, C]."""
    lib = load_library()
    out = torch.empty((n_seq * L, C), dtype=_BF16, device=qkv.device)
    _check(_launch(("attention_bf16", (n_seq, L, C), heads), qkv.device, lib.yolosod_attention_bf16,
                   _dev(qkv, "qkv", _BF16), _dev(out, "out", _BF16), n_seq, L, C, heads, _stream(qkv.device)),
           "attention_bf16")
    return out
