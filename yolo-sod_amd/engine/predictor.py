"""Inference driver for tensor batches (the reference's predictor hot loop, minus the absent ``ultralytics/data``).

Reference flow (``engine/predictor.py:116-143, 219-304`` and ``models/yolo/detect/predict.py:23-41``):
``preprocess`` (tensor input: ``.to(device).float()``, no /255, no letterbox) -> ``AutoBackend`` forward of the
fused model -> ``postprocess`` = ``non_max_suppression`` + ``scale_boxes`` (same-shape input: clip to the image).

MI355X additions:
* :meth:`DetectionPredictor.predict_padded` never syncs the host: NMS returns fixed-shape ``[B, max_det, 6]``
  rows + counts, so a batch is one stream-ordered sequence of launches (graph-capturable). ``__call__`` (which syncs
  for the per-image lists anyway) also reads the split-range guard and redoes a batch whose operands left the fp16-split
  kernels' range on the exact fp32 kernels; predict_padded callers read ``_hip.split_range_flag()`` themselves.
* Data parallel inference: one process per GPU; :func:`shard_bounds` splits images across ranks (no data-path
  collective), :func:`gather_detections` is the single exchange step - ONE all-gather of a packed int32 buffer per
  image holding the padded detections, the kept anchor indices and the count (RCCL over xGMI with backend ``nccl``;
  ``gloo`` on CPU for tests): one collective latency instead of three, ~8.4 KB per image at max_det 300.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.distributed as dist

from .. import _hip
from ..utils import ops


@dataclass
class Detections:
    """Per-image result: ``boxes`` [n, 6] = (x1, y1, x2, y2, conf, cls) clipped to the image, ``index`` anchors."""

    boxes: torch.Tensor
    index: torch.Tensor
    orig_shape: tuple


class DetectionPredictor:
    def __init__(self, model, conf=0.25, iou=0.7, max_det=300, classes=None, agnostic_nms=False,
                 multi_label=False):
        self.model = model
        self.conf, self.iou, self.max_det = conf, iou, max_det
        self.classes, self.agnostic, self.multi_label = classes, agnostic_nms, multi_label
        p = next(model.parameters())
        self.device, self.dtype = p.device, p.dtype

    def preprocess(self, im: torch.Tensor) -> torch.Tensor:
        """predictor.py:123-134 tensor branch: ``.to(device)``, ``.half()`` if the model is fp16 else ``.float()`` -
        here the model's dtype (bf16 in the bf16 config)."""
        return im.to(self.device, non_blocking=True).to(self.dtype)

    @torch.inference_mode()
    def predict_padded(self, im: torch.Tensor):
        """(out [B, max_det, 6] clipped, counts [B] int32, index [B, max_det] int32) without host sync."""
        x = self.preprocess(im)
        preds = self.model(x)
        y = preds[0] if isinstance(preds, (list, tuple)) else preds
        # in_place=False: the reference's postprocess rewrites preds[:, :4] to xyxy (ops.py:167, in_place=True) and
        # then drops preds; y is local here too, so the rewrite (17 MB at bs 32) is skipped - same detections
        out, counts, index = ops.non_max_suppression_padded(
            y, self.conf, self.iou, classes=self.classes, agnostic=self.agnostic, multi_label=self.multi_label,
            max_det=self.max_det, in_place=False)
        ops.clip_boxes(out[..., :4], x.shape[2:])  # scale_boxes with gain 1 / pad 0 (same-shape tensor input)
        return out, counts, index

    def predict_padded_guarded(self, im: torch.Tensor):
        """:meth:`predict_padded`, then the split-range guard (reads one flag word: a host sync): a batch in which an
        operand left the fp16-split kernels' range (|v| > 65504, or NaN) is redone on the exact fp32 MFMA kernels."""
        out, counts, index = self.predict_padded(im)
        if self.dtype == torch.float32 and _hip.split_range_flag(reset=True, device=self.device):
            with _hip.exact_fp32_matrix():
                out, counts, index = self.predict_padded(im)
            _hip.split_range_flag(reset=True, device=self.device)
        return out, counts, index

    def __call__(self, im: torch.Tensor):
        out, counts, index = self.predict_padded_guarded(im)
        n = counts.cpu().tolist()
        shape = tuple(im.shape[2:])
        return [Detections(out[i, : n[i]], index[i, : n[i]], shape) for i in range(len(n))]


def shard_bounds(n: int, rank: int, world: int):
    """Contiguous, balanced image shard [lo, hi) of rank ``rank``."""
    base, rem = divmod(n, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def pack_detections(out: torch.Tensor, counts: torch.Tensor, index: torch.Tensor | None = None) -> torch.Tensor:
    """One int32 row per image: the [D, 6] fp32 rows (bit patterns), then the [D] kept anchor indices (if given),
    then the count - [B, 6D (+ D) + 1], contiguous (the single buffer the exchange step all-gathers)."""
    B, D = out.shape[:2]
    parts = [out.float().reshape(B, D * 6).contiguous().view(torch.int32)]
    if index is not None:
        parts.append(index.to(torch.int32).reshape(B, D))
    parts.append(counts.to(torch.int32).reshape(B, 1))
    return torch.cat(parts, 1).contiguous()


def unpack_detections(packed: torch.Tensor, D: int, with_index: bool):
    """Inverse of :func:`pack_detections`: (out [B, D, 6] fp32, counts [B] int32[, index [B, D] int32])."""
    B = packed.shape[0]
    out = packed[:, : 6 * D].contiguous().view(torch.float32).reshape(B, D, 6)
    counts = packed[:, -1].contiguous()
    if not with_index:
        return out, counts
    return out, counts, packed[:, 6 * D: 7 * D].contiguous()


def gather_detections(out: torch.Tensor, counts: torch.Tensor, index: torch.Tensor | None = None, group=None):
    """All-gather padded detections of equal-size shards: [B_local, D, 6] + [B_local] (+ the kept anchor indices
    [B_local, D]) -> [world*B_local, ...] in rank order, as ONE collective on the packed buffer
    (:func:`pack_detections`). Returns (out, counts) or (out, counts, index)."""
    world = dist.get_world_size(group)
    packed = pack_detections(out, counts, index)
    g = torch.empty((world * packed.shape[0], packed.shape[1]), dtype=packed.dtype, device=packed.device)
    dist.all_gather_into_tensor(g, packed, group=group)
    return unpack_detections(g, out.shape[1], index is not None)


def sharded_predict(predict_padded, n_images: int, images, group=None, split_guard: bool = True):
    """Data-parallel inference over ``n_images`` global images, one process per GPU.

    ``images(lo, hi)`` returns this rank's shard (global images [lo, hi), ``shard_bounds``) - each rank
    materialises only its own images; ``predict_padded(x) -> (out [b, D, 6], counts [b], index [b, D])`` is the
    rank-local path (``DetectionPredictor.predict_padded``). Shards are padded to the largest shard (count 0,
    index -1) so one fixed-size all-gather serves uneven splits. Returns (out [n_images, D, 6], counts [n_images],
    index [n_images, D]) in global image order on every rank: the kept anchor indices of every image
    (``models/yolo/detect/predict.py:23-41`` per image) survive the exchange.

    ``split_guard``: after the rank-local step on a GPU, the split-range flag is read (a host sync) and a shard whose
    operands left the fp16-split kernels' range is redone on the exact fp32 kernels before the exchange, as
    :meth:`DetectionPredictor.__call__` does for one process."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    lo, hi = shard_bounds(n_images, rank, world)
    x = images(lo, hi)
    out, counts, index = predict_padded(x)[:3]
    model_dtype = getattr(getattr(predict_padded, "__self__", None), "dtype", torch.float32)  # bf16: no split kernels
    if split_guard and out.is_cuda and model_dtype == torch.float32 and _hip.split_range_flag(reset=True,
                                                                                              device=out.device):
        with _hip.exact_fp32_matrix():
            out, counts, index = predict_padded(x)[:3]
        _hip.split_range_flag(reset=True, device=out.device)
    smax = -(-n_images // world)
    if out.shape[0] < smax:
        pad = smax - out.shape[0]
        out = torch.cat([out, out.new_zeros((pad, *out.shape[1:]))])
        counts = torch.cat([counts, counts.new_zeros((pad,))])
        index = torch.cat([index, index.new_full((pad, *index.shape[1:]), -1)])
    g_out, g_cnt, g_idx = gather_detections(out, counts, index, group)
    if n_images % world:
        keep = torch.cat([torch.arange(r * smax, r * smax + (b - a)) for r in range(world)
                          for a, b in [shard_bounds(n_images, r, world)]])
        g_out, g_cnt, g_idx = (t[keep.to(t.device)] for t in (g_out, g_cnt, g_idx))
    return g_out, g_cnt, g_idx


def seeded_images(lo: int, hi: int, imgsz: int, seed: int = 1000, device=None) -> torch.Tensor:
    """Synthetic input batch of global images [lo, hi): image i = torch.rand(3, imgsz, imgsz) from a generator
    seeded ``seed + i``, so every rank's shard is a slice of one global batch whatever the world size."""
    x = torch.empty((hi - lo, 3, imgsz, imgsz))
    for k, i in enumerate(range(lo, hi)):
        x[k] = torch.rand(3, imgsz, imgsz, generator=torch.Generator().manual_seed(seed + i))
    return x if device is None else x.to(device)
