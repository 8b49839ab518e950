"""Checkpoint ingest for the reference's ``.pt`` files, without executing anything from the file.

Reference format (``engine/trainer.py:513-536``): ``torch.save({"ema": deepcopy(model).half(), "model": None,
"train_args": vars(args), "epoch": ..., ...})`` - a pickled ``ultralytics.nn.tasks.DetectionModel`` module tree in
fp16. The reference reads it with ``torch.load(weights_only=False)`` (``nn/tasks.py:824-900`` torch_safe_load),
i.e. it imports and runs whatever globals the pickle names, then ``attempt_load_one_weight`` (``:941-975``) takes
``ckpt.get("ema") or ckpt["model"]``, ``.float()``, ``fuse()``, ``eval()``.

Here:
1. ``torch.serialization.get_unsafe_globals_in_checkpoint`` lists the globals the pickle needs *without* unpickling;
2. ``torch.nn.modules.*`` module classes are allowed as themselves (library code: unpickling a module only calls
   ``cls.__new__`` and ``Module.__setstate__``); every other global (``ultralytics.*`` classes, argument namespaces,
   ...) is replaced by an inert ``nn.Module`` stub registered under the same qualified name;
3. ``torch.load(weights_only=True)`` rebuilds the tree of stubs. Their ``state_dict()`` carries the reference's key
   names (``model.9.window_attn.attn.in_proj_weight`` ...), and ``.yaml`` the model dict it was built from;
4. :func:`attempt_load_one_weight` builds this package's ``DetectionModel`` from that dict, loads the fp32 state
   (strict), fuses and moves it to the device - the same steps as the reference.

:func:`save_checkpoint` writes the same layout (stub classes under the reference's class paths), for tests and for
moving weights between processes.
"""
from __future__ import annotations

import contextlib
import copy
import sys
import types
from datetime import datetime
from pathlib import Path

import torch
import torch.nn as nn

from . import modules as M
from .tasks import DetectionModel

__all__ = ("load_checkpoint", "checkpoint_model_state", "attempt_load_one_weight", "save_checkpoint", "REF_CLASS_PATH")

# this package's classes -> the reference's class paths (ultralytics/nn/modules/*.py, nn/tasks.py)
REF_CLASS_PATH = {
    M.Conv: "ultralytics.nn.modules.conv.Conv",
    M.DWConv: "ultralytics.nn.modules.conv.DWConv",
    M.Concat: "ultralytics.nn.modules.conv.Concat",
    M.C2f: "ultralytics.nn.modules.block.C2f",
    M.Bottleneck: "ultralytics.nn.modules.block.Bottleneck",
    M.SPPF: "ultralytics.nn.modules.block.SPPF",
    M.DFL: "ultralytics.nn.modules.block.DFL",
    M.Detect: "ultralytics.nn.modules.head.Detect",
    M.SE: "ultralytics.nn.modules.smallobj_modules.SE",
    M.CBAM_Block: "ultralytics.nn.modules.cbam_block.CBAM_Block",
    M.ChannelAttention: "ultralytics.nn.modules.cbam_block.ChannelAttention",
    M.SpatialAttention: "ultralytics.nn.modules.cbam_block.SpatialAttention",
    M.CA_Block: "ultralytics.nn.modules.ca_block.CA_Block",
    M.h_sigmoid: "ultralytics.nn.modules.ca_block.h_sigmoid",
    M.A2_Attn: "ultralytics.nn.modules.a2_attn.A2_Attn",
    M.SwinBlock: "ultralytics.nn.modules.blocks_transformer.SwinBlock",
    M.WindowAttention: "ultralytics.nn.modules.blocks_transformer.WindowAttention",
    DetectionModel: "ultralytics.nn.tasks.DetectionModel",
}


class _Stub(nn.Module):
    """Inert stand-in for a pickled class: accepts any constructor arguments, keeps the unpickled state."""

    def __init__(self, *args, **kwargs):  # noqa: D401 - REDUCE of e.g. a namespace passes arguments
        super().__init__()
        self._stub_args = args

    def __setstate__(self, state):
        if isinstance(state, dict):
            super().__setstate__(state)
        else:  # non-dict state (e.g. a tuple): keep it, never interpret it
            super().__setstate__({})
            self._stub_state = state


_STUBS: dict[str, type] = {}


def _stub_class(qualname: str) -> type:
    """One stub class per qualified name, with __module__/__qualname__ set so the unpickler maps that global to it."""
    if qualname not in _STUBS:
        mod, _, name = qualname.rpartition(".")
        _STUBS[qualname] = type(name, (_Stub,), {"__module__": mod, "__qualname__": name})
    return _STUBS[qualname]


def _torch_nn_class(qualname: str):
    """The real class for a ``torch.nn.modules.*`` module class name, else None."""
    mod, _, name = qualname.rpartition(".")
    if not mod.startswith("torch.nn.modules."):
        return None
    try:
        m = __import__(mod, fromlist=[name])
    except ImportError:
        return None
    cls = getattr(m, name, None)
    return cls if isinstance(cls, type) and issubclass(cls, nn.Module) else None


def load_checkpoint(path) -> dict:
    """Unpickle a reference checkpoint with ``weights_only=True``; foreign classes become inert stubs."""
    path = Path(path)
    if not path.exists():
        raise FileNotFoundError(path)
    needed = torch.serialization.get_unsafe_globals_in_checkpoint(str(path))
    allow = []
    for q in needed:
        cls = _torch_nn_class(q)
        allow.append(cls if cls is not None else _stub_class(q))
    with torch.serialization.safe_globals(allow):
        ckpt = torch.load(str(path), map_location="cpu", weights_only=True)
    if not isinstance(ckpt, dict):  # torch.save(model) files (tasks.py:893-898): wrap like the reference
        ckpt = {"model": getattr(ckpt, "model", ckpt)}
    return ckpt


def checkpoint_model_state(ckpt: dict):
    """(model yaml dict, fp32 state_dict, stride) of ``ckpt.get("ema") or ckpt["model"]`` (tasks.py:946)."""
    m = ckpt.get("ema") or ckpt.get("model")
    if m is None:
        raise KeyError("checkpoint has neither 'ema' nor 'model'")
    cfg = getattr(m, "yaml", None)
    if not isinstance(cfg, dict):
        raise ValueError("checkpoint model carries no yaml dict; cannot rebuild its graph")
    sd = {k: (v.float() if v.is_floating_point() else v) for k, v in m.state_dict().items()}
    stride = getattr(m, "stride", None)
    return copy.deepcopy(cfg), sd, stride


def attempt_load_one_weight(weight, device="cuda", fuse: bool = True, registry=None):
    """(model, ckpt) like nn/tasks.py:941-975: rebuild the graph from the embedded YAML, load the fp32 weights
    (strict key match), fuse Conv+BN, eval, move to ``device``."""
    ckpt = load_checkpoint(weight)
    cfg, sd, stride = checkpoint_model_state(ckpt)
    model = DetectionModel(cfg, registry=registry, probe_stats=False)
    missing, unexpected = model.load_state_dict(sd, strict=False)
    if missing or unexpected:
        raise KeyError(f"checkpoint / graph mismatch: missing {missing[:5]}..., unexpected {unexpected[:5]}...")
    if stride is not None and not torch.equal(torch.as_tensor(stride, dtype=model.stride.dtype), model.stride):
        raise ValueError(f"checkpoint strides {stride} != graph strides {model.stride.tolist()}")
    model.args = {k: v for k, v in (ckpt.get("train_args") or {}).items()} if isinstance(ckpt.get("train_args"), dict) else {}
    model.pt_path = str(weight)
    if fuse:
        model.fuse()
    return model.to(device).eval(), ckpt


@contextlib.contextmanager
def _ref_modules_registered():
    """Make the reference class paths importable for pickle's save-side lookup (stub classes only)."""
    added, prior = [], []
    absent = object()
    for q in set(REF_CLASS_PATH.values()):
        mod, _, name = q.rpartition(".")
        parts = mod.split(".")
        for i in range(1, len(parts) + 1):
            pm = ".".join(parts[:i])
            if pm not in sys.modules:
                sys.modules[pm] = types.ModuleType(pm)
                added.append(pm)
        # a real (already imported) reference module keeps its class: remember it and put it back afterwards
        prior.append((sys.modules[mod], name, getattr(sys.modules[mod], name, absent)))
        setattr(sys.modules[mod], name, _stub_class(q))
    try:
        yield
    finally:
        for m, name, old in reversed(prior):
            if old is absent:
                with contextlib.suppress(AttributeError):
                    delattr(m, name)
            else:
                setattr(m, name, old)
        for pm in added:
            sys.modules.pop(pm, None)


def _to_reference_tree(model: nn.Module) -> nn.Module:
    """Deep copy of ``model`` whose modules are re-classed as stubs under the reference class paths (state kept)."""
    tree = copy.deepcopy(model).cpu()
    for mod in tree.modules():
        q = REF_CLASS_PATH.get(type(mod))
        if q is not None:
            mod.__class__ = _stub_class(q)
    return tree


def save_checkpoint(model: DetectionModel, path, **meta) -> Path:
    """Write ``model`` (unfused) in the reference trainer's checkpoint layout (fp16 ``ema``)."""
    if any(isinstance(m, M.Conv) and m.is_fused() for m in model.modules()):
        raise ValueError("save_checkpoint needs the unfused model (Conv + BatchNorm), as the trainer saves it")
    tree = _to_reference_tree(model).half()
    ckpt = {"epoch": -1, "best_fitness": None, "model": None, "ema": tree, "updates": None, "optimizer": None,
            "train_args": {}, "train_metrics": {}, "train_results": {}, "date": datetime.now().isoformat(),
            "version": "8.3.63", "license": "AGPL-3.0 (https://ultralytics.com/license)",
            "docs": "https://docs.ultralytics.com"}
    ckpt.update(meta)
    path = Path(path)
    with _ref_modules_registered():
        torch.save(ckpt, str(path))
    return path
