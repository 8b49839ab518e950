"""Build the gfx950 HIP library ``lib/libyolosod_hip.so`` in-tree (hipcc, no cmake).

Run ``python yolo-sod_amd/build.py`` or call :func:`build`. Object files go to ``build/`` next to this file;
rebuilds are incremental on source / header mtimes.
"""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
OBJ = PKG / "build"
LIB = PKG / "lib" / "libyolosod_hip.so"
INCLUDE = PKG.parent / "include"
ARCH = os.environ.get("YOLOSOD_ARCH", "gfx950")

# per-file extra flags: the decode / NMS arithmetic must not be contracted into FMAs (bit-exact NMS indices)
EXTRA = {"detect.hip": ["-ffp-contract=off"], "nms.hip": ["-ffp-contract=off"]}
COMMON = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-variable",
          "-Wno-unused-function", f"-I{INCLUDE}", f"-I{CSRC}"]


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.sep not in c or Path(c).exists()):
            return c
    raise RuntimeError("hipcc not found")


TORCH_OPS_SRC = CSRC / "torch_ops.cpp"
TORCH_OPS_LIB = PKG / "lib" / "yolosod_torch_ops.so"


def build_torch_ops(verbose: bool = False, force: bool = False) -> Path:
    """torch.ops.yolosod.* (csrc/torch_ops.cpp): a torch.utils.cpp_extension library over libyolosod_hip.so, built
    in-tree (build/torch_ops, ninja) and copied next to the HIP library (lib/, which ships to the GPU box)."""
    import shutil

    deps = [TORCH_OPS_SRC, INCLUDE / "yolosod_hip.h"]
    if (not force and TORCH_OPS_LIB.exists()
            and TORCH_OPS_LIB.stat().st_mtime >= max(d.stat().st_mtime for d in deps)):
        return TORCH_OPS_LIB
    from torch.utils import cpp_extension

    bdir = OBJ / "torch_ops"
    bdir.mkdir(parents=True, exist_ok=True)
    so = cpp_extension.load(
        name="yolosod_torch_ops", sources=[str(TORCH_OPS_SRC)], extra_include_paths=[str(INCLUDE), "/opt/rocm/include"],
        extra_cflags=["-O2", "-D__HIP_PLATFORM_AMD__"],
        extra_ldflags=[f"-L{LIB.parent}", "-lyolosod_hip", "-L/opt/rocm/lib", "-lamdhip64", "-lc10_hip", r"-Wl,-rpath,\$$ORIGIN:\$$ORIGIN/../../lib"],  # \$$: ninja + shell escape
        build_directory=str(bdir), is_python_module=False, verbose=verbose)
    built = bdir / "yolosod_torch_ops.so"
    shutil.copy2(built, TORCH_OPS_LIB)
    return TORCH_OPS_LIB


def build(verbose: bool = False, force: bool = False) -> Path:
    srcs = sorted(CSRC.glob("*.hip"))
    headers = list(CSRC.glob("*.h")) + list(INCLUDE.glob("*.h"))
    hdr_mtime = max((h.stat().st_mtime for h in headers), default=0.0)
    OBJ.mkdir(exist_ok=True)
    LIB.parent.mkdir(exist_ok=True)
    hipcc = _hipcc()
    procs = []
    objs = []
    for s in srcs:
        o = OBJ / (s.stem + ".o")
        objs.append(o)
        if not force and o.exists() and o.stat().st_mtime >= max(s.stat().st_mtime, hdr_mtime):
            continue
        cmd = [hipcc, *COMMON, *EXTRA.get(s.name, []), "-c", str(s), "-o", str(o)]
        if verbose:
            print(" ".join(cmd), flush=True)
        procs.append((s, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)))
    failed = []
    for s, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            failed.append((s, out))
        elif verbose and out.strip():
            print(out)
    if failed:
        msg = "\n".join(f"--- {s.name}\n{out}" for s, out in failed)
        raise RuntimeError(f"hipcc failed:\n{msg}")
    lib_mtime = LIB.stat().st_mtime if LIB.exists() else 0.0
    if force or procs or not LIB.exists() or any(o.stat().st_mtime > lib_mtime for o in objs):
        # soname: a same-soname copy loaded first (YOLOSOD_LIB_AB) also satisfies the torch-op library's NEEDED entry
        cmd = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-Wl,-soname,libyolosod_hip.so", *map(str, objs),
               "-o", str(LIB)]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    build_torch_ops(verbose=verbose, force=force)
    return LIB


if __name__ == "__main__":
    print(build(verbose=True, force="--force" in sys.argv))
