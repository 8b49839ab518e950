"""Import helper: the package lives in the directory ``yolo-sod_amd/`` (not a valid identifier), so it is loaded
from its path and registered in ``sys.modules`` as ``yolosod_amd``."""
import importlib.util
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent
PKG_DIR = ROOT / "yolo-sod_amd"


def load():
    if "yolosod_amd" in sys.modules:
        return sys.modules["yolosod_amd"]
    spec = importlib.util.spec_from_file_location("yolosod_amd", PKG_DIR / "__init__.py",
                                                  submodule_search_locations=[str(PKG_DIR)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["yolosod_amd"] = mod
    try:
        spec.loader.exec_module(mod)
    except BaseException:
        sys.modules.pop("yolosod_amd", None)
        raise
    return mod


yolosod_amd = load()
