"""CPU: ISA guards on hot kernels (hipcc -S for gfx950, no GPU). A buffer resource that the compiler cannot prove
wave-uniform makes it wrap every buffer load in a waterfall loop (v_readfirstlane + s_cbranch_execnz per load): the
1x1 kernel's virtual-concat build had 144 of them and ran 3x slower. The loops of these kernels are few and fixed."""
import re
import shutil
import subprocess
from pathlib import Path

import pytest

CSRC = Path(__file__).resolve().parents[1] / "yolo-sod_amd" / "csrc"
HIPCC = shutil.which("hipcc") or ("/opt/rocm/bin/hipcc" if Path("/opt/rocm/bin/hipcc").exists() else None)


def _kernel_isa(src, tmp_path):
    out = tmp_path / (src + ".s")
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "--cuda-device-only", "-S", f"-I{CSRC}", "-o", str(out),
                    str(CSRC / src)], check=True, capture_output=True, timeout=300)
    text = out.read_text()
    kernels = {}
    for m in re.finditer(r"^(_Z[^:\s]+):", text, re.M):
        end = text.find("s_endpgm", m.end())
        kernels[m.group(1)] = text[m.end():end]
    return kernels


@pytest.mark.skipif(HIPCC is None, reason="hipcc not available")
@pytest.mark.parametrize("src,pattern", [("conv1x1x2.hip", "conv1x1_x2_kernel"), ("conv3x3.hip", "conv3x3_p_kernel"),
                                         ("conv3x3s2.hip", "conv3x3s2_t2_kernel")])
def test_no_waterfall_loops(src, pattern, tmp_path):
    """A waterfall loop costs one v_readfirstlane per buffer load (the bad build: 272 in one kernel); the good builds
    keep a handful (the resources' base / size)."""
    ks = {k: v for k, v in _kernel_isa(src, tmp_path).items() if pattern in k}
    assert ks, f"no {pattern} in {src}"
    for name, body in ks.items():
        rfl, loops = body.count("v_readfirstlane"), body.count("s_cbranch_execnz")
        assert rfl <= 16 and loops <= 16, f"{name}: {rfl} readfirstlane, {loops} exec-mask loops (waterfall loads?)"
