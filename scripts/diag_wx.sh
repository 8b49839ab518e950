#!/bin/bash
# Per-stage timeline of the C = 256 fp16-split Swin kernel (swin_wx): builds diag/lib_diag.so here with
# -DYS_DIAG_STAMPS (s_memtime of wave 0 at each stage boundary, first 256 windows), then on the GPU box:
#   python scripts/diag_wx.py
set -e
cd "$(dirname "$0")/.."
mkdir -p diag
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -Iinclude -Iyolo-sod_amd/csrc -DYS_DIAG_STAMPS \
  -c yolo-sod_amd/csrc/swin_x3.hip -o diag/swin_x3_diag.o
objs=$(ls yolo-sod_amd/build/*.o | grep -v swin_x3.o)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -Wl,-soname,libyolosod_hip.so $objs diag/swin_x3_diag.o -o diag/lib_diag.so
echo built diag/lib_diag.so
