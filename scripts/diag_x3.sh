#!/bin/bash
# Per-stage timelines of the fp16-split Swin kernels: builds ablib/lib_diag.so here with -DYS_DIAG_STAMPS (s_memtime
# of wave 0 at each stage boundary, first 256 windows; ablib/ travels to the GPU box), then there:
#   YOLOSOD_LIB_AB=ablib/lib_diag.so python scripts/diag_x3.py      (C = 64, swin_x3_kernel)
#   YOLOSOD_LIB_AB=ablib/lib_diag.so python scripts/diag_wx.py      (C = 256, swin_wx_kernel)
set -e
cd "$(dirname "$0")/.."
mkdir -p ablib
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -Iinclude -Iyolo-sod_amd/csrc -DYS_DIAG_STAMPS \
  -c yolo-sod_amd/csrc/swin_x3.hip -o ablib/swin_x3_diag.o
objs=$(ls yolo-sod_amd/build/*.o | grep -v swin_x3.o)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -Wl,-soname,libyolosod_hip.so $objs ablib/swin_x3_diag.o -o ablib/lib_diag.so
rm -f ablib/swin_x3_diag.o
echo built ablib/lib_diag.so
