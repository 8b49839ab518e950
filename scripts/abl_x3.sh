#!/bin/bash
# Ablation builds of the C = 64 fp16-split Swin kernel (timing sensitivity only; their results are wrong):
# ablib/lib_abl_<name>.so for each -D flag. Run on the GPU box: bash scripts/abl_x3_run.sh
set -e
cd "$(dirname "$0")/.."
mkdir -p ablib
objs=$(ls yolo-sod_amd/build/*.o | grep -v swin_x3.o)
for f in ${ABL_FLAGS:-GELU MLPMFMA EXP WLOAD DW}; do
  /opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -Iinclude -Iyolo-sod_amd/csrc -DYS_ABL_$f -DYS_$f \
    -c yolo-sod_amd/csrc/swin_x3.hip -o /tmp/abl_$f.o
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -Wl,-soname,libyolosod_hip.so $objs /tmp/abl_$f.o \
    -o ablib/lib_abl_$f.so
done
echo built
