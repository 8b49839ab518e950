#!/bin/bash
# Per-phase timeline of nms_select / nms_resolve: builds ab_nms/lib_nms_diag.so here with -DYS_DIAG_STAMPS (s_memtime
# of thread 0 at phase boundaries, images 0..31; ab_nms/ travels to the GPU box), then there:
#   YOLOSOD_LIB_AB=ab_nms/lib_nms_diag.so python scripts/diag_nms.py [loads...]
set -e
cd "$(dirname "$0")/.."
mkdir -p ab_nms
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -ffp-contract=off -Iinclude -Iyolo-sod_amd/csrc \
  -DYS_DIAG_STAMPS -c yolo-sod_amd/csrc/nms.hip -o ab_nms/nms_diag.o
objs=$(ls yolo-sod_amd/build/*.o | grep -v '/nms.o')
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -Wl,-soname,libyolosod_hip.so $objs ab_nms/nms_diag.o -o ab_nms/lib_nms_diag.so
rm -f ab_nms/nms_diag.o
echo built ab_nms/lib_nms_diag.so
