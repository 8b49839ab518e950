/*
 * ORACLE - TEST INFRASTRUCTURE ONLY. Never linked into or called by the product path (yolo-sod_amd/).
 *
 * CPU restatement of torchvision==0.20.1 `torchvision.ops.nms` (CPU kernel, third-party dependency of the
 * reference pinned in requirements.txt:62, called at ultralytics/utils/ops.py:296). The dependency is absent
 * from /root/reference and from this image, so this follows its published algorithm:
 *   order  = scores sorted descending, stable (ties: lower input index first)
 *   areas  = (x2 - x1) * (y2 - y1)                       (fp32, no +1)
 *   greedy : for i in order, if not suppressed: keep i; for later j not suppressed:
 *              w = max(0, min(x2i,x2j) - max(x1i,x1j)), h likewise, inter = w*h,
 *              ovr = inter / (area_i + area_j - inter);  suppress j if (double)ovr > iou_threshold
 * Compiled with -ffp-contract=off so that fp32 rounding matches a non-FMA x86-64 build.
 * Parity at this boundary is "unpinned" by reference fixtures (no reference test asserts NMS outputs); the
 * ultralytics wrapper around it (ops.py:167-316) IS pinned by tests/golden fixtures.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct { float s; int64_t i; } key_t_;

static int cmp_desc_stable(const void* a, const void* b) {
  const key_t_* x = (const key_t_*)a;
  const key_t_* y = (const key_t_*)b;
  if (x->s > y->s) return -1;
  if (x->s < y->s) return 1;
  return (x->i < y->i) ? -1 : (x->i > y->i);
}

/* boxes: n x 4 (x1,y1,x2,y2), scores: n. Writes kept indices (into the input) to keep, returns count. */
int64_t nms_ref(const float* boxes, const float* scores, int64_t n, double iou_threshold, int64_t* keep) {
  if (n <= 0) return 0;
  key_t_* order = (key_t_*)malloc(sizeof(key_t_) * n);
  float* areas = (float*)malloc(sizeof(float) * n);
  unsigned char* sup = (unsigned char*)calloc(n, 1);
  for (int64_t i = 0; i < n; ++i) {
    order[i].s = scores[i];
    order[i].i = i;
    const float* b = boxes + 4 * i;
    areas[i] = (b[2] - b[0]) * (b[3] - b[1]);
  }
  qsort(order, n, sizeof(key_t_), cmp_desc_stable);
  int64_t nk = 0;
  for (int64_t _i = 0; _i < n; ++_i) {
    const int64_t i = order[_i].i;
    if (sup[i]) continue;
    keep[nk++] = i;
    const float* bi = boxes + 4 * i;
    const float ix1 = bi[0], iy1 = bi[1], ix2 = bi[2], iy2 = bi[3], iarea = areas[i];
    for (int64_t _j = _i + 1; _j < n; ++_j) {
      const int64_t j = order[_j].i;
      if (sup[j]) continue;
      const float* bj = boxes + 4 * j;
      const float xx1 = ix1 > bj[0] ? ix1 : bj[0];
      const float yy1 = iy1 > bj[1] ? iy1 : bj[1];
      const float xx2 = ix2 < bj[2] ? ix2 : bj[2];
      const float yy2 = iy2 < bj[3] ? iy2 : bj[3];
      const float dw = xx2 - xx1, dh = yy2 - yy1;
      const float w = 0.0f > dw ? 0.0f : dw;
      const float h = 0.0f > dh ? 0.0f : dh;
      const float inter = w * h;
      const float ovr = inter / (iarea + areas[j] - inter);
      if ((double)ovr > iou_threshold) sup[j] = 1;
    }
  }
  free(order);
  free(areas);
  free(sup);
  return nk;
}
