// Torch-op registration of the hot-path kernel families ("a torch.utils.cpp_extension module ... thin
// wrappers registered as torch ops"): torch.ops.yolosod.{se_fwd, cbam_fwd, ca_fwd, a2_fwd, swin_fwd,
// detect_head_fwd, detect_decode_fwd, nms_batched}.
//
// Each op validates its tensors with TORCH_CHECK (RuntimeError in Python, as the reference's own asserts /
// exceptions surface, e.g. a2_attn.py:24), allocates its output and workspace with at::empty on the input's device
// (PyTorch's caching allocator, stream-ordered on the current stream: graph-capture safe), and calls the C ABI of
// libyolosod_hip.so (include/yolosod_hip.h) on c10::hip::getCurrentHIPStream(). Activations are fp32 or bf16
// (the bf16 model config); the bf16 entry points take bf16 GEMM weights for Swin / A2 and fp32 elsewhere. Meta
// kernels give shapes without a GPU (the model's stride probe / tracing).
#include <torch/library.h>
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>

#include "yolosod_hip.h"

namespace {

using at::Tensor;

void* sp(const c10::hip::HIPStream& s) { return (void*)s.stream(); }

void check_rc(int rc, const char* what) {
  TORCH_CHECK(rc == 0, "yolosod_amd.", what, " failed (rc=", rc, "): ", yolosod_last_error());
}

// element count of the per-plane partials a producing epilogue emits for SE / CBAM (yolosod_plane_parts)
int64_t partials_numel(int B, int C, int H, int W) {
  long seg = 0;
  const int parts = yolosod_plane_parts((long)H * W, &seg);
  return (int64_t)B * C * parts;
}

bool act_bf16(const Tensor& x, const char* what) {
  TORCH_CHECK(x.is_cuda(), what, ": HIP kernel requires a GPU tensor (got ", x.device(), "); no CPU fallback");
  TORCH_CHECK(x.dim() == 4, what, ": expected [B, C, H, W], got ", x.sizes());
  TORCH_CHECK(x.is_contiguous(), what, ": expected a contiguous tensor");
  TORCH_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16, what,
              ": activations must be float32 or bfloat16, got ", x.scalar_type());
  return x.scalar_type() == at::kBFloat16;
}

// pointer of a parameter after checking device, dtype, contiguity and element count
const void* par(const Tensor& t, const Tensor& x, const char* name, int64_t numel, at::ScalarType dt = at::kFloat) {
  TORCH_CHECK(t.device() == x.device(), name, ": on ", t.device(), ", activations on ", x.device());
  TORCH_CHECK(t.scalar_type() == dt, name, ": expected ", dt, ", got ", t.scalar_type());
  TORCH_CHECK(t.is_contiguous(), name, ": expected a contiguous tensor");
  TORCH_CHECK(numel < 0 || t.numel() == numel, name, ": expected ", numel, " elements, got ", t.numel());
  return t.data_ptr();
}

Tensor workspace(size_t bytes, const Tensor& x) {
  return at::empty({(int64_t)std::max<size_t>(bytes, 256)}, x.options().dtype(at::kByte));
}

Tensor se_fwd(const Tensor& x, const Tensor& fc1_w, const Tensor& fc1_b, const Tensor& fc2_w, const Tensor& fc2_b,
              const c10::optional<Tensor>& psum) {
  const bool bf = act_bf16(x, "se_fwd");
  c10::DeviceGuard guard(x.device());
  const int B = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3), hid = fc1_w.size(0);
  Tensor y = at::empty_like(x);
  Tensor ws = workspace(yolosod_se_workspace(B, C, H, W), x);
  const float* ps = psum ? (const float*)par(*psum, x, "psum", partials_numel(B, C, H, W)) : nullptr;
  auto st = c10::hip::getCurrentHIPStream(x.get_device());
  const float* w1 = (const float*)par(fc1_w, x, "fc1.weight", (int64_t)hid * C);
  const float* b1 = (const float*)par(fc1_b, x, "fc1.bias", hid);
  const float* w2 = (const float*)par(fc2_w, x, "fc2.weight", (int64_t)C * hid);
  const float* b2 = (const float*)par(fc2_b, x, "fc2.bias", C);
  int rc;
  if (bf)
    rc = yolosod_se_forward_bf16((const uint16_t*)x.data_ptr(), (uint16_t*)y.data_ptr(), B, C, H, W, w1, b1, w2, b2,
                                 hid, ps, ws.data_ptr(), ws.numel(), sp(st));
  else if (ps)
    rc = yolosod_se_forward_pre((const float*)x.data_ptr(), (float*)y.data_ptr(), B, C, H, W, w1, b1, w2, b2, hid, ps,
                                ws.data_ptr(), ws.numel(), sp(st));
  else
    rc = yolosod_se_forward((const float*)x.data_ptr(), (float*)y.data_ptr(), B, C, H, W, w1, b1, w2, b2, hid,
                            ws.data_ptr(), ws.numel(), sp(st));
  check_rc(rc, "se_fwd");
  return y;
}

Tensor cbam_fwd(const Tensor& x, const Tensor& fc0_w, const Tensor& fc2_w, const Tensor& sa_w,
                const c10::optional<Tensor>& psum, const c10::optional<Tensor>& pmax) {
  const bool bf = act_bf16(x, "cbam_fwd");
  TORCH_CHECK(psum.has_value() == pmax.has_value(), "cbam_fwd: give both producer partials or neither");
  c10::DeviceGuard guard(x.device());
  const int B = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3), hid = fc0_w.size(0);
  Tensor y = at::empty_like(x);
  Tensor ws = workspace(yolosod_cbam_workspace(B, C, H, W), x);
  auto st = c10::hip::getCurrentHIPStream(x.get_device());
  const float* w0 = (const float*)par(fc0_w, x, "fc.0.weight", (int64_t)hid * C);
  const float* w2 = (const float*)par(fc2_w, x, "fc.2.weight", (int64_t)C * hid);
  const float* sa = (const float*)par(sa_w, x, "conv1.weight", 98);
  const int64_t nparts = partials_numel(B, C, H, W);  // the producer layout the kernels read: B * C * parts
  const float* ps = psum ? (const float*)par(*psum, x, "psum", nparts) : nullptr;
  const float* pm = pmax ? (const float*)par(*pmax, x, "pmax", nparts) : nullptr;
  int rc;
  if (bf)
    rc = yolosod_cbam_forward_bf16((const uint16_t*)x.data_ptr(), (uint16_t*)y.data_ptr(), B, C, H, W, w0, w2, hid,
                                   sa, ps, pm, ws.data_ptr(), ws.numel(), sp(st));
  else if (ps)
    rc = yolosod_cbam_forward_pre((const float*)x.data_ptr(), (float*)y.data_ptr(), B, C, H, W, w0, w2, hid, sa, ps,
                                  pm, ws.data_ptr(), ws.numel(), sp(st));
  else
    rc = yolosod_cbam_forward((const float*)x.data_ptr(), (float*)y.data_ptr(), B, C, H, W, w0, w2, hid, sa,
                              ws.data_ptr(), ws.numel(), sp(st));
  check_rc(rc, "cbam_fwd");
  return y;
}

Tensor ca_fwd(const Tensor& x, const Tensor& conv1_w, const Tensor& conv1_b, const Tensor& bn_w, const Tensor& bn_b,
              const Tensor& bn_mean, const Tensor& bn_var, double bn_eps, const Tensor& convh_w, const Tensor& convh_b,
              const Tensor& convw_w, const Tensor& convw_b, const c10::optional<Tensor>& yin) {
  const bool bf = act_bf16(x, "ca_fwd");
  c10::DeviceGuard guard(x.device());
  const int B = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3), mip = conv1_w.size(0);
  Tensor y = at::empty_like(x);
  Tensor ws = workspace(yolosod_ca_workspace(B, C, H, W), x);
  auto st = c10::hip::getCurrentHIPStream(x.get_device());
  const float* p[10] = {
      (const float*)par(conv1_w, x, "conv1.weight", (int64_t)mip * C), (const float*)par(conv1_b, x, "conv1.bias", mip),
      (const float*)par(bn_w, x, "bn1.weight", mip), (const float*)par(bn_b, x, "bn1.bias", mip),
      (const float*)par(bn_mean, x, "bn1.running_mean", mip), (const float*)par(bn_var, x, "bn1.running_var", mip),
      (const float*)par(convh_w, x, "conv_h.weight", (int64_t)C * mip), (const float*)par(convh_b, x, "conv_h.bias", C),
      (const float*)par(convw_w, x, "conv_w.weight", (int64_t)C * mip), (const float*)par(convw_b, x, "conv_w.bias", C)};
  const float* yi = yin ? (const float*)par(*yin, x, "yin", (int64_t)B * C * (H + W)) : nullptr;
  int rc;
  if (bf)
    rc = yolosod_ca_forward_bf16((const uint16_t*)x.data_ptr(), (uint16_t*)y.data_ptr(), B, C, H, W, p[0], p[1], mip,
                                 p[2], p[3], p[4], p[5], (float)bn_eps, p[6], p[7], p[8], p[9], yi, ws.data_ptr(),
                                 ws.numel(), sp(st));
  else if (yi)
    rc = yolosod_ca_forward_pre((const float*)x.data_ptr(), (float*)y.data_ptr(), B, C, H, W, p[0], p[1], mip, p[2],
                                p[3], p[4], p[5], (float)bn_eps, p[6], p[7], p[8], p[9], yi, ws.data_ptr(), ws.numel(),
                                sp(st));
  else
    rc = yolosod_ca_forward((const float*)x.data_ptr(), (float*)y.data_ptr(), B, C, H, W, p[0], p[1], mip, p[2], p[3],
                            p[4], p[5], (float)bn_eps, p[6], p[7], p[8], p[9], ws.data_ptr(), ws.numel(), sp(st));
  check_rc(rc, "ca_fwd");
  return y;
}

// A2's fused LN / QKV / attention kernel's prepared in_proj weights (yolosod_a2_prepare) as a uint8 tensor, made
// once per parameter version by the caller (nn/modules.A2_Attn caches it) and passed to a2_fwd.
Tensor a2_prep(const Tensor& x, int64_t num_areas, int64_t num_heads, const Tensor& proj_w, const Tensor& ln_w,
               const Tensor& ln_b, const Tensor& in_w, const Tensor& in_b) {
  TORCH_CHECK(!act_bf16(x, "a2_prep"), "a2_prep: the prepared path is the fp32 config's");
  c10::DeviceGuard guard(x.device());
  const int C = x.size(1), W = x.size(3);
  const size_t bytes = yolosod_a2_prep_bytes(C, num_heads, num_areas, W);
  TORCH_CHECK(bytes > 0, "a2_prep: C=", C, " heads=", num_heads, " L=", num_areas * W, " has no fused kernel");
  Tensor prep = at::empty({(int64_t)bytes}, x.options().dtype(at::kByte));
  auto st = c10::hip::getCurrentHIPStream(x.get_device());
  check_rc(yolosod_a2_prepare(C, (const float*)par(proj_w, x, "proj.weight", (int64_t)C * C),
                              (const float*)par(ln_w, x, "layer_norm.weight", C),
                              (const float*)par(ln_b, x, "layer_norm.bias", C),
                              (const float*)par(in_w, x, "in_proj_weight", 3LL * C * C),
                              (const float*)par(in_b, x, "in_proj_bias", 3 * C), prep.data_ptr(), bytes, sp(st)),
           "a2_prep");
  return prep;
}

Tensor a2_fwd(const Tensor& x, int64_t num_areas, int64_t num_heads, const Tensor& proj_w, const Tensor& proj_b,
              const Tensor& ln_w, const Tensor& ln_b, double ln_eps, const Tensor& in_w, const Tensor& in_b,
              const c10::optional<Tensor>& mo_w, const c10::optional<Tensor>& mo_b, const Tensor& op_w,
              const Tensor& op_b, const c10::optional<Tensor>& prep) {
  const bool bf = act_bf16(x, "a2_fwd");
  c10::DeviceGuard guard(x.device());
  const int B = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(C % num_heads == 0, "A2_Attn: C=", C, " not divisible by num_heads=", num_heads);
  TORCH_CHECK(mo_w.has_value() == mo_b.has_value(), "a2_fwd: out_proj weight and bias must both be given or neither");
  Tensor y = at::empty_like(x);
  auto st = c10::hip::getCurrentHIPStream(x.get_device());
  const auto gw = bf ? at::kBFloat16 : at::kFloat;
  const void* pw = par(proj_w, x, "proj.weight", (int64_t)C * C, gw);
  const float* pb = (const float*)par(proj_b, x, "proj.bias", C);
  const float* lw = (const float*)par(ln_w, x, "layer_norm.weight", C);
  const float* lb = (const float*)par(ln_b, x, "layer_norm.bias", C);
  const void* iw = par(in_w, x, "in_proj_weight", 3LL * C * C, gw);
  const float* ib = (const float*)par(in_b, x, "in_proj_bias", 3 * C);
  const void* ow = par(op_w, x, "out_proj.weight", (int64_t)C * C, gw);
  const float* ob = (const float*)par(op_b, x, "out_proj.bias", C);
  int rc;
  if (bf) {
    TORCH_CHECK(!mo_w.has_value(), "a2_fwd: the bf16 path takes the pre-multiplied output weights only");
    Tensor ws = workspace(yolosod_a2_workspace_bf16(B, C, H, W, num_areas), x);
    rc = yolosod_a2_forward_bf16((const uint16_t*)x.data_ptr(), (uint16_t*)y.data_ptr(), B, C, H, W, num_areas,
                                 num_heads, (const uint16_t*)pw, pb, lw, lb, (float)ln_eps, (const uint16_t*)iw, ib,
                                 (const uint16_t*)ow, ob, ws.data_ptr(), ws.numel(), sp(st));
  } else {
    Tensor ws = workspace(yolosod_a2_workspace(B, C, H, W, num_areas), x);
    const float* mw = mo_w ? (const float*)par(*mo_w, x, "attention.out_proj.weight", (int64_t)C * C) : nullptr;
    const float* mb = mo_b ? (const float*)par(*mo_b, x, "attention.out_proj.bias", C) : nullptr;
    const size_t pbytes = yolosod_a2_prep_bytes(C, num_heads, num_areas, W);
    if (prep && pbytes > 0 && !mo_w) {
      TORCH_CHECK((size_t)prep->numel() == pbytes && prep->scalar_type() == at::kByte && prep->device() == x.device() &&
                      prep->is_contiguous(),
                  "a2_fwd: prep must be the ", pbytes, "-byte block of a2_prep on ", x.device());
      rc = yolosod_a2_forward_prepared((const float*)x.data_ptr(), (float*)y.data_ptr(), B, C, H, W, num_areas,
                                       num_heads, (const float*)pw, pb, lw, lb, (float)ln_eps, (const float*)iw, ib,
                                       (const float*)ow, ob, prep->data_ptr(), pbytes, ws.data_ptr(), ws.numel(),
                                       sp(st));
    } else {
      rc = yolosod_a2_forward((const float*)x.data_ptr(), (float*)y.data_ptr(), B, C, H, W, num_areas, num_heads,
                              (const float*)pw, pb, lw, lb, (float)ln_eps, (const float*)iw, ib, mw, mb,
                              (const float*)ow, ob, ws.data_ptr(), ws.numel(), sp(st));
    }
  }
  check_rc(rc, "a2_fwd");
  return y;
}

// The fp16-split Swin kernels' prepared parameters (weight planes, folds) as a uint8 tensor, made once per parameter
// version by the caller (nn/modules.SwinBlock caches it) and passed to swin_fwd_prepared.
Tensor swin_prep(const Tensor& x, int64_t num_heads, const Tensor& ln1_w, const Tensor& ln1_b, const Tensor& in_w,
                 const Tensor& in_b, const Tensor& out_w, const Tensor& ln2_w, const Tensor& ln2_b, const Tensor& m1_w,
                 const Tensor& m1_b, const Tensor& m2_w, const Tensor& pw_w, const Tensor& bn_w, const Tensor& bn_b,
                 const Tensor& bn_mean, const Tensor& bn_var, double bn_eps) {
  TORCH_CHECK(!act_bf16(x, "swin_prep"), "swin_prep: the prepared path is the fp32 config's");
  c10::DeviceGuard guard(x.device());
  const int C = x.size(1), hid = m1_w.size(0);
  const size_t bytes = yolosod_swin_prep_bytes(C, num_heads, hid);
  TORCH_CHECK(bytes > 0, "swin_prep: C=", C, " heads=", num_heads, " hidden=", hid, " has no prepared path");
  Tensor prep = at::empty({(int64_t)bytes}, x.options().dtype(at::kByte));
  auto st = c10::hip::getCurrentHIPStream(x.get_device());
  const int rc = yolosod_swin_prepare(
      C, num_heads, hid, (const float*)par(ln1_w, x, "norm1.weight", C), (const float*)par(ln1_b, x, "norm1.bias", C),
      (const float*)par(in_w, x, "in_proj_weight", 3LL * C * C), (const float*)par(in_b, x, "in_proj_bias", 3 * C),
      (const float*)par(out_w, x, "out_proj.weight", (int64_t)C * C), (const float*)par(ln2_w, x, "norm2.weight", C),
      (const float*)par(ln2_b, x, "norm2.bias", C), (const float*)par(m1_w, x, "mlp.0.weight", (int64_t)hid * C),
      (const float*)par(m1_b, x, "mlp.0.bias", hid), (const float*)par(m2_w, x, "mlp.2.weight", (int64_t)C * hid),
      (const float*)par(pw_w, x, "pw.weight", (int64_t)C * C), (const float*)par(bn_w, x, "bn.weight", C),
      (const float*)par(bn_b, x, "bn.bias", C), (const float*)par(bn_mean, x, "bn.running_mean", C),
      (const float*)par(bn_var, x, "bn.running_var", C), (float)bn_eps, prep.data_ptr(), bytes, sp(st));
  check_rc(rc, "swin_prep");
  return prep;
}

Tensor swin_fwd_prepared(const Tensor& x, const Tensor& prep, int64_t num_heads, int64_t window, const Tensor& dw_w,
                         double ln1_eps, const Tensor& out_b, double ln2_eps, int64_t hid, const Tensor& m2_b) {
  TORCH_CHECK(!act_bf16(x, "swin_fwd_prepared"), "swin_fwd_prepared: fp32 activations only");
  c10::DeviceGuard guard(x.device());
  const int B = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const size_t bytes = yolosod_swin_prep_bytes(C, num_heads, hid);
  TORCH_CHECK(bytes > 0 && (size_t)prep.numel() == bytes && prep.scalar_type() == at::kByte &&
                  prep.device() == x.device() && prep.is_contiguous(),
              "swin_fwd_prepared: prep must be the ", bytes, "-byte block of swin_prep on ", x.device());
  TORCH_CHECK((int64_t)C * H * W < (1LL << 30), "swin_fwd_prepared: one image of ", C, "x", H, "x", W,
              " is too large for the prepared kernels (use swin_fwd)");
  Tensor y = at::empty_like(x);
  auto st = c10::hip::getCurrentHIPStream(x.get_device());
  Tensor ws = workspace(yolosod_swin_prepared_workspace(B, C, H, W, num_heads, window, hid), x);
  const int rc = yolosod_swin_forward_prepared(
      (const float*)x.data_ptr(), (float*)y.data_ptr(), B, C, H, W, num_heads, window,
      (const float*)par(dw_w, x, "dw.weight", 9LL * C), (float)ln1_eps, (const float*)par(out_b, x, "out_proj.bias", C),
      (float)ln2_eps, hid, (const float*)par(m2_b, x, "mlp.2.bias", C), prep.data_ptr(), bytes, ws.data_ptr(),
      ws.numel(), sp(st));
  check_rc(rc, "swin_fwd_prepared");
  return y;
}

Tensor swin_fwd(const Tensor& x, int64_t num_heads, int64_t window, const Tensor& dw_w, const Tensor& ln1_w,
                const Tensor& ln1_b, double ln1_eps, const Tensor& in_w, const Tensor& in_b, const Tensor& out_w,
                const Tensor& out_b, const Tensor& ln2_w, const Tensor& ln2_b, double ln2_eps, const Tensor& m1_w,
                const Tensor& m1_b, const Tensor& m2_w, const Tensor& m2_b, const Tensor& pw_w, const Tensor& bn_w,
                const Tensor& bn_b, const Tensor& bn_mean, const Tensor& bn_var, double bn_eps) {
  const bool bf = act_bf16(x, "swin_fwd");
  c10::DeviceGuard guard(x.device());
  const int B = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3), hid = m1_w.size(0);
  TORCH_CHECK(C % num_heads == 0, "SwinBlock: C=", C, " not divisible by num_heads=", num_heads);
  Tensor y = at::empty_like(x);
  auto st = c10::hip::getCurrentHIPStream(x.get_device());
  const auto gw = bf ? at::kBFloat16 : at::kFloat;
  const float* f[13] = {
      (const float*)par(dw_w, x, "dw.weight", 9LL * C), (const float*)par(ln1_w, x, "norm1.weight", C),
      (const float*)par(ln1_b, x, "norm1.bias", C), (const float*)par(in_b, x, "in_proj_bias", 3 * C),
      (const float*)par(out_b, x, "out_proj.bias", C), (const float*)par(ln2_w, x, "norm2.weight", C),
      (const float*)par(ln2_b, x, "norm2.bias", C), (const float*)par(m1_b, x, "mlp.0.bias", hid),
      (const float*)par(m2_b, x, "mlp.2.bias", C), (const float*)par(bn_w, x, "bn.weight", C),
      (const float*)par(bn_b, x, "bn.bias", C), (const float*)par(bn_mean, x, "bn.running_mean", C),
      (const float*)par(bn_var, x, "bn.running_var", C)};
  const void* g[5] = {par(in_w, x, "in_proj_weight", 3LL * C * C, gw), par(out_w, x, "out_proj.weight", (int64_t)C * C, gw),
                      par(m1_w, x, "mlp.0.weight", (int64_t)hid * C, gw), par(m2_w, x, "mlp.2.weight", (int64_t)C * hid, gw),
                      par(pw_w, x, "pw.weight", (int64_t)C * C, gw)};
  int rc;
  if (bf) {
    Tensor ws = workspace(yolosod_swin_workspace_bf16(B, C, H, W, num_heads, window, hid), x);
    rc = yolosod_swin_forward_bf16((const uint16_t*)x.data_ptr(), (uint16_t*)y.data_ptr(), B, C, H, W, num_heads,
                                   window, f[0], f[1], f[2], (float)ln1_eps, (const uint16_t*)g[0], f[3],
                                   (const uint16_t*)g[1], f[4], f[5], f[6], (float)ln2_eps, (const uint16_t*)g[2], f[7],
                                   hid, (const uint16_t*)g[3], f[8], (const uint16_t*)g[4], f[9], f[10], f[11], f[12],
                                   (float)bn_eps, ws.data_ptr(), ws.numel(), sp(st));
  } else {
    Tensor ws = workspace(yolosod_swin_workspace_v2(B, C, H, W, num_heads, window, hid), x);
    rc = yolosod_swin_forward((const float*)x.data_ptr(), (float*)y.data_ptr(), B, C, H, W, num_heads, window, f[0],
                              f[1], f[2], (float)ln1_eps, (const float*)g[0], f[3], (const float*)g[1], f[4], f[5], f[6],
                              (float)ln2_eps, (const float*)g[2], f[7], hid, (const float*)g[3], f[8],
                              (const float*)g[4], f[9], f[10], f[11], f[12], (float)bn_eps, ws.data_ptr(), ws.numel(),
                              sp(st));
  }
  check_rc(rc, "swin_fwd");
  return y;
}

// levels [l0, l1) of the fused Detect tail + decode into y [B, 4+nc, A] (A over all levels; l1 < 0: all levels,
// y allocated here when undefined)
static Tensor detect_head_run(at::TensorList box_feats, at::TensorList cls_feats, at::TensorList box_w,
                              at::TensorList box_b, at::TensorList cls_w, at::TensorList cls_b,
                              at::ArrayRef<double> strides, int64_t nc, int64_t reg_max, Tensor y, int64_t l0,
                              int64_t l1) {
  const int nl = box_feats.size();
  TORCH_CHECK(nl >= 1 && nl <= 4 && cls_feats.size() == (size_t)nl && box_w.size() == (size_t)nl &&
                  box_b.size() == (size_t)nl && cls_w.size() == (size_t)nl && cls_b.size() == (size_t)nl &&
                  strides.size() == (size_t)nl,
              "detect_head_fwd: 1..4 levels with one tensor of each kind per level");
  if (l1 < 0) l1 = nl;
  TORCH_CHECK(0 <= l0 && l0 < l1 && l1 <= nl, "detect_head: level range [", l0, ", ", l1, ") outside [0, ", nl, ")");
  const Tensor& x0 = box_feats[0];
  const bool bf = act_bf16(x0, "detect_head_fwd");
  c10::DeviceGuard guard(x0.device());
  const int B = x0.size(0), c2 = x0.size(1), c3 = cls_feats[0].size(1);
  const void* fb[4];
  const void* fc[4];
  const float *wb[4], *bb[4], *wc[4], *bc[4];
  int hs[4], wsz[4];
  float st_[4];
  int64_t A = 0;
  for (int i = 0; i < nl; ++i) {
    const Tensor& b = box_feats[i];
    const Tensor& c = cls_feats[i];
    TORCH_CHECK(b.device() == x0.device() && c.device() == x0.device(), "detect_head_fwd: level ", i,
                " features on ", b.device(), " / ", c.device(), ", level 0 on ", x0.device());
    TORCH_CHECK(act_bf16(b, "box_feats") == bf && act_bf16(c, "cls_feats") == bf && b.size(0) == B &&
                    b.size(1) == c2 && c.size(1) == c3 && b.size(2) == c.size(2) && b.size(3) == c.size(3),
                "detect_head_fwd: level ", i, " features ", b.sizes(), " / ", c.sizes(), " mismatch");
    fb[i] = b.data_ptr();
    fc[i] = c.data_ptr();
    wb[i] = (const float*)par(box_w[i], x0, "box_w", 4 * reg_max * c2);
    bb[i] = (const float*)par(box_b[i], x0, "box_b", 4 * reg_max);
    wc[i] = (const float*)par(cls_w[i], x0, "cls_w", nc * c3);
    bc[i] = (const float*)par(cls_b[i], x0, "cls_b", nc);
    hs[i] = b.size(2);
    wsz[i] = b.size(3);
    st_[i] = (float)strides[i];
    A += (int64_t)hs[i] * wsz[i];
  }
  if (!y.defined()) y = at::empty({B, 4 + nc, A}, x0.options().dtype(at::kFloat));
  TORCH_CHECK(y.device() == x0.device() && y.scalar_type() == at::kFloat && y.is_contiguous() && y.dim() == 3 &&
                  y.size(0) == B && y.size(1) == 4 + nc && y.size(2) == A,
              "detect_head: y must be a contiguous fp32 [", B, ", ", 4 + nc, ", ", A, "] tensor on ", x0.device());
  auto st = c10::hip::getCurrentHIPStream(x0.get_device());
  const int rc = yolosod_detect_head_levels(nl, (int)l0, (int)l1, fb, fc, c2, c3, wb, bb, wc, bc, hs, wsz, st_, B,
                                            nc, reg_max, y.data_ptr<float>(), bf ? 1 : 0, sp(st));
  check_rc(rc, "detect_head_fwd");
  return y;
}

Tensor detect_head_fwd(at::TensorList box_feats, at::TensorList cls_feats, at::TensorList box_w, at::TensorList box_b,
                       at::TensorList cls_w, at::TensorList cls_b, at::ArrayRef<double> strides, int64_t nc,
                       int64_t reg_max) {
  return detect_head_run(box_feats, cls_feats, box_w, box_b, cls_w, cls_b, strides, nc, reg_max, Tensor(), 0, -1);
}

// levels [l0, l1) into the caller's y (the executor: the levels whose towers are done, then the last one)
void detect_head_into(Tensor y, int64_t l0, int64_t l1, at::TensorList box_feats, at::TensorList cls_feats,
                      at::TensorList box_w, at::TensorList box_b, at::TensorList cls_w, at::TensorList cls_b,
                      at::ArrayRef<double> strides, int64_t nc, int64_t reg_max) {
  detect_head_run(box_feats, cls_feats, box_w, box_b, cls_w, cls_b, strides, nc, reg_max, y, l0, l1);
}

Tensor detect_decode_fwd(at::TensorList maps, at::ArrayRef<double> strides, int64_t nc, int64_t reg_max) {
  const int nl = maps.size();
  TORCH_CHECK(nl >= 1 && nl <= 4 && strides.size() == (size_t)nl, "detect_decode_fwd: 1..4 levels");
  const Tensor& x0 = maps[0];
  TORCH_CHECK(!act_bf16(x0, "detect_decode_fwd"), "detect_decode_fwd: the decode takes fp32 maps");
  c10::DeviceGuard guard(x0.device());
  const int B = x0.size(0);
  const float* mp[4];
  int hs[4], wsz[4];
  float st_[4];
  int64_t A = 0;
  for (int i = 0; i < nl; ++i) {
    TORCH_CHECK(!act_bf16(maps[i], "maps") && maps[i].size(0) == B && maps[i].size(1) == 4 * reg_max + nc,
                "detect_decode_fwd: map ", i, " has shape ", maps[i].sizes());
    mp[i] = maps[i].data_ptr<float>();
    hs[i] = maps[i].size(2);
    wsz[i] = maps[i].size(3);
    st_[i] = (float)strides[i];
    A += (int64_t)hs[i] * wsz[i];
  }
  Tensor y = at::empty({B, 4 + nc, A}, x0.options());
  auto st = c10::hip::getCurrentHIPStream(x0.get_device());
  check_rc(yolosod_detect_decode(nl, mp, hs, wsz, st_, B, nc, reg_max, y.data_ptr<float>(), sp(st)),
           "detect_decode_fwd");
  return y;
}

std::tuple<Tensor, Tensor, Tensor> nms_batched(const Tensor& pred, double conf_thres, double iou_thres,
                                               const c10::optional<Tensor>& classes, bool agnostic, bool multi_label,
                                               int64_t max_det, int64_t max_nms, double max_wh, bool in_place) {
  TORCH_CHECK(pred.is_cuda() && pred.scalar_type() == at::kFloat && pred.is_contiguous() && pred.dim() == 3,
              "nms_batched: prediction must be a contiguous float32 GPU tensor [B, 4+nc, A], got ", pred.sizes());
  c10::DeviceGuard guard(pred.device());
  const int B = pred.size(0), nc = pred.size(1) - 4, A = pred.size(2);
  auto f = pred.options();
  Tensor out = at::empty({B, max_det, 6}, f);
  Tensor counts = at::empty({B}, f.dtype(at::kInt));
  Tensor index = at::empty({B, max_det}, f.dtype(at::kInt));
  Tensor ws = workspace(yolosod_nms_workspace_v2(B, nc, A, multi_label, max_det), pred);
  const int* cls = nullptr;
  int ncls = 0;
  if (classes) {
    TORCH_CHECK(classes->device() == pred.device() && classes->scalar_type() == at::kInt && classes->is_contiguous(),
                "nms_batched: classes must be a contiguous int32 tensor on the prediction's device");
    cls = classes->data_ptr<int>();
    ncls = classes->numel();
  }
  auto st = c10::hip::getCurrentHIPStream(pred.get_device());
  check_rc(yolosod_nms(pred.data_ptr<float>(), B, nc, A, (float)conf_thres, iou_thres, cls, ncls, agnostic, multi_label,
                       max_det, max_nms, (float)max_wh, in_place ? 1 : 0, out.data_ptr<float>(), counts.data_ptr<int>(),
                       index.data_ptr<int>(), ws.data_ptr(), ws.numel(), sp(st)),
           "nms_batched");
  return {out, counts, index};
}

// ---- shape-only (Meta) kernels ----
Tensor mafn_meta(const Tensor& x) { return at::empty_like(x); }

}  // namespace

TORCH_LIBRARY(yolosod, m) {
  m.def("se_fwd(Tensor x, Tensor fc1_w, Tensor fc1_b, Tensor fc2_w, Tensor fc2_b, Tensor? psum) -> Tensor");
  m.def("cbam_fwd(Tensor x, Tensor fc0_w, Tensor fc2_w, Tensor sa_w, Tensor? psum, Tensor? pmax) -> Tensor");
  m.def("ca_fwd(Tensor x, Tensor conv1_w, Tensor conv1_b, Tensor bn_w, Tensor bn_b, Tensor bn_mean, Tensor bn_var, "
        "float bn_eps, Tensor convh_w, Tensor convh_b, Tensor convw_w, Tensor convw_b, Tensor? yin) -> Tensor");
  m.def("a2_fwd(Tensor x, int num_areas, int num_heads, Tensor proj_w, Tensor proj_b, Tensor ln_w, Tensor ln_b, "
        "float ln_eps, Tensor in_w, Tensor in_b, Tensor? mo_w, Tensor? mo_b, Tensor op_w, Tensor op_b, "
        "Tensor? prep=None) -> Tensor");
  m.def("a2_prep(Tensor x, int num_areas, int num_heads, Tensor proj_w, Tensor ln_w, Tensor ln_b, Tensor in_w, "
        "Tensor in_b) -> Tensor");
  m.def("swin_fwd(Tensor x, int num_heads, int window, Tensor dw_w, Tensor ln1_w, Tensor ln1_b, float ln1_eps, "
        "Tensor in_w, Tensor in_b, Tensor out_w, Tensor out_b, Tensor ln2_w, Tensor ln2_b, float ln2_eps, "
        "Tensor m1_w, Tensor m1_b, Tensor m2_w, Tensor m2_b, Tensor pw_w, Tensor bn_w, Tensor bn_b, Tensor bn_mean, "
        "Tensor bn_var, float bn_eps) -> Tensor");
  m.def("swin_prep(Tensor x, int num_heads, Tensor ln1_w, Tensor ln1_b, Tensor in_w, Tensor in_b, Tensor out_w, "
        "Tensor ln2_w, Tensor ln2_b, Tensor m1_w, Tensor m1_b, Tensor m2_w, Tensor pw_w, Tensor bn_w, Tensor bn_b, "
        "Tensor bn_mean, Tensor bn_var, float bn_eps) -> Tensor");
  m.def("swin_fwd_prepared(Tensor x, Tensor prep, int num_heads, int window, Tensor dw_w, float ln1_eps, "
        "Tensor out_b, float ln2_eps, int hid, Tensor m2_b) -> Tensor");
  m.def("detect_head_fwd(Tensor[] box_feats, Tensor[] cls_feats, Tensor[] box_w, Tensor[] box_b, Tensor[] cls_w, "
        "Tensor[] cls_b, float[] strides, int nc, int reg_max) -> Tensor");
  m.def("detect_head_into(Tensor(a!) y, int l0, int l1, Tensor[] box_feats, Tensor[] cls_feats, Tensor[] box_w, "
        "Tensor[] box_b, Tensor[] cls_w, Tensor[] cls_b, float[] strides, int nc, int reg_max) -> ()");
  m.def("detect_decode_fwd(Tensor[] maps, float[] strides, int nc, int reg_max) -> Tensor");
  m.def("nms_batched(Tensor(a!) pred, float conf_thres, float iou_thres, Tensor? classes, bool agnostic, "
        "bool multi_label, int max_det, int max_nms, float max_wh, bool in_place=True) -> (Tensor, Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(yolosod, CUDA, m) {
  m.impl("se_fwd", se_fwd);
  m.impl("cbam_fwd", cbam_fwd);
  m.impl("ca_fwd", ca_fwd);
  m.impl("a2_fwd", a2_fwd);
  m.impl("a2_prep", a2_prep);
  m.impl("swin_fwd", swin_fwd);
  m.impl("swin_prep", swin_prep);
  m.impl("swin_fwd_prepared", swin_fwd_prepared);
  m.impl("detect_head_fwd", detect_head_fwd);
  m.impl("detect_head_into", detect_head_into);
  m.impl("detect_decode_fwd", detect_decode_fwd);
  m.impl("nms_batched", nms_batched);
}

TORCH_LIBRARY_IMPL(yolosod, Meta, m) {
  m.impl("se_fwd", [](const Tensor& x, const Tensor&, const Tensor&, const Tensor&, const Tensor&,
                      const c10::optional<Tensor>&) { return mafn_meta(x); });
  m.impl("cbam_fwd", [](const Tensor& x, const Tensor&, const Tensor&, const Tensor&, const c10::optional<Tensor>&,
                        const c10::optional<Tensor>&) { return mafn_meta(x); });
  m.impl("ca_fwd", [](const Tensor& x, const Tensor&, const Tensor&, const Tensor&, const Tensor&, const Tensor&,
                      const Tensor&, double, const Tensor&, const Tensor&, const Tensor&, const Tensor&,
                      const c10::optional<Tensor>&) { return mafn_meta(x); });
  m.impl("a2_fwd", [](const Tensor& x, int64_t, int64_t, const Tensor&, const Tensor&, const Tensor&, const Tensor&,
                      double, const Tensor&, const Tensor&, const c10::optional<Tensor>&, const c10::optional<Tensor>&,
                      const Tensor&, const Tensor&, const c10::optional<Tensor>&) { return mafn_meta(x); });
  m.impl("swin_fwd", [](const Tensor& x, int64_t, int64_t, const Tensor&, const Tensor&, const Tensor&, double,
                        const Tensor&, const Tensor&, const Tensor&, const Tensor&, const Tensor&, const Tensor&, double,
                        const Tensor&, const Tensor&, const Tensor&, const Tensor&, const Tensor&, const Tensor&,
                        const Tensor&, const Tensor&, const Tensor&, double) { return mafn_meta(x); });
  m.impl("swin_fwd_prepared", [](const Tensor& x, const Tensor&, int64_t, int64_t, const Tensor&, double,
                                 const Tensor&, double, int64_t, const Tensor&) { return mafn_meta(x); });
  m.impl("detect_head_fwd", [](at::TensorList bf, at::TensorList, at::TensorList, at::TensorList, at::TensorList,
                               at::TensorList, at::ArrayRef<double>, int64_t nc, int64_t) {
    int64_t A = 0;
    for (const auto& t : bf) A += t.size(2) * t.size(3);
    return at::empty({bf[0].size(0), 4 + nc, A}, bf[0].options().dtype(at::kFloat));
  });
  m.impl("detect_decode_fwd", [](at::TensorList maps, at::ArrayRef<double>, int64_t nc, int64_t) {
    int64_t A = 0;
    for (const auto& t : maps) A += t.size(2) * t.size(3);
    return at::empty({maps[0].size(0), 4 + nc, A}, maps[0].options().dtype(at::kFloat));
  });
  m.impl("nms_batched", [](const Tensor& pred, double, double, const c10::optional<Tensor>&, bool, bool,
                           int64_t max_det, int64_t, double, bool) {
    const int64_t B = pred.size(0);
    auto f = pred.options();
    return std::make_tuple(at::empty({B, max_det, 6}, f), at::empty({B}, f.dtype(at::kInt)),
                           at::empty({B, max_det}, f.dtype(at::kInt)));
  });
}
