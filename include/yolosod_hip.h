/*
 * yolosod_hip.h - C ABI of the MI355X (gfx950) hot path of YOLO-SOD inference.
 *
 * Library: yolo-sod_amd/lib/libyolosod_hip.so  (built by `python -m yolosod_amd.build` / __graft_entry__.build()).
 *
 * Conventions (every entry point):
 *   - all tensor arguments are DEVICE pointers to contiguous fp32 (or int32) buffers in the reference's layout
 *     (NCHW feature maps, PyTorch Linear/Conv weight layouts), allocated and owned by the caller;
 *   - `workspace` is a caller-owned device buffer of at least yolosod_<op>_workspace(...) bytes;
 *   - `stream` is a hipStream_t; launches are stream-ordered, nothing synchronises the host;
 *   - return 0 on success, nonzero on error (message in yolosod_last_error(), thread-local).
 *   - outputs never alias inputs, except yolosod_nms with in_place=1 which rewrites pred[:, 0:4] to xyxy,
 *     mirroring non_max_suppression(in_place=True).
 *
 * Each entry point replaces one reference interface (quitedob/yolo-sod, file:line):
 */
#ifndef YOLOSOD_HIP_H
#define YOLOSOD_HIP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

int yolosod_abi_version(void);
const char* yolosod_last_error(void);
/* Per-device state (the split-range flag word), allocated and zeroed eagerly; idempotent. Call once per device before
 * the first launch on it (and before any stream capture): a launch on a device never initialised allocates the state
 * itself, synchronously. Returns 0, or < 0 on error. The current device is restored. */
int yolosod_init(int device);

/* SE / SE_Block.forward            ultralytics/nn/modules/smallobj_modules.py:84-92
 * y = x * sigmoid(fc2(relu(fc1(mean_hw(x)))));  fc1: [hidden,C]+[hidden], fc2: [C,hidden]+[C]. */
size_t yolosod_se_workspace(int B, int C, int H, int W);
int yolosod_se_forward(const float* x, float* y, int B, int C, int H, int W, const float* fc1_w, const float* fc1_b,
                       const float* fc2_w, const float* fc2_b, int hidden, void* workspace, size_t workspace_bytes,
                       void* stream);

/* CBAM_Block.forward               ultralytics/nn/modules/cbam_block.py:52-55 (ChannelAttention :19-23,
 * SpatialAttention :32-37).  fc0: [hidden,C] (channel_attention.fc.0), fc2: [C,hidden] (fc.2), sa_w: [1,2,7,7]. */
size_t yolosod_cbam_workspace(int B, int C, int H, int W);
int yolosod_cbam_forward(const float* x, float* y, int B, int C, int H, int W, const float* fc0_w,
                         const float* fc2_w, int hidden, const float* sa_w, void* workspace, size_t workspace_bytes,
                         void* stream);

/* CA_Block.forward                 ultralytics/nn/modules/ca_block.py:38-59 (bn1 in eval mode, not fused). */
size_t yolosod_ca_workspace(int B, int C, int H, int W);
int yolosod_ca_forward(const float* x, float* y, int B, int C, int H, int W, const float* conv1_w,
                       const float* conv1_b, int mip, const float* bn_w, const float* bn_b, const float* bn_mean,
                       const float* bn_var, float bn_eps, const float* convh_w, const float* convh_b,
                       const float* convw_w, const float* convw_b, void* workspace, size_t workspace_bytes,
                       void* stream);

/* A2_Attn.forward (Conv layers in fused form, nn/tasks.py:227-255)   ultralytics/nn/modules/a2_attn.py:35-69
 * proj / oproj: [C,C] fused conv weight + bias (SiLU), MHA: in_proj [3C,C]+[3C], out_proj [C,C]+[C]. */
size_t yolosod_a2_workspace(int B, int C, int H, int W, int num_areas);
int yolosod_a2_forward(const float* x, float* y, int B, int C, int H, int W, int num_areas, int num_heads,
                       const float* proj_w, const float* proj_b, const float* ln_w, const float* ln_b, float ln_eps,
                       const float* in_proj_w, const float* in_proj_b, const float* mha_out_w,
                       const float* mha_out_b, const float* oproj_w, const float* oproj_b, void* workspace,
                       size_t workspace_bytes, void* stream);
/* The fused LN -> QKV -> attention kernel of the fp16-split path (csrc/a2_fused.hip; head dim 64, areas * W <= 160)
 * and the proj + SiLU + pooling kernel (area groups whose rows fit 400 pixels; any sequence length) take the weights
 * prepared once: yolosod_a2_prep_bytes (0 = the shape takes neither fused kernel), yolosod_a2_prepare (in_proj with the LayerNorm affine folded and the
 * BN-folded proj conv, split into fp16 planes; re-run when one of them changes), yolosod_a2_forward_prepared (the forward of yolosod_a2_forward with the pre-multiplied output
 * weights, on that block; the workspace is yolosod_a2_workspace). yolosod_a2_forward prepares per call instead. */
size_t yolosod_a2_prep_bytes(int C, int num_heads, int num_areas, int W);
int yolosod_a2_prepare(int C, const float* proj_w, const float* ln_w, const float* ln_b, const float* in_proj_w,
                       const float* in_proj_b, void* prep, size_t prep_bytes, void* stream);
int yolosod_a2_forward_prepared(const float* x, float* y, int B, int C, int H, int W, int num_areas, int num_heads,
                                const float* proj_w, const float* proj_b, const float* ln_w, const float* ln_b,
                                float ln_eps, const float* in_proj_w, const float* in_proj_b, const float* oproj_w,
                                const float* oproj_b, const void* prep, size_t prep_bytes, void* workspace,
                                size_t workspace_bytes, void* stream);

/* SwinBlock.forward                ultralytics/nn/modules/blocks_transformer.py:150-171 (WindowAttention
 * :100-131, window_partition :8-47, window_reverse :49-79).  dw: [C,1,3,3]; in_proj [3C,C]; mlp1 [hid,C];
 * mlp2 [C,hid]; pw [C,C,1,1]; bn in eval mode (not fused by fuse()). */
size_t yolosod_swin_workspace(int B, int C, int H, int W, int window, int mlp_hidden);
/* heads-aware query: small when the fused per-window kernel handles the shape (C in {32,64,128}, <=49 tokens) */
size_t yolosod_swin_workspace_v2(int B, int C, int H, int W, int num_heads, int window, int mlp_hidden);
int yolosod_swin_forward(const float* x, float* y, int B, int C, int H, int W, int num_heads, int window,
                         const float* dw_w, const float* ln1_w, const float* ln1_b, float ln1_eps,
                         const float* in_proj_w, const float* in_proj_b, const float* out_proj_w,
                         const float* out_proj_b, const float* ln2_w, const float* ln2_b, float ln2_eps,
                         const float* mlp1_w, const float* mlp1_b, int mlp_hidden, const float* mlp2_w,
                         const float* mlp2_b, const float* pw_w, const float* bn_w, const float* bn_b,
                         const float* bn_mean, const float* bn_var, float bn_eps, void* workspace,
                         size_t workspace_bytes, void* stream);
/* The same forward with the parameter preparation (weight split into fp16 planes with the LayerNorm affines folded,
 * BN fold) done once by the caller and kept across calls, for the shapes of the fp16-split kernels (7x7 windows,
 * C = 64 / 2 heads and C = 256 / 4 heads, mlp_hidden = 2C): yolosod_swin_prep_bytes returns the block's size (0 when
 * (C, heads, hidden) has no such kernel), yolosod_swin_prepare fills a caller-owned block from the parameters of
 * yolosod_swin_forward (re-run it whenever a parameter changes), yolosod_swin_forward_prepared runs the block with a
 * caller-owned scratch of yolosod_swin_prepared_workspace bytes (C = 64: T after the attention residual, token-major,
 * between the attention kernel and the token-tiled MLP kernel). The block also keeps the weights' split-range result,
 * which every forward on it reports again (yolosod_split_range_flag). One image's C*H*W must stay below 2^30. */
size_t yolosod_swin_prep_bytes(int C, int num_heads, int mlp_hidden);
size_t yolosod_swin_prepared_workspace(int B, int C, int H, int W, int num_heads, int window, int mlp_hidden);
int yolosod_swin_prepare(int C, int num_heads, int mlp_hidden, const float* ln1_w, const float* ln1_b,
                         const float* in_proj_w, const float* in_proj_b, const float* out_proj_w, const float* ln2_w,
                         const float* ln2_b, const float* mlp1_w, const float* mlp1_b, const float* mlp2_w,
                         const float* pw_w, const float* bn_w, const float* bn_b, const float* bn_mean,
                         const float* bn_var, float bn_eps, void* prep, size_t prep_bytes, void* stream);
int yolosod_swin_forward_prepared(const float* x, float* y, int B, int C, int H, int W, int num_heads, int window,
                                  const float* dw_w, float ln1_eps, const float* out_proj_b, float ln2_eps,
                                  int mlp_hidden, const float* mlp2_b, const void* prep, size_t prep_bytes,
                                  void* workspace, size_t workspace_bytes, void* stream);

/* Producer-side statistics for the channel gates (SE smallobj_modules.py:87, CBAM cbam_block.py:14-17): a conv
 * epilogue that also writes its output's per-plane partial sums (+ maxes when pmax != NULL) in the segmentation
 * yolosod_plane_parts returns (parts per plane, floats per part), and SE / CBAM entry points that take them instead
 * of re-reading x (bitwise the same gate inputs up to summation order). */
int yolosod_plane_parts(long HW, long* seg);
int yolosod_bias_act_stats(const float* y, long y_bstride, float* out, long out_bstride, const float* bias,
                           const float* res, long res_bstride, int B, int C, long HW, int act, int parts, long seg,
                           float* psum, float* pmax, void* stream);
int yolosod_se_forward_pre(const float* x, float* y, int B, int C, int H, int W, const float* fc1_w,
                           const float* fc1_b, const float* fc2_w, const float* fc2_b, int hidden, const float* psum,
                           void* workspace, size_t workspace_bytes, void* stream);
int yolosod_cbam_forward_pre(const float* x, float* y, int B, int C, int H, int W, const float* fc0_w,
                             const float* fc2_w, int hidden, const float* sa_w, const float* psum, const float* pmax,
                             void* workspace, size_t workspace_bytes, void* stream);
/* CA_Block (ca_block.py:43-44): the producing conv's epilogue also writes the pooled row means (over W) and column
 * means (over H) of its output, yin[B][C][H+W]; the CA entry point then runs the gate and the apply pass only.
 * W % 4 == 0, W <= 1024. */
int yolosod_bias_act_capool(const float* y, long y_bstride, float* out, long out_bstride, const float* bias,
                            const float* res, long res_bstride, int B, int C, int H, int W, int act, float* yin,
                            void* stream);
/* Nearest 2x upsample (nn.Upsample(None, 2, 'nearest') rows of the neck YAML) of x [B, C, h, w] into a channel
 * slice of the following Concat's buffer (out batch stride in elements): the neck glue's copy, not a hot-path op.
 * elem_bytes 4 (fp32) / 2 (bf16); w % 4 == 0 and 16-byte aligned pointers / strides. */
int yolosod_upsample2x(const void* x, void* out, long out_bstride, int B, int C, int h, int w, int elem_bytes,
                       void* stream);
int yolosod_ca_forward_pre(const float* x, float* y, int B, int C, int H, int W, const float* conv1_w,
                           const float* conv1_b, int mip, const float* bn_w, const float* bn_b, const float* bn_mean,
                           const float* bn_var, float bn_eps, const float* convh_w, const float* convh_b,
                           const float* convw_w, const float* convw_b, const float* yin, void* workspace,
                           size_t workspace_bytes, void* stream);

/* MambaBlock (GLU fallback)        ultralytics/nn/modules/blocks_mamba.py:84-113 (Conv1x1BN, GLUBlock), :198-236
 * (forward without mamba_ssm); arg rule nn/tasks.py:1122-1127 (MambaBlock(c, c_hidden, seq_reduction)).
 * y = x + SiLU(BN_o(W_o . up_nearest(GLU(avg_pool_r(SiLU(BN_i(W_i . x)))))))  with
 * GLU(p) = W_pw2 . SiLU(BN(dw3x3(sigmoid(g) * a))), [a; g] = W_pw1 . p. All BatchNorms in eval form (not folded by
 * the reference's fuse()). x, y: [B, C, H, W]; c_hidden = ch; reduction r >= 1 (pool kernel = stride = r, floor;
 * nearest upsample back to H x W). C and ch multiples of 32. */
size_t yolosod_mamba_glu_workspace(int B, int C, int H, int W, int ch, int reduction);
int yolosod_mamba_glu_forward(const float* x, float* y, int B, int C, int H, int W, int ch, int reduction,
                              const float* in_w, const float* in_bn_w, const float* in_bn_b, const float* in_bn_mean,
                              const float* in_bn_var, float in_bn_eps, const float* pw1_w, const float* dw_w,
                              const float* bn_w, const float* bn_b, const float* bn_mean, const float* bn_var,
                              float bn_eps, const float* pw2_w, const float* out_w, const float* out_bn_w,
                              const float* out_bn_b, const float* out_bn_mean, const float* out_bn_var,
                              float out_bn_eps, void* workspace, size_t workspace_bytes, void* stream);

/* Detect._inference (decode)       ultralytics/nn/modules/head.py:100-131, DFL block.py:79-82,
 * make_anchors / dist2bbox utils/tal.py:333-357.
 * maps: host array of nl device pointers, map i = [B, 4*reg_max+nc, heights[i], widths[i]];
 * y: [B, 4+nc, A] (xywh * stride, sigmoid scores), A = sum_i heights[i]*widths[i]. */
int yolosod_detect_decode(int nl, const float* const* maps, const int* heights, const int* widths,
                          const float* strides, int B, int nc, int reg_max, float* y, void* stream);

/* Detect head tail fused with the decode (head.py:45-48,70 + the decode above): the last 1x1 convs
 * of the box tower (box_w [64][c2], box_b [64]) and class tower (cls_w [nc][c3], cls_b [nc]) applied to the tower
 * features box_feat[i] [B][c2][H_i][W_i], cls_feat[i] [B][c3][H_i][W_i] (fp32 NCHW, contiguous), then DFL /
 * dist2bbox / sigmoid -> y [B][4+nc][A]; the [B][64+nc][H][W] raw maps are never materialised.
 * Supports reg_max 16, c2 64, c3 64 or 128, nc <= 16. */
int yolosod_detect_head(int nl, const float* const* box_feat, const float* const* cls_feat, int c2, int c3,
                        const float* const* box_w, const float* const* box_b, const float* const* cls_w,
                        const float* const* cls_b, const int* heights, const int* widths, const float* strides, int B,
                        int nc, int reg_max, float* y, void* stream);

/* non_max_suppression + torchvision.ops.nms   ultralytics/utils/ops.py:167-316 (nms call :296).
 * pred: [B, 4+nc, A] xywh (rewritten to xyxy in place when in_place); classes: device int32[n_classes] or NULL;
 * out: [B, max_det, 6] rows (x1,y1,x2,y2,conf,cls) in kept order, zero padded; counts: [B];
 * out_index: [B, max_det] anchor index of each kept row (-1 padded). max_det 1..2^20 (the reference has no cap,
 * ops.py:297); the workspace depends on max_det above 1024 (_v2), the original query covers max_det <= 1024. */
size_t yolosod_nms_workspace(int B, int nc, int A, int multi_label);
size_t yolosod_nms_workspace_v2(int B, int nc, int A, int multi_label, int max_det);
int yolosod_nms(float* pred, int B, int nc, int A, float conf_thres, double iou_thres, const int* classes,
                int n_classes, int agnostic, int multi_label, int max_det, int max_nms, float max_wh, int in_place,
                float* out, int* counts, int* out_index, void* workspace, size_t workspace_bytes, void* stream);

/* Conv epilogue for the PyTorch-ROCm backbone convs (not a reference hot-path op; conv.py:37-55 + block.py:343-356
 * + Concat): out[b*out_bstride + c*HW + p] = act(y[b*y_bstride + c*HW + p] + bias[c]) (+ res[...]); act 0 id, 1 SiLU.
 * Writes into channel slices of a concat buffer via out_bstride; in place allowed. */
int yolosod_bias_act(const float* y, long y_bstride, float* out, long out_bstride, const float* bias,
                     const float* res, long res_bstride, int B, int C, long HW, int act, void* stream);

/* yolosod_bias_act that also stores channels [c2lo, C) of the result packed in out2 ([B, C - c2lo, HW], batch
 * stride out2_bstride): C2f's Bottleneck chain (block.py:249-253, :343-356) reads channel slices of the concat
 * buffer, which MIOpen would otherwise make contiguous with a copy pass per Bottleneck. */
int yolosod_bias_act_dual(const float* y, long y_bstride, float* out, long out_bstride, const float* bias,
                          const float* res, long res_bstride, float* out2, long out2_bstride, int c2lo, int B, int C,
                          long HW, int act, void* stream);

/* Detect head tower conv (ultralytics/nn/modules/head.py:43-57, conv.py:37-55): 3x3 / stride 1 /
 * pad 1 conv with 64 outputs + folded-BN bias + SiLU, fp32 NCHW in and out, as an implicit GEMM on fp16 two-term
 * split MFMA (csrc/conv3x3.hip). Replaces torch.nn.functional.conv2d (MIOpen) + the bias / SiLU epilogue for those
 * convs. Cin a multiple of 32 (<= 2048). The weights [64][Cin][3][3] are prepared once per version into a caller-
 * owned block of yolosod_conv3x3_prep_bytes(Cin) bytes (0: unsupported Cin). */
size_t yolosod_conv3x3_prep_bytes(int cin);
int yolosod_conv3x3_prepare(const float* w, int cin, void* prep, size_t prep_bytes, void* stream);
int yolosod_conv3x3_silu(const float* x, float* y, int B, int cin, int H, int W, const float* bias, const void* prep,
                         size_t prep_bytes, void* stream);
/* General form (the neck's C2f Bottleneck convs too): Cout 32 or a multiple of 64 (<= 512); the output image b at
 * y + b*y_bstride (a concat slice), res (or NULL) added after the activation (Bottleneck shortcut); _xs: the input image
 * b at x + b*x_bstride (a channel slice, e.g. of the C2f's own buffer); _ex: contiguous x. */
size_t yolosod_conv3x3_prep_bytes_ex(int cin, int cout);
int yolosod_conv3x3_prepare_ex(const float* w, int cin, int cout, void* prep, size_t prep_bytes, void* stream);
int yolosod_conv3x3_silu_ex(const float* x, float* y, long y_bstride, const float* res, long res_bstride, int B,
                            int cin, int cout, int H, int W, const float* bias, const void* prep, size_t prep_bytes,
                            void* stream);
int yolosod_conv3x3_silu_xs(const float* x, long x_bstride, float* y, long y_bstride, const float* res, long res_bstride,
                            int B, int cin, int cout, int H, int W, const float* bias, const void* prep,
                            size_t prep_bytes, void* stream);

/* Thin fused 1x1 convolution of the backbone (conv.py:37-55 after fuse(), 1x1 case): out = SiLU(W x + bias) (+ res)
 * for Cout in {64, 128}, Cin in {64, 96, 128, 192, 256}, HW % 64 == 0; x / out / res may be channel slices (batch
 * strides, multiples of 4); out2 (optional, NULL) = packed copy of channels [c2lo, Cout). Other shapes: error. */
int yolosod_conv1x1_thin(const float* x, long x_bs, const float* w, const float* bias, float* out, long out_bs,
                         const float* res, long res_bs, float* out2, long out2_bs, int c2lo, int B, int Cin, int Cout,
                         long HW, void* stream);

/* SPPF's pooling pyramid (block.py SPPF: three chained MaxPool2d(5, 1, 2) + torch.cat) in one pass over the concat
 * buffer z [B][4C][H][W] (image b at z + b*z_bstride, images contiguous): channels [C, 4C) <- the 5 / 9 / 13-window max
 * pools (clipped to the image; = the chained pools) of channels [0, C), which cv1 wrote. H*W <= 4096. */
int yolosod_sppf_pool(float* z, long z_bstride, int B, int C, int H, int W, void* stream);

/* yolosod_conv1x1_thin (no res) over a virtual concat [x; x2]: channels [0, k1) from x, [k1, Cin) from x2 (any split);
 * bit-identical to the materialised concat. */
int yolosod_conv1x1_thin_cat(const float* x, long x_bs, const float* x2, long x2_bs, int k1, const float* w,
                             const float* bias, float* out, long out_bs, float* out2, long out2_bs, int c2lo, int B,
                             int Cin, int Cout, long HW, void* stream);

/* yolosod_conv1x1_thin (no res / out2) that also emits the output's per-plane statistics for a following SE / CBAM
 * gate in the psum / pmax[B*Cout*parts] layout of yolosod_se_forward_pre / yolosod_cbam_forward_pre (parts =
 * yolosod_plane_parts(HW); plane total in k = 0, 0 / -inf in k > 0); pmax may be NULL; tile_ws = 2*B*Cout*(HW/64)
 * floats of scratch. */
int yolosod_conv1x1_thin_stats(const float* x, long x_bs, const float* w, const float* bias, float* out, long out_bs,
                               int B, int Cin, int Cout, long HW, int parts, float* psum, float* pmax, float* tile_ws,
                               void* stream);

/* 1x1 convolution (stride 1, groups 1) of the backbone as an fp32 MFMA GEMM with the epilogue fused:
 * out[b*out_bs + m*HW + p] = act(sum_k w[m][k] x[b*x_bs + k*HW + p] + bias[m]) (+ res[...]); Cin % 32 == 0. */
int yolosod_conv1x1(const float* x, long x_bs, const float* w, const float* bias, float* out, long out_bs,
                    const float* res, long res_bs, int B, int Cin, int Cout, long HW, int act, void* stream);

/* Building blocks, exported for unit tests (no single reference interface):
 * C(b,m,n) = act(sum_k A(b,m,k) B(b,k,n) + bias) + res;  A K-contiguous; B K- or N-contiguous. */
int yolosod_gemm_f32(const float* A, long a_bs, int lda, const float* B, long b_bs, int ldb, int b_kcontig, float* C,
                     long c_bs, int ldc, int M, int N, int K, int batch, const float* bias, int bias_mode, int act,
                     const float* res, void* stream);
int yolosod_layernorm(const float* x, float* y, long rows, int C, const float* w, const float* b, float eps,
                      void* stream);
int yolosod_attention(const float* qkv, float* out, long n_seq, int L, int C, int heads, void* stream);

/* Test hook: 1 routes SwinBlock shapes the fused per-window kernel covers (C 64/128, heads 2/4, window <= 7x7,
 * mlp 2C) through it (default), 0 forces the decomposed GEMM path for every shape. */
void yolosod_debug_set_swin_fused(int on);
/* Test hook: 1 (default; env YOLOSOD_SWIN_X3=0 turns it off) routes 7x7-window SwinBlocks with C = 64 / 2 heads and
 * C = 256 / 4 heads through the kernels that run every matrix product as fp16 two-term splits on the fp16 matrix
 * cores at fp32 accuracy (csrc/swin_x3.hip), 0 through the exact-fp32-MFMA fused kernels. */
int yolosod_debug_set_swin_x3(int on);
/* The yolosod_debug_set_* switches that return int return the previous state. */
/* Test hook: pixels per area group of the A2 proj + SiLU + pooling kernel (the launcher takes the fewest area groups
 * whose row bands fit; 208 by default - two workgroups per CU; <= 0 restores 208). Same
 * results for every cap. Returns the previous cap. */
int yolosod_debug_set_a2_pool_px(int px);
/* Test hook: 1 (default; env YOLOSOD_HEAD_X2=0 turns it off) runs the Detect head's 1x1 convs as fp16 two-term
 * splits on the fp16 matrix cores (detect_head_x2_kernel), 0 on the exact fp32 MFMA (detect_head_lds_kernel). */
int yolosod_debug_set_head_x2(int on);
/* Test hooks: A2_Attn's GEMMs as fp16 two-term splits on v_mfma_f32_32x32x16_f16 (1, default; env YOLOSOD_A2_X2=0
 * turns it off) or exact fp32 MFMA (0); yolosod_debug_set_gemm_x2(1) makes every yolosod_gemm_f32 / internal fp32 GEMM
 * call take the split products, 0 restores the callers' choice. */
int yolosod_debug_set_a2_x2(int on);
/* Test hook: A2_Attn's split path through the fused kernels (1, default:
 * proj + SiLU + pooling, then LN + QKV + attention, csrc/a2_fused.hip) or the decomposed GEMM path (0). */
int yolosod_debug_set_a2_fused(int on);
/* Test hook: A2_Attn's proj + SiLU + pooling kernel with 128 / 256 output channels per workgroup (1, default)
 * or with 64 (0); returns the previous state. */
int yolosod_debug_set_a2_pool_wide(int on);
/* The SE gate only, sigmoid(fc2(relu(fc1(mean_hw(x)))))   smallobj_modules.py:87-90, into gate [B][C], for a consumer
 * that applies y = x * gate itself (yolosod_conv3x3s2_silu); psum: x's per-plane partial sums from its producer
 * (yolosod_bias_act_stats) or NULL (a statistics pass over x). workspace: yolosod_se_workspace bytes. */
int yolosod_se_gate(const float* x, int B, int C, int H, int W, const float* fc1_w, const float* fc1_b,
                    const float* fc2_w, const float* fc2_b, int hidden, const float* psum, float* gate, void* workspace,
                    size_t workspace_bytes, void* stream);
/* The CBAM gates only   cbam_block.py:14-23,33-37: ca [B][C] and sa [B][H][W] (sa from the channel statistics of
 * x * ca), for a consumer that applies y = (x * ca) * sa itself; psum / pmax from the producer or both NULL.
 * workspace: yolosod_cbam_workspace bytes. */
int yolosod_cbam_gates(const float* x, int B, int C, int H, int W, const float* fc0_w, const float* fc2_w, int hidden,
                       const float* sa_w, const float* psum, const float* pmax, float* ca, float* sa, void* workspace,
                       size_t workspace_bytes, void* stream);
/* 3x3 / stride 2 / pad 1 conv + bias + SiLU with the producing MAFN gate applied while the input is staged
 * (csrc/conv3x3s2.hip): y = SiLU(conv3x3_s2((x * gc) * gp, W) + bias), the consumer Conv of SE_Block L1 (gc = the SE
 * gate, smallobj_modules.py:92) and of CBAM_Block L4 (gc = ca, gp = sa, cbam_block.py:53-54) in the paper YAML, with the
 * gate's output never written. fp16 two-term split MFMA at fp32 accuracy; Cout 64 or 128 (_out: multiples of 128 up to
 * 512 too), Cin a multiple of 32 (<= 2048),
 * Ho = (H + 1) / 2, Wo = (W + 1) / 2 with Wo % 4 == 0; x [B][cin][H][W] (B*cin*H*W*4 < 2^32), gc [B][cin] 16-byte
 * aligned or NULL, gp [B][H][W] or NULL, y [B][cout][Ho][Wo]. Weights prepared once per parameter version into a
 * caller-owned block of yolosod_conv3x3s2_prep_bytes(cin, cout) bytes (0: unsupported). Replaces the gate's apply pass
 * + torch.nn.functional.conv2d (MIOpen) + the bias / SiLU epilogue. */
size_t yolosod_conv3x3s2_prep_bytes(int cin, int cout);
int yolosod_conv3x3s2_prepare(const float* w, int cin, int cout, void* prep, size_t prep_bytes, void* stream);
int yolosod_conv3x3s2_silu(const float* x, float* y, int B, int cin, int cout, int H, int W, const float* bias,
                           const float* gc, const float* gp, const void* prep, size_t prep_bytes, void* stream);
/* The same with image b's output [cout][Ho][Wo] at y + b * y_bstride (y_bstride >= cout*Ho*Wo, a multiple of 4, y
 * 16-byte aligned): a channel slice of a concat buffer (nn/tasks.py concat elision). Cout may also be any multiple of
 * 128 up to 512 (the PAN neck's stride-2 convs, layers 29 / 33 / 36 of the paper YAML). */
int yolosod_conv3x3s2_silu_out(const float* x, float* y, long y_bstride, int B, int cin, int cout, int H, int W,
                               const float* bias, const float* gc, const float* gp, const void* prep,
                               size_t prep_bytes, void* stream);
/* 1x1 / stride 1 conv + bias + SiLU on the fp16 two-term split MFMA at fp32 accuracy (csrc/conv1x1x2.hip): the PAN
 * neck's wide 1x1 convs (C2f cv1 / cv2, lateral convs; conv.py:37-55, block.py:249-253). Cout a multiple of 128 (<= 1024),
 * Cin a multiple of 32 (<= 4096, weights padded to 128), HW % 4 == 0. x image b at x + b*x_bstride ([cin][HW]); y image
 * b at y + b*y_bstride ([cout][HW], a concat slice when the stride is larger); y2 (or NULL): channels [c2lo, cout)
 * stored again at y2 + b*y2_bstride (C2f's first Bottleneck input). Replaces MIOpen's fp32 GEMM + the bias / SiLU pass. */
size_t yolosod_conv1x1x2_prep_bytes(int cin, int cout);
int yolosod_conv1x1x2_prepare(const float* w, int cin, int cout, void* prep, size_t prep_bytes, void* stream);
int yolosod_conv1x1x2_silu(const float* x, long x_bstride, float* y, long y_bstride, float* y2, long y2_bstride,
                           int c2lo, int B, int cin, int cout, int HW, const float* bias, const void* prep,
                           size_t prep_bytes, void* stream);
/* The same over a virtual concat [x; x2] (block.py:249-253: the C2f cv1 after a neck Concat): channels [0, k1) from x
 * (image b at x + b*x_bstride), [k1, cin) from x2 (image b at x2 + b*x2_bstride), k1 a multiple of 128; x2 NULL:
 * yolosod_conv1x1x2_silu. Bit-identical to the materialised concat. */
int yolosod_conv1x1x2_silu_cat(const float* x, long x_bstride, const float* x2, long x2_bstride, int k1, float* y,
                               long y_bstride, float* y2, long y2_bstride, int c2lo, int B, int cin, int cout, int HW,
                               const float* bias, const void* prep, size_t prep_bytes, void* stream);
/* Timing hook: ablation variants of the stride-2 conv kernel at Cout 64 with a channel gate (csrc/conv3x3s2.hip; WRONG
 * results for abl != 0 - scripts/bench_conv3x3s2.py only). Returns the previous value. */
int yolosod_debug_set_conv3x3s2_abl(int abl);
/* Timing hook: ablation variants of the 3x3 conv kernel (csrc/conv3x3.hip; WRONG results for any abl != 0 and
 * != 16 - scripts/bench_conv3x3.py only). Returns the previous value. */
int yolosod_debug_set_conv3x3_abl(int abl);
void yolosod_debug_set_gemm_x2(int on);
/* Test hook: the bf16 decomposed SwinBlock's depthwise conv + token layout and LN1 in one pass
 * (swin_tokens_ln_bf16_kernel, 1, default) or as two kernels (0);
 * bit-identical. Returns the previous state. */
int yolosod_debug_set_swin_tokln(int on);
/* Test hook: the fp16 two-term split of the fp32-accurate matrix kernels (common.h split2) on npair pairs of v:
 * h[i] = the fp16 pair (fp16(v[2i]), fp16(v[2i+1])), l[i] = (fp16(v[2i] - h.lo), fp16(v[2i+1] - h.hi)), as 2 x 16-bit
 * patterns per uint32 (low half = even element). Device pointers. */
int yolosod_debug_split_f16(const float* v, uint32_t* h, uint32_t* l, long npair, void* stream);
/* Split-range guard of the fp32-accurate fp16-split kernels (Swin x3 / wx and their weight preparation, Detect head
 * x2, the X2 GEMMs): fp16 represents |v| < 65520 only, so every split site records the largest magnitude it split and
 * a kernel that saw one beyond 65504 (or a NaN) sets the current device's flag word. Returns 1 if set since the last
 * reset, 0 if not, < 0 on error; synchronises `stream` first; reset != 0 clears it. A caller that sees 1 redoes the
 * work on the exact-fp32-MFMA kernels (the yolosod_debug_set_*(0) switches; DetectionPredictor does). */
int yolosod_split_range_flag(int reset, void* stream);

/* ---------------------------------------------------------------------------------------------------------------
 * bf16 model config (BASELINE configs[4]): `model.to(torch.bfloat16)` after fuse() - AutoBackend's fp16
 * route (autobackend.py:145-156, predictor im.half()) with bfloat16. Activations (x, y, res, out2, tower features)
 * and the GEMM weights of Swin / A2 are bf16 bit patterns (uint16_t, torch.bfloat16 layout); every other parameter,
 * the statistics / partials and Detect's output are fp32. Arithmetic is fp32 (bf16 MFMA with fp32 accumulation for
 * the GEMMs and attention); each stored tensor is rounded once (nearest even). Same argument meaning and workspace
 * queries as the fp32 entry points above unless noted.
 * ------------------------------------------------------------------------------------------------------------- */
#include <stdint.h>

/* SE (smallobj_modules.py:84-92); psum = producer partials (yolosod_bias_act_stats_bf16) or NULL. */
int yolosod_se_forward_bf16(const uint16_t* x, uint16_t* y, int B, int C, int H, int W, const float* fc1_w,
                            const float* fc1_b, const float* fc2_w, const float* fc2_b, int hidden, const float* psum,
                            void* workspace, size_t workspace_bytes, void* stream);
/* CBAM (cbam_block.py:52-55); psum / pmax both NULL or both the producer's partials. */
int yolosod_cbam_forward_bf16(const uint16_t* x, uint16_t* y, int B, int C, int H, int W, const float* fc0_w,
                              const float* fc2_w, int hidden, const float* sa_w, const float* psum, const float* pmax,
                              void* workspace, size_t workspace_bytes, void* stream);
/* CA (ca_block.py:38-59); yin = producer's pooled means (yolosod_bias_act_capool_bf16) or NULL. */
int yolosod_ca_forward_bf16(const uint16_t* x, uint16_t* y, int B, int C, int H, int W, const float* conv1_w,
                            const float* conv1_b, int mip, const float* bn_w, const float* bn_b, const float* bn_mean,
                            const float* bn_var, float bn_eps, const float* convh_w, const float* convh_b,
                            const float* convw_w, const float* convw_b, const float* yin, void* workspace,
                            size_t workspace_bytes, void* stream);
/* SwinBlock.forward (blocks_transformer.py:150-171): in_proj_w [3C][C], out_proj_w [C][C], mlp1_w [hid][C],
 * mlp2_w [C][hid], pw_w [C][C] bf16; C % 64 == 0, head dim 32 / 64 / 128. */
size_t yolosod_swin_workspace_bf16(int B, int C, int H, int W, int num_heads, int window, int mlp_hidden);
int yolosod_swin_forward_bf16(const uint16_t* x, uint16_t* y, int B, int C, int H, int W, int num_heads, int window,
                              const float* dw_w, const float* ln1_w, const float* ln1_b, float ln1_eps,
                              const uint16_t* in_proj_w, const float* in_proj_b, const uint16_t* out_proj_w,
                              const float* out_proj_b, const float* ln2_w, const float* ln2_b, float ln2_eps,
                              const uint16_t* mlp1_w, const float* mlp1_b, int mlp_hidden, const uint16_t* mlp2_w,
                              const float* mlp2_b, const uint16_t* pw_w, const float* bn_w, const float* bn_b,
                              const float* bn_mean, const float* bn_var, float bn_eps, void* workspace,
                              size_t workspace_bytes, void* stream);
/* A2_Attn.forward (a2_attn.py:35-69), residual form, pre-multiplied output weights (oproj_w = Wconv . Wmha,
 * oproj_b = Wconv . bmha + bconv); proj_w / in_proj_w / oproj_w bf16; head dim 32 / 64 / 128, H*W % 8 == 0. */
size_t yolosod_a2_workspace_bf16(int B, int C, int H, int W, int num_areas);
int yolosod_a2_forward_bf16(const uint16_t* x, uint16_t* y, int B, int C, int H, int W, int num_areas, int num_heads,
                            const uint16_t* proj_w, const float* proj_b, const float* ln_w, const float* ln_b,
                            float ln_eps, const uint16_t* in_proj_w, const float* in_proj_b, const uint16_t* oproj_w,
                            const float* oproj_b, void* workspace, size_t workspace_bytes, void* stream);
/* Detect head tail + decode (as yolosod_detect_head) of levels [l0, l1) only, into y laid out for all nl levels
 * (the anchor offsets and A of every level; the other levels' slices of y are not written and their feature
 * pointers not read). bf16 != 0: bf16 tower features (uint16_t patterns). Lets a caller decode the levels whose
 * tower convolutions are done while the last level's still run (head.py:70 per level + _inference :100-131). */
int yolosod_detect_head_levels(int nl, int l0, int l1, const void* const* box_feat, const void* const* cls_feat, int c2,
                               int c3, const float* const* box_w, const float* const* box_b, const float* const* cls_w,
                               const float* const* cls_b, const int* heights, const int* widths, const float* strides,
                               int B, int nc, int reg_max, float* y, int bf16, void* stream);
/* Detect head tail + decode (as yolosod_detect_head) on bf16 tower features; weights, biases and y fp32. */
int yolosod_detect_head_bf16(int nl, const uint16_t* const* box_feat, const uint16_t* const* cls_feat, int c2, int c3,
                             const float* const* box_w, const float* const* box_b, const float* const* cls_w,
                             const float* const* cls_b, const int* heights, const int* widths, const float* strides,
                             int B, int nc, int reg_max, float* y, void* stream);
/* Conv epilogues on bf16 maps (yolosod_bias_act / _dual / _stats / _capool); out2 NULL = no second store. The
 * statistics are fp32 sums / maxes / means of the stored (rounded) values. */
int yolosod_bias_act_bf16(const uint16_t* y, long y_bstride, uint16_t* out, long out_bstride, const float* bias,
                          const uint16_t* res, long res_bstride, uint16_t* out2, long out2_bstride, int c2lo, int B,
                          int C, long HW, int act, void* stream);
int yolosod_bias_act_stats_bf16(const uint16_t* y, long y_bstride, uint16_t* out, long out_bstride, const float* bias,
                                const uint16_t* res, long res_bstride, int B, int C, long HW, int act, int parts,
                                long seg, float* psum, float* pmax, void* stream);
int yolosod_bias_act_capool_bf16(const uint16_t* y, long y_bstride, uint16_t* out, long out_bstride,
                                 const float* bias, const uint16_t* res, long res_bstride, int B, int C, int H, int W,
                                 int act, float* yin, void* stream);
/* Test hooks: bf16 GEMM (bf16 out, fp32 accumulation; K % 64 == 0) and attention over contiguous sequences. */
int yolosod_gemm_bf16(const uint16_t* A, long a_bs, int lda, const uint16_t* B, long b_bs, int ldb, int b_kcontig,
                      uint16_t* C, long c_bs, int ldc, int M, int N, int K, int batch, const float* bias,
                      int bias_mode, int act, const uint16_t* res, void* stream);
int yolosod_attention_bf16(const uint16_t* qkv, uint16_t* out, long n_seq, int L, int C, int heads, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* YOLOSOD_HIP_H */
