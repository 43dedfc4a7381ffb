/*
 * rn.h -- C-ABI of the MI355X-native ResNet/ResNeXt training runtime (librn.so).
 *
 * This is the drop-in boundary that replaces the MXNet runtime (libmxnet.so of the
 * huangzehao/incubator-mxnet-bk fork) underneath the reference's Python training harness.
 * The reference never calls a C API directly: every op below replaces what MXNet ran for
 * one `mx.sym.<Op>` node of the reference graphs (symbol/resnet.py, symbol/resnext.py,
 * symbol/resnet_int8.py) when core/solver.py drove Module.forward / backward / update.
 * The `mxnet` shim shipped in resnet.mxnet_amd/mxnet binds these entry points with ctypes
 * (resnet.mxnet_amd/rn/lib.py); INTEGRATION.md shows the binding.
 *
 * Conventions
 *  - Every entry returns 0 on success and -1 on failure; rn_last_error() returns the
 *    thread-local message (mirrors MXNet's `-1` + MXGetLastError C-API convention).
 *  - No entry point allocates device memory or synchronises: all work is enqueued on the
 *    caller's HIP stream (`rn_stream_t` = hipStream_t), so a caller may capture it in a graph.
 *  - Activations are NHWC ("rows" = N*H*W pixels, channel-contiguous) with the channel
 *    stride padded to a multiple of 8 elements; weights are KRSC (fwd) / CRSK (dgrad).
 *  - dtype: RN_BF16 (bf16 storage, fp32 accumulate) or RN_F32 (exact fp32 MFMA path,
 *    used for parity runs). Parameters, gradients, BN statistics are always fp32.
 */
#ifndef RN_H_
#define RN_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* rn_stream_t; /* hipStream_t */

enum rn_dtype { RN_BF16 = 0, RN_F32 = 1 };

/* ---------------------------------------------------------------------------------------
 * Convolution / FullyConnected (implicit GEMM on MFMA).
 * Replaces mx.sym.Convolution (symbol/resnet.py:14-31,93; symbol/resnext.py:17-38,83) and
 * mx.sym.FullyConnected (symbol/resnet.py:115) = a 1x1 convolution over a 1x1 image.
 * ------------------------------------------------------------------------------------- */
typedef struct rn_conv_desc {
  int32_t dtype;                  /* rn_dtype of x, w (compute copy), y                     */
  int32_t n, h, w;                /* input batch and spatial size                             */
  int32_t c;                      /* input channel STRIDE (multiple of 8)                     */
  int32_t c_real;                 /* logical input channels (<= c)                            */
  int32_t k;                      /* output channels (num_filter / num_hidden)                */
  int32_t k_pad;                  /* output channel stride (multiple of 8, >= k)              */
  int32_t r, s;                   /* kernel height, width                                     */
  int32_t stride_h, stride_w;
  int32_t pad_h, pad_w;
  int32_t groups;                 /* num_group (ResNeXt grouped conv)                         */
  int32_t p, q;                   /* output spatial size, filled by rn_conv_desc_init         */
  int32_t grouped_direct;         /* filled by rn_conv_desc_init: 1 = this grouped 3x3 runs the
                                     direct v_dot2 kernels with compact weight copies (see
                                     rn_conv_pack_numel); fixed for the descriptor's lifetime    */
} rn_conv_desc;

/* Validate and fill p, q (MXNet 'valid' convention: p = (h + 2*pad - r)/stride + 1). */
int rn_conv_desc_init(rn_conv_desc* d);

/* y[n,p,q,k] = sum_{r,s,c} x[n,p*sh-ph+r,q*sw-pw+s,c] * w[k,r,s,c] (+ bias[k]) (+ add_src)
 * w: compute copy, KRSC, channel stride c. y_dtype lets the FC head write fp32 logits.
 * add_src (may alias y, or NULL) implements the residual `conv3 + shortcut` and req='add'. */
int rn_conv_fwd(const rn_conv_desc* d, const void* x, const void* w_krsc, void* y, int32_t y_dtype,
                const void* add_src, const float* bias, rn_stream_t stream);

/* rn_conv_fwd that also emits the BatchNorm statistics of y for a following BatchNorm in
 * training mode (saves the statistics pass over y): part = float[rn_conv_bnstats_blocks(d)][3][k_pad]
 * per-block partials (S1, S2, pivot), consumed by rn_bn_fwd_train_part with rows_blk = 128. */
int rn_conv_fwd_bnstats(const rn_conv_desc* d, const void* x, const void* w_krsc, void* y, int32_t y_dtype,
                        const void* add_src, const float* bias, float* part, rn_stream_t stream);
int64_t rn_conv_bnstats_blocks(const rn_conv_desc* d);
/* Rows each BatchNorm partial block of the conv kernel covers (mode 0 fwd / 1 dgrad): 128, or half
 * the tile rows of the 256/224-row tiles. rn_bn_fwd_train_part's rows_blk. */
int32_t rn_conv_bn_part_rows(const rn_conv_desc* d, int32_t mode);
/* Kernel variant the bf16 forward (mode 0, plain: no bias / input transform) or data-gradient
 * (mode 1) of `d` runs: the column count of its 256-row tile (256, 128 or 64), or 0 for the
 * 128-row kernel. Lets a caller enable the BatchNorm epilogue fusions only where they pay (the
 * 64-column tile has none: with a fused epilogue those layers run the 128-row kernel). */
int32_t rn_conv_tile(const rn_conv_desc* d, int32_t mode);
/* Int8 forward of a quantized convolution (resnet_int8 / attach_quantize_node graphs: conv over
 * Quantization_int8(data) and Quantization_int8(weight), symbol/int8_api.py:120-151). x_codes /
 * w_codes are the int8 codes (value = code * unit; NHWC / KRSC, channel stride d->c bytes, a multiple
 * of 16) and x_unit / w_unit device pointers to the per-tensor units: y = unit_x * unit_w * sum of
 * int8 products, accumulated exactly in int32 by v_mfma_i32_16x16x64_i8 (+ add_src), stored as
 * y_dtype. part (nullable): the BatchNorm statistics partials of y as rn_conv_fwd_bnstats, with
 * rn_conv_bn_part_rows(d, 2) rows per block; rn_conv_tile(d, 2) is this kernel's tile columns. */
int rn_conv_fwd_i8(const rn_conv_desc* d, const void* x_codes, const void* w_codes, void* y, int32_t y_dtype,
                   const void* add_src, const float* x_unit, const float* w_unit, float* part,
                   rn_stream_t stream);
/* rn_conv_fwd_i8 that also writes part_mm[block][k_pad]: per channel, the max of the stored output
 * over the rows of each BatchNorm partial block -- the MIN where mm_sign[channel] < 0 (mm_sign
 * nullable: the max everywhere; the consuming BatchNorm's gamma, whose sign is its scale's) -- part
 * required, blocks of rn_conv_bn_part_rows(d, 2) rows: what rn_bn_desc.xmm reads. */
int rn_conv_fwd_i8_mm(const rn_conv_desc* d, const void* x_codes, const void* w_codes, void* y, int32_t y_dtype,
                      const void* add_src, const float* x_unit, const float* w_unit, float* part, float* part_mm,
                      const float* mm_sign, rn_stream_t stream);
/* w_codes[k][r][s][c] = round(w[k][r][s][c] / unit) (int8, zero for c >= c_real): the int8 compute
 * copy of a per-tensor quantized weight from the fp32 master (unit from rn_quant_int8_fwd_codes). */
int rn_conv_weight_pack_i8(const rn_conv_desc* d, const float* w_master, const float* unit, void* w_codes,
                           rn_stream_t stream);

/* rn_conv_bwd_data that also reduces the BatchNorm+ReLU backward of the BN whose output gradient
 * this call completes (dx here = d(bn output), bn_x = the BN input, bn_mean / bn_scale / bn_shift =
 * its saved mean and the scale/shift of its forward): part[rn_conv_bnred_blocks(d)][c][2] receives
 * per-output-block (sum dz, sum dz*(x - mean)), dz = dx * [bn_x*scale + shift > 0] (relu != 0);
 * rn_bn_bwd_part then finishes the BN backward without its own reduction pass over x and dy.
 * dx = NULL (no add_src; the 224/256-row tile): the reduction only, nothing is stored (the first
 * pass of rn_conv_bwd_data_bnapply's recompute). */
int rn_conv_bwd_data_bnred(const rn_conv_desc* d, const void* dy, const void* w_crsk, void* dx, const void* add_src,
                           const void* bn_x, const float* bn_mean, const float* bn_scale, const float* bn_shift,
                           int32_t relu, float* part, rn_stream_t stream);
/* rn_conv_bwd_data_bnred whose BN output feeds a Quantization_int8 (rn_bn_desc.clip): the reduction's
 * dz also carries the quantizer's straight-through clip, dz = dx * [y > 0] * [y < *clip]. */
int rn_conv_bwd_data_bnred_clip(const rn_conv_desc* d, const void* dy, const void* w_crsk, void* dx,
                                const void* add_src, const void* bn_x, const float* bn_mean, const float* bn_scale,
                                const float* bn_shift, int32_t relu, const float* clip, float* part,
                                rn_stream_t stream);
/* A stage-first unit's act1 read by two Quantization_int8 (symbol/resnet_int8.py: conv1's and the
 * shortcut's, each with its own threshold): the later of the two data gradients writes dx = bf16(
 * [y < *clip] * bf16(its gradient) + [y < *clip2] * other), y = bf16(bn_x * scale + shift) -- both
 * straight-through clips, as rn_bn_bwd forms them from rn_bn_desc.dy / dy2 -- and reduces the BN+ReLU
 * backward from it (part, as rn_conv_bwd_data_bnred); the BN then runs rn_bn_bwd_part on dx with no clip.
 * other: the first quantizer's stored gradient (read only). bf16, dense, an LDS-DMA tile. */
int rn_conv_bwd_data_bnred_clip2(const rn_conv_desc* d, const void* dy, const void* w_crsk, void* dx,
                                 const void* other, const void* bn_x, const float* bn_mean, const float* bn_scale,
                                 const float* bn_shift, const float* clip, const float* clip2, float* part,
                                 rn_stream_t stream);
/* The BatchNorm(+ReLU) backward of the BN whose output gradient this convolution's data gradient is,
 * APPLIED in the epilogue to the recomputed gradient: dx = A (dz - mean(dz)) - A2 (x - mean)
 * (+ add_src), dz = g relu'(x scale + shift) (relu != 0), g = conv_transpose(dy, w) rounded as
 * rn_conv_bwd_data would store it, coef from rn_bn_bwd_finalize over the partials of a
 * reduction-only rn_conv_bwd_data_bnred (dx = NULL) of the same convolution. Bit-identical to
 * rn_conv_bwd_data + rn_bn_bwd_part. For cheap data gradients (a 1x1 convolution whose input has
 * more channels than its output, the pre-activation units' conv1, symbol/resnet.py:17-20): the
 * BN-width gradient is never written nor read back. bf16, the 224/256-row tile (rn_conv_tile(d, 1)
 * >= 128). */
int rn_conv_bwd_data_bnapply(const rn_conv_desc* d, const void* dy, const void* w_crsk, void* dx,
                             const void* add_src, const void* bn_x, const float* coef, const float* bn_scale,
                             const float* bn_shift, int32_t relu, rn_stream_t stream);
int64_t rn_conv_bnred_blocks(const rn_conv_desc* d);

/* rn_conv_fwd whose input is the PRE-BatchNorm tensor of a BatchNorm+ReLU (pre-activation
 * units, symbol/resnet.py:17-31): the kernel stages max(x*in_scale[c] + in_shift[c], 0) (the
 * coefficients rn_bn_fwd_train / rn_bn_fwd_infer computed), so the BN+ReLU output is never
 * written. in_scale/in_shift nullable (plain conv); part: as rn_conv_fwd_bnstats, nullable. */
int rn_conv_fwd_x(const rn_conv_desc* d, const void* x, const void* w_krsc, void* y, int32_t y_dtype,
                  const void* add_src, const float* bias, const float* in_scale, const float* in_shift,
                  float* part, rn_stream_t stream);

/* dx = conv_transpose(dy, w) (+ add_src). w_crsk is the CRSK re-layout made by
 * rn_conv_weight_pack (row count c, K stride k_pad). */
int rn_conv_bwd_data(const rn_conv_desc* d, const void* dy, const void* w_crsk, void* dx,
                     const void* add_src, rn_stream_t stream);

/* dw_krsc (fp32, KRSC with channel stride c_real/groups, see rn_conv_weight_numel) += x^T * dy.
 * Accumulates with fp32 atomics: the caller zeroes dw once per step. */
int rn_conv_bwd_filter(const rn_conv_desc* d, const void* x, const void* dy, float* dw,
                       rn_stream_t stream);

/* rn_conv_bwd_filter with a workspace for the split-M partial tiles: the large-tile LDS-DMA kernels
 * store each split's tile into ws (no atomics) and a reduction pass adds the splits into dw.
 * rn_conv_wgrad_ws_bytes(d) = the bytes that takes (0: this conv's kernel adds with atomics);
 * a smaller ws falls back to the atomic epilogue. ws: 16-byte aligned, device memory. */
int64_t rn_conv_wgrad_ws_bytes(const rn_conv_desc* d);
int rn_conv_bwd_filter_ws(const rn_conv_desc* d, const void* x, const void* dy, float* dw, void* ws,
                          int64_t ws_bytes, rn_stream_t stream);
/* The weight gradient of an int8 convolution (symbol/resnet_int8.py: Quantization_int8 on the data, then
 * Convolution; MXNet's backward multiplies dy by the fake-quantized values x = unit * code) from the
 * input's int8 codes (x_codes: NHWC, c channels, as rn_quant_int8_fwd_codes* write them) and its unit
 * (x_unit: one fp32, device): dw += *x_unit * sum dy * code -- the codes widened to bf16 exactly, the
 * unit applied once per tile, so the bf16 fake-quantized values need not exist. On the streaming
 * 1x1 kernel and the 128 / 256-column LDS-DMA tiles: rn_conv_wgrad_i8_supported(d) = 1 where this applies
 * (bf16, dense, c % 16 == 0, c_real == c; a 1x1 stride-1 conv with K, C in {64, 128, 256}, K x C <= 32768,
 * or > 64 output channels and columns -- not stage 1's 3x3 image-band shape); ws as rn_conv_bwd_filter_ws,
 * sized by rn_conv_wgrad_i8_ws_bytes(d) (-1 where unsupported). */
int32_t rn_conv_wgrad_i8_supported(const rn_conv_desc* d);
int64_t rn_conv_wgrad_i8_ws_bytes(const rn_conv_desc* d);
int rn_conv_bwd_filter_i8(const rn_conv_desc* d, const void* x_codes, const float* x_unit, const void* dy, float* dw,
                          void* ws, int64_t ws_bytes, rn_stream_t stream);
/* rn_conv_bwd_filter_ws over the same BN+ReLU-on-load input as rn_conv_fwd_x (x = the BatchNorm
 * input; the 1x1 convolutions run the LDS-DMA tiles with the transform on their B fragments). */
int rn_conv_bwd_filter_x(const rn_conv_desc* d, const void* x, const void* dy, float* dw, const float* in_scale,
                         const float* in_shift, void* ws, int64_t ws_bytes, rn_stream_t stream);

/* Number of fp32 elements of the master weight (K x R x S x c_real/groups, KRSC). */
int64_t rn_conv_weight_numel(const rn_conv_desc* d);

#define RN_GROUP_BLOCK 64
/* Elements of the compute copy written by rn_conv_weight_pack: which = 0 (w_krsc) or 1 (w_crsk). */
int64_t rn_conv_pack_numel(const rn_conv_desc* d, int32_t which);

/* From the fp32 KRSC master weight, write the compute copies: w_krsc (dtype, channel stride
 * c) and w_crsk (dtype, c rows, K stride k_pad). Either output may be NULL.
 * Grouped (groups > 1, symbol/resnext.py:23-25 num_group=32): the copies are block-diagonal
 * over RN_GROUP_BLOCK-wide column blocks -- for output column j the reduction runs over the
 * channels of the groups that j's 64-column block touches, zero outside j's own group
 * (w_krsc: [k][r][s][cblk], w_crsk: [c][r][s][kblk]); sizes from rn_conv_pack_numel.
 * Except where the direct grouped kernel runs (bf16, 3x3 pad 1, c = k, 4 channels per group at
 * stride 1 or 2, or 8 per group at stride 2 -- forward and data gradient; d->grouped_direct, which
 * rn_conv_desc_init sets from rn_set_tuning 15 at that time): that
 * mode's copy is compact, [c/8][tap][8][G] with G = c/groups -- w_krsc[k/8][tap][k%8][c'] =
 * w[k][tap][c'], w_crsk[c/8][tap][c%8][k'] = w[g*G + k'][8 - tap][c - g*G], g = c/G -- and
 * rn_conv_fwd / rn_conv_bwd_data multiply it with v_dot2_f32_bf16 (no bias, statistics or BN fusions). */
int rn_conv_weight_pack(const rn_conv_desc* d, const float* w_master, void* w_krsc, void* w_crsk,
                        rn_stream_t stream);
/* rn_conv_weight_pack for count layers (host arrays: descs[i], w_masters[i], w_krsc[i], w_crsk[i],
 * the last two nullable): the grouped layers' copies in one launch per 32 copies (the grouped
 * weights are repacked after every update -- a ResNeXt-50 step's 33 separate launches were ~6 us
 * each on its critical path), dense layers through rn_conv_weight_pack. Same bytes as per layer;
 * the grouped layers of one call share a dtype. */
int rn_conv_weight_pack_multi(const rn_conv_desc* descs, const float* const* w_masters, void* const* w_krsc,
                              void* const* w_crsk, int32_t count, rn_stream_t stream);

/* Stem: explicit im2col of an NCHW fp32 image (the `data` input, train.py:70-73) with an
 * optional per-channel affine (bn_data, symbol/resnet.py:90) into cols[m][kc] (dtype),
 * kc = round_up(r*s*c_real, 32). conv0 then runs as a 1x1 conv over cols. */
int rn_im2col_nchw(const rn_conv_desc* d, const float* x_nchw, const float* scale,
                   const float* shift, void* cols, int32_t kc, rn_stream_t stream);

/* Quantized stem (symbol/resnet_int8.py:96-98, int8_api.py:133-136): conv0 reads
 * Quantization_int8(bn_data(x)). Updates the activation minmax state (EMA of max|affine(x)|,
 * when is_train) and writes the im2col matrix of the fake-quantized affine input.
 * ws: >= 2 floats. */
int rn_im2col_nchw_quant(const rn_conv_desc* d, const float* x_nchw, const float* scale,
                         const float* shift, float* minmax, int32_t is_train, float ema_decay,
                         int32_t first_batch, int32_t nbits, float* ws, void* cols, int32_t kc,
                         rn_stream_t stream);
/* The activation STE zeroes the gradient of clipped inputs (|affine(x)| >= minmax):
 * dbeta[c] -= sum over clipped (n,c,h,w) of (conv0 data-gradient), with w_q the fp32 KRSC
 * quantized weight conv0 ran with. Run after rn_stem_shift_grad. Limits: c_real <= 8, k <= 64 and
 * a multiple of 4, at most 4 x 4 taps per input pixel, x and dy 16-byte aligned. */
int rn_stem_quant_clip_grad(const rn_conv_desc* d, const float* x_nchw, const float* scale,
                            const float* shift, const float* minmax, const void* dy, const float* w_q,
                            float* dbeta, rn_stream_t stream);
/* The same clip gradient as a weight gradient (bf16 NHWC-8 stem image x8, 2 * c_real <= 8): dbeta[c]
 * -= sum_{k,r,s} w_q[k,r,s,c] * D[k,r,s,c], D = the stem convolution's weight gradient over the clip
 * mask of channel c (1 where !(-t < x*scale + shift < t) on the fp32 input, t = *minmax).
 * rn_stem_clip_mask writes the masks into x8's channels c_real .. 2 c_real - 1 (after the forward read
 * x8; rn_stem_prepare rewrites them to zero next step); rn_stem_clip_wgrad computes the weight
 * gradient over the real and mask channels into ext (float[k * r * s * 2 c_real], zeroed here),
 * dw += its real part (ws / ws_bytes: the slab workspace, rn_stem_clip_wgrad_ws_bytes);
 * rn_stem_clip_dbeta subtracts the mask part's dot product from dbeta (after rn_stem_shift_grad).
 * rn_stem_clip_supported: 1 where these apply. */
int32_t rn_stem_clip_supported(const rn_conv_desc* d);
int rn_stem_clip_mask(const rn_conv_desc* d, const float* x_nchw, const float* scale, const float* shift,
                      const float* minmax, void* x8, rn_stream_t stream);
int64_t rn_stem_clip_wgrad_ws_bytes(const rn_conv_desc* d);
int rn_stem_clip_wgrad(const rn_conv_desc* d, const void* x8, const void* dy, float* dw, float* ext, void* ws,
                       int64_t ws_bytes, rn_stream_t stream);
/* rn_stem_clip_wgrad over one image chunk (d, x8, dy: the chunk's descriptor and rows): ext is zeroed by
 * the first chunk (first = 1), every chunk adds its weight gradient into ext, and the last (last = 1)
 * adds the real part into dw -- so each chunk's gradient starts as soon as its rows of the stem's
 * BatchNorm backward are applied (rn_bn_bwd_apply_rows), on the weight-gradient stream. */
int rn_stem_clip_wgrad_chunk(const rn_conv_desc* d, const void* x8, const void* dy, float* dw, float* ext, void* ws,
                             int64_t ws_bytes, int32_t first, int32_t last, rn_stream_t stream);
int rn_stem_clip_dbeta(const rn_conv_desc* d, const float* ext, const float* w_q, float* dbeta,
                       rn_stream_t stream);

/* d(beta) of a BN feeding the stem conv, without the stem dgrad:
 * dbeta[c] += sum_{k,r,s} w[k,r,s,c] * sum_{n,p,q valid(r,s)} dy[n,p,q,k].
 * ws: float workspace of p*q*k_pad + p*s*k + k*r*s elements. */
int rn_stem_shift_grad(const rn_conv_desc* d, const void* dy, const float* w_master, float* dbeta,
                       float* ws, rn_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * BatchNorm (+ fused ReLU) -- replaces mx.sym.BatchNorm + mx.sym.Activation('relu')
 * (symbol/resnet.py:12-23,90-96,111-112).
 * ------------------------------------------------------------------------------------- */
typedef struct rn_bn_desc {
  int32_t dtype;     /* dtype of x / y / dy / dx                              */
  int64_t m;         /* rows = N*H*W                                          */
  int32_t c;         /* channel stride (multiple of 8)                        */
  int32_t c_real;    /* channels that carry parameters                        */
  float eps;
  float momentum;    /* moving = moving*momentum + batch*(1-momentum)         */
  int32_t fix_gamma; /* gamma := 1, dgamma := 0                                */
  int32_t relu;      /* fuse Activation(relu) on the output                   */
  /* nullable (backward only, with relu): device pointer to the threshold t of the Quantization_int8
   * that alone consumes this BN's output (the int8 graph, symbol/resnet_int8.py via int8_api.py:
   * 133-136). Its straight-through backward (clip_grad_quantization_int8.py: zero where |y| >= t) is
   * folded into this BN's backward: dz = dy * [y > 0] * [y < t], y = the output as stored. */
  const float* clip;
  /* nullable (rn_bn_bwd / rn_bn_bwd_global only, with relu and clip): a SECOND Quantization_int8 of
   * this BN's output (symbol/resnet_int8.py: a stage's first unit quantizes act1 for conv1 and for
   * the shortcut conv, each with its own threshold), its threshold and its output gradient. Both
   * straight-through backwards fold in: dz = [y > 0] * round(dy * [y < *clip] + dy2 * [y < *clip2]),
   * round = to the storage type, as two rn_quant_int8_bwd calls summing into one buffer store it. */
  const float* clip2;
  const void* dy2;
  /* nullable (rn_quant_int8_fwd_codes_bn[2] with relu only): per-block per-channel extremes of x,
   * [xmm_blocks][c], from the producing int8 convolution's epilogue (rn_conv_fwd_i8_mm with mm_sign =
   * this BN's gamma): the max where scale >= 0, else the min. y = relu(x*scale + shift) is monotone in
   * x per channel, so the quantizers' max|y| comes from these instead of a pass over x; bit-identical. */
  const float* xmm;
  int64_t xmm_blocks;
} rn_bn_desc;

/* Workspace (bytes) needed by rn_bn_fwd_train / rn_bn_bwd. */
int64_t rn_bn_workspace_bytes(const rn_bn_desc* d);

/* Training forward: batch stats (biased variance), moving-stat update, y = act(x*scale+shift).
 * save_mean/save_invstd/scale/shift are fp32 [c_real] outputs kept for backward.
 * y may be NULL (stats only). */
int rn_bn_fwd_train(const rn_bn_desc* d, const void* x, void* y, const float* gamma,
                    const float* beta, float* moving_mean, float* moving_var, float* save_mean,
                    float* save_invstd, float* scale, float* shift, void* ws, rn_stream_t stream);

/* Inference forward with moving statistics (use_global_stats / is_train=False). */
/* Stem input: conv0 reads bn_data(data) (symbol/resnet.py:90-93, fix_gamma BatchNorm over the
 * NCHW fp32 batch). Writes the NHWC-8 compute copy out[n*h*w][8] (d->dtype; channels >= c are 0)
 * of the normalised input. mode 0: batch statistics (training; moving stats updated, save_* and
 * scale/shift written); 1: moving statistics (inference / use_global_stats); 2: no BatchNorm.
 * d: dtype, m = n*h*w, c = 8, c_real = c, eps, momentum, fix_gamma. ws: 2*c*256 floats. */
int rn_stem_prepare(const rn_bn_desc* d, const float* x_nchw, int32_t n, int32_t c, int32_t h, int32_t w, void* out,
                    int32_t mode, const float* gamma, const float* beta, float* moving_mean, float* moving_var,
                    float* save_mean, float* save_invstd, float* scale, float* shift, void* ws, rn_stream_t stream);
/* The same as the zero-bordered NHWC4 image out[n][h + ph][w + pw][4] of hp x wp pixels (bf16; the
 * caller zeroes the border once) that the padded-NHWC4 stem path reads. */
int rn_stem_prepare_p4(const rn_bn_desc* d, const float* x_nchw, int32_t n, int32_t c, int32_t h, int32_t w,
                       void* out, int32_t hp, int32_t wp, int32_t ph, int32_t pw, int32_t mode,
                       const float* gamma, const float* beta, float* moving_mean, float* moving_var,
                       float* save_mean, float* save_invstd, float* scale, float* shift, void* ws,
                       rn_stream_t stream);
/* conv0 over that image (bf16, c_real <= 4, k <= 64, r, s <= 8): the reduction runs over
 * k = (r * 8 + s) * 4 + c (rows and taps padded to 8, channels to 4: 256 instead of the NHWC-8
 * layout's r * s * 8), with no in-image tests (the border is zero). d: the conv0 descriptor
 * (c = 8 as for rn_stem_prepare, c_real = 3); hp >= (p-1)*stride_h + 8, wp >= (q-1)*stride_w + 8.
 * w4: [k][8][8][4] from rn_stem_weight_pack_p4 (master [k][r][s][c_real] fp32).
 * rn_stem_conv_wgrad_p4 ADDS dW into dw ([k][r][s][c_real] fp32). */
int32_t rn_stem_p4_supported(const rn_conv_desc* d, int32_t hp, int32_t wp);
int rn_stem_weight_pack_p4(const rn_conv_desc* d, const float* w_master, void* w4, rn_stream_t stream);
int rn_stem_conv_fwd_p4(const rn_conv_desc* d, const void* x4, const void* w4, void* y, int32_t hp, int32_t wp,
                        rn_stream_t stream);
/* rn_stem_conv_fwd_p4 that also emits the statistics of y for the BatchNorm after the stem (bn0,
 * symbol/resnet.py:94): part = float[rn_stem_bnstats_blocks(d, hp, wp)][3][64] (S1, S2, pivot per block, as
 * rn_conv_fwd_bnstats), each block n*p*q / blocks rows, consumed by rn_bn_fwd_train_part with ld = 64.
 * rn_stem_bnstats_blocks returns 0 where the band kernel cannot give every block the same rows (then the
 * call is refused: run the statistics pass). */
int rn_stem_conv_fwd_p4_bnstats(const rn_conv_desc* d, const void* x4, const void* w4, void* y, int32_t hp,
                                int32_t wp, float* part, rn_stream_t stream);
int64_t rn_stem_bnstats_blocks(const rn_conv_desc* d, int32_t hp, int32_t wp);
int rn_stem_conv_wgrad_p4(const rn_conv_desc* d, const void* x4, const void* dy, float* dw, int32_t hp,
                          int32_t wp, rn_stream_t stream);

/* rn_bn_fwd_train with the batch statistics already reduced per row block by the producer
 * (rn_conv_fwd_bnstats): fp64 merge of part[nblk][3][ld] -> coefficients, moving stats, then
 * y = bn(x) (+relu) when y != NULL. ws: rn_bn_workspace_bytes(d) (rows_blk = 128). */
int rn_bn_fwd_train_part(const rn_bn_desc* d, const float* part, int64_t nblk, int32_t rows_blk, int32_t ld,
                         const void* x, void* y, const float* gamma, const float* beta, float* moving_mean,
                         float* moving_var, float* save_mean, float* save_invstd, float* scale, float* shift,
                         void* ws, rn_stream_t stream);
/* rn_bn_bwd with the reduction already done by the producer of dy (rn_conv_bwd_data_bnred):
 * finalize over part[nrb][c][2], then dx = BN-backward(dy) (+ add_src). ws: >= 4*c floats + 16 B. */
int rn_bn_bwd_part(const rn_bn_desc* d, const float* part, int64_t nrb, const void* x, const void* dy, void* dx,
                   const void* add_src, const float* gamma, const float* save_mean, const float* save_invstd,
                   const float* scale, const float* shift, float* dgamma, float* dbeta, void* ws,
                   rn_stream_t stream);
/* The finalize half of rn_bn_bwd_part: dgamma / dbeta and coef[c][4] = {A = gamma*invstd, mean(dz),
 * A2 = gamma*invstd^2*sum(dz*xhat)/m, mean} (16-byte aligned), from which dx = A (dz - mean(dz)) -
 * A2 (x - mean) (+ add). For rn_conv_bwd_data_bnapply. */
int rn_bn_bwd_finalize(const rn_bn_desc* d, const float* part, int64_t nrb, const float* gamma,
                       const float* save_mean, const float* save_invstd, float* dgamma, float* dbeta, float* coef,
                       rn_stream_t stream);
int rn_bn_fwd_infer(const rn_bn_desc* d, const void* x, void* y, const float* gamma,
                    const float* beta, const float* moving_mean, const float* moving_var,
                    float* scale, float* shift, rn_stream_t stream);

/* The post-activation unit tail (symbol/resnext.py:40-47, symbol/resnet.py:63-74):
 * y = act(bf16(xa*scale_a + shift_a) + b), b = bf16(xb*scale_b + shift_b) (the shortcut's
 * BatchNorm) or, with scale_b = shift_b = NULL, xb itself; each BatchNorm output rounded to the
 * storage type as rn_bn_apply stores it, so the result equals rn_bn_apply + rn_eltwise_add bit for
 * bit while the BatchNorm outputs are never written. act = ReLU when relu != 0. */
int rn_bn_apply_add(const rn_bn_desc* d, const void* xa, const float* scale_a, const float* shift_a,
                    const void* xb, const float* scale_b, const float* shift_b, void* y, int32_t relu,
                    rn_stream_t stream);
/* Its backward: g = dy * [y > 0] (the ReLU after the add) written once, and in the same pass the
 * backward reductions of the BatchNorm(s) feeding the add: part_a[nrb][c][2] = {sum g,
 * sum g*(xa - mean_a)} per row block (and part_b for xb / mean_b, the shortcut's BN; or all three
 * NULL), nrb = rn_bn_reduce_blocks(d); rn_bn_bwd_part(d, part, nrb, x, g, ...) finalizes and applies. */
int64_t rn_bn_reduce_blocks(const rn_bn_desc* d);
int rn_relu_bwd_bnred(const rn_bn_desc* d, const void* y, const void* dy, void* g, const void* xa,
                      const float* mean_a, float* part_a, const void* xb, const float* mean_b, float* part_b,
                      rn_stream_t stream);
/* Apply y = act(x*scale + shift) with precomputed per-channel scale/shift. */
int rn_bn_apply(const rn_bn_desc* d, const void* x, void* y, const float* scale,
                const float* shift, rn_stream_t stream);

/* Backward through [relu o] BN: dz = relu ? dy*(x*scale+shift > 0) : dy,
 * dgamma = sum(dz*xhat) (0 if fix_gamma), dbeta = sum(dz),
 * dx = gamma*invstd*(dz - mean(dz) - xhat*mean(dz*xhat)) (+ add_src). dgamma/dbeta written. */
int rn_bn_bwd(const rn_bn_desc* d, const void* x, const void* dy, void* dx, const void* add_src,
              const float* gamma, const float* save_mean, const float* save_invstd,
              const float* scale, const float* shift, float* dgamma, float* dbeta, void* ws,
              rn_stream_t stream);
/* dx rows [row0, row0 + rows) of rn_bn_bwd, from the coefficients an rn_bn_bwd call with dx = NULL
 * (reductions and dgamma/dbeta only) left in ws -- same d, x, dy, ws. Lets a consumer of dx start on
 * the first rows while later ones are applied (the stem: its weight gradient per image chunk on the
 * side stream). Bit-identical to rn_bn_bwd's dx. row0 * c a multiple of 16 bytes; no dy2. */
int rn_bn_bwd_apply_rows(const rn_bn_desc* d, const void* x, const void* dy, void* dx, const void* add_src,
                         const float* scale, const float* shift, const void* ws, int64_t row0, int64_t rows,
                         rn_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * Pooling -- mx.sym.Pooling (symbol/resnet.py:97 max 3x3/s2/p1; :113 global avg).
 * ------------------------------------------------------------------------------------- */
enum rn_pool_type { RN_POOL_MAX = 0, RN_POOL_AVG = 1 };
typedef struct rn_pool_desc {
  int32_t dtype;
  int32_t n, h, w, c;   /* c = channel stride */
  int32_t r, s, stride_h, stride_w, pad_h, pad_w;
  int32_t type;         /* rn_pool_type */
  int32_t global_pool;  /* ignores r/s/stride/pad like MXNet */
  int32_t p, q;         /* filled by rn_pool_desc_init */
} rn_pool_desc;
int rn_pool_desc_init(rn_pool_desc* d);
/* argmax: uint8 tap index per output element (max pool only; may be NULL for avg). */
int rn_pool_fwd(const rn_pool_desc* d, const void* x, void* y, uint8_t* argmax, rn_stream_t stream);
/* rn_pool_fwd over the output of the producing BatchNorm+ReLU (the stem's bn0 -> relu0 -> pool0 and the
 * final bn1 -> relu1 -> global pool, symbol/resnet.py:94-97,111-113), applied while loading: x = the BN
 * input, each element max(x * in_scale + in_shift, 0) rounded to the storage type as rn_bn_apply stores it,
 * so y and argmax are bit-identical to rn_bn_apply followed by rn_pool_fwd, and the activation is never
 * written or read back. */
int rn_pool_fwd_x(const rn_pool_desc* d, const void* x, void* y, uint8_t* argmax, const float* in_scale,
                  const float* in_shift, rn_stream_t stream);
int rn_pool_bwd(const rn_pool_desc* d, const void* dy, const uint8_t* argmax, void* dx,
                const void* add_src, rn_stream_t stream);
/* rn_pool_bwd that also reduces the backward of the BatchNorm(+ReLU) whose output the pool read (the
 * stem's bn0 -> relu0 -> pool0, symbol/resnet.py:94-97), as rn_conv_bwd_data_bnred does: dx here =
 * d(bn output), bn_x = the BN input; part[rn_pool_bwd_bnred_blocks(d)][c][2] receives per-block
 * (sum dz, sum dz*(x - mean)), dz = dx * [bn_x*scale + shift > 0] (relu != 0) on the stored dx, for
 * rn_bn_bwd_part. bf16, the 3x3 / stride-2 / pad-1 max pool with H = 2P and W = 2Q, c / 8 dividing 256. */
int rn_pool_bwd_bnred(const rn_pool_desc* d, const void* dy, const uint8_t* argmax, void* dx,
                      const void* add_src, const void* bn_x, const float* bn_mean, const float* bn_scale,
                      const float* bn_shift, int32_t relu, float* part, rn_stream_t stream);
/* Partial blocks of rn_pool_bwd_bnred for d; 0 where it does not apply. */
int64_t rn_pool_bwd_bnred_blocks(const rn_pool_desc* d);

/* ---------------------------------------------------------------------------------------
 * SoftmaxOutput -- mx.sym.SoftmaxOutput (symbol/resnet.py:118-120): forward = probabilities,
 * backward = grad_scale*(p - onehot(label)) with normalization 'null'. Also accumulates
 * stats[0] += sum CE loss, stats[1] += top-1 hits, stats[2] += top-5 hits (device side,
 * so the metric does not force a host sync every step).
 * ------------------------------------------------------------------------------------- */
int rn_softmax_output(int32_t grad_dtype, int32_t batch, int32_t ncls, int32_t ld,
                      const float* logits, const float* label, float* prob, void* dlogits,
                      float grad_scale, float* stats, rn_stream_t stream);

/* out[j] (=|+=) sum_i x[i*ld + j], j < c  (FullyConnected bias gradient). */
int rn_col_sum(int32_t dtype, int64_t m, int32_t c, int32_t ld, const void* x, float* out,
               int32_t accumulate, rn_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * Optimizer -- MXNet SGD momentum (train.py:186-194, core/solver.py:80-82):
 *   g = rescale_grad*grad (clipped if clip > 0);  mom = momentum*mom - lr*(g + wd*w);  w += mom
 * over a flat fp32 parameter buffer described by a per-tensor table in device memory
 * (offset, numel, wd). lr may be taken from a device scalar (lr_dev != NULL) so that a
 * captured graph can replay with a schedule.  w_lowp (optional, dtype lowp_dtype) receives
 * the updated weights in the compute precision.
 * ------------------------------------------------------------------------------------- */
int rn_sgd_mom_update(int32_t ntensors, const int64_t* offsets, const int64_t* numels,
                      const float* wds, float* w, const float* g, float* mom, void* w_lowp,
                      int32_t lowp_dtype, float lr, const float* lr_dev, float momentum,
                      float rescale_grad, float clip, rn_stream_t stream);

/* Compute copies of one parameter tensor written by rn_sgd_mom_update_pack (layouts of
 * rn_conv_weight_pack, dense convolutions / FullyConnected only). krsc == NULL: plain tensor. */
typedef struct rn_wpack {
  void* krsc;     /* [k][rs][c] copy (channel stride c), or NULL                          */
  void* crsk;     /* [c][rs][kpad] copy, or NULL                                          */
  int32_t k, rs;  /* output channels, taps                                                */
  int32_t creal;  /* input channels of the master tensor ([k][rs][creal])                */
  int32_t c;      /* channel stride of the KRSC copy                                      */
  int32_t kpad;   /* output-channel stride of the CRSK copy                               */
  int32_t pad_;
} rn_wpack;

/* rn_sgd_mom_update fused with the weight packs: the same update, and for every tensor whose
 * `packs` entry (device table, ntensors entries) names copies, the updated weight written to
 * them in lowp_dtype -- replaces rn_sgd_mom_update + one rn_conv_weight_pack per layer.
 * work: device table of nwork int32x4 items, one workgroup each: {tensor, start, 0, 0} = the
 * 4096 elements from `start` of a tensor without a CRSK copy; {tensor, k0, tap, c0} = the
 * 64 x 64 (k, c) tile of one tap of a tensor with one (rn_sgd_pack_work builds the table). */
int rn_sgd_mom_update_pack(int32_t ntensors, const int64_t* offsets, const int64_t* numels,
                           const float* wds, float* w, const float* g, float* mom,
                           const rn_wpack* packs, const int32_t* work, int32_t nwork,
                           int32_t lowp_dtype, float lr, const float* lr_dev, float momentum,
                           float rescale_grad, float clip, rn_stream_t stream);
/* Host helper: fills `work` (host memory, capacity max_items x 4) for the tensors described by
 * numels / packs (host copies); returns the item count, or -1 if max_items is too small. */
int32_t rn_sgd_pack_work(int32_t ntensors, const int64_t* numels, const rn_wpack* packs, int32_t* work,
                         int32_t max_items);

/* ---------------------------------------------------------------------------------------
 * Data movement helpers.
 * ------------------------------------------------------------------------------------- */
/* Backward through [relu o] BN with GLOBAL statistics (use_global_stats=True; config.fix_bn ->
 * core/graph_optimize.py:114-157 fix_bn, train.py:106-109): the forward normalised with the moving
 * statistics (rn_bn_fwd_infer wrote scale/shift), which are constants: dz as in rn_bn_bwd,
 * dgamma = sum(dz*xhat) (0 if fix_gamma), dbeta = sum(dz), dx = gamma/sqrt(moving_var+eps)*dz
 * (+ add_src), xhat = (x - moving_mean)/sqrt(moving_var+eps). Moving statistics are not updated. */
int rn_bn_bwd_global(const rn_bn_desc* d, const void* x, const void* dy, void* dx, const void* add_src,
                     const float* gamma, const float* moving_mean, const float* moving_var,
                     const float* scale, const float* shift, float* dgamma, float* dbeta, void* ws,
                     rn_stream_t stream);
/* NCHW fp32 -> NHWC dtype with channel stride c_pad (zero padding). */
int rn_nchw_to_nhwc(int32_t n, int32_t c, int32_t h, int32_t w, int32_t c_pad, const float* src,
                    void* dst, int32_t dst_dtype, rn_stream_t stream);
/* Element-wise cast between fp32 and bf16 (n elements). */
int rn_cast(int64_t n, const void* src, int32_t src_dtype, void* dst, int32_t dst_dtype,
            rn_stream_t stream);
/* dst = act(a + b) (b may be NULL: dst = act(a)); act = relu if relu != 0. Residual
 * `bn3 + shortcut` (+ Activation) of the post-activation graphs (symbol/resnext.py:45-46,
 * symbol/resnet.py:70-74) and the unfused elementwise add. dst may alias a or b. */
int rn_eltwise_add(int64_t n, int32_t dtype, const void* a, const void* b, void* dst, int32_t relu,
                   rn_stream_t stream);
/* dx = dy * (y > 0) (+ add_src): Activation('relu') backward from its output. */
int rn_relu_bwd(int64_t n, int32_t dtype, const void* y, const void* dy, void* dx,
                const void* add_src, rn_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * Int8 fake quantization -- mx.sym.contrib.Quantization_int8 (symbol/int8_api.py:133-136),
 * semantics from symbol/quant_ops.py:12-42 / clip_grad_quantization_int8.py:14-67.
 * ------------------------------------------------------------------------------------- */
/* out = round(clip(x, -t, t) / (t/qmax)) * (t/qmax) with t = max|x| (weights) or the EMA
 * minmax state (activations, updated in place when is_train). ws: >= 4096 floats whose ws[0] is
 * zero on entry (a zeroed buffer; every quantizer call leaves it zero, so one workspace serves all). */
int rn_quant_int8_fwd(int32_t dtype, int64_t n, const void* x, void* out, float* minmax,
                      int32_t is_weight, int32_t is_train, float ema_decay, int32_t first_batch,
                      int32_t nbits, float* ws, rn_stream_t stream);
/* rn_quant_int8_fwd that also writes the int8 codes round(clip(x)/unit) (codes nullable: values
 * only; n a multiple of 16 when set) and unit[0] = t/qmax (kept for the int8 convolution; nbits <= 8).
 * out (nullable when codes is set) gets the fake-quantized values as rn_quant_int8_fwd. */
int rn_quant_int8_fwd_codes(int32_t dtype, int64_t n, const void* x, void* out, void* codes, float* unit,
                            float* minmax, int32_t is_weight, int32_t is_train, float ema_decay,
                            int32_t first_batch, int32_t nbits, float* ws, rn_stream_t stream);
/* The activation Quantization_int8 of a BatchNorm(+ReLU) output that only the quantizer reads
 * (symbol/resnet_int8.py's bn -> relu -> Quantization_int8 -> conv), the BatchNorm applied on load:
 * y = [relu](x*scale + shift) (d->relu) rounded to d->dtype as rn_bn_apply stores it, then
 * rn_quant_int8_fwd_codes(y) with is_weight = 0 -- bit-identical to that pair, but y is never
 * written nor re-read. scale / shift from rn_bn_fwd_train[_part] / rn_bn_fwd_infer with y = NULL;
 * d->c a multiple of 16; codes required, out nullable (codes only: the values are expanded where
 * they are read, by rn_quant_int8_expand -- the int8 graph's weight gradients). */
int rn_quant_int8_fwd_codes_bn(const rn_bn_desc* d, const void* x, const float* scale, const float* shift,
                               void* out, void* codes, float* unit, float* minmax, int32_t is_train,
                               float ema_decay, int32_t first_batch, int32_t nbits, float* ws,
                               rn_stream_t stream);
/* The same for the two quantizers of one BatchNorm output (rn_bn_desc.dy2): one max|y| pass, both
 * threshold states updated from it, one pass writing both quantizers' values and codes. */
int rn_quant_int8_fwd_codes_bn2(const rn_bn_desc* d, const void* x, const float* scale, const float* shift,
                                void* out, void* codes, float* unit, float* minmax, float ema_decay,
                                int32_t nbits, void* out2, void* codes2, float* unit2, float* minmax2,
                                float ema_decay2, int32_t nbits2, int32_t is_train, int32_t first_batch,
                                float* ws, rn_stream_t stream);
/* out[i] = codes[i] * unit[0] rounded to dtype: the fake-quantized values of an activation quantizer
 * from its int8 codes and unit (rn_quant_int8_fwd_codes*), bit-identical to the out those calls write.
 * The int8 graph defers them to the weight-gradient stream, just before the weight gradient that
 * reads them (the forward writes 1 byte per element instead of 3). n a multiple of 16; codes / out
 * 16-byte aligned. */
int rn_quant_int8_expand(int32_t dtype, int64_t n, const void* codes, const float* unit, void* out,
                         rn_stream_t stream);
/* One weight of rn_weight_quant_pack: the fp32 master (KRSC, c_real channels) of a Quantization_int8
 * weight (int8_api.py:131-132, per-tensor threshold t = max|w|) and the copies written from it. */
typedef struct rn_wquant_item {
  const float* master; /* k * rs * c_real fp32                                         */
  float* qw;           /* fake-quantized copy round(w/unit)*unit, unit = t/qmax (required) */
  float* unit;         /* nullable: unit                                                */
  float* minmax;       /* nullable: the threshold state (:= t)                          */
  int8_t* w_codes;     /* nullable: int8 codes, KRSC, channel stride c (rn_conv_weight_pack_i8) */
  void* w_crsk;        /* nullable: data-gradient compute copy of qw, dense CRSK with k_pad
                        * stride (rn_conv_weight_pack's w_crsk), dtype of the call            */
  int32_t k, rs, c_real, c, k_pad, nbits;
} rn_wquant_item;
/* Every weight quantizer of a network in three launches (max|w| of each tensor, the thresholds, the
 * copies) instead of rn_quant_int8_fwd_codes + rn_conv_weight_pack + rn_conv_weight_pack_i8 per
 * weight: bit-identical to those. items: DEVICE array of count entries; ws: >= 2*count floats (the
 * quantizers' shared workspace: the first count are cleared on entry and left zero, whatever the
 * activation quantizers left in them). The padding of w_codes /
 * w_crsk (channels >= c_real, columns >= k) is not written (zero from their first pack). */
int rn_weight_quant_pack(const rn_wquant_item* items, int32_t count, int32_t dtype, float* ws,
                         rn_stream_t stream);
/* STE backward: dx = dy (weights) or dy * (|x| <= t) (activations). */
int rn_quant_int8_bwd(int32_t dtype, int64_t n, const void* x, const void* dy, void* dx,
                      const float* minmax, int32_t is_weight, const void* add_src,
                      rn_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * Runtime.
 * ------------------------------------------------------------------------------------- */
const char* rn_last_error(void);
/* Kernel-variant switches (A/B measurements): 0 = wgrad LDS-DMA staging (default off),
 * 1 = igemm LDS-DMA staging (default off: measured slower), 2 = wgrad split-M target blocks per CU
 * (default: occupancy), 3 = diagnostic build only (RN_DIAG=1; refused by librn.so):
 * igemm A operand from one L1-resident chunk (wrong results; isolates memory latency),
 * 4 = igemm 256-row tiles (0 auto, 1 off, 2 force 256x256, 3 force 256x128, 5 no 256x64),
 * 5 = wgrad variant (0 auto: 128x128 LDS-DMA tiles where K and the column count exceed 64; 1 = 256-column
 *     LDS-DMA tiles, measured slower; 3 = the register-staged kernel only),
 * 6 = diagnostic build only: wgrad skips its dW epilogue (wrong results; isolates the atomic adds),
 * 7 = diagnostic build only: igemm 256-row tile schedule experiments (bit mask; 0 = default; bits 4,
 *     8, 16, 32, 64, 128, 256, 512 drop waits / DMAs / the epilogue / the stores / the epilogue's LDS
 *     staging writes (16x16 tiles) / its BatchNorm partial math / its loads / its staging reads: wrong
 *     results),
 * 8 = igemm 256-row tile MFMA shape (0 = 32x32x16, 1 = 16x16x32),
 * 9 = igemm 224-row tiles for the 256/128-column tiles (0 = on, 1 = 256 rows),
 * 10 = igemm 256-row-family persistent grid: workgroups (a multiple of 8) that walk the tiles of a
 *      larger grid, so one tile's output stores drain while the next tile loads (default 512; 0 = one
 *      tile per workgroup),
 * 11 = the 4-wave one-buffer 224x128 conv tile, two workgroups per CU (0 auto: forward 1x1 layers of
 *      >= 1024 tiles; 1 off; 2 every 1x1 pad-0 conv; 3 one-K-tile forward layers only, the round-4 rule),
 * 12 = 3x3 / stride-2 max-pool backward over 2x2 input blocks (0 = on where H = 2P, W = 2Q; 1 = the
 *      per-pixel gather),
 * 13 = grouped convolutions with equal channels in and out per group (<= 32): skip the MFMAs of the
 *      block-diagonal tile's zero blocks (0 = on, 1 = off),
 * 14 = the same for their bf16 weight gradients (64 x 64 tile: only the two diagonal 32 x 32 blocks,
 *      each wave one of them over half of each M stage; 0 = on, 1 = off, 2 = on, the
 *      diagonal blocks on two of the four waves),
 * 15 = grouped convolutions with 4 channels per group (ResNeXt 32x4d stage 1; 8 per group at
 *      stride 2, stage 2 unit 1): the direct v_dot2 kernels and their weight copies (0 = on, 1 = the block-diagonal
 *      64-column tiles; set it before rn_conv_weight_pack: the copies of the two paths differ),
 * 16 = 1: block barriers around the LDS staging of the 224/256-row tiles' epilogue (default 0: each
 *      wave waits only for its own staged rows; the paired-row BatchNorm-statistics epilogue keeps
 *      its barriers either way),
 * 17 = deterministic weight gradients (1 = on): every M-split of every weight gradient stores its
 *      partial tile into the workspace slab (rn_conv_bwd_filter_ws / _x; rn_conv_wgrad_ws_bytes is
 *      > 0 for every layer then, fp32 included) and one pass sums the splits in a fixed order, instead
 *      of fp32 atomic adds; the FullyConnected forward's split-K atomics are off. Bitwise
 *      run-to-run reproducible steps (the parity tests' mode),
 * 18 = cache hints of the BatchNorm apply passes (rn_bn_fwd_train / _part / rn_bn_apply outputs,
 *      rn_bn_bwd / _part data gradients), bit mask: 1 = nontemporal 16-byte stores, 2 = nontemporal
 *      loads, 4 (with 2) = nontemporal loads in the reduction / residual-tail passes too
 *      (rn_bn_bwd's reduction, rn_relu_bwd_bnred, rn_bn_apply_add), 8 = the BatchNorm-folded int8
 *      quantizer pass (rn_quant_int8_fwd_codes_bn / _bn2: x loads, the fake-quantized copy's stores;
 *      measured slower: C5 24.1 -> 25.1 ms per step), 16 = the 224/256-row conv tiles' output stores
 *      (rn_conv_fwd* / rn_conv_bwd_data*), 32 = the apply passes' stores write-through (sc1) instead of
 *      bit 1's hint (no dirty lines left in the XCD L2s; round 6, four pairs on one box: C2 18.85 ->
 *      18.82, 18.91 -> 18.86, 18.88 -> 18.82, 18.89 -> 18.85 ms; C4 26.75 -> 26.60, C5 21.21 -> 21.11),
 *      64 = the int8 quantizer pass's stores (codes, fake-quantized copy) write-through (measured
 *      slower, four pairs on one box: C5 21.16 -> 21.26, 21.14 -> 21.26, 21.21 -> 21.26, 21.12 -> 21.25 ms).
 *      Default 55. The same bits either way: only the cache policy changes,
 * 19 = the slice-resident weight gradients (rn_conv_bwd_filter[_ws / _x]; a workgroup keeps its dW
 *      slice for all of its images in registers, so dy and x are read once per slice; they need the
 *      slab workspace, rn_conv_wgrad_ws_bytes): the image-band kernels of the 3x3 stride-1 pad-1
 *      convolutions -- dense with C = K in {64, 128, 256, 512}, and grouped (32 groups) with 4 / 8 / 16
 *      channels per group -- and the streaming kernel of the 1x1 stride-1 ones with K, C in
 *      {64, 128, 256} and K x C <= 32768: 0 = on (default; the dense band kernel for C = 64 only),
 *      1 = the tiled kernels, 2 = on, the dense band kernel for C = 128..512 too (measured slower),
 * 20 = conv tile schedule A/B bits: 1 = static priority of the 8-wave tiles' second half (waves 4-7 at
 *      s_setprio 1 for the whole kernel; default off), 2 = the 224-row tiles issue the DMAs of the A
 *      rows past the tile too (default: skipped, those rows are never read),
 * 21 = the CUs the weight gradients size their split-M grids for, in percent of the device's (default
 *      50; 0 = 100): fewer splits, fewer partial slabs to reduce, for kernels that share the chip with
 *      the data-gradient stream (measured, ResNet-50 at batch 256: 100 % 20.83 / 20.80 ms per step,
 *      75 % 20.74, 50 % 20.09 / 20.04, 25 % 23.85; on another box 55 % 21.01 / 21.03, 50 % 20.63 /
 *      20.60, 45 % 20.48 / 20.44, 40 % 20.67; round 6, timed without event packets: 50 % 18.82 / 18.83,
 *      45 % 19.08 / 19.03, 55 % 18.95). Set before the workspaces are sized
 *      (rn_conv_wgrad_ws_bytes),
 * 23 = the same percent for the grouped image-band weight gradients only (0 = key 21's),
 * 24 = 1: rn_bn_fwd_train_part always merges and finalizes in two launches (default 0: one launch where
 *      the partials form at most 4 merge groups, bit-identical),
 * 25 = 1: the weight-gradient slab reduction always runs its general kernel (default 0: one thread per
 *      16-byte column with every split in flight where there are <= 16 splits; the same sums),
 * 27 = 1: the 1x1 / stride-1 data gradients reducing over K = 64 or 128 into C >= 128 channels (the pre-activation
 *      units' conv1) on the 224-row tiles (default 0: dgrad1x1_stream_kernel, which streams their rows with the
 *      weights in registers -- with the BN-backward reduction, and with the BN backward applied);
 *      27 = 2: that kernel with 32 channels per wave (default 64 where C % 256 == 0),
 * 26 = 1: the 3x3 / stride-1 / pad-1 64 -> 64 convolutions (forward, data gradient) and the stem's 7x7 /
 *      stride-2 64-channel forward (rn_stem_conv_fwd_p4) on the implicit-GEMM tile (default 0:
 *      conv3x3c64_band_kernel and stem_band_kernel, image bands and the weights in LDS); 26 = 2: the stem
 *      only on the tile,
 * 22 = 1: the BatchNorm-folded int8 quantizers (rn_quant_int8_fwd_codes_bn[2]) form every quotient
 *      v / unit by division (default 0: v * (1 / unit), the division only where that product lies
 *      within 2^-21 |v / unit| of a half-integer -- the same codes bit for bit, fewer instructions). */
int rn_set_tuning(int32_t key, int32_t value);
int32_t rn_version(void);
/* Build id baked in at compile time: a hash of the sources (csrc/*.hip, csrc/*.h, include/rn.h) and the
 * compiler flags this library was built from (rn/build.py: source_hash). The host refuses to run a library
 * whose id differs from the tree's, so a stale prebuilt cannot be tested silently. Same role as the
 * reference's pin to one MXNet fork build (README.md:7). */
const char* rn_build_id(void);
/* Number of compute units of the current device (for split heuristics / reporting). */
int32_t rn_device_cu_count(void);

/* ---------------------------------------------------------------------------------------
 * Diagnostic build only (RN_DIAG=1 at build time: librn_diag.so, never the shipped librn.so).
 * ------------------------------------------------------------------------------------- */
#ifdef RN_DIAG
/* Diagnostic twin of rn_sgd_mom_update_pack: every global index is checked against
 * lim = {nparam, then per tensor the KRSC and CRSK copy sizes}; out-of-range accesses are
 * skipped and flagged (bit mask) in *flag (device int). */
int rn_sgd_mom_update_pack_checked(int32_t ntensors, const int64_t* offsets, const int64_t* numels,
                                   const float* wds, float* w, const float* g, float* mom,
                                   const rn_wpack* packs, const int32_t* work, int32_t nwork,
                                   int32_t lowp_dtype, float lr, float momentum, float rescale_grad,
                                   const int64_t* lim, int32_t* flag, rn_stream_t stream);
#endif /* RN_DIAG */

#ifdef __cplusplus
}
#endif

#endif /* RN_H_ */
