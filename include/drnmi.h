/*
 * drnmi.h — C-ABI of the MI355X-native DRN-D segmentation hot path.
 *
 * Every entry point takes device pointers, plain sizes and a hipStream_t (passed
 * as void*), launches asynchronously on that stream and returns 0 on success or
 * a negative drnmi_status on a rejected argument / a positive hipError_t on a
 * launch failure.  No torch or C++ types cross this boundary; the Python host
 * layer (drnmi/_lib.py) binds it with ctypes, and any other FFI (cgo, JNI,
 * N-API) can bind it the same way.
 *
 * The reference (thejasvi-konduru/video-seg-model-compress) has no native code
 * and no FFI: its hot path is PyTorch ATen ops called from Python.  Each entry
 * point below names the reference code it replaces (file:line in the reference).
 *
 * Layouts: activations are NHWC with a power-of-two channel stride >= 8;
 * weights are packed [cout_pad][k_pad] with k = (kh*ks + kw)*cin + ci.
 * dtype codes: DRNMI_F32 (fp32 parity mode), DRNMI_BF16 (bf16 perf mode).
 */
#ifndef DRNMI_H
#define DRNMI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI version of the argument structs below (drnmi_conv_args, drnmi_wgrad_args).  The structs
 * have grown by appended fields (x2.. in version 2, ws / ws_bytes in version 3); a caller built
 * against another header must not pass them: check drnmi_abi_version() == DRNMI_ABI_VERSION and
 * drnmi_conv_args_size() == sizeof(drnmi_conv_args) once after loading the library (drnmi/_lib.py
 * does, and refuses a mismatched library). */
#define DRNMI_ABI_VERSION 5
int32_t drnmi_abi_version(void);
int64_t drnmi_conv_args_size(void);

enum drnmi_dtype { DRNMI_F32 = 0, DRNMI_BF16 = 1, DRNMI_U8 = 2, DRNMI_I64 = 3, DRNMI_I8 = 4, DRNMI_F32X3 = 5 };
/* DRNMI_F32X3 (conv dtype only, the "fp32x" precision mode): x, res and y are fp32 NHWC as in
 * DRNMI_F32, wgt is three bf16 planes [3][cout_pad][k_pad] with w = w1 + w2 + w3 (an exact split
 * of the fp32 weight), and the conv runs fp32-accurate arithmetic on the bf16 MFMA pipe: each
 * fp32 activation is split the same way in registers and the six products above 2^-24 are
 * accumulated in fp32 (csrc/conv_x6.hip).  Requires cin >= 32 (power of two), ks 1 or 3,
 * out_dtype DRNMI_F32. */

enum drnmi_status {
  DRNMI_OK = 0,
  DRNMI_EINVAL = -1,     /* bad shape / stride / dtype combination */
  DRNMI_ENOTSUP = -2,    /* no kernel instantiated for this configuration */
};

/* One fused convolution: y = act(conv(x, w) * scale + shift [+ res]).
 * Replaces conv3x3 + BatchNorm2d + ReLU (+ residual add) of the reference:
 *   lmodels/drn.py:27-29   conv3x3
 *   lmodels/drn.py:49-65   BasicBlock.forward (conv-bn-relu, conv-bn, += residual, relu)
 *   lmodels/drn.py:86-106  Bottleneck.forward (1x1 / 3x3 / 1x1 + residual)
 *   lmodels/drn.py:132-137 layer0 (7x7 stem) ; :181-186 downsample (1x1 stride s + BN)
 *   lmodels/drn.py:201-211 _make_conv_layers (conv-bn-relu stacks, layer1/2/7/8)
 *   lmodels/drnseg.py:278-284 seg (1x1 conv + bias, scale = 1, shift = bias)
 * Output addressing: y[img*y_sn + pixel*y_sp + c*y_sc] (pixel = oh*wo + ow), so
 * the same kernel writes NHWC activations or the NCHW fp32 logits tensor. */
typedef struct drnmi_conv_args {
  const void* x;       /* NHWC input [n][h][w][cin]                                   */
  const void* wgt;     /* packed weights [cout_pad][k_pad]                            */
  const float* scale;  /* [cout_pad] folded BN scale, or NULL = 1 (scale pre-folded    */
                       /* into wgt; lets the bf16 kernels start from shift + res)    */
  const float* shift;  /* [cout_pad] folded BN shift (or conv bias)                   */
  const void* res;     /* optional NHWC residual [n*ho*wo][cout] in x's dtype, or NULL */
  void* y;             /* output                                                      */
  int64_t y_sn, y_sp, y_sc; /* output strides in elements                          */
  int32_t n, h, w, cin;     /* cin: channel stride of x, power of two >= 8          */
  int32_t ho, wo, cout, cout_pad;
  int32_t ks, stride, pad, dil;
  int32_t k, k_pad;         /* k = ks*ks*cin ; k_pad = round_up(k, 32)              */
  int32_t relu;             /* 1: ReLU after the (optional) residual add            */
  int32_t dtype;            /* DRNMI_BF16 or DRNMI_F32: x, w, res                   */
  int32_t out_dtype;        /* DRNMI_BF16 or DRNMI_F32: y                           */
  int32_t tile;             /* tile id (drnmi_conv_tile_name), -1 = auto            */
  int32_t algo;             /* DRNMI_ALGO_IGEMM or DRNMI_ALGO_PATCH (see below)     */
  int32_t src_u8;           /* PATCH only: x is uint8 HWC3 frames, normalised on load */
  int32_t bgr;              /* src_u8: swap channel 0 and 2 on read                  */
  float mean[3], std[3];    /* src_u8: (u8 / 255 - mean[c]) / std[c], fp32          */
  const uint32_t* unit_mask; /* optional block-sparsity map of wgt (drnmi_weight_unit_mask):  */
                             /* bit (rb, ku) = 0 -> rows 16rb..16rb+15 x packed K columns   */
                             /* 32ku..32ku+31 are all zero and their MFMAs are skipped      */
                             /* (bf16 LDS-DMA kernels; NULL = dense).  Results are bit-     */
                             /* identical to the dense kernel on the same weights.          */
  /* W8A8 (dtype DRNMI_I8: x, wgt, res int8; per-tensor symmetric activations, per-channel  */
  /* weights; BASELINE config C5).  acc = int32 sum; v = float(acc) * scale[c] + shift[c];  */
  /* v += float(res) * res_scale; ReLU; out_dtype DRNMI_I8 stores                           */
  /* clamp(rint(v * out_scale), -127, 127), BF16 / F32 store v.  Each step is one fp32        */
  /* rounding (no fused multiply-add), so a scalar restatement reproduces it bit for bit.  */
  /* scale must be non-NULL for int8.  Ignored for other dtypes.                             */
  float res_scale;
  float out_scale;            /* 1 / (scale of the int8 output activation)                */
  /* Fused second input (bf16 LDS-DMA kernels, x2 != NULL): y = act(conv(x, w) + conv1x1_s(x2, w2)
   * * scale + shift) as ONE implicit GEMM over the concatenated K [ks*ks*cin | cin2]; wgt rows hold
   * [w | w2] (k = ks*ks*cin + cin2).  This folds a BasicBlock / Bottleneck 1x1 downsample
   * (lmodels/drn.py:181-186, its BN scale folded into w2, shifts summed) into the block's last
   * conv, so the residual branch is never written to HBM.  x2: NHWC [n][h2][w2][cin2], sampled at
   * (oh*stride2, ow*stride2); res must be NULL.  x2 = NULL: unused.  Two accepted forms:
   *   conv_big (cin >= 256 tiles): cin2 % 64 == 0 and k_pad == k;
   *   conv_halo (stride-1 3x3 with cin = cout 64 or 128, layer3/layer4): cin2 == 32 or 64,
   *     k_pad = round_up(k, 64) with zero columns after w2, scale == NULL (BN scales folded
   *     into the weights, shifts summed in shift).  Other combinations return
   *     DRNMI_ENOTSUP.                                                                       */
  const void* x2;
  int32_t cin2, h2, w2, stride2;
  /* Optional fp32 scratch (16-B aligned) of the F32X3 kernel (conv_x6): a launch given one takes
   * the training plan -- a tile variant and split-K count chosen for grids that leave CUs idle
   * (the K range split over gridDim.y workgroups per tile, their partial sums land here and a
   * second kernel adds them in split order and applies the epilogue).  Size:
   * drnmi_conv_workspace_bytes (0 = the plan is the inference one: pass NULL).  ws = NULL keeps
   * the inference plan (the inference engine's launches); other dtypes ignore it. */
  void* ws;
  int64_t ws_bytes;
  /* Optional train-mode BN statistics of the stored output (F32X3 conv_x6 launches that do not
   * split K: drnmi_conv_stats_rows(args) > 0): the epilogue writes per-channel fp64 partial sums
   * of y and y^2, one row per 64-pixel wave slice, as [2][rows][cout] (sums, then sums of
   * squares), in a fixed order.  drnmi_bn_stats_partials_f32 turns them into the batch mean /
   * invstd with the same finalize as drnmi_bn_stats_f32 (mean, biased variance, invstd, running-
   * stat update; semantic_seg.py:166-230's train-mode BatchNorm2d after the conv), without reading
   * y again.  The fp64 sums are added in a different fixed order than drnmi_bn_stats_f32's row
   * splits, so the two agree to fp32 rounding, not bit for bit.  NULL: off. */
  double* stats;
  /* Optional output row stride in elements (F32X3 conv_x6 launches only): y(n, oh, ow, c) =
   * y[n*y_sn + oh*y_sr + ow*y_sp + c*y_sc]; a residual then has y's layout.  0 = rows packed
   * (oh*wo*y_sp).  A stride-2 conv's data gradient runs as four of these launches, one per output
   * parity class, writing every other pixel of every other row (drnmi_dgrad_s2_class_planes).  With
   * y_sr != 0 the output size is free (ho x wo need not follow the conv formula): taps past the
   * input's edges read zeros. */
  int64_t y_sr;
} drnmi_conv_args;

/* Algorithms behind drnmi_conv2d_bn_act:
 *  DRNMI_ALGO_IGEMM  NHWC implicit GEMM (any power-of-two cin >= 8, any ks/stride/dil; bf16 or
 *                    fp32).  tile -1 picks the bf16 LDS-DMA kernel (tiles 4..7: 128/256/64/64
 *                    output channels x 256 pixels, tile 6 with 32-channel K steps, tile 7 with
 *                    64; cin >= 64, ks 1 or 3) when it applies, else a
 *                    register-staged tile 0..3 by cout.  Whole 256-pixel output rows (3x3, stride
 *                    1, cin % 128 == 0) route to the strip tiles: 19 conv_stag (256 / 128
 *                    channels, 8 waves with staggered SIMD partners), 22 conv_w1 (the same tile
 *                    as 4 waves of 128 x 128, one per SIMD; auto at cin >= 512 without residual),
 *                    23 conv_w1h (128 x 128 tiles, two workgroups per CU; auto at cout 128) --
 *                    all with the same K order, so bit-identical.  int8 (dtype DRNMI_I8) takes
 *                    19 / 22 / 23 as its int8 forms (auto: 23 at cin, cout <= 256, else 19).
 *  DRNMI_ALGO_PATCH  bf16-only small-channel direct conv for the full-resolution layers
 *                    (lmodels/drn.py:132-137 layer0, :201-211 layer1/layer2): the input tile
 *                    plus halo is staged once in LDS and reused by all ks*ks taps; weights stay
 *                    in registers; the MFMA puts output channels on rows so each lane stores 4
 *                    contiguous channels (coalesced NHWC stores).  Supports dil = 1,
 *                    (cin, cout, ks, stride) in {(8,16,7,1), (16,16,3,1), (16,32,3,2), (32,64,3,2)},
 *                    no residual, packed NHWC output; and the
 *                    fused stem src_u8 = 1 with (cin = 4, cout = 16, ks = 7, stride = 1): weights
 *                    packed [cout_pad][224] with k = kh*32 + kw*4 + c (kw < 8, c < 4; kw = 7 and
 *                    c = 3 are zero), which also replaces the frame-ingest kernel. */
enum drnmi_algo { DRNMI_ALGO_IGEMM = 0, DRNMI_ALGO_PATCH = 1 };

int drnmi_conv2d_bn_act(const drnmi_conv_args* args, void* stream);

/* Rows of the args->stats partials this launch writes (4 per 256-pixel tile), or 0 when it
 * cannot produce them (not conv_x6, or a split-K plan: compute the statistics from y). */
int64_t drnmi_conv_stats_rows(const drnmi_conv_args* args);

/* Bytes of args->ws the training plan of these arguments needs (0: the inference plan; 256: a
 * different tile variant, no split; else S x M x cout x 4 for S split-K partitions; -1: NULL).
 * Only DRNMI_F32X3 implicit-GEMM launches use it (drnmi/train.py passes it for the fp32x
 * fine-tune); the plan depends on the geometry alone, so a size queried once per layer holds for
 * every step. */
int64_t drnmi_conv_workspace_bytes(const drnmi_conv_args* args);

/* Fused stem + layer1 (bf16, csrc/patch_conv.hip stem_l1_kernel): replaces the two launches
 *   drnmi_conv2d_bn_act(stem); drnmi_conv2d_bn_act(next)
 * of lmodels/drn.py:132-137 (layer0 7x7 3->16 + BN + ReLU on the uint8 frame) and :201-211
 * (layer1 3x3 16->16 + BN + ReLU) with one, bit-identical to them; the stem output is never
 * written (stem->y is ignored).  stem: the src_u8 = 1 PATCH contract above (cin 4, cout 16,
 * ks 7, pad 3, k = k_pad = 224); next: cin 16, cout 16, ks 3, stride 1, pad 1, dil 1,
 * k = 144, k_pad >= 160, no residual, packed NHWC bf16 output, same n/h/w as the stem.
 * DRNMI_EINVAL for anything else.  drnmi_stem_layer1_kernel_name: "stem_l1_kernel" or NULL. */
int drnmi_stem_layer1(const drnmi_conv_args* stem, const drnmi_conv_args* next, void* stream);
const char* drnmi_stem_layer1_kernel_name(const drnmi_conv_args* stem, const drnmi_conv_args* next);

/* Fused video front (bf16 perf mode, csrc/front.hip front_kernel): uint8 HWC3 frames -> layer0
 * (7x7 3->16 + BN + ReLU, lmodels/drn.py:132-137, on the normalised frame of data_transforms.py:
 * 109-125, 256-281) -> layer1 (3x3 16->16 + BN + ReLU, drn.py:201-211) -> layer2 (3x3 stride 2
 * 16->32 + BN + ReLU) in one launch: neither the 16-channel full-resolution stem output nor
 * layer1's is ever written; the layer2 output y is NHWC bf16 [n][(h+1)/2][(w+1)/2][32].
 * Arithmetic: the stem runs f16 MFMAs on the exact frame bytes (1024 + u8 is exact in f16) with the
 * normalisation and the stem's BN scale folded into f16 weights w * scale / (255 std[c]); the
 * offset 1024 and the mean term are subtracted through a per-border-case shift (the reference
 * zero-pads in normalised space, so the shift depends on which taps fall inside the image);
 * layer1 / layer2 are bf16 MFMAs (BN scale folded into bf16 weights) on bf16 activations.
 *   drnmi_front_pack: HOST function, no GPU: packs the three convs' OIHW fp32 weights (w0
 *     [16][3][7][7], w1 [16][16][3][3], w2 [32][16][3][3]), their folded BN scale/shift
 *     (scale*: NULL = 1), mean/std (3 each, per model channel) and bgr into a host buffer of
 *     drnmi_front_pack_bytes() bytes that the caller copies to the device once.
 *   drnmi_video_front_u8: frames [n][h][w][3] uint8 (bgr as packed), pack = the device copy;
 *     requires w % 4 == 0, h >= 8, w >= 8, n*h*w*3 < 2^31 (DRNMI_EINVAL otherwise).
 *   drnmi_front_supported: 1 if drnmi_video_front_u8 takes (n, h, w).
 * Replaces ToTensorVideoImage + Normalize + layer0 + layer1 + layer2 of the seg_video loop
 * (seg_video_old_no_plot.py:157-169 -> lmodels/drnseg.py:295-299 -> drn.py:213-259). */
int64_t drnmi_front_pack_bytes(void);
int drnmi_front_pack(const float* w0, const float* scale0, const float* shift0, const float* w1, const float* scale1,
                     const float* shift1, const float* w2, const float* scale2, const float* shift2,
                                      const float* mean3, const float* std3, int32_t bgr, void* out_host);
int drnmi_front_supported(int32_t n, int32_t h, int32_t w);

/* Fused 64-channel BasicBlock (lmodels/drn.py:49-65 with inplanes = planes = 64, stride 1,
 * dilation 1, no downsample: DRN-D-22 layer3.1, D-38 layer3.1/3.2):
 *   y = relu(bn2(conv3x3(relu(bn1(conv3x3(x))))) + x), bf16 NHWC [n][h][w][64] in and out, eval BN
 *   (scale folded into the weights, shift added; fp32 accumulation).
 * The intermediate never reaches HBM (csrc/block64.hip).  `pack`: device copy of the blob that the
 * HOST function drnmi_block64_pack(w1, scale1, shift1, w2, scale2, shift2, out) builds from the two
 * convs' OIHW fp32 weights [64][64][3][3] and per-channel BN scale / shift (fp32 [64] each);
 * drnmi_block64_pack_bytes() bytes.  x and y must not alias. */
int64_t drnmi_block64_pack_bytes(void);
int drnmi_block64_pack(const float* w1, const float* scale1, const float* shift1, const float* w2,
                       const float* scale2, const float* shift2, void* out_host);
int drnmi_block64_supported(int32_t n, int32_t h, int32_t w);
int drnmi_basic_block64(const void* x, const void* pack, void* y, int32_t n, int32_t h, int32_t w, void* stream);
int drnmi_video_front_u8(const uint8_t* frames, const void* pack, void* y, int32_t n, int32_t h, int32_t w,
                         void* stream);

/* Block-sparsity map of packed weights [rows_pad][k_pad] (dtype F32 or BF16): one bit per
 * 16-row x 32-column unit, bit = 1 iff any element of the unit is nonzero (+-0 count as zero);
 * layout: row-block rb owns words [rb*W, rb*W + W), W = ceil(k_pad / 32 / 32), unit ku at bit
 * ku % 32 of word ku / 32.  mask must hold (rows_pad / 16) * W words; *nonzero_units (device
 * int32, NULL-able) receives the count of nonzero units.  This is how pruner masks reach the
 * MFMA path: MFMA runs only on the dense-within-block sub-tiles (BlockPruner blocks of whole
 * kernels, BlockPruner.py:139-241, with block_width a multiple of 32 input channels map 1:1 to
 * units; narrower blocks skip where neighbouring blocks are both pruned). */
int drnmi_weight_unit_mask(const void* wgt, int32_t dtype, int32_t rows_pad, int32_t k_pad, uint32_t* mask,
                           int32_t* nonzero_units, void* stream);

/* W8A8 helpers (BASELINE config C5; csrc/quant.hip).  The reference has no quantisation code
 * (SURVEY.md C5 row): the scheme is ours.  Activations are per-tensor symmetric int8.
 *   drnmi_quantize_i8: y[i] = clamp(rint(x[i] * inv_scale), -127, 127) over n elements
 *     (x BF16 or F32, n % 8 == 0; one fp32 multiply, round-half-even) -- the bf16 -> int8
 *     boundary in front of the first int8 conv.
 *   drnmi_absmax: *out = max |x[i]| (device float; calibration of the activation scales). */
int drnmi_quantize_i8(const void* x, int32_t dtype, int8_t* y, int64_t n, float inv_scale, void* stream);
int drnmi_absmax(const void* x, int32_t dtype, int64_t n, float* out, void* stream);

/* Name of the kernel (template instance) drnmi_conv2d_bn_act would launch for these
 * arguments, e.g. "conv_big_kernel<3, 128, 2, 2>"; NULL if none.  No launch, no GPU needed.
 * (Used by bench.py to attribute timed launches to kernels as rocprofv3 names them.) */
const char* drnmi_conv_kernel_name(const drnmi_conv_args* args);

/* Name of a tile configuration ("128x128", ...) or NULL; count via drnmi_conv_num_tiles. */
const char* drnmi_conv_tile_name(int tile);
int drnmi_conv_num_tiles(void);

/* Frame ingest: uint8 HWC frames -> normalised NHWC (channel stride 8, c>=3 zero).
 * Replaces ToTensorVideoImage + Normalize (data_transforms.py:256-281, :109-125;
 * constants info.json:1): v = (u8 / 255 - mean[c]) / std[c] in fp32, then cast.
 * bgr != 0 swaps channel order on read (seg_video_old_no_plot.py:125 feeds cv2's
 * BGR frames as "RGB"; bgr = 0 reproduces that quirk when given cv2 frames). */
/* mean3 / std3 are HOST pointers to 3 floats (passed by value to the kernel). */
int drnmi_frame_ingest_u8(const uint8_t* frames, void* out, int32_t n, int32_t h, int32_t w,
                          const float* mean3, const float* std3, int32_t bgr,
                          int32_t out_dtype, void* stream);

/* fp32 NCHW [n][c][h][w] -> NHWC [n][h][w][c_pad] in out_dtype, zero-filling c..c_pad-1.
 * The boundary conversion for DRNSeg.forward(x) (lmodels/drnseg.py:295-299 takes NCHW fp32). */
int drnmi_nchw_to_nhwc(const float* x, void* out, int32_t n, int32_t c, int32_t h, int32_t w,
                       int32_t c_pad, int32_t out_dtype, void* stream);

/* NHWC [n][h][w][c_stride] (first c channels) -> fp32 NCHW [n][c][h][w]. Debug/parity taps. */
int drnmi_nhwc_to_nchw(const void* x, float* out, int32_t n, int32_t c, int32_t h, int32_t w,
                       int32_t c_stride, int32_t in_dtype, void* stream);

/* Fused up x8 + LogSoftmax(dim=1) + argmax over classes.
 * Replaces the depthwise ConvTranspose2d(c, c, 16, stride 8, pad 4, groups=c) with the
 * bilinear fill_up_weights kernel, the LogSoftmax and torch.max(final, 1):
 *   lmodels/drnseg.py:257-266, :285-299 ; semantic_seg.py:445 ; seg_video_old_no_plot.py:166
 * logits: fp32 NCHW [n][c][h][w]; up_w: fp32 [16][16] (one depthwise plane, all planes equal);
 * logprobs: fp32 NCHW [n][c][8h][8w] or NULL; labels: [n][8h][8w] uint8 or int64 (label_dtype)
 * or NULL.  Ties in argmax resolve to the lowest class index. */
int drnmi_up8_logsoftmax_argmax(const float* logits, const float* up_w, float* logprobs,
                                void* labels, int32_t label_dtype, int32_t n, int32_t c,
                                int32_t h, int32_t w, void* stream);

/* Labels-only form of the same head (the video path: no log-prob planes) on NHWC logits: fp32
 * [n][h][w][cs] rows, classes 0..c-1 first (cs % 4 == 0, cs >= c, 16-B aligned), as the seg conv
 * writes them with y_sp = cs, y_sc = 1.  Same per-pixel arithmetic, near-tie fallback and argmax
 * order as drnmi_up8_logsoftmax_argmax: identical labels.  c == 19 (else DRNMI_ENOTSUP). */
int drnmi_up8_labels_nhwc(const float* logits, int32_t cs, const float* up_w, void* labels, int32_t label_dtype,
                          int32_t n, int32_t c, int32_t h, int32_t w, void* stream);

/* The labels-only video path with the seg classifier (1x1 c_in -> 19 + bias, lmodels/drnseg.py:278-284)
 * folded into the epilogue of the last 3x3 conv (D-22 layer8): `a` is that conv's argument block
 * exactly as for drnmi_conv2d_bn_act (bf16, scale folded, no residual / x2, cout % 256 == 0, a shape
 * the staggered strip tile takes) but its activation is NOT stored (a->y unused); instead each
 * 256-channel block's partial logits go to partials[cout / 256][n*ho*wo][20] (fp32, 16-B aligned):
 * partial_b[m][k] = sum over the block's channels c of seg_w[k][c] * bf16(relu(conv)[m][c]).
 * seg_w: packed bf16 [seg_rows >= 32][seg_k_pad] (rows 19.. zero).  DRNMI_ENOTSUP if the conv does
 * not take the staggered tile.  It runs on the one-wave-per-SIMD tile (conv_w1_seg_kernel /
 * conv_w1_i8_seg_kernel); a->tile == 19 forces the staggered one (the same partials, bit for bit).
 * int8 nets (a->dtype DRNMI_I8, out_dtype DRNMI_I8, the W8A8 epilogue of drnmi_conv2d_bn_act, no
 * residual): seg_w is the int8 seg conv's packed weights and the partials are int32,
 * partial_b[m][k] = sum over the block's channels c of seg_w[k][c] * q8[m][c], q8 = the int8 value
 * the conv would store; the int8 seg conv's fp32 output is then (float)(partial_0 + partial_1) *
 * seg_scale[k] + seg_shift[k] (drnmi_up8_labels_seg2_i8). */
int drnmi_conv_stag_seg(const drnmi_conv_args* a, const void* seg_w, int32_t seg_k_pad, int32_t seg_rows,
                        void* partials, void* stream);
/* The kernel drnmi_conv_stag_seg launches for these arguments (as rocprofv3 names it), or NULL. */
const char* drnmi_conv_stag_seg_kernel_name(const drnmi_conv_args* a);

/* Labels from those partials: logit[k] = (bias[k] + partial_0[k]) + partial_1[k] (bias: >= cs
 * floats), then the labels-only head's arithmetic (drnmi_up8_labels_nhwc).  partials: [2][n][h][w][cs]. */
int drnmi_up8_labels_seg2(const float* partials, int32_t cs, const float* bias, const float* up_w, void* labels,
                          int32_t label_dtype, int32_t n, int32_t c, int32_t h, int32_t w, void* stream);

/* int8 nets: logit[k] = (float)(partial_0[k] + partial_1[k]) * scale[k] + shift[k] (fmul then fadd,
 * the int8 seg conv's epilogue: identical logits), then the same head.  partials: int32
 * [2][n][h][w][cs]; scale, shift: >= cs floats. */
int drnmi_up8_labels_seg2_i8(const int32_t* partials, int32_t cs, const float* scale, const float* shift,
                             const float* up_w, void* labels, int32_t label_dtype, int32_t n, int32_t c, int32_t h,
                             int32_t w, void* stream);

/* Same head for DRNSeg(use_torch_up=True): nn.UpsamplingBilinear2d(scale_factor=8) (bilinear,
 * align_corners=True; lmodels/drnseg.py:285-287) + LogSoftmax + argmax.  Source index and
 * weights follow ATen's CPU kernel: scale = (in-1)/(out-1) in fp32, i0 = floor(scale*dst),
 * i1 = i0 + (i0 < in-1), l1 = scale*dst - i0.  Output [n][c][8h][8w]. */
int drnmi_up8_bilinear_logsoftmax_argmax(const float* logits, float* logprobs, void* labels,
                                         int32_t label_dtype, int32_t n, int32_t c, int32_t h, int32_t w,
                                         void* stream);

/* Bilinear resize with Pillow's arithmetic (Image.resize(size, BILINEAR): separable, horizontal
 * pass first, the filter support widened by the downscale factor; coefficient tables computed on
 * the device exactly as Pillow's precompute_coeffs).  Bit-identical to Pillow 12.
 *   drnmi_resize_bilinear_u8: uint8 HWC3 frames [n][h][w][3] -> [n][oh][ow][3]; 8-bit fixed point
 *     with 22 fractional bits and a uint8 intermediate (Pillow's 8bpc path).  Replaces
 *     T.Resize((300, 300)) on each decoded frame (seg_video_old_no_plot.py:126-127).
 *   drnmi_resize_bilinear_f32: fp32 planes [planes][h][w] -> [planes][oh][ow]; fp32 x double
 *     summed in double, fp32 intermediate (Pillow's 'F' mode).  accumulate != 0: dst += result in
 *     fp32.  Replaces resize_4d_tensor + the scale sum of test_ms (semantic_seg.py:471-504, :540).
 *   ws: device workspace of drnmi_resize_workspace_bytes(n or planes, h, w, oh, ow, 3 or 4) bytes.
 *   drnmi_argmax_nchw_f32: labels[n][p] = first index of the max over c of x[n][c][p] (numpy
 *     argmax(axis=1), semantic_seg.py:543), uint8 or int64 labels. */
int64_t drnmi_resize_workspace_bytes(int32_t n, int32_t h, int32_t w, int32_t oh, int32_t ow, int32_t elem_bytes);
int drnmi_resize_bilinear_u8(const uint8_t* src, int32_t n, int32_t h, int32_t w, uint8_t* dst, int32_t oh, int32_t ow,
                             void* ws, int64_t ws_bytes, void* stream);
int drnmi_resize_bilinear_f32(const float* src, int32_t planes, int32_t h, int32_t w, float* dst, int32_t oh,
                              int32_t ow, int32_t accumulate, void* ws, int64_t ws_bytes, void* stream);
int drnmi_argmax_nchw_f32(const float* x, int32_t n, int32_t c, int64_t hw, void* labels, int32_t label_dtype,
                          void* stream);

/* Multi-tensor in-place mask apply: w[t][i] *= m[t][i] for every tensor t.
 * Replaces Pruner.apply_masks (pruners/Pruner.py:17-20, same body BlockPruner.py:27-30,
 * SRMBRepMasker.py:20-23): one launch for all masked layers instead of one ATen mul_ per
 * layer plus a state_dict() rebuild per layer. */
int drnmi_mask_apply_f32(int32_t ntensors, float* const* weights, const float* const* masks,
                         const int64_t* numels, void* stream);

/* Same, with bit-packed masks: bit i of word i/32 of masks[t] keeps element i. */
int drnmi_mask_apply_bits_f32(int32_t ntensors, float* const* weights,
                              const uint32_t* const* mask_bits, const int64_t* numels,
                              void* stream);

/* Eval: accumulate the nclass x nclass confusion matrix hist[label*nclass + pred] += 1 over the
 * pixels with 0 <= label < nclass and pred < nclass (int64 hist, NOT cleared: accumulates across
 * calls like the reference's running hist).  Replaces fast_hist (semantic_seg.py:293-296) used by
 * test()/val_miou() (:455, :655).  pred/label dtypes: DRNMI_U8 or DRNMI_I64; nclass <= 32. */
int drnmi_confusion_matrix(const void* pred, int32_t pred_dtype, const void* label, int32_t label_dtype,
                           int64_t npix, int32_t nclass, int64_t* hist, void* stream);

/* ======================================================================================
 * Fine-tune (train-mode) path, fp32 — csrc/train.hip.
 * Replaces the reference training step (semantic_seg.py:166-230): model.train() forward
 * with batch-statistics BatchNorm (lmodels/drn.py:7), CrossEntropyLoss(ignore_index=255) on
 * the log-probs (semantic_seg.py:817, :197-198), loss.backward(), torch.optim.SGD(momentum,
 * weight_decay) (:963-966, :212) and Pruner.apply_masks (:213-214, pruners/Pruner.py:17-20).
 * Conv forward and data-gradient passes go through drnmi_conv2d_bn_act (fp32): dgrad is a
 * stride-1 conv of dy with weights packed by drnmi_pack_conv_weight(mode = 1), after
 * drnmi_zero_insert_f32 for stride-s convs.  All reductions are fp64, fixed order
 * (bit-reproducible).  Workspaces are caller-provided device buffers of the queried size.
 * ====================================================================================== */

/* OIHW fp32 weights -> packed [rows_pad][k_pad] (out_dtype F32 or BF16), zero elsewhere.
 * mode 0 (forward):  row = co, k = (kh*ks + kw)*kin_stride + ci, value w[co][ci][kh][kw] *
 *                    row_scale[co] (row_scale may be NULL = 1; folds an eval BN scale).
 * mode 1 (dgrad):    row = ci, k = (kh*ks + kw)*kin_stride + co, value
 *                    w[co][ci][ks-1-kh][ks-1-kw] (transposed, spatially flipped).
 * Replaces the host-side permute/pad of the conv weights (lmodels/drn.py:27-29 layout). */
int drnmi_pack_conv_weight(const float* w, int32_t cout, int32_t cin, int32_t ks, int32_t kin_stride,
                           int32_t rows_pad, int32_t k_pad, int32_t mode, const float* row_scale,
                           int32_t out_dtype, void* out, void* stream);

/* Batched form of drnmi_pack_conv_weight (F32 output) + drnmi_split3_bf16 for a whole network:
 * one launch packs every entry of a device-resident table (the fine-tune re-packs all forward
 * and data-gradient weights after each SGD step; per layer that was 4 launches of ~6 us).
 * table: DEVICE memory, n entries of DRNMI_PACK_ENTRY_WORDS int64 each:
 *   [0] w (const float*), [1] out (float* [rows_pad][k_pad]), [2] planes (bf16 [3][rows_pad*k_pad]
 *   or 0), [3] cout, [4] cin, [5] ks, [6] kin_stride, [7] rows_pad, [8] k_pad, [9] mode (0 | 1,
 *   as drnmi_pack_conv_weight, no row scale), [10] first element index of the entry (prefix sum
 *   of rows_pad*k_pad over the entries before it), [11] 0.
 * total = sum of rows_pad*k_pad.  Values are bit-identical to the per-layer calls.
 * Limits: n <= 512, ks <= 7, kin_stride and k_pad multiples of 4, out / planes 16-B aligned.
 * drnmi_pack_table_check validates a HOST copy of the table before it is uploaded. */
#define DRNMI_PACK_ENTRY_WORDS 12
int drnmi_pack_table_check(const int64_t* table_host, int32_t n, int64_t* total_out);
int drnmi_pack_conv_weights_batched(const int64_t* table, int32_t n, int64_t total, void* stream);

/* Workspace bytes for the per-channel reductions over `rows` x `channels` (power of two >= 4). */
int64_t drnmi_reduce_workspace_bytes(int64_t rows, int32_t channels);

/* Train-mode BatchNorm2d statistics over rows of NHWC y [rows][C]: mean, invstd =
 * 1/sqrt(biased_var + eps); if running_mean/var are given: r = (1-momentum)*r + momentum*batch
 * (running_var with the unbiased variance), and *num_batches_tracked += 1 (if non-NULL). */
int drnmi_bn_stats_f32(const float* y, int64_t rows, int32_t C, float eps, float momentum,
                       float* mean, float* invstd, float* running_mean, float* running_var,
                       int64_t* num_batches_tracked, void* ws, void* stream);

/* Weight planes of parity class (a, b) of a stride-2 conv's data gradient (the transpose of
 * lmodels/drn.py's strided conv3x3 / downsample 1x1 in the fine-tune backward): gathered from the
 * dgrad's packed bf16 planes `planes` ([3][rows][k_pad], drnmi_pack_conv_weight mode 1 + split3,
 * k = tap' * kst + co, taps flipped, pad_d = dil*(ks-1) - pad) into `out` [3][rows][k_pad_c] for a
 * ksc x ksc stride-1 conv of dy: tap (khc, kwc) = flipped tap ((pad_d - a) mod 2 + 2 khc, likewise
 * for b), zero where the class has fewer taps.  Launch the class conv with F32X3, x = dy, pad 0,
 * y = dx + (a * W + b) * cs, y_sp = 2 cs, y_sr = 2 W cs, y_sn = H W cs: the four classes together
 * are bit-identical to the conv of the zero-inserted dy (drnmi_zero_insert_f32).  kst % 8 == 0. */
int drnmi_dgrad_s2_class_planes(const void* planes, int32_t rows, int32_t k_pad, int32_t kst, int32_t ks,
                                int32_t pad_d, int32_t a, int32_t b, int32_t ksc, void* out, int32_t k_pad_c,
                                void* stream);

/* drnmi_bn_stats_f32 from the partial sums a conv epilogue wrote (drnmi_conv_args.stats:
 * [2][G][C] fp64, G = drnmi_conv_stats_rows): the same finalize (mean, biased variance, invstd,
 * running-stat update) over `rows` pixels. */
int drnmi_bn_stats_partials_f32(const double* partials, int64_t G, int64_t rows, int32_t C, float eps,
                                float momentum, float* mean, float* invstd, float* running_mean,
                                float* running_var, int64_t* num_batches_tracked, void* stream);

/* z = relu?(((y - mean) * invstd) * gamma + beta [+ res]) over [rows][C]; gamma/beta/res NULL-able.
 * (BasicBlock / Bottleneck tail: lmodels/drn.py:49-65, :86-106.)  mean/invstd/gamma/beta must be
 * 16-byte aligned (DRNMI_EINVAL otherwise). */
int drnmi_bn_act_f32(const float* y, const float* mean, const float* invstd, const float* gamma,
                     const float* beta, const float* res, int32_t relu, int64_t rows, int32_t C,
                     float* z, void* stream);

/* Backward of drnmi_bn_act_f32 (train-mode BN): dr = dz * (relu ? z > 0 : 1);
 * dbeta = sum dr, dgamma = sum dr * xhat; dy = gamma*invstd*(dr - mean(dr) - xhat*mean(dr*xhat));
 * dres (NULL-able) = dr (or += dr with dres_accumulate).  dy may alias dz.
 * grad_accumulate: dgamma/dbeta += instead of =.  mean must be 16-byte aligned. */
int drnmi_bn_act_bwd_f32(const float* dz, const float* z, const float* y, const float* mean,
                         const float* invstd, const float* gamma, int32_t relu, int64_t rows,
                         int32_t C, float* dy, float* dres, int32_t dres_accumulate, float* dgamma,
                         float* dbeta, int32_t grad_accumulate, void* ws, void* stream);

/* drnmi_bn_act_bwd_f32 for a residual-free BN + ReLU (relu = 1, res = NULL, dres = NULL) without z:
 * the mask z > 0 is recomputed from y with the forward's own arithmetic (bn_act's rounding order),
 * so it is bit-identical to reading z and each pass reads one fp32 tensor less.  gamma / beta as
 * given to drnmi_bn_act_f32 (NULL-able); mean/invstd/gamma/beta 16-byte aligned.
 * (semantic_seg.py:166-230 backward through lmodels/drn.py:49-65 / :86-106's bn + relu.) */
int drnmi_bn_relu_bwd_y_f32(const float* dz, const float* y, const float* mean, const float* invstd,
                            const float* gamma, const float* beta, int64_t rows, int32_t C, float* dy,
                            float* dgamma, float* dbeta, int32_t grad_accumulate, void* ws, void* stream);

/* out[c] (+)= sum over rows of x[row][c], c < cvalid (row stride C).  Conv-bias gradient
 * (seg 1x1 + bias, lmodels/drnseg.py:278-284). */
int drnmi_channel_sum_f32(const float* x, int64_t rows, int32_t C, int32_t cvalid, float* out,
                          int32_t accumulate, void* ws, void* stream);

/* Weight gradient of a conv: dw[co][ci][kh][kw] (+)= sum_pixels dy[pix][co] * x[tap(pix)][ci].
 * dy: NHWC [n*ho*wo][dy_stride] (first cout valid), x: NHWC [n][h][w][cin_stride]. */
typedef struct drnmi_wgrad_args {
  const float* dy;
  const float* x;
  float* dw;             /* OIHW [cout][cin][ks][ks] fp32 (the parameter's .grad)          */
  void* ws;              /* workspace, ws_bytes >= drnmi_conv_wgrad_workspace_bytes()      */
  int64_t ws_bytes;
  int32_t n, h, w, cin, cin_stride, ho, wo, cout, dy_stride;
  int32_t ks, stride, pad, dil;
  int32_t accumulate;    /* 1: dw += ; 0: dw =                                            */
} drnmi_wgrad_args;
int64_t drnmi_conv_wgrad_workspace_bytes(const drnmi_wgrad_args* args);    /* room for either kernel */
int64_t drnmi_conv_wgrad_f32_workspace_bytes(const drnmi_wgrad_args* args);/* drnmi_conv_wgrad_f32 only */
int drnmi_conv_wgrad_f32(const drnmi_wgrad_args* args, void* stream);
/* The same weight gradient in fp32-class split-bf16 arithmetic (the fp32x fine-tune: exact 3-way
 * bf16 split of dy and x, the six products above 2^-24 on the bf16 MFMA, fp32 accumulation);
 * same arguments, workspace and errors.  semantic_seg.py:166-230 backward. */
int drnmi_conv_wgrad_f32x3(const drnmi_wgrad_args* args, void* stream);
/* fp32 w[n] -> bf16 out[3][n] with w = out[0] + out[1] + out[2] exactly (round to nearest even at
 * each step): the three weight planes of a DRNMI_F32X3 launch. */
int drnmi_split3_bf16(const float* w, int64_t n, void* out, void* stream);

/* out[n][y][x][c] = dy[n][y/s][x/s][c] where y, x are multiples of s (and inside dy), else 0;
 * out is [n][hu][wu][c] (c % 4 == 0).  Input of the stride-1 dgrad conv of a stride-s conv. */
int drnmi_zero_insert_f32(const float* dy, int32_t n, int32_t ho, int32_t wo, int32_t c, int32_t stride,
                          int32_t hu, int32_t wu, float* out, void* stream);

/* Head backward: du = grad_scale * (g_lp - exp(lp) * sum_c g_lp) (LogSoftmax, dim 1), then
 * dlogits = up^T(du) [+ grad_scale * g_logits] — the transpose of the fixed bilinear ConvTranspose2d(k16,
 * s8, p4) (lmodels/drnseg.py:285-299).  g_logprobs/logprobs/du_ws: NCHW [n][c][8h][8w];
 * dlogits/g_logits: [n][c][h][w]; g_logprobs NULL = logits-only gradient. */
int drnmi_up8_lsm_bwd_f32(const float* g_logprobs, const float* logprobs, const float* g_logits,
                          const float* up_w, float grad_scale, int32_t n, int32_t c, int32_t h,
                          int32_t w, float* du_ws, float* dlogits, void* stream);

/* Head backward of the use_torch_up head (bilinear align_corners=True x8): du as above, then
 * dlogits = bilinear^T(du) [+ grad_scale * g_logits] (a fixed-order gather, no atomics). */
int drnmi_up8_bilinear_lsm_bwd_f32(const float* g_logprobs, const float* logprobs, const float* g_logits,
                                   float grad_scale, int32_t n, int32_t c, int32_t h, int32_t w, float* du_ws,
                                   float* dlogits, void* stream);

/* CrossEntropyLoss(ignore_index) applied to log-probs [n][c][hw] with int64 targets [n][hw]:
 * loss[0] = mean over target != ignore of (logsumexp(lp) - lp[target]) (NaN if a target is out
 * of range), count[0] = number of counted pixels.  Device scalars; ws of drnmi_ce_workspace_bytes. */
int64_t drnmi_ce_workspace_bytes(void);
int drnmi_ce_loss_f32(const float* logprobs, const int64_t* target, int32_t n, int32_t c, int64_t hw,
                      int64_t ignore_index, float* loss, float* count, void* ws, void* stream);
/* g_logprobs = dloss[0] / count[0] * (softmax(lp) - onehot(target)), 0 on ignored pixels. */
int drnmi_ce_loss_bwd_f32(const float* logprobs, const int64_t* target, int32_t n, int32_t c, int64_t hw,
                          int64_t ignore_index, const float* dloss, const float* count,
                          float* g_logprobs, void* stream);

/* Multi-tensor torch.optim.SGD step (semantic_seg.py:963-966, torch semantics: d = g + wd*w;
 * buf = first ? d : momentum*buf + (1-dampening)*d; d = nesterov ? d + momentum*buf : buf;
 * w -= lr*d) with the pruner mask fused: w *= bit (mask_bits[t] NULL-able; NULL array = none).
 * params/grads/momentum_bufs/numels/mask_bits/first_step are HOST arrays of device pointers. */
int drnmi_sgd_step_f32(int32_t ntensors, float* const* params, const float* const* grads,
                       float* const* momentum_bufs, const int64_t* numels,
                       const uint32_t* const* mask_bits, const int32_t* first_step, float lr,
                       float momentum, float dampening, float weight_decay, int32_t nesterov,
                       void* stream);

/* Library version string, e.g. "drnmi 0.1.0 gfx950". */
const char* drnmi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* DRNMI_H */
