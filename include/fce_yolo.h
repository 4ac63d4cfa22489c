/*
 * fce_yolo.h — C-ABI of the MI355X-native FCE-YOLOv11 inference path (libfceyolo.so).
 *
 * Plain C: pointers, sizes and POD descriptors only; no torch or C++ types.  Every
 * function returns an int status (FCE_OK = 0); on failure fce_last_error() returns a
 * thread-local message.  No C++ exception crosses this ABI.  Device pointers are HIP
 * device allocations owned by the caller unless stated otherwise; `stream` is a
 * hipStream_t passed as void* (NULL = the null stream).  Nothing here synchronises or
 * allocates inside a launch function, so every op may be captured into a hipGraph.
 *
 * Which reference interface each entry point replaces (ShioMisaka/fce-yolo, ultralytics/):
 *   fce_conv2d            nn/modules/conv.py:39-89 Conv.forward_fuse (+BN fold torch_utils.py:237-267),
 *                         conv.py:185-200 DWConv, head.py:86-107 the Detect 1x1 nn.Conv2d,
 *                         block.py:474-476 Bottleneck residual, conv.py:616-641 Concat (channel-offset
 *                         writes), block.py:303-307 C2f chunk (channel-offset reads), nn.Upsample (up=1 reads)
 *   fce_maxpool_chain     block.py:228-232 SPPF's three chained MaxPool2d(5,1,2)
 *   fce_weighted_add      nn/modules/fce_block.py:40-63 BiFPN_Concat weighted fusion (Identity branches)
 *   fce_bicoordcrossatt   nn/modules/fce_block.py:183-284 BiCoordCrossAtt.forward
 *   fce_coordatt          nn/modules/fce_block.py:65-116  CoordAtt.forward
 *   fce_coordcrossatt     nn/modules/fce_block.py:119-180 CoordCrossAtt.forward
 *   fce_psa_attention     nn/modules/block.py:1284-1304   Attention.forward (softmax(q^T k) v + pe(v))
 *   fce_detect_decode     nn/modules/head.py:149-167 Detect._inference, block.py:76-79 DFL,
 *                         utils/tal.py:352-376 make_anchors / dist2bbox
 *   fce_nms               utils/nms.py:13-166 non_max_suppression + :239-296 TorchNMS.nms
 *   fce_copy              the NCHW <-> NHWC / fp32 <-> fp16 edges a drop-in module needs
 *   fce_net_*             nn/tasks.py:160-188 BaseModel._predict_once (graph executor) and
 *                         nn/autobackend.py:667-700 / :912-926 (forward, warmup) in hipGraph form
 */
#ifndef FCE_YOLO_H
#define FCE_YOLO_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FCE_ABI_VERSION 7

/* status codes */
#define FCE_OK 0
#define FCE_ERR_INVALID 1     /* bad argument / shape */
#define FCE_ERR_HIP 2         /* HIP runtime error */
#define FCE_ERR_UNSUPPORTED 3 /* valid but not implemented configuration */

/* dtypes / layouts / activations / epilogues */
#define FCE_F16 0
#define FCE_F32 1
#define FCE_U8 2
#define FCE_NHWC 0
#define FCE_NCHW 1
#define FCE_ACT_NONE 0
#define FCE_ACT_SILU 1
#define FCE_EPI_STORE 0  /* y = act(conv + b) [+ residual]                      */
#define FCE_EPI_WSTORE 1 /* y = alpha * act(conv + b)          (first BiFPN term)  */
#define FCE_EPI_ACCUM 2  /* y = y + alpha * act(conv + b)      (later BiFPN terms) */

/* A 4-D activation view.  NHWC views may be a channel slice [coff, coff+c) of a buffer
 * holding `cstride` channels per pixel (this is how Concat / chunk / split are free).
 * NCHW views are dense (cstride = c, coff = 0). */
typedef struct fce_tensor {
  void* data;
  int dtype;  /* FCE_F16 | FCE_F32 | FCE_U8 */
  int layout; /* FCE_NHWC | FCE_NCHW */
  int n, c, h, w;
  int cstride;
  int coff;
} fce_tensor;

const char* fce_last_error(void);
int fce_abi_version(void);
/* number of visible HIP devices (0 without a GPU); never fails */
int fce_device_count(void);

/* ---------------------------------------------------------------- convolution */
typedef struct fce_conv_desc {
  int cin, cout, k, stride; /* square kernel, pad = k/2 (conv.py:30-36 autopad) */
  int groups;               /* 1 = dense, cin (== cout) = depthwise               */
  int act;                  /* FCE_ACT_*                                          */
  int up;                   /* input read through nearest x(1<<up) upsampling     */
  int epilogue;             /* FCE_EPI_*                                          */
  const float* fusion_w;    /* BiFPN raw weights (device, fp32): alpha =          */
  int fusion_n, fusion_i;   /*   relu(w[i]) / (sum_j relu(w[j]) + 1e-4)           */
} fce_conv_desc;

/* Bytes of the packed fp16 weight image the conv kernels read (dense: MFMA fragment order;
 * depthwise / stem: tap-major fp32). */
size_t fce_conv_weight_bytes(const fce_conv_desc* d);
/* Host-side packing of an OIHW fp32 weight (BN already folded) into that image. */
int fce_conv_pack_weights(const fce_conv_desc* d, const float* w_oihw, void* packed_host);
/* y = conv(x) with the desc's epilogue.  x: NHWC f16 (or NCHW f16/f32/u8 when cin <= 4:
 * the stem path), y: NHWC f16 or f32, residual: NHWC f16 or NULL.  bias: cout fp32. */
int fce_conv2d(const fce_conv_desc* d, const fce_tensor* x, const void* w_packed, const float* bias,
               const fce_tensor* residual, const fce_tensor* y, void* stream);

/* Kernel variants of a conv (register tiles / LDS-tiled kernels / depthwise variants) for input width
 * in_w; every variant computes each output with the same summation order, so all give bitwise the
 * same result — the executor times them at plan and keeps the fastest.  Returns the count (<= cap). */
int fce_conv_variants(const fce_conv_desc* d, int in_w, int* codes, int cap);
/* fce_conv2d with an explicit variant code from fce_conv_variants (-1 = heuristic). */
int fce_conv2d_variant(const fce_conv_desc* d, const fce_tensor* x, const void* w_packed, const float* bias,
                       const fce_tensor* residual, const fce_tensor* y, int variant, void* stream);
/* fce_conv2d_variant of a plain 1x1 conv whose epilogue also stores output channels [dup_lo, dup_lo + dup->c)
 * into the dense view dup (the C2f / C3k2 cv1 duplicate store of fce_net_add_conv_dup; dup_lo, dup->c % 8 == 0):
 * every variant's store path writes the same fp16 values to both. */
int fce_conv2d_variant_dup(const fce_conv_desc* d, const fce_tensor* x, const void* w_packed, const float* bias,
                           const fce_tensor* residual, const fce_tensor* y, int variant, const fce_tensor* dup,
                           int dup_lo, void* stream);

/* Detect tail fused into the last 1x1 conv of a branch (head.py:149-167): part 0 = box branch
 * (4*reg_max logits -> DFL expectation -> xywh * stride into pred rows 0..3), part 1 = cls branch
 * (nc logits -> sigmoid into pred rows 4..).  pred: (N, 4+nc, anchors) fp32; this level's anchors
 * start at anchor_offset. */
typedef struct fce_detect_epi {
  float* pred;
  int anchors, anchor_offset, nc, reg_max, part;
  float stride;
  /* optional (NULL = off): per-anchor best-class key (n, anchors) uint64 = score bits << 32 | (~class),
   * the argmax of utils/nms.py:91-104 (first maximum) produced by the cls epilogue with an atomic max;
   * the box epilogue (part 0) of the same level zeroes it first.  fce_nms_best consumes it. */
  unsigned long long* best;
} fce_detect_epi;
int fce_conv2d_detect(const fce_conv_desc* d, const fce_tensor* x, const void* w_packed, const float* bias,
                      const fce_detect_epi* e, void* stream);

/* ---------------------------------------------------------------- pre / post processing */
/* One decoded source image (uint8 HWC BGR, device memory) and its letterbox placement, as computed by
 * the reference's LetterBox (data/augment.py:1555-1610; auto=False, center=True, scaleup=True). */
typedef struct fce_letterbox_img {
  const uint8_t* src;
  int h0, w0, row_stride;  /* source rows of row_stride bytes */
  int new_h, new_w;        /* resized (unpadded) size */
  int top, left;           /* placement on the canvas */
} fce_letterbox_img;
/* predictor.py:151-201 preprocess on the device: resize (cv2 INTER_LINEAR u8 semantics), pad with
 * pad_value, BGR -> RGB; dst = uint8 NCHW (n, 3, H, W), the engine's u8 network input.  imgs: n
 * descriptors in device memory. */
int fce_letterbox(const fce_letterbox_img* imgs, int n, uint8_t* dst, int H, int W, int pad_value, void* stream);
/* utils/ops.py:102-176 scale_boxes + clip_boxes per image (ratio_pad=None form): for slot k < counts[b]
 * of dets (n, max_det, 6): xyxy -= (pad_x, pad_y), /= gain, clamped to [0, w0] x [0, h0]. */
typedef struct fce_box_scale {
  float gain;
  int pad_x, pad_y, h0, w0;
} fce_box_scale;
int fce_scale_boxes(float* dets, const int32_t* counts, int n, int max_det, const fce_box_scale* params, void* stream);

/* ---------------------------------------------------------------- pooling / fusion */
/* SPPF chain: y1 = maxpool_k(x), y2 = maxpool_k(y1), y3 = maxpool_k(y2), stride 1, -inf pad. */
int fce_maxpool_chain(const fce_tensor* x, const fce_tensor* y1, const fce_tensor* y2, const fce_tensor* y3, int k,
                      void* stream);
/* BiFPN identity branch: y = (accumulate ? y : 0) + alpha_i * up(x). */
int fce_weighted_add(const fce_tensor* x, int up, const float* fusion_w, int fusion_n, int fusion_i, int accumulate,
                     const fce_tensor* y, void* stream);

/* ---------------------------------------------------------------- FCE coordinate attention */
typedef struct fce_coord_desc {
  int inp, oup, mid, heads; /* mid = dim_head*heads (BiCoord) / mip (CoordAtt, CoordCrossAtt) */
  float scale;              /* softmax scale                                                  */
  /* fp32 device weights of the 1x1 convs, TRANSPOSED: [in][out] row-major; biases [out].  Usage:
   *   BiCoordCrossAtt: w[0..5] = proj_q_h, proj_k_h, proj_v_h, proj_q_w, proj_k_w, proj_v_w (inp x mid),
   *                    w[6] = out_h, w[7] = out_w (mid x oup)
   *   CoordAtt:        w[0] = cv1 (inp x mid, BN folded, SiLU), w[1] = cv_h, w[2] = cv_w (mid x oup)
   *   CoordCrossAtt:   w[0] = cv1 (inp x mid), w[1..3] = q_conv, k_conv, v_conv (mid x mid), w[4] = proj */
  const float* w[8];
  const float* b[8];
  /* identity 1x1 conv when inp != oup (packed with fce_conv_pack_weights), else NULL */
  const void* id_w;
  const float* id_b;
} fce_coord_desc;

size_t fce_coord_workspace_bytes(const fce_coord_desc* d, int n, int h, int w);
int fce_bicoordcrossatt(const fce_coord_desc* d, const fce_tensor* x, const fce_tensor* y, void* ws, size_t ws_bytes,
                        void* stream);
int fce_coordatt(const fce_coord_desc* d, const fce_tensor* x, const fce_tensor* y, void* ws, size_t ws_bytes,
                 void* stream);
int fce_coordcrossatt(const fce_coord_desc* d, const fce_tensor* x, const fce_tensor* y, void* ws, size_t ws_bytes,
                      void* stream);

/* ---------------------------------------------------------------- C2PSA attention */
/* qkv: NHWC f16 with heads*(2*key_dim+head_dim) channels ([q|k|v] per head, block.py:1296);
 * y: NHWC f16 with heads*head_dim channels = softmax(q^T k * key_dim^-0.5) v + pe(v);
 * pe_w: 9 x (heads*head_dim) fp32 depthwise taps, BN folded — the layout fce_conv_pack_weights
 * produces for the depthwise desc (tap-major); pe_b: fp32 (heads*head_dim).
 * Only key_dim 32 / head_dim 64 (C2PSA: num_heads = c // 64, attn_ratio 0.5). */
int fce_psa_attention(const fce_tensor* qkv, int heads, int key_dim, int head_dim, const float* pe_w,
                      const float* pe_b, const fce_tensor* y, void* stream);

/* ---------------------------------------------------------------- Detect */
/* box[i]: NHWC f32 (4*reg_max ch), cls[i]: NHWC f32 (nc ch) for level i; out: (N, 4+nc, A) fp32,
 * A = sum_i h_i*w_i; rows 0-3 = xywh * stride (DFL expectation, fp32), rows 4.. = sigmoid(cls). */
int fce_detect_decode(const fce_tensor* box, const fce_tensor* cls, int nl, const float* strides, int reg_max,
                      float* out, void* stream);

/* ---------------------------------------------------------------- fused blocks */
/* C3k2 with c3k = False and one Bottleneck repeat (block.py:1064-1084, C2f.forward :303-307,
 * Bottleneck.forward :474-476): y = SiLU(cv2([a | b | m])), [a | b] = SiLU(cv1(x)),
 * m = SiLU(m.cv2(SiLU(m.cv1(b)))) + b, in one kernel (t / h / m stay in LDS).  w / b: the four convs'
 * packed weights (fce_conv_pack_weights) and BN-folded biases, in the order cv1 (cin -> 2c, 1x1),
 * m.cv1 (c -> c_mid, 3x3), m.cv2 (c_mid -> c, 3x3), cv2 (3c -> cout, 1x1); all SiLU.  Bitwise equal
 * to the four fce_conv2d calls.  fce_c3k2_supported: channel limits (c, c_mid, cout <= 128, ...). */
typedef struct fce_c3k2_desc {
  int cin, c, c_mid, cout;
  const void* w[4];
  const float* b[4];
} fce_c3k2_desc;
int fce_c3k2_supported(const fce_c3k2_desc* d);
int fce_c3k2(const fce_c3k2_desc* d, const fce_tensor* x, const fce_tensor* y, void* stream);

/* Detect cls branch of one level (head.py:86-107, legacy = False: DWConv(c0, c0, 3) -> Conv(c0, c3, 1) ->
 * DWConv(c3, c3, 3) -> Conv(c3, c3, 1) -> nn.Conv2d(c3, nc, 1), all but the last with SiLU) ending in the cls
 * epilogue of fce_conv2d_detect (e->part 1: sigmoid into pred rows 4.., the best-class key), in one kernel (t1..t4
 * stay in LDS).  w / b in the order dw1, pw1, dw2, pw2, cls: the five convs' fce_conv_pack_weights images (the
 * depthwise ones fp32 [9][c]) and BN-folded biases.  Bitwise equal to the five fce_conv2d / fce_conv2d_detect calls.
 * fce_detect_cls_supported: the instantiated (c0, c3, nc).  ABI v6. */
typedef struct fce_dcls_desc {
  int c0, c3, nc;
  const void* w[5];
  const float* b[5];
} fce_dcls_desc;
int fce_detect_cls_supported(const fce_dcls_desc* d);
int fce_detect_cls(const fce_dcls_desc* d, const fce_tensor* x, const fce_detect_epi* e, void* stream);

/* The backbone's first two convs (yaml rows 0-1: Conv(3, c0, 3, 2) -> Conv(c0, c1, 3, 2), both SiLU) in one
 * kernel: x NCHW 3-channel f16 / f32 / u8 (as fce_conv2d's stem), y NHWC f16 at a quarter of the input size; the
 * stem's output stays in LDS.  w / b: the two convs' fce_conv_pack_weights images and BN-folded biases.  Bitwise equal
 * to the two fce_conv2d calls.  fce_stem_fused_supported: the instantiated (c0, c1).  ABI v6. */
typedef struct fce_stem2_desc {
  int c0, c1;
  const void* w[2];
  const float* b[2];
} fce_stem2_desc;
int fce_stem_fused_supported(const fce_stem2_desc* d);
int fce_stem_fused(const fce_stem2_desc* d, const fce_tensor* x, const fce_tensor* y, void* stream);

/* A chain of n (1 or 2) Bottlenecks with the shortcut (block.py Bottleneck.forward :474-476: x = SiLU(cv2(SiLU(cv1(x))))
 * + x, cv1 3x3 c -> c_mid, cv2 3x3 c_mid -> c) in one kernel: C3k.m (block.py:1087-1108, n = 2, c_mid = c) and the
 * Bottleneck of C3k2(c3k = False) (:1064-1084, n = 1).  x, y NHWC f16 views of c channels; the intermediates stay in
 * LDS.  w / b: the 2 n convs' fce_conv_pack_weights images and BN-folded biases in chain order (cv1, cv2 of the first
 * Bottleneck, then of the second).  Bitwise equal to the 2 n fce_conv2d calls.  fce_bneck_supported: the instantiated
 * (c, c_mid, n); fce_bneck_fused also needs an instantiation for the map width (else FCE_ERR_INVALID).  ABI v7. */
typedef struct fce_bneck_desc {
  int c, c_mid, n, shortcut;
  const void* w[4];
  const float* b[4];
} fce_bneck_desc;
int fce_bneck_supported(const fce_bneck_desc* d);
int fce_bneck_fused(const fce_bneck_desc* d, const fce_tensor* x, const fce_tensor* y, void* stream);

/* Two chained 1x1 stride-1 convs in one kernel: h = act1(W1 x1 + b1) (+ r1) into the view h, then y = act2(W2 x2 +
 * b2) (+ r2) where x2 is a view of the SAME buffer as h whose channels overlapping h come straight from op 1 (the
 * pairs of C3k2 / C3k and C2PSA, block.py:303-307, :340, :1455-1464).  h is written to HBM when h_store (another op
 * reads it).  dup (nullable): op 2's output channels [dup_lo, dup_lo + dup.c) stored a second time (as
 * fce_conv2d_variant_dup).  act: FCE_ACT_SILU / FCE_ACT_NONE; w / b: the two convs' fce_conv_pack_weights images and
 * biases.  epi1: op 1's epilogue, FCE_EPI_STORE (0), or FCE_EPI_WSTORE / FCE_EPI_ACCUM with the BiFPN weights fw
 * (device, fn of them, this input's index fi) as fce_conv_desc takes them: op 1 is then a BiFPN_Concat realign conv
 * (fce_block.py:57-63) whose weighted sum op 2 reads (ACCUM: h's previous contents are read and added).  Bitwise
 * equal to the two fce_conv2d calls.  fce_pw2_supported: the instantiated channel counts.  ABI v7. */
typedef struct fce_pw2_desc {
  int cin1, cout1, cin2, cout2;
  int act[2];
  const void* w[2];
  const float* b[2];
  int epi1;
  const float* fw;
  int fn, fi;
} fce_pw2_desc;
int fce_pw2_supported(const fce_pw2_desc* d);
int fce_pw2(const fce_pw2_desc* d, const fce_tensor* x1, const fce_tensor* r1, const fce_tensor* h, int h_store,
            const fce_tensor* x2, const fce_tensor* r2, const fce_tensor* y, const fce_tensor* dup, int dup_lo,
            void* stream);

/* ---------------------------------------------------------------- NMS */
size_t fce_nms_workspace_bytes(int n, int anchors, int max_nms);
/* pred: (N, 4+nc, A) fp32.  dets: N x max_det x 6 (x1,y1,x2,y2,conf,cls), keep: N x max_det
 * anchor indices, counts: N.  Bit-exact with the reference for distinct scores; ties in the
 * score sort are broken by ascending anchor index. */
int fce_nms(const float* pred, int n, int nc, int anchors, float conf_thres, float iou_thres, int max_det,
            int max_nms, float max_wh, void* ws, size_t ws_bytes, float* dets, int64_t* keep, int32_t* counts,
            void* stream);
/* fce_nms with the per-anchor best-class keys (fce_detect_epi::best) of the forward that wrote pred:
 * the class arg-max pass over pred's nc rows (nms.py:91-104) is skipped.  Same results as fce_nms. */
int fce_nms_best(const float* pred, const unsigned long long* best, int n, int nc, int anchors, float conf_thres,
                 float iou_thres, int max_det, int max_nms, float max_wh, void* ws, size_t ws_bytes, float* dets,
                 int64_t* keep, int32_t* counts, void* stream);

/* Non-default arguments of non_max_suppression (utils/nms.py:13-29), ABI v4:
 *   agnostic     nms.py:141   class offset c = cls * 0 (one NMS over all classes);
 *   multi_label  nms.py:116-120  one candidate per (anchor, class) with score > conf_thres, in (anchor, class)
 *                order (torch.where), when nc > 1; the workspace then holds anchors * nc candidates;
 *   classes      nms.py:128-132  keep only candidates whose class is in the host list (class ids < 1024).
 * best (optional, the forward's best-class keys) is ignored with multi_label.  Bit-exact with the reference
 * for distinct scores, like fce_nms. */
typedef struct fce_nms_opts {
  float conf_thres, iou_thres;
  int max_det, max_nms;
  float max_wh;
  int agnostic, multi_label;
  const int32_t* classes; /* host array, or NULL for every class */
  int nclasses;
} fce_nms_opts;
size_t fce_nms_workspace_bytes_ex(int n, int nc, int anchors, const fce_nms_opts* o);
int fce_nms_ex(const float* pred, const unsigned long long* best, int n, int nc, int anchors, const fce_nms_opts* o,
               void* ws, size_t ws_bytes, float* dets, int64_t* keep, int32_t* counts, void* stream);

/* ---------------------------------------------------------------- layout / dtype edges */
/* dst = src with layout / dtype conversion (same n,c,h,w). */
int fce_copy(const fce_tensor* src, const fce_tensor* dst, void* stream);

/* ---------------------------------------------------------------- whole-graph executor */
typedef struct fce_net fce_net;
fce_net* fce_net_create(void);
void fce_net_destroy(fce_net* net);
/* Activation buffer: `c` channels at (H >> shift, W >> shift); dtype FCE_F16 or FCE_F32. */
int fce_net_add_buffer(fce_net* net, int c, int shift, int dtype);
/* ops reference buffers by id; channel slices by (coff, c).  -1 = the network input. */
int fce_net_add_conv(fce_net* net, const fce_conv_desc* d, int in_buf, int in_coff, int out_buf, int out_coff,
                     int res_buf, int res_coff, const void* w_packed, const float* bias);
/* fce_net_add_conv whose output channels [dup_lo, dup_lo + dup_c) are ALSO stored into buffer dup (exactly
 * dup_c channels, same spatial size): a 1x1 conv with a plain fp16 store, 8-aligned channel ranges (ABI v5).
 * The C2f / C3k2 lowering gives the chunk its bottlenecks read (block.py:303-307) a dense copy, so their 3x3
 * convs read whole cache lines instead of a 16- or 32-channel slice of the concat record. */
int fce_net_add_conv_dup(fce_net* net, const fce_conv_desc* d, int in_buf, int in_coff, int out_buf, int out_coff,
                         int res_buf, int res_coff, const void* w_packed, const float* bias, int dup_buf, int dup_lo,
                         int dup_c);
int fce_net_add_maxpool_chain(fce_net* net, int buf, int in_coff, int c, int k);
int fce_net_add_weighted_add(fce_net* net, int in_buf, int in_coff, int c, int up, const float* fusion_w,
                             int fusion_n, int fusion_i, int accumulate, int out_buf, int out_coff);
int fce_net_add_coord(fce_net* net, int kind /*0 BiCoord,1 CoordAtt,2 CoordCross*/, const fce_coord_desc* d,
                      int in_buf, int in_coff, int out_buf, int out_coff);
int fce_net_add_psa_attention(fce_net* net, int qkv_buf, int heads, int key_dim, int head_dim, const float* pe_w,
                              const float* pe_b, int out_buf, int out_coff);
int fce_net_add_c3k2(fce_net* net, const fce_c3k2_desc* d, int in_buf, int in_coff, int out_buf, int out_coff);
/* The fused C3k2 as an ALTERNATIVE to the nops conv ops just added (its cv1, m.cv1, m.cv2, cv2, writing the same
 * output): exactly one form runs.  The fused form is active until fce_net_plan's autotune times both on the
 * planned shapes and keeps the faster (FCE_FUSE_C3K2=1: keep the fused form).  Both forms are bitwise equal. */
int fce_net_add_c3k2_alt(fce_net* net, const fce_c3k2_desc* d, int in_buf, int in_coff, int out_buf, int out_coff,
                         int first_op, int nops);
/* 1 = op i (an fce_net_add_c3k2_alt op) runs fused, 0 = its convs run, -1 = not such an op */
int fce_net_c3k2_form(const fce_net* net, int i);
int fce_net_set_c3k2_form(fce_net* net, int i, int fused);
/* The fused Detect cls branch (fce_detect_cls) as an ALTERNATIVE to the nops (= 5) ops just added: the branch's two
 * depthwise and two 1x1 fce_net_add_conv ops and its cls fce_net_add_conv_detect, one chain from (in_buf, in_coff)
 * with the weights of d.  Exactly one form runs; the plan-time autotune keeps the faster (FCE_FUSE_DCLS=1: the fused
 * form).  ABI v6. */
int fce_net_add_detect_cls_alt(fce_net* net, const fce_dcls_desc* d, int in_buf, int in_coff, int first_op, int nops);
/* The fused stem pair (fce_stem_fused) as an ALTERNATIVE to the nops (= 2) ops just added: the stem conv reading the
 * network input and the stride-2 3x3 conv reading all of its output.  fce_net_plan keeps the two convs when any other
 * op reads the stem's output buffer; otherwise the autotune keeps the faster form (FCE_FUSE_STEM=1: fused).  ABI v6. */
int fce_net_add_stem_alt(fce_net* net, const fce_stem2_desc* d, int first_op, int nops);
/* The fused Bottleneck chain (fce_bneck_fused) as an ALTERNATIVE to the nops (= 2 n) conv ops just added: the chain's
 * 3x3 convs, the first reading (in_buf, in_coff), the last writing (out_buf, out_coff), each odd one adding the input of
 * its Bottleneck.  fce_net_plan keeps the convs when no instantiation covers the planned map width; otherwise the
 * autotune keeps the faster form (FCE_FUSE_BNECK=1: fused).  ABI v7. */
int fce_net_add_bneck_alt(fce_net* net, const fce_bneck_desc* d, int in_buf, int in_coff, int out_buf, int out_coff,
                          int first_op, int nops);
/* The fused 1x1 pair (fce_pw2) as an ALTERNATIVE to the two conv ops just added (first_op, first_op + 1: the second
 * reading channels of the first's output buffer); fce_net_plan decides whether h must still be stored (another op
 * reads it) and the autotune keeps the faster form (FCE_FUSE_PW2=1: fused).  ABI v7. */
int fce_net_add_pw2_alt(fce_net* net, const fce_pw2_desc* d, int first_op);
/* Any alternative op (fused C3k2 or fused Detect cls branch): 1 = the fused form runs, 0 = the ops it replaces run,
 * -1 = op i is not an alternative.  ABI v6. */
int fce_net_alt_form(const fce_net* net, int i);
int fce_net_set_alt_form(fce_net* net, int i, int fused);
/* 1 when op i belongs to the inactive form of an alternative (it launches nothing; profile / op_info report 0) */
int fce_net_op_skipped(const fce_net* net, int i);
/* map_bufs[i]: f32 buffer of level i holding cat(box 4*reg_max, cls nc) channels (head.py:122) */
int fce_net_add_detect(fce_net* net, int nl, const int* map_bufs, const float* strides, int reg_max);
/* Fused Detect tail conv (see fce_conv2d_detect) writing the forward's pred output; `level` orders
 * the anchor blocks (offsets are resolved at plan time). */
int fce_net_add_conv_detect(fce_net* net, const fce_conv_desc* d, int in_buf, int in_coff, int part, int level,
                            float stride, int nc, int reg_max, const void* w_packed, const float* bias);
/* allocate the arena for (batch, H, W); invalidates any captured graph.  Times every candidate kernel
 * variant of every conv and keeps the fastest unless the environment sets FCE_AUTOTUNE=0. */
int fce_net_plan(fce_net* net, int batch, int h, int w);
/* fce_net_plan with explicit options instead of the environment (ABI v5):
 * FCE_PLAN_NO_AUTOTUNE keeps the heuristic variants (e.g. a second executor that copies another's picks). */
#define FCE_PLAN_NO_AUTOTUNE 1
int fce_net_plan_ex(fce_net* net, int batch, int h, int w, int flags);
size_t fce_net_arena_bytes(const fce_net* net);
int fce_net_num_anchors(const fce_net* net);
/* input: NCHW f16/f32/u8 (u8 is divided by 255 in the stem); pred: (batch, 4+nc, A) fp32.
 * graph=1 captures the whole forward into a hipGraph on first use for these pointers and
 * replays it afterwards (re-captured if the pointers change). */
int fce_net_forward(fce_net* net, const fce_tensor* input, float* pred, int graph, void* stream);
/* fce_net_forward that also writes the per-anchor best-class keys (batch, A) uint64 for fce_nms_best
 * (best may be NULL).  fce_net_profile runs with the keys of the most recent forward. */
int fce_net_forward_best(fce_net* net, const fce_tensor* input, float* pred, unsigned long long* best, int graph,
                         void* stream);
/* Fork point for overlapping work with the forward (SURVEY §8(e) double-buffered batches): after
 * fce_net_set_fork(net, op), every direct-launch forward records an event after op `op` (at the end
 * with graph replay / multiple streams / op = -1), and fce_net_wait_fork(net, stream) makes `stream`
 * wait for the most recent such event.  fce_net_fork_hint = the first op at the coarsest resolution. */
int fce_net_fork_hint(const fce_net* net);
int fce_net_set_fork(fce_net* net, int op);
int fce_net_wait_fork(fce_net* net, void* stream);
/* Eager run in which every kernel is launched with its own (start, stop) event pair
 * (hipExtLaunchKernelGGL): ms[i] = summed kernel execution time of op i, launches[i] (nullable) = its
 * kernel count (cap entries each). */
int fce_net_profile(fce_net* net, const fce_tensor* input, float* pred, float* ms, int* launches, int cap,
                    void* stream);
int fce_net_num_ops(const fce_net* net);
/* name (kernel family), algorithmic bytes and flops of op i at the planned size (before fce_net_plan: the name,
 * zero bytes and flops) */
int fce_net_op_info(const fce_net* net, int i, char* name, int name_cap, double* bytes, double* flops);
int fce_net_buffer(const fce_net* net, int id, fce_tensor* out);
/* kernel variant code the plan-time autotune chose for op i (-1 = heuristic / not tunable) */
int fce_net_op_variant(const fce_net* net, int i);
/* Candidate kernel variants of conv op i (as fce_conv_variants, for the planned shapes); 0 for other ops. */
int fce_net_op_variants(const fce_net* net, int i, int* codes, int cap);
/* Pin conv op i to a candidate variant (-1 = heuristic), e.g. to replay a tuning recorded elsewhere or to
 * check variants against each other; results are bitwise the same for every candidate. */
int fce_net_set_op_variant(fce_net* net, int i, int code);
/* k-th autotune measurement of the last plan: op index, variant code, ms per run; returns 0 past the end */
int fce_net_tune_record(const fce_net* net, int k, int* op, int* code, float* ms);

#ifdef __cplusplus
}
#endif
#endif /* FCE_YOLO_H */
