// C-ABI entry points (include/fce_yolo.h) and the native whole-graph executor.
//
// The executor restates BaseModel._predict_once (reference ultralytics/nn/tasks.py:160-188) as a
// flat list of kernel launches over an NHWC fp16 arena whose buffers are planned once per
// (batch, H, W): every layer output, every C2f/C3/SPPF/C2PSA concat buffer and the fp32 Detect
// maps live at fixed offsets, so one forward is a fixed launch sequence that is captured into a
// hipGraph and replayed (AutoBackend.forward / warmup, nn/autobackend.py:667-700, :912-926).
#include <algorithm>
#include <exception>
#include <memory>
#include <vector>

#include "common.h"

namespace fce {

// kernels (other translation units)
size_t conv_weight_bytes(const fce_conv_desc& d);
int conv_pack(const fce_conv_desc& d, const float* w, void* out);
int conv2d(const fce_conv_desc& d, const fce_tensor& x, const void* w, const float* bias, const fce_tensor* res,
           const fce_tensor& y, hipStream_t s, int tile = -1, const fce_tensor* dup = nullptr, int duplo = 0);
int conv2d_detect(const fce_conv_desc& d, const fce_tensor& x, const void* w, const float* bias,
                  const fce_detect_epi& e, hipStream_t s, int tile = -1);
int conv_tile_candidates(const fce_conv_desc& d, int det_box, int in_w, int* out, int cap);
int maxpool_chain(const fce_tensor& x, const fce_tensor& y1, const fce_tensor& y2, const fce_tensor& y3, int k,
                  hipStream_t s);
int weighted_add(const fce_tensor& x, int up, const float* fw, int fn, int fi, int accumulate, const fce_tensor& y,
                 hipStream_t s);
int copy(const fce_tensor& src, const fce_tensor& dst, hipStream_t s);
size_t coord_ws_bytes(const fce_coord_desc& d, int n, int h, int w);
int bicoordcrossatt(const fce_coord_desc& d, const fce_tensor& x, const fce_tensor& y, void* ws, size_t wsb,
                    hipStream_t s);
int coordatt(const fce_coord_desc& d, const fce_tensor& x, const fce_tensor& y, void* ws, size_t wsb, hipStream_t s);
int coordcrossatt(const fce_coord_desc& d, const fce_tensor& x, const fce_tensor& y, void* ws, size_t wsb,
                  hipStream_t s);
int psa_attention(const fce_tensor& qkv, int heads, int key_dim, int head_dim, const float* pe_w, const float* pe_b,
                  const fce_tensor& y, hipStream_t s);
int detect_decode(const fce_tensor* box, const fce_tensor* cls, int nl, const float* strides, int reg_max,
                  float* out, hipStream_t s);
size_t nms_ws_bytes(int n, int A, int max_nms);
size_t nms_ws_bytes_ex(int n, int nc, int A, int max_nms, int multi);
int nms(const float* pred, const unsigned long long* best, int n, int nc, int A, float conf, float iou, int max_det,
        int max_nms, float max_wh, void* ws, size_t ws_bytes, float* dets, int64_t* keep, int32_t* counts,
        hipStream_t s, int multi = 0, const int32_t* classes = nullptr, int nclasses = 0);

bool c3k2_fused_ok(const fce_c3k2_desc& d);
int c3k2_fused(const fce_c3k2_desc& d, const fce_tensor& x, const fce_tensor& y, hipStream_t s);
bool detect_cls_fused_ok(const fce_dcls_desc& d);
bool stem_fused_ok(const fce_stem2_desc& d);
bool stem_fused_fits(const fce_stem2_desc& d, int h, int w);
int stem_fused(const fce_stem2_desc& d, const fce_tensor& x, const fce_tensor& y, hipStream_t s);
int detect_cls_fused(const fce_dcls_desc& d, const fce_tensor& x, const fce_detect_epi& e, hipStream_t s);
bool bneck_fused_ok(const fce_bneck_desc& d);
bool bneck_fused_fits(const fce_bneck_desc& d, int h, int w);
int bneck_fused(const fce_bneck_desc& d, const fce_tensor& x, const fce_tensor& y, hipStream_t s);
bool pw2_fused_ok(const fce_pw2_desc& d);
int pw2_fused(const fce_pw2_desc& d, const fce_tensor& x1, const fce_tensor* r1, const fce_tensor& h, int h_store,
              const fce_tensor& x2, const fce_tensor* r2, const fce_tensor& y, const fce_tensor* dup, int dup_lo,
              hipStream_t s);

int letterbox(const fce_letterbox_img* imgs, int n, uint8_t* dst, int H, int W, int pad, hipStream_t s);
int scale_boxes(float* dets, const int32_t* counts, int n, int max_det, const fce_box_scale* sc, hipStream_t s);

static thread_local std::string g_err;
static thread_local LaunchProbe* g_probe = nullptr;
LaunchProbe*& probe_slot() { return g_probe; }
void set_error(const std::string& m) { g_err = m; }
int fail(int code, const std::string& m) {
  g_err = m;
  return code;
}
int check_nhwc(const fce_tensor* t, const char* name, int dtype) {
  if (!t) return fail(FCE_ERR_INVALID, std::string(name) + ": null tensor");
  if (t->layout != FCE_NHWC || t->dtype != dtype) return fail(FCE_ERR_INVALID, std::string(name) + ": wrong layout/dtype");
  return FCE_OK;
}

}  // namespace fce

using namespace fce;

#define FCE_GUARD(...)                                     \
  try {                                                    \
    __VA_ARGS__                                            \
  } catch (const std::exception& e) {                      \
    return fail(FCE_ERR_INVALID, std::string("exception: ") + e.what()); \
  } catch (...) {                                          \
    return fail(FCE_ERR_INVALID, "unknown exception");     \
  }

extern "C" {

const char* fce_last_error(void) { return g_err.c_str(); }
int fce_abi_version(void) { return FCE_ABI_VERSION; }
int fce_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

size_t fce_conv_weight_bytes(const fce_conv_desc* d) { return d ? conv_weight_bytes(*d) : 0; }
int fce_conv_pack_weights(const fce_conv_desc* d, const float* w, void* out) {
  FCE_CHECK(d && w && out, "fce_conv_pack_weights: null argument");
  FCE_GUARD(return conv_pack(*d, w, out);)
}
int fce_conv2d(const fce_conv_desc* d, const fce_tensor* x, const void* w, const float* bias, const fce_tensor* res,
               const fce_tensor* y, void* stream) {
  FCE_CHECK(d && x && w && bias && y, "fce_conv2d: null argument");
  FCE_GUARD(return conv2d(*d, *x, w, bias, res, *y, S(stream));)
}
int fce_conv_variants(const fce_conv_desc* d, int in_w, int* codes, int cap) {
  if (!d || !codes || cap <= 0) return 0;
  return conv_tile_candidates(*d, 0, in_w, codes, cap);
}
int fce_conv2d_variant(const fce_conv_desc* d, const fce_tensor* x, const void* w, const float* bias,
                       const fce_tensor* res, const fce_tensor* y, int variant, void* stream) {
  FCE_CHECK(d && x && w && bias && y, "fce_conv2d_variant: null argument");
  FCE_GUARD(return conv2d(*d, *x, w, bias, res, *y, S(stream), variant);)
}
int fce_conv2d_variant_dup(const fce_conv_desc* d, const fce_tensor* x, const void* w, const float* bias,
                           const fce_tensor* res, const fce_tensor* y, int variant, const fce_tensor* dup, int dup_lo,
                           void* stream) {
  FCE_CHECK(d && x && w && bias && y && dup, "fce_conv2d_variant_dup: null argument");
  FCE_CHECK(d->k == 1 && d->groups == 1 && d->epilogue == FCE_EPI_STORE && dup->dtype == FCE_F16 &&
                dup->layout == FCE_NHWC && dup_lo >= 0 && dup_lo % 8 == 0 && dup->c % 8 == 0 &&
                dup_lo + dup->c <= d->cout && dup->n == y->n && dup->h == y->h && dup->w == y->w,
            "fce_conv2d_variant_dup: the duplicate store needs a plain 1x1 conv and an aligned f16 view of y's size");
  FCE_GUARD(return conv2d(*d, *x, w, bias, res, *y, S(stream), variant, dup, dup_lo);)
}
int fce_c3k2_supported(const fce_c3k2_desc* d) { return d && c3k2_fused_ok(*d) ? 1 : 0; }
int fce_c3k2(const fce_c3k2_desc* d, const fce_tensor* x, const fce_tensor* y, void* stream) {
  FCE_CHECK(d && x && y, "fce_c3k2: null argument");
  FCE_GUARD(return c3k2_fused(*d, *x, *y, S(stream));)
}
int fce_detect_cls_supported(const fce_dcls_desc* d) { return d && detect_cls_fused_ok(*d) ? 1 : 0; }
int fce_detect_cls(const fce_dcls_desc* d, const fce_tensor* x, const fce_detect_epi* e, void* stream) {
  FCE_CHECK(d && x && e, "fce_detect_cls: null argument");
  FCE_GUARD(return detect_cls_fused(*d, *x, *e, S(stream));)
}
int fce_bneck_supported(const fce_bneck_desc* d) { return d && bneck_fused_ok(*d) ? 1 : 0; }
int fce_bneck_fused(const fce_bneck_desc* d, const fce_tensor* x, const fce_tensor* y, void* stream) {
  FCE_CHECK(d && x && y, "fce_bneck_fused: null argument");
  FCE_GUARD(return bneck_fused(*d, *x, *y, S(stream));)
}
int fce_pw2_supported(const fce_pw2_desc* d) { return d && pw2_fused_ok(*d) ? 1 : 0; }
int fce_pw2(const fce_pw2_desc* d, const fce_tensor* x1, const fce_tensor* r1, const fce_tensor* h, int h_store,
            const fce_tensor* x2, const fce_tensor* r2, const fce_tensor* y, const fce_tensor* dup, int dup_lo,
            void* stream) {
  FCE_CHECK(d && x1 && h && x2 && y, "fce_pw2: null argument");
  FCE_GUARD(return pw2_fused(*d, *x1, r1, *h, h_store, *x2, r2, *y, dup, dup_lo, S(stream));)
}
int fce_stem_fused_supported(const fce_stem2_desc* d) { return d && stem_fused_ok(*d) ? 1 : 0; }
int fce_stem_fused(const fce_stem2_desc* d, const fce_tensor* x, const fce_tensor* y, void* stream) {
  FCE_CHECK(d && x && y, "fce_stem_fused: null argument");
  FCE_GUARD(return stem_fused(*d, *x, *y, S(stream));)
}
int fce_conv2d_detect(const fce_conv_desc* d, const fce_tensor* x, const void* w, const float* bias,
                      const fce_detect_epi* e, void* stream) {
  FCE_CHECK(d && x && w && bias && e, "fce_conv2d_detect: null argument");
  FCE_GUARD(return conv2d_detect(*d, *x, w, bias, *e, S(stream));)
}
int fce_maxpool_chain(const fce_tensor* x, const fce_tensor* y1, const fce_tensor* y2, const fce_tensor* y3, int k,
                      void* stream) {
  FCE_CHECK(x && y1 && y2 && y3, "fce_maxpool_chain: null argument");
  FCE_GUARD(return maxpool_chain(*x, *y1, *y2, *y3, k, S(stream));)
}
int fce_weighted_add(const fce_tensor* x, int up, const float* fw, int fn, int fi, int accumulate, const fce_tensor* y,
                     void* stream) {
  FCE_CHECK(x && y, "fce_weighted_add: null argument");
  FCE_GUARD(return weighted_add(*x, up, fw, fn, fi, accumulate, *y, S(stream));)
}
size_t fce_coord_workspace_bytes(const fce_coord_desc* d, int n, int h, int w) {
  return d ? coord_ws_bytes(*d, n, h, w) : 0;
}
int fce_bicoordcrossatt(const fce_coord_desc* d, const fce_tensor* x, const fce_tensor* y, void* ws, size_t wsb,
                        void* stream) {
  FCE_CHECK(d && x && y, "fce_bicoordcrossatt: null argument");
  FCE_GUARD(return bicoordcrossatt(*d, *x, *y, ws, wsb, S(stream));)
}
int fce_coordatt(const fce_coord_desc* d, const fce_tensor* x, const fce_tensor* y, void* ws, size_t wsb,
                 void* stream) {
  FCE_CHECK(d && x && y, "fce_coordatt: null argument");
  FCE_GUARD(return coordatt(*d, *x, *y, ws, wsb, S(stream));)
}
int fce_coordcrossatt(const fce_coord_desc* d, const fce_tensor* x, const fce_tensor* y, void* ws, size_t wsb,
                      void* stream) {
  FCE_CHECK(d && x && y, "fce_coordcrossatt: null argument");
  FCE_GUARD(return coordcrossatt(*d, *x, *y, ws, wsb, S(stream));)
}
int fce_psa_attention(const fce_tensor* qkv, int heads, int kd, int hd, const float* pe_w, const float* pe_b,
                      const fce_tensor* y, void* stream) {
  FCE_CHECK(qkv && y && pe_w && pe_b, "fce_psa_attention: null argument");
  FCE_GUARD(return psa_attention(*qkv, heads, kd, hd, pe_w, pe_b, *y, S(stream));)
}
int fce_detect_decode(const fce_tensor* box, const fce_tensor* cls, int nl, const float* strides, int reg_max,
                      float* out, void* stream) {
  FCE_CHECK(box && cls && strides && out, "fce_detect_decode: null argument");
  FCE_GUARD(return detect_decode(box, cls, nl, strides, reg_max, out, S(stream));)
}
size_t fce_nms_workspace_bytes(int n, int anchors, int max_nms) { return nms_ws_bytes(n, anchors, max_nms); }
int fce_nms(const float* pred, int n, int nc, int A, float conf, float iou, int max_det, int max_nms, float max_wh,
            void* ws, size_t wsb, float* dets, int64_t* keep, int32_t* counts, void* stream) {
  FCE_CHECK(pred && dets && keep && counts, "fce_nms: null argument");
  FCE_GUARD(return nms(pred, nullptr, n, nc, A, conf, iou, max_det, max_nms, max_wh, ws, wsb, dets, keep, counts,
                       S(stream));)
}
int fce_nms_best(const float* pred, const unsigned long long* best, int n, int nc, int A, float conf, float iou,
                 int max_det, int max_nms, float max_wh, void* ws, size_t wsb, float* dets, int64_t* keep,
                 int32_t* counts, void* stream) {
  FCE_CHECK(pred && best && dets && keep && counts, "fce_nms_best: null argument");
  FCE_GUARD(return nms(pred, best, n, nc, A, conf, iou, max_det, max_nms, max_wh, ws, wsb, dets, keep, counts,
                       S(stream));)
}
size_t fce_nms_workspace_bytes_ex(int n, int nc, int anchors, const fce_nms_opts* o) {
  return o ? nms_ws_bytes_ex(n, nc, anchors, o->max_nms, o->multi_label) : 0;
}
int fce_nms_ex(const float* pred, const unsigned long long* best, int n, int nc, int A, const fce_nms_opts* o, void* ws,
               size_t wsb, float* dets, int64_t* keep, int32_t* counts, void* stream) {
  FCE_CHECK(pred && o && dets && keep && counts, "fce_nms_ex: null argument");
  FCE_GUARD(return nms(pred, best, n, nc, A, o->conf_thres, o->iou_thres, o->max_det, o->max_nms,
                       o->agnostic ? 0.f : o->max_wh, ws, wsb, dets, keep, counts, S(stream), o->multi_label,
                       o->classes, o->nclasses);)
}
int fce_letterbox(const fce_letterbox_img* imgs, int n, uint8_t* dst, int H, int W, int pad_value, void* stream) {
  FCE_GUARD(return letterbox(imgs, n, dst, H, W, pad_value, S(stream));)
}
int fce_scale_boxes(float* dets, const int32_t* counts, int n, int max_det, const fce_box_scale* params,
                    void* stream) {
  FCE_GUARD(return scale_boxes(dets, counts, n, max_det, params, S(stream));)
}
int fce_copy(const fce_tensor* src, const fce_tensor* dst, void* stream) {
  FCE_CHECK(src && dst, "fce_copy: null argument");
  FCE_GUARD(return copy(*src, *dst, S(stream));)
}

}  // extern "C"

// ============================================================================ executor
namespace {

enum OpKind { OP_CONV, OP_MAXPOOL, OP_WADD, OP_COORD, OP_PSA, OP_DETECT, OP_CONV_DETECT, OP_C3K2, OP_DCLS, OP_STEM2, OP_BNECK, OP_PW2 };

struct BufDesc {
  int c, shift, dtype;
  size_t offset = 0, bytes = 0;
};

struct OpDesc {
  OpKind kind;
  fce_conv_desc conv{};
  fce_coord_desc coord{};
  int coord_kind = 0;
  int in = -1, in_coff = 0, in_c = 0;
  int out = -1, out_coff = 0;
  int res = -1, res_coff = 0;
  const void* w = nullptr;
  const float* b = nullptr;
  int k = 0, up = 0, accumulate = 0;
  const float* fw = nullptr;
  int fn = 0, fi = 0;
  int heads = 0, key_dim = 0, head_dim = 0;
  const float* pe_w = nullptr;
  const float* pe_b = nullptr;
  int nl = 0;
  int box[4] = {0, 0, 0, 0}, cls[4] = {0, 0, 0, 0};
  float strides[4] = {0, 0, 0, 0};
  int reg_max = 16;
  int part = 0, level = 0, nc = 0;  // OP_CONV_DETECT, OP_DCLS (part 1)
  fce_c3k2_desc c3k2{};              // OP_C3K2
  fce_dcls_desc dcls{};              // OP_DCLS
  fce_stem2_desc stem2{};            // OP_STEM2
  fce_bneck_desc bneck{};            // OP_BNECK
  fce_pw2_desc pw2{};                // OP_PW2: op 1 = in / res / out (h), op 2 = in2 / res2 / out2 / dup
  int in2 = -1, in2_coff = 0, res2 = -1, res2_coff = 0, out2 = -1, out2_coff = 0, h_store = 1;
  int tile = -1;                     // dense conv register tile (autotuned at plan), -1 = heuristic
  int dup = -1, dup_lo = 0, dup_c = 0;  // OP_CONV duplicate store of out channels [dup_lo, +dup_c) into buffer dup
  // alternative forms: an OP_C3K2 / OP_DCLS added by fce_net_add_c3k2_alt / fce_net_add_detect_cls_alt computes the
  // same output as ops [alt_first, alt_first + alt_n) (its four convs / its five ops); exactly one form runs, the
  // other's ops are skipped (plan-time choice)
  int alt_first = -1, alt_n = 0;
  bool alt_locked = false;  // the alternative cannot run in this net (fce_net_plan found a reason): the ops it replaces run
  bool skip = false;
};

}  // namespace

struct fce_net {
  std::vector<BufDesc> bufs;
  std::vector<OpDesc> ops;
  struct TuneRec {
    int op, code;
    float ms;
  };
  std::vector<TuneRec> tune_log;  // plan-time autotune measurements (fce_net_tune_record)
  int batch = 0, H = 0, W = 0;
  char* arena = nullptr;
  size_t arena_bytes = 0;
  void* ws = nullptr;
  size_t ws_bytes = 0;
  int anchors = 0, nc = 0;
  int level_off[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  // captured forwards, one per (input, pred, stream, input dtype / channels): a double-buffered caller
  // (engine.Pipeline alternates two pred buffers) replays its graphs instead of recapturing
  struct Captured {
    hipGraph_t graph;
    hipGraphExec_t exec;
    const void* in;
    float* out;
    unsigned long long* best;
    hipStream_t stream;
    int dtype, c;
    unsigned long long used;
  };
  static constexpr int kMaxGraphs = 4;
  unsigned long long* cur_best = nullptr;  // best-class key output of the current forward (or null)
  // fork point: after op fork_op of a direct-launch forward, mid_ev is recorded on the forward's stream
  // (a side stream can start concurrent work -- the previous batch's NMS -- where the forward leaves
  // CUs idle); with graph replay, multiple streams or fork_op < 0 it is recorded at the end instead
  int fork_op = -1;
  hipEvent_t mid_ev = nullptr;
  std::vector<Captured> graphs;
  unsigned long long graph_clock = 0;
  // multi-stream capture: side streams + one event per op (+ fork), created on first capture
  std::vector<hipStream_t> side;
  std::vector<hipEvent_t> op_ev;
  hipEvent_t fork_ev = nullptr;
  hipStream_t own = nullptr;                   // capture/replay stream when the caller passes the null stream
  hipEvent_t join_ev[2] = {nullptr, nullptr};  // caller -> own, own -> caller

  void drop_streams() {
    for (hipEvent_t e : op_ev) (void)hipEventDestroy(e);
    op_ev.clear();
    if (fork_ev) (void)hipEventDestroy(fork_ev);
    fork_ev = nullptr;
    for (hipStream_t q : side) (void)hipStreamDestroy(q);
    side.clear();
    for (hipEvent_t& e : join_ev) {
      if (e) (void)hipEventDestroy(e);
      e = nullptr;
    }
    if (own) (void)hipStreamDestroy(own);
    own = nullptr;
  }

  static void destroy(Captured& c) {
    if (c.exec) (void)hipGraphExecDestroy(c.exec);
    if (c.graph) (void)hipGraphDestroy(c.graph);
  }
  void drop_graph() {  // every captured forward (the plan, a buffer or an op variant changed)
    for (Captured& c : graphs) destroy(c);
    graphs.clear();
  }
  void release() {
    drop_graph();
    if (arena) (void)hipFree(arena);
    if (ws) (void)hipFree(ws);
    arena = nullptr;
    ws = nullptr;
    arena_bytes = ws_bytes = 0;
  }
  ~fce_net() {
    release();
    drop_streams();
    if (mid_ev) (void)hipEventDestroy(mid_ev);
  }

  fce_tensor view(int id, int coff, int c) const {
    const BufDesc& b = bufs[id];
    fce_tensor t{};
    t.data = arena + b.offset;
    t.dtype = b.dtype;
    t.layout = FCE_NHWC;
    t.n = batch;
    t.c = c;
    t.h = H >> b.shift;
    t.w = W >> b.shift;
    t.cstride = b.c;
    t.coff = coff;
    return t;
  }
};

namespace {

int op_input_view(const fce_net* net, const OpDesc& op, const fce_tensor& input, fce_tensor* out) {
  if (op.in < 0) {
    *out = input;
    return FCE_OK;
  }
  *out = net->view(op.in, op.in_coff, op.in_c);
  return FCE_OK;
}

int run_op_impl(fce_net* net, const OpDesc& op, const fce_tensor& input, float* pred, hipStream_t s) {
  fce_tensor x;
  op_input_view(net, op, input, &x);
  switch (op.kind) {
    case OP_CONV: {
      fce_tensor y = net->view(op.out, op.out_coff, op.conv.cout);
      fce_tensor r;
      const fce_tensor* rp = nullptr;
      if (op.res >= 0) {
        r = net->view(op.res, op.res_coff, op.conv.cout);
        rp = &r;
      }
      if (op.dup >= 0) {
        const fce_tensor dv = net->view(op.dup, 0, op.dup_c);
        return conv2d(op.conv, x, op.w, op.b, rp, y, s, op.tile, &dv, op.dup_lo);
      }
      return conv2d(op.conv, x, op.w, op.b, rp, y, s, op.tile);
    }
    case OP_MAXPOOL: {
      const int c = op.in_c;
      fce_tensor y1 = net->view(op.in, op.in_coff + c, c), y2 = net->view(op.in, op.in_coff + 2 * c, c),
                 y3 = net->view(op.in, op.in_coff + 3 * c, c);
      return maxpool_chain(x, y1, y2, y3, op.k, s);
    }
    case OP_WADD: {
      fce_tensor y = net->view(op.out, op.out_coff, op.in_c);
      return weighted_add(x, op.up, op.fw, op.fn, op.fi, op.accumulate, y, s);
    }
    case OP_COORD: {
      fce_tensor y = net->view(op.out, op.out_coff, op.coord.oup);
      if (op.coord_kind == 0) return bicoordcrossatt(op.coord, x, y, net->ws, net->ws_bytes, s);
      if (op.coord_kind == 1) return coordatt(op.coord, x, y, net->ws, net->ws_bytes, s);
      return coordcrossatt(op.coord, x, y, net->ws, net->ws_bytes, s);
    }
    case OP_PSA: {
      fce_tensor y = net->view(op.out, op.out_coff, op.heads * op.head_dim);
      return psa_attention(x, op.heads, op.key_dim, op.head_dim, op.pe_w, op.pe_b, y, s);
    }
    case OP_C3K2: {
      fce_tensor y = net->view(op.out, op.out_coff, op.c3k2.cout);
      return c3k2_fused(op.c3k2, x, y, s);
    }
    case OP_CONV_DETECT: {
      fce_detect_epi e{pred, net->anchors, net->level_off[op.level], op.nc, op.reg_max, op.part, op.strides[0],
                       net->cur_best};
      return conv2d_detect(op.conv, x, op.w, op.b, e, s, op.tile);
    }
    case OP_STEM2: {
      fce_tensor y = net->view(op.out, op.out_coff, op.stem2.c1);
      return stem_fused(op.stem2, x, y, s);
    }
    case OP_BNECK: {
      fce_tensor y = net->view(op.out, op.out_coff, op.bneck.c);
      return bneck_fused(op.bneck, x, y, s);
    }
    case OP_PW2: {
      const fce_pw2_desc& d = op.pw2;
      const fce_tensor h = net->view(op.out, op.out_coff, d.cout1);
      const fce_tensor x2 = net->view(op.in2, op.in2_coff, d.cin2);
      const fce_tensor y = net->view(op.out2, op.out2_coff, d.cout2);
      fce_tensor r1{}, r2{}, dv{};
      if (op.res >= 0) r1 = net->view(op.res, op.res_coff, d.cout1);
      if (op.res2 >= 0) r2 = net->view(op.res2, op.res2_coff, d.cout2);
      if (op.dup >= 0) dv = net->view(op.dup, 0, op.dup_c);
      return pw2_fused(d, x, op.res >= 0 ? &r1 : nullptr, h, op.h_store, x2, op.res2 >= 0 ? &r2 : nullptr, y,
                       op.dup >= 0 ? &dv : nullptr, op.dup_lo, s);
    }
    case OP_DCLS: {
      fce_detect_epi e{pred, net->anchors, net->level_off[op.level], op.nc, op.reg_max, 1, op.strides[0],
                       net->cur_best};
      return detect_cls_fused(op.dcls, x, e, s);
    }
    case OP_DETECT: {
      fce_tensor bx[4], cl[4];
      for (int i = 0; i < op.nl; ++i) {
        const int c = net->bufs[op.box[i]].c;
        bx[i] = net->view(op.box[i], 0, 4 * op.reg_max);
        cl[i] = net->view(op.cls[i], 4 * op.reg_max, c - 4 * op.reg_max);
      }
      return detect_decode(bx, cl, op.nl, op.strides, op.reg_max, pred, s);
    }
  }
  return fail(FCE_ERR_INVALID, "unknown op");
}

// an op of the inactive form of an alternative launches nothing
int run_op(fce_net* net, const OpDesc& op, const fce_tensor& input, float* pred, hipStream_t s) {
  return op.skip ? FCE_OK : run_op_impl(net, op, input, pred, s);
}

int run_all(fce_net* net, const fce_tensor& input, float* pred, hipStream_t s, bool fork = false) {
  for (size_t i = 0; i < net->ops.size(); ++i) {
    int st = run_op(net, net->ops[i], input, pred, s);
    if (st) return st;
    if (fork && int(i) == net->fork_op) FCE_HIP_CHECK(hipEventRecord(net->mid_ev, s));
  }
  return FCE_OK;
}

// ---- dependency DAG for multi-stream graph capture
// Every op touches buffer channel ranges (reads / writes); two ops conflict when they touch
// overlapping ranges of the same buffer and at least one writes.  The coordinate-attention ops
// share the executor workspace (pseudo buffer WS); Detect tails write disjoint blocks of pred.
struct Access {
  int buf, c0, c1;
  bool write;
};
static constexpr int kBufPred = -2, kBufWs = -3, kBufBest = -4;

static void op_accesses(const fce_net* net, const OpDesc& op, std::vector<Access>& a) {
  a.clear();
  if (op.skip) return;
  switch (op.kind) {
    case OP_CONV:
      if (op.in >= 0) a.push_back({op.in, op.in_coff, op.in_coff + op.conv.cin, false});
      if (op.res >= 0) a.push_back({op.res, op.res_coff, op.res_coff + op.conv.cout, false});
      a.push_back({op.out, op.out_coff, op.out_coff + op.conv.cout, true});
      if (op.dup >= 0) a.push_back({op.dup, 0, op.dup_c, true});
      break;
    case OP_MAXPOOL:
      a.push_back({op.in, op.in_coff, op.in_coff + op.in_c, false});
      a.push_back({op.in, op.in_coff + op.in_c, op.in_coff + 4 * op.in_c, true});
      break;
    case OP_WADD:
      a.push_back({op.in, op.in_coff, op.in_coff + op.in_c, false});
      a.push_back({op.out, op.out_coff, op.out_coff + op.in_c, true});
      break;
    case OP_COORD:
      a.push_back({op.in, op.in_coff, op.in_coff + op.coord.inp, false});
      a.push_back({op.out, op.out_coff, op.out_coff + op.coord.oup, true});
      a.push_back({kBufWs, 0, 1, true});
      break;
    case OP_PSA:
      a.push_back({op.in, op.in_coff, op.in_coff + op.in_c, false});
      a.push_back({op.out, op.out_coff, op.out_coff + op.heads * op.head_dim, true});
      break;
    case OP_C3K2:
      a.push_back({op.in, op.in_coff, op.in_coff + op.c3k2.cin, false});
      a.push_back({op.out, op.out_coff, op.out_coff + op.c3k2.cout, true});
      break;
    case OP_CONV_DETECT:
      a.push_back({op.in, op.in_coff, op.in_coff + op.conv.cin, false});
      a.push_back({kBufPred, 2 * op.level + op.part, 2 * op.level + op.part + 1, true});
      a.push_back({kBufBest, op.level, op.level + 1, true});  // box zeroes, cls maxes: keep them ordered
      break;
    case OP_STEM2:
      a.push_back({op.out, op.out_coff, op.out_coff + op.stem2.c1, true});
      break;
    case OP_BNECK:
      a.push_back({op.in, op.in_coff, op.in_coff + op.bneck.c, false});
      a.push_back({op.out, op.out_coff, op.out_coff + op.bneck.c, true});
      break;
    case OP_PW2:
      a.push_back({op.in, op.in_coff, op.in_coff + op.pw2.cin1, false});
      if (op.res >= 0) a.push_back({op.res, op.res_coff, op.res_coff + op.pw2.cout1, false});
      if (op.pw2.epi1 == FCE_EPI_ACCUM) a.push_back({op.out, op.out_coff, op.out_coff + op.pw2.cout1, false});
      a.push_back({op.out, op.out_coff, op.out_coff + op.pw2.cout1, true});
      a.push_back({op.in2, op.in2_coff, op.in2_coff + op.pw2.cin2, false});
      if (op.res2 >= 0) a.push_back({op.res2, op.res2_coff, op.res2_coff + op.pw2.cout2, false});
      a.push_back({op.out2, op.out2_coff, op.out2_coff + op.pw2.cout2, true});
      if (op.dup >= 0) a.push_back({op.dup, 0, op.dup_c, true});
      break;
    case OP_DCLS:
      a.push_back({op.in, op.in_coff, op.in_coff + op.dcls.c0, false});
      a.push_back({kBufPred, 2 * op.level + 1, 2 * op.level + 2, true});
      a.push_back({kBufBest, op.level, op.level + 1, true});
      break;
    case OP_DETECT:
      for (int i = 0; i < op.nl; ++i) a.push_back({op.box[i], 0, net->bufs[op.box[i]].c, false});
      a.push_back({kBufPred, 0, 1 << 20, true});
      break;
  }
}

static bool conflict(const std::vector<Access>& x, const std::vector<Access>& y) {
  for (const Access& p : x)
    for (const Access& q : y)
      if (p.buf == q.buf && (p.write || q.write) && p.c0 < q.c1 && q.c0 < p.c1) return true;
  return false;
}

// Scheduling of the op DAG onto the net's streams: an op goes to the stream of its most recent
// dependency when that stream has not moved on, otherwise to the stream idle longest, and waits
// (hipStreamWaitEvent) on every dependency recorded on another stream, so independent branches (the
// Detect levels / box and cls chains, the P3 head against the neck's P4/P5 path) run concurrently.
// Launched directly: multi-stream stream capture crashed the ROCm 7 runtime here (4 streams), and a
// captured linear graph replays slower than direct launches (measured).
int run_all_streams(fce_net* net, const fce_tensor& input, float* pred, hipStream_t s, int nstreams) {
  const int nops = int(net->ops.size());
  while (int(net->side.size()) < nstreams) {
    hipStream_t q = nullptr;
    FCE_HIP_CHECK(hipStreamCreateWithFlags(&q, hipStreamNonBlocking));
    net->side.push_back(q);
  }
  while (int(net->op_ev.size()) < nops) {
    hipEvent_t e = nullptr;
    FCE_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    net->op_ev.push_back(e);
  }
  if (!net->fork_ev) FCE_HIP_CHECK(hipEventCreateWithFlags(&net->fork_ev, hipEventDisableTiming));
  std::vector<hipStream_t> st(net->side.begin(), net->side.begin() + nstreams);
  FCE_HIP_CHECK(hipEventRecord(net->fork_ev, s));
  for (int k = 0; k < nstreams; ++k) FCE_HIP_CHECK(hipStreamWaitEvent(st[k], net->fork_ev, 0));
  std::vector<std::vector<Access>> acc(nops);
  for (int j = 0; j < nops; ++j) op_accesses(net, net->ops[j], acc[j]);
  std::vector<int> stream_of(nops, 0), last_on(nstreams, -1);
  std::vector<int> deps;
  for (int j = 0; j < nops; ++j) {
    deps.clear();
    for (int i = 0; i < j; ++i)
      if (conflict(acc[i], acc[j])) deps.push_back(i);
    int pick = -1;
    for (int t = int(deps.size()) - 1; t >= 0 && pick < 0; --t) {
      const int k = stream_of[deps[t]];
      if (last_on[k] == deps[t]) pick = k;  // continue the chain on its own stream
    }
    if (pick < 0) {  // the stream whose last op is oldest
      pick = 0;
      for (int k = 1; k < nstreams; ++k)
        if (last_on[k] < last_on[pick]) pick = k;
    }
    for (int i : deps)
      if (stream_of[i] != pick || i > last_on[pick]) FCE_HIP_CHECK(hipStreamWaitEvent(st[pick], net->op_ev[i], 0));
    const int rc = run_op(net, net->ops[j], input, pred, st[pick]);
    if (rc) return rc;
    FCE_HIP_CHECK(hipEventRecord(net->op_ev[j], st[pick]));
    stream_of[j] = pick;
    last_on[pick] = j;
  }
  for (int k = 0; k < nstreams; ++k)
    if (last_on[k] >= 0) FCE_HIP_CHECK(hipStreamWaitEvent(s, net->op_ev[last_on[k]], 0));
  return FCE_OK;
}

void op_cost(const fce_net* net, const OpDesc& op, std::string* name, double* bytes, double* flops) {
  const double N = net->batch;
  auto hw = [&](int id) { return double(net->H >> net->bufs[id].shift) * double(net->W >> net->bufs[id].shift); };
  *bytes = 0;
  *flops = 0;
  if (op.skip) {  // the inactive form of an alternative: its name, no work
    double b, f;
    OpDesc live = op;
    live.skip = false;
    op_cost(net, live, name, &b, &f);
    return;
  }
  switch (op.kind) {
    case OP_CONV: {
      const fce_conv_desc& d = op.conv;
      const double ohw = hw(op.out);
      const double ihw = op.in >= 0 ? hw(op.in) : double(net->H) * net->W;
      const int in_bytes = op.in >= 0 ? 2 : 2;  // f16 network input in the bench
      const bool dw = d.groups > 1;
      const bool stem = !dw && d.cin <= 4;
      *name = stem ? "conv_stem" : dw ? "dwconv3x3" : (d.k == 3 ? "conv3x3_mfma" : "conv1x1_mfma");
      const int osz = net->bufs[op.out].dtype == FCE_F32 ? 4 : 2;
      *bytes = N * ihw * d.cin * in_bytes + N * ohw * d.cout * osz + double(conv_weight_bytes(d));
      if (op.res >= 0) *bytes += N * ohw * d.cout * 2;
      if (op.dup >= 0) *bytes += N * ohw * op.dup_c * 2;
      if (d.epilogue == FCE_EPI_ACCUM) *bytes += N * ohw * d.cout * 2;
      *flops = 2.0 * N * ohw * d.cout * d.k * d.k * (dw ? 1 : d.cin);
      break;
    }
    case OP_CONV_DETECT: {
      const fce_conv_desc& d = op.conv;
      const double px = N * hw(op.in);
      *name = op.part == 0 ? "conv1x1_detect_box" : "conv1x1_detect_cls";
      *bytes = px * d.cin * 2 + px * (op.part == 0 ? 4 : d.cout) * 4 + double(conv_weight_bytes(d));
      *flops = 2.0 * px * d.cout * d.cin;
      break;
    }
    case OP_MAXPOOL:
      *name = "maxpool_chain";
      *bytes = N * hw(op.in) * op.in_c * 2 * 4;
      break;
    case OP_WADD:
      *name = "bifpn_weighted_add";
      *bytes = N * hw(op.out) * op.in_c * 2 * (op.accumulate ? 3 : 2) / (op.up ? 1.6 : 1.0);
      break;
    case OP_COORD: {
      const char* nm[3] = {"bicoordcrossatt", "coordatt", "coordcrossatt"};
      *name = nm[op.coord_kind];
      const double px = N * hw(op.in);
      *bytes = px * op.coord.inp * 2 * 2 + px * op.coord.oup * 2;  // 2 reads (pool, gate) + 1 write
      const double L = double(net->H >> net->bufs[op.in].shift) + double(net->W >> net->bufs[op.in].shift);
      *flops = 2.0 * N * (3.0 * op.coord.mid * op.coord.inp * L + op.coord.oup * op.coord.mid * L);
      break;
    }
    case OP_STEM2: {  // one read of the f16 input, one write of the second conv's output, both convs' weights
      const fce_stem2_desc& d = op.stem2;
      *name = "stem_fused";
      const double ohw = hw(op.out), ihw = double(net->H) * net->W;
      const fce_conv_desc c0{3, d.c0, 3, 2, 1, FCE_ACT_SILU, 0, FCE_EPI_STORE, nullptr, 0, 0};
      const fce_conv_desc c1{d.c0, d.c1, 3, 2, 1, FCE_ACT_SILU, 0, FCE_EPI_STORE, nullptr, 0, 0};
      *bytes = N * ihw * 3 * 2 + N * ohw * d.c1 * 2 + double(conv_weight_bytes(c0)) + double(conv_weight_bytes(c1));
      *flops = 2.0 * N * (ihw / 4.0 * d.c0 * 27.0 + ohw * d.c1 * 9.0 * d.c0);
      break;
    }
    case OP_DCLS: {  // one read of x, one write of the fp32 scores, the five ops' weights
      const fce_dcls_desc& d = op.dcls;
      *name = "detect_cls_fused";
      const double px = N * hw(op.in);
      const fce_conv_desc cs[5] = {{d.c0, d.c0, 3, 1, d.c0, FCE_ACT_SILU, 0, FCE_EPI_STORE, nullptr, 0, 0},
                                   {d.c0, d.c3, 1, 1, 1, FCE_ACT_SILU, 0, FCE_EPI_STORE, nullptr, 0, 0},
                                   {d.c3, d.c3, 3, 1, d.c3, FCE_ACT_SILU, 0, FCE_EPI_STORE, nullptr, 0, 0},
                                   {d.c3, d.c3, 1, 1, 1, FCE_ACT_SILU, 0, FCE_EPI_STORE, nullptr, 0, 0},
                                   {d.c3, d.nc, 1, 1, 1, FCE_ACT_NONE, 0, FCE_EPI_STORE, nullptr, 0, 0}};
      *bytes = px * d.c0 * 2 + px * d.nc * 4;
      for (const fce_conv_desc& c : cs) *bytes += double(conv_weight_bytes(c));
      *flops = 2.0 * px * (9.0 * d.c0 + double(d.c0) * d.c3 + 9.0 * d.c3 + double(d.c3) * d.c3 + double(d.c3) * d.nc);
      break;
    }
    case OP_PW2: {  // x1, op 2's inputs that are not op 1's output, the residuals, y (+ h when stored), both weights
      const fce_pw2_desc& d = op.pw2;
      *name = "pw2_fused";
      const double px = N * hw(op.in);
      const fce_conv_desc c1{d.cin1, d.cout1, 1, 1, 1, d.act[0], 0, FCE_EPI_STORE, nullptr, 0, 0};
      const fce_conv_desc c2{d.cin2, d.cout2, 1, 1, 1, d.act[1], 0, FCE_EPI_STORE, nullptr, 0, 0};
      const int lo = std::max(op.in2_coff, op.out_coff), hi = std::min(op.in2_coff + d.cin2, op.out_coff + d.cout1);
      const int over = op.in2 == op.out ? std::max(0, hi - lo) : 0;
      *bytes = px * 2 * (d.cin1 + (d.cin2 - over) + d.cout2 + (op.h_store ? d.cout1 : 0) + (op.res >= 0 ? d.cout1 : 0) +
                         (d.epi1 == FCE_EPI_ACCUM ? d.cout1 : 0) +
                         (op.res2 >= 0 ? d.cout2 : 0) + (op.dup >= 0 ? op.dup_c : 0)) +
               double(conv_weight_bytes(c1)) + double(conv_weight_bytes(c2));
      *flops = 2.0 * px * (double(d.cin1) * d.cout1 + double(d.cin2) * d.cout2);
      break;
    }
    case OP_BNECK: {  // one read of x, one write of y, the 2 n convs' weights
      const fce_bneck_desc& d = op.bneck;
      *name = "bneck_fused";
      const double px = N * hw(op.in);
      const fce_conv_desc c1{d.c, d.c_mid, 3, 1, 1, FCE_ACT_SILU, 0, FCE_EPI_STORE, nullptr, 0, 0};
      const fce_conv_desc c2{d.c_mid, d.c, 3, 1, 1, FCE_ACT_SILU, 0, FCE_EPI_STORE, nullptr, 0, 0};
      *bytes = px * d.c * 2 * 2 + d.n * (double(conv_weight_bytes(c1)) + double(conv_weight_bytes(c2)));
      *flops = 2.0 * px * d.n * (9.0 * d.c * d.c_mid + 9.0 * d.c_mid * d.c);
      break;
    }
    case OP_C3K2: {  // one read of x, one write of y, the four convs' weights
      const fce_c3k2_desc& d = op.c3k2;
      *name = "c3k2_fused";
      const double px = N * hw(op.in);
      const fce_conv_desc cs[4] = {{d.cin, 2 * d.c, 1, 1, 1, FCE_ACT_SILU, 0, FCE_EPI_STORE, nullptr, 0, 0},
                                   {d.c, d.c_mid, 3, 1, 1, FCE_ACT_SILU, 0, FCE_EPI_STORE, nullptr, 0, 0},
                                   {d.c_mid, d.c, 3, 1, 1, FCE_ACT_SILU, 0, FCE_EPI_STORE, nullptr, 0, 0},
                                   {3 * d.c, d.cout, 1, 1, 1, FCE_ACT_SILU, 0, FCE_EPI_STORE, nullptr, 0, 0}};
      *bytes = px * (d.cin + d.cout) * 2;
      for (const fce_conv_desc& c : cs) *bytes += double(conv_weight_bytes(c));
      *flops = 2.0 * px * (d.cin * 2.0 * d.c + 9.0 * d.c * d.c_mid + 9.0 * d.c_mid * d.c + 3.0 * d.c * d.cout);
      break;
    }
    case OP_PSA: {
      *name = "psa_attention";
      const double t = hw(op.in);
      *bytes = N * t * op.heads * (2 * op.key_dim + op.head_dim) * 2 + N * t * op.heads * op.head_dim * 2;
      *flops = 2.0 * N * op.heads * t * t * (op.key_dim + op.head_dim);
      break;
    }
    case OP_DETECT: {
      *name = "detect_decode";
      double a = 0;
      for (int i = 0; i < op.nl; ++i) a += hw(op.box[i]);
      *bytes = N * a * (4 * op.reg_max + net->nc) * 4 + N * a * (4 + net->nc) * 4;
      break;
    }
  }
}

// the active form of an alternative: the fused op, or the ops it replaces
void set_alt_form(fce_net* net, OpDesc& op, bool fused) {
  if (op.skip != !fused) net->drop_graph();  // captured forwards hold the other form's launches
  op.skip = !fused;
  for (int j = op.alt_first; j < op.alt_first + op.alt_n; ++j) net->ops[j].skip = fused;
}

}  // namespace

extern "C" {

fce_net* fce_net_create(void) {
  try {
    return new fce_net();
  } catch (...) {
    set_error("fce_net_create: allocation failed");
    return nullptr;
  }
}
void fce_net_destroy(fce_net* net) { delete net; }

int fce_net_fork_hint(const fce_net* net) {
  // the op after which the forward runs at its coarsest resolution (stride 32): from there on the
  // forward's kernels are small and leave most CUs idle
  if (!net) return -1;
  int best = -1, shift = -1;
  for (size_t i = 0; i < net->ops.size(); ++i) {
    const OpDesc& op = net->ops[i];
    if (op.kind == OP_CONV && op.out >= 0 && net->bufs[op.out].shift > shift) {
      shift = net->bufs[op.out].shift;
      best = int(i);
    }
  }
  return best;
}

int fce_net_set_fork(fce_net* net, int op) {
  FCE_CHECK(net && op >= -1 && op < int(net->ops.size()), "fce_net_set_fork: bad op");
  if (!net->mid_ev) FCE_HIP_CHECK(hipEventCreateWithFlags(&net->mid_ev, hipEventDisableTiming));
  net->fork_op = op;
  net->drop_graph();
  return FCE_OK;
}

int fce_net_wait_fork(fce_net* net, void* stream) {
  FCE_CHECK(net && net->mid_ev, "fce_net_wait_fork: call fce_net_set_fork first");
  FCE_HIP_CHECK(hipStreamWaitEvent(S(stream), net->mid_ev, 0));
  return FCE_OK;
}

int fce_net_add_buffer(fce_net* net, int c, int shift, int dtype) {
  FCE_CHECK(net && c > 0 && shift >= 0 && shift <= 8 && (dtype == FCE_F16 || dtype == FCE_F32),
            "fce_net_add_buffer: bad argument");
  net->drop_graph();
  net->bufs.push_back(BufDesc{c, shift, dtype});
  return int(net->bufs.size()) - 1;
}

static int valid_buf(const fce_net* net, int id, bool allow_input) {
  return (allow_input && id == -1) || (id >= 0 && id < int(net->bufs.size()));
}

int fce_net_add_conv(fce_net* net, const fce_conv_desc* d, int in, int in_coff, int out, int out_coff, int res,
                     int res_coff, const void* w, const float* b) {
  FCE_CHECK(net && d && w && b, "fce_net_add_conv: null argument");
  FCE_CHECK(valid_buf(net, in, true) && valid_buf(net, out, false) && (res == -1 || valid_buf(net, res, false)),
            "fce_net_add_conv: bad buffer id");
  OpDesc op;
  op.kind = OP_CONV;
  op.conv = *d;
  op.in = in;
  op.in_coff = in_coff;
  op.in_c = d->cin;
  op.out = out;
  op.out_coff = out_coff;
  op.res = res;
  op.res_coff = res_coff;
  op.w = w;
  op.b = b;
  net->drop_graph();
  net->ops.push_back(op);
  return FCE_OK;
}

int fce_net_add_conv_dup(fce_net* net, const fce_conv_desc* d, int in, int in_coff, int out, int out_coff, int res,
                         int res_coff, const void* w, const float* b, int dup, int dup_lo, int dup_c) {
  FCE_CHECK(net && valid_buf(net, dup, false) && dup_c > 0 && dup_c % 8 == 0 && dup_lo >= 0 && dup_lo % 8 == 0 &&
                d && d->k == 1 && dup_lo + dup_c <= d->cout && net->bufs[dup].c == dup_c &&
                net->bufs[dup].dtype == FCE_F16,
            "fce_net_add_conv_dup: bad duplicate-store buffer or channel range");
  // every check before the op is added: a failed call leaves the op list unchanged
  FCE_CHECK(valid_buf(net, out, false) && net->bufs[dup].shift == net->bufs[out].shift,
            "fce_net_add_conv_dup: dup buffer size differs");
  const int st = fce_net_add_conv(net, d, in, in_coff, out, out_coff, res, res_coff, w, b);
  if (st) return st;
  OpDesc& op = net->ops.back();
  op.dup = dup;
  op.dup_lo = dup_lo;
  op.dup_c = dup_c;
  return FCE_OK;
}

int fce_net_add_maxpool_chain(fce_net* net, int buf, int in_coff, int c, int k) {
  FCE_CHECK(net && valid_buf(net, buf, false), "fce_net_add_maxpool_chain: bad buffer");
  OpDesc op;
  op.kind = OP_MAXPOOL;
  op.in = buf;
  op.in_coff = in_coff;
  op.in_c = c;
  op.k = k;
  net->drop_graph();
  net->ops.push_back(op);
  return FCE_OK;
}

int fce_net_add_weighted_add(fce_net* net, int in, int in_coff, int c, int up, const float* fw, int fn, int fi,
                             int accumulate, int out, int out_coff) {
  FCE_CHECK(net && fw && valid_buf(net, in, false) && valid_buf(net, out, false), "fce_net_add_weighted_add: bad arg");
  OpDesc op;
  op.kind = OP_WADD;
  op.in = in;
  op.in_coff = in_coff;
  op.in_c = c;
  op.up = up;
  op.fw = fw;
  op.fn = fn;
  op.fi = fi;
  op.accumulate = accumulate;
  op.out = out;
  op.out_coff = out_coff;
  net->drop_graph();
  net->ops.push_back(op);
  return FCE_OK;
}

int fce_net_add_coord(fce_net* net, int kind, const fce_coord_desc* d, int in, int in_coff, int out, int out_coff) {
  FCE_CHECK(net && d && kind >= 0 && kind <= 2 && valid_buf(net, in, false) && valid_buf(net, out, false),
            "fce_net_add_coord: bad argument");
  OpDesc op;
  op.kind = OP_COORD;
  op.coord_kind = kind;
  op.coord = *d;
  op.in = in;
  op.in_coff = in_coff;
  op.in_c = d->inp;
  op.out = out;
  op.out_coff = out_coff;
  net->drop_graph();
  net->ops.push_back(op);
  return FCE_OK;
}

int fce_net_add_psa_attention(fce_net* net, int qkv, int heads, int kd, int hd, const float* pe_w, const float* pe_b,
                              int out, int out_coff) {
  FCE_CHECK(net && pe_w && pe_b && valid_buf(net, qkv, false) && valid_buf(net, out, false),
            "fce_net_add_psa_attention: bad argument");
  OpDesc op;
  op.kind = OP_PSA;
  op.in = qkv;
  op.in_coff = 0;
  op.in_c = heads * (2 * kd + hd);
  op.heads = heads;
  op.key_dim = kd;
  op.head_dim = hd;
  op.pe_w = pe_w;
  op.pe_b = pe_b;
  op.out = out;
  op.out_coff = out_coff;
  net->drop_graph();
  net->ops.push_back(op);
  return FCE_OK;
}

int fce_net_add_c3k2_alt(fce_net* net, const fce_c3k2_desc* d, int in, int in_coff, int out, int out_coff,
                         int first_op, int nops) {
  FCE_CHECK(net && nops >= 1 && first_op >= 0 && first_op + nops == int(net->ops.size()),
            "fce_net_add_c3k2_alt: the alternative must be the last ops added");
  for (int j = first_op; j < first_op + nops; ++j)
    FCE_CHECK(net->ops[j].kind == OP_CONV && !net->ops[j].skip && net->ops[j].alt_first < 0,
              "fce_net_add_c3k2_alt: the alternative must be plain conv ops");
  const int st = fce_net_add_c3k2(net, d, in, in_coff, out, out_coff);
  if (st) return st;
  OpDesc& op = net->ops.back();
  op.alt_first = first_op;
  op.alt_n = nops;
  set_alt_form(net, op, true);  // fused until the plan-time autotune says otherwise
  return FCE_OK;
}

int fce_net_c3k2_form(const fce_net* net, int i) {
  if (!net || i < 0 || i >= int(net->ops.size())) return -1;
  const OpDesc& op = net->ops[i];
  return op.kind == OP_C3K2 && op.alt_first >= 0 ? (op.skip ? 0 : 1) : -1;
}

int fce_net_set_c3k2_form(fce_net* net, int i, int fused) {
  FCE_CHECK(fce_net_c3k2_form(net, i) >= 0, "fce_net_set_c3k2_form: not a fused C3k2 op with an alternative");
  set_alt_form(net, net->ops[i], fused != 0);
  return FCE_OK;
}

int fce_net_alt_form(const fce_net* net, int i) {
  if (!net || i < 0 || i >= int(net->ops.size())) return -1;
  const OpDesc& op = net->ops[i];
  return op.alt_first >= 0 ? (op.skip ? 0 : 1) : -1;
}

int fce_net_set_alt_form(fce_net* net, int i, int fused) {
  FCE_CHECK(fce_net_alt_form(net, i) >= 0, "fce_net_set_alt_form: not a fused op with an alternative");
  FCE_CHECK(!fused || !net->ops[i].alt_locked, "fce_net_set_alt_form: this fused op cannot run in this net");
  set_alt_form(net, net->ops[i], fused != 0);
  return FCE_OK;
}

int fce_net_add_bneck_alt(fce_net* net, const fce_bneck_desc* d, int in, int in_coff, int out, int out_coff,
                          int first_op, int nops) {
  FCE_CHECK(net && d && valid_buf(net, in, false) && valid_buf(net, out, false) && (d->n == 1 || d->n == 2) &&
                nops == 2 * d->n && first_op >= 0 && first_op + nops == int(net->ops.size()),
            "fce_net_add_bneck_alt: the alternative must be the last 2 n ops added");
  FCE_CHECK(bneck_fused_ok(*d), "fce_net_add_bneck_alt: unsupported channel configuration");
  const OpDesc* o = &net->ops[first_op];
  for (int j = 0; j < nops; ++j) {
    const fce_conv_desc& c = o[j].conv;
    const bool odd = j % 2 == 1;
    FCE_CHECK(o[j].kind == OP_CONV && !o[j].skip && o[j].alt_first < 0 && o[j].dup < 0 && c.k == 3 && c.stride == 1 &&
                  c.groups == 1 && c.up == 0 && c.act == FCE_ACT_SILU && c.epilogue == FCE_EPI_STORE &&
                  c.cin == (odd ? d->c_mid : d->c) && c.cout == (odd ? d->c : d->c_mid) && o[j].w == d->w[j] &&
                  o[j].b == d->b[j],
              "fce_net_add_bneck_alt: the ops are not this chain's 3x3 SiLU convs (shapes, weights or epilogues differ)");
    // chain: conv j reads conv j - 1's whole output (the first reads the input); every odd conv adds its
    // Bottleneck's input (the input of conv j - 1) as the residual; only the last writes the given output
    const int src = j == 0 ? in : o[j - 1].out, src_off = j == 0 ? in_coff : o[j - 1].out_coff;
    FCE_CHECK(o[j].in == src && o[j].in_coff == src_off, "fce_net_add_bneck_alt: the ops must form one chain");
    if (odd)
      FCE_CHECK(o[j].res == o[j - 1].in && o[j].res_coff == o[j - 1].in_coff,
                "fce_net_add_bneck_alt: every second conv must add its Bottleneck's input");
    else
      FCE_CHECK(o[j].res < 0, "fce_net_add_bneck_alt: the first conv of a Bottleneck has no residual");
  }
  FCE_CHECK(o[nops - 1].out == out && o[nops - 1].out_coff == out_coff,
            "fce_net_add_bneck_alt: the last conv must write the given output");
  OpDesc op;
  op.kind = OP_BNECK;
  op.bneck = *d;
  op.in = in;
  op.in_coff = in_coff;
  op.in_c = d->c;
  op.out = out;
  op.out_coff = out_coff;
  op.alt_first = first_op;
  op.alt_n = nops;
  net->drop_graph();
  net->ops.push_back(op);
  set_alt_form(net, net->ops.back(), true);  // fused until the plan-time autotune (or the map width) says otherwise
  return FCE_OK;
}

int fce_net_add_pw2_alt(fce_net* net, const fce_pw2_desc* d, int first_op) {
  FCE_CHECK(net && d && first_op >= 0 && first_op + 2 == int(net->ops.size()),
            "fce_net_add_pw2_alt: the alternative must be the last two ops added");
  FCE_CHECK(pw2_fused_ok(*d), "fce_net_add_pw2_alt: unsupported channel configuration");
  const OpDesc& o1 = net->ops[first_op];
  const OpDesc& o2 = net->ops[first_op + 1];
  const int cins[2] = {d->cin1, d->cin2}, couts[2] = {d->cout1, d->cout2};
  for (int j = 0; j < 2; ++j) {
    const OpDesc& o = j ? o2 : o1;
    const fce_conv_desc& c = o.conv;
    FCE_CHECK(o.kind == OP_CONV && !o.skip && o.alt_first < 0 && o.in >= 0 && c.k == 1 && c.stride == 1 &&
                  c.groups == 1 && c.up == 0 && c.epilogue == (j ? FCE_EPI_STORE : d->epi1) && c.act == d->act[j] &&
                  (j || d->epi1 == FCE_EPI_STORE ||
                   (c.fusion_w == d->fw && c.fusion_n == d->fn && c.fusion_i == d->fi)) &&
                  c.cin == cins[j] &&
                  c.cout == couts[j] && o.w == d->w[j] && o.b == d->b[j] && net->bufs[o.out].dtype == FCE_F16 &&
                  net->bufs[o.in].dtype == FCE_F16 && net->bufs[o.in].shift == net->bufs[o1.in].shift,
              "fce_net_add_pw2_alt: the two ops are not this pair's 1x1 convs (shapes, weights or epilogues differ)");
  }
  FCE_CHECK(o1.dup < 0, "fce_net_add_pw2_alt: op 1 has a duplicate store");
  const int lo = std::max(o2.in_coff, o1.out_coff), hi = std::min(o2.in_coff + d->cin2, o1.out_coff + d->cout1);
  FCE_CHECK(o2.in == o1.out && hi > lo, "fce_net_add_pw2_alt: op 2 must read channels of op 1's output buffer");
  OpDesc op;
  op.kind = OP_PW2;
  op.pw2 = *d;
  op.in = o1.in;
  op.in_coff = o1.in_coff;
  op.in_c = d->cin1;
  op.res = o1.res;
  op.res_coff = o1.res_coff;
  op.out = o1.out;
  op.out_coff = o1.out_coff;
  op.in2 = o2.in;
  op.in2_coff = o2.in_coff;
  op.res2 = o2.res;
  op.res2_coff = o2.res_coff;
  op.out2 = o2.out;
  op.out2_coff = o2.out_coff;
  op.dup = o2.dup;
  op.dup_lo = o2.dup_lo;
  op.dup_c = o2.dup_c;
  op.h_store = 1;  // fce_net_plan clears it when nothing else reads h
  op.alt_first = first_op;
  op.alt_n = 2;
  net->drop_graph();
  net->ops.push_back(op);
  set_alt_form(net, net->ops.back(), true);  // fused until the plan-time autotune says otherwise
  return FCE_OK;
}

int fce_net_add_stem_alt(fce_net* net, const fce_stem2_desc* d, int first_op, int nops) {
  FCE_CHECK(net && d && nops == 2 && first_op >= 0 && first_op + nops == int(net->ops.size()),
            "fce_net_add_stem_alt: the alternative must be the last two ops added");
  FCE_CHECK(stem_fused_ok(*d), "fce_net_add_stem_alt: unsupported channel configuration");
  const OpDesc& s0 = net->ops[first_op];
  const OpDesc& s1 = net->ops[first_op + 1];
  const fce_conv_desc &c0 = s0.conv, &c1 = s1.conv;
  FCE_CHECK(s0.kind == OP_CONV && s1.kind == OP_CONV && !s0.skip && !s1.skip && s0.alt_first < 0 && s1.alt_first < 0,
            "fce_net_add_stem_alt: the alternative must be two conv ops");
  FCE_CHECK(s0.in == -1 && c0.cin == 3 && c0.cout == d->c0 && c0.k == 3 && c0.stride == 2 && c0.groups == 1 &&
                c0.act == FCE_ACT_SILU && c0.epilogue == FCE_EPI_STORE && s0.res < 0 && s0.dup < 0 && s0.w == d->w[0] &&
                s0.b == d->b[0],
            "fce_net_add_stem_alt: the first op must be the 3x3 stride-2 SiLU stem on the network input");
  FCE_CHECK(s1.in == s0.out && s1.in_coff == s0.out_coff && c1.cin == d->c0 && c1.cout == d->c1 && c1.k == 3 &&
                c1.stride == 2 && c1.groups == 1 && c1.up == 0 && c1.act == FCE_ACT_SILU &&
                c1.epilogue == FCE_EPI_STORE && s1.res < 0 && s1.dup < 0 && s1.w == d->w[1] && s1.b == d->b[1],
            "fce_net_add_stem_alt: the second op must be the 3x3 stride-2 SiLU conv of the stem's output");
  OpDesc op;
  op.kind = OP_STEM2;
  op.stem2 = *d;
  op.in = -1;
  op.in_c = 3;
  op.out = s1.out;
  op.out_coff = s1.out_coff;
  op.alt_first = first_op;
  op.alt_n = nops;
  net->drop_graph();
  net->ops.push_back(op);
  set_alt_form(net, net->ops.back(), true);  // fused until the plan-time autotune says otherwise
  return FCE_OK;
}

int fce_net_add_detect_cls_alt(fce_net* net, const fce_dcls_desc* d, int in, int in_coff, int first_op, int nops) {
  FCE_CHECK(net && d && valid_buf(net, in, false) && nops == 5 && first_op >= 0 &&
                first_op + nops == int(net->ops.size()),
            "fce_net_add_detect_cls_alt: the alternative must be the last five ops added");
  FCE_CHECK(detect_cls_fused_ok(*d), "fce_net_add_detect_cls_alt: unsupported channel configuration");
  const OpDesc* o = &net->ops[first_op];
  for (int j = 0; j < 5; ++j)
    FCE_CHECK(!o[j].skip && o[j].alt_first < 0 && o[j].kind == (j < 4 ? OP_CONV : OP_CONV_DETECT),
              "fce_net_add_detect_cls_alt: the alternative must be four conv ops and a conv-detect op");
  const int ks[5] = {3, 1, 3, 1, 1}, cin[5] = {d->c0, d->c0, d->c3, d->c3, d->c3};
  const int cout[5] = {d->c0, d->c3, d->c3, d->c3, d->nc};
  for (int j = 0; j < 5; ++j) {
    const fce_conv_desc& c = o[j].conv;
    FCE_CHECK(c.k == ks[j] && c.cin == cin[j] && c.cout == cout[j] && c.stride == 1 && c.up == 0 &&
                  c.groups == (ks[j] == 3 ? c.cin : 1) && c.act == (j < 4 ? FCE_ACT_SILU : FCE_ACT_NONE) &&
                  c.epilogue == FCE_EPI_STORE && o[j].w == d->w[j] && o[j].b == d->b[j],
              "fce_net_add_detect_cls_alt: the five ops are not this branch (shapes, activations or weights differ)");
  }
  // the chain: x -> dw1 -> pw1 -> dw2 -> pw2 -> cls, each reading the previous op's whole output
  FCE_CHECK(o[0].in == in && o[0].in_coff == in_coff && o[0].res < 0 && o[0].dup < 0,
            "fce_net_add_detect_cls_alt: the first op must read the given input");
  for (int j = 1; j < 5; ++j)
    FCE_CHECK(o[j].in == o[j - 1].out && o[j].in_coff == o[j - 1].out_coff && o[j].res < 0 && o[j].dup < 0,
              "fce_net_add_detect_cls_alt: the five ops must form one chain");
  FCE_CHECK(o[4].part == 1 && o[4].nc == d->nc, "fce_net_add_detect_cls_alt: the last op must be the cls tail");
  OpDesc op;
  op.kind = OP_DCLS;
  op.dcls = *d;
  op.in = in;
  op.in_coff = in_coff;
  op.in_c = d->c0;
  op.level = o[4].level;
  op.strides[0] = o[4].strides[0];
  op.nc = o[4].nc;
  op.reg_max = o[4].reg_max;
  op.part = 1;
  op.alt_first = first_op;
  op.alt_n = nops;
  net->drop_graph();
  net->ops.push_back(op);
  set_alt_form(net, net->ops.back(), true);  // fused until the plan-time autotune says otherwise
  return FCE_OK;
}

int fce_net_op_skipped(const fce_net* net, int i) {
  return net && i >= 0 && i < int(net->ops.size()) && net->ops[i].skip ? 1 : 0;
}

int fce_net_add_c3k2(fce_net* net, const fce_c3k2_desc* d, int in, int in_coff, int out, int out_coff) {
  FCE_CHECK(net && d && valid_buf(net, in, false) && valid_buf(net, out, false), "fce_net_add_c3k2: bad argument");
  FCE_CHECK(c3k2_fused_ok(*d), "fce_net_add_c3k2: unsupported channel configuration");
  OpDesc op;
  op.kind = OP_C3K2;
  op.c3k2 = *d;
  op.in = in;
  op.in_coff = in_coff;
  op.in_c = d->cin;
  op.out = out;
  op.out_coff = out_coff;
  net->drop_graph();
  net->ops.push_back(op);
  return FCE_OK;
}

int fce_net_add_detect(fce_net* net, int nl, const int* maps, const float* strides, int reg_max) {
  FCE_CHECK(net && maps && strides && nl >= 1 && nl <= 4, "fce_net_add_detect: bad argument");
  OpDesc op;
  op.kind = OP_DETECT;
  op.nl = nl;
  for (int i = 0; i < nl; ++i) {
    FCE_CHECK(valid_buf(net, maps[i], false), "fce_net_add_detect: bad buffer");
    FCE_CHECK(net->bufs[maps[i]].dtype == FCE_F32 && net->bufs[maps[i]].c > 4 * reg_max, "detect maps must be f32");
    op.box[i] = maps[i];
    op.cls[i] = maps[i];
    op.strides[i] = strides[i];
  }
  op.in = maps[0];
  op.reg_max = reg_max;
  net->nc = net->bufs[maps[0]].c - 4 * reg_max;
  net->drop_graph();
  net->ops.push_back(op);
  return FCE_OK;
}

int fce_net_add_conv_detect(fce_net* net, const fce_conv_desc* d, int in, int in_coff, int part, int level,
                            float stride, int nc, int reg_max, const void* w, const float* b) {
  FCE_CHECK(net && d && w && b && valid_buf(net, in, false), "fce_net_add_conv_detect: bad argument");
  FCE_CHECK(part == 0 || part == 1, "fce_net_add_conv_detect: part must be 0 (box) or 1 (cls)");
  FCE_CHECK(level >= 0 && level < 8, "fce_net_add_conv_detect: level out of range");
  OpDesc op;
  op.kind = OP_CONV_DETECT;
  op.conv = *d;
  op.in = in;
  op.in_coff = in_coff;
  op.in_c = d->cin;
  op.part = part;
  op.level = level;
  op.strides[0] = stride;
  op.nc = nc;
  op.reg_max = reg_max;
  op.w = w;
  op.b = b;
  net->nc = nc;
  net->drop_graph();
  net->ops.push_back(op);
  return FCE_OK;
}

// Plan-time tile autotuning: every dense conv is timed (on the planned shapes, arena contents) with
// each candidate register tile and keeps the fastest.  Small maps favour fewer, fuller tiles (L2
// traffic) over occupancy in ways a closed-form rule does not capture reliably.
static int autotune(fce_net* net) {
  hipStream_t ts = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  float* pred = nullptr;
  int st = FCE_OK;
  int nc = 0;
  for (const OpDesc& op : net->ops)
    if (op.kind == OP_CONV_DETECT) nc = std::max(nc, op.nc);
  // a dummy network input (f16 NCHW, zeros) for timing the alternatives that read it (the fused stem pair)
  void* tin = nullptr;
  bool need_in = false;
  for (const OpDesc& op : net->ops) need_in |= op.kind == OP_STEM2 && op.alt_first >= 0 && !op.alt_locked;
  auto cleanup = [&]() {
    if (tin) (void)hipFree(tin);
    if (pred) (void)hipFree(pred);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (ts) (void)hipStreamDestroy(ts);
  };
  if (hipStreamCreateWithFlags(&ts, hipStreamNonBlocking) != hipSuccess || hipEventCreate(&e0) != hipSuccess ||
      hipEventCreate(&e1) != hipSuccess ||
      (nc > 0 && hipMalloc(reinterpret_cast<void**>(&pred), size_t(net->batch) * (4 + nc) * std::max(net->anchors, 1) *
                                                                 sizeof(float)) != hipSuccess)) {
    cleanup();
    return fail(FCE_ERR_HIP, "fce_net_plan: autotune setup failed");
  }
  fce_tensor none{};
  fce_tensor input{};
  if (need_in) {
    const size_t nb = size_t(net->batch) * 3 * net->H * net->W * sizeof(_Float16);
    if (hipMalloc(&tin, nb) != hipSuccess || hipMemset(tin, 0, nb) != hipSuccess) {
      cleanup();
      return fail(FCE_ERR_HIP, "fce_net_plan: autotune input allocation failed");
    }
    input = fce_tensor{tin, FCE_F16, FCE_NCHW, net->batch, 3, net->H, net->W, 3, 0};
  }
  for (OpDesc& op : net->ops) {
    if (!(op.kind == OP_CONV && op.in >= 0) && op.kind != OP_CONV_DETECT) continue;
    int cand[128];
    const int nc_ = conv_tile_candidates(op.conv, op.kind == OP_CONV_DETECT && op.part == 0,
                                         net->W >> net->bufs[op.in].shift, cand, 128);
    if (nc_ <= 1) continue;
    float best_ms = 1e30f;
    int best = -1;
    for (int i = 0; i < nc_ && st == FCE_OK; ++i) {
      op.tile = cand[i];
      for (int r = 0; r < 2 && st == FCE_OK; ++r) st = run_op_impl(net, op, none, pred, ts);
      if (st) break;
      // best of two 3-launch windows: one window alone let clock / co-tenant noise flip close picks
      float ms = 1e30f;
      for (int t = 0; t < 2 && st == FCE_OK; ++t) {
        (void)hipEventRecord(e0, ts);
        for (int r = 0; r < 3 && st == FCE_OK; ++r) st = run_op_impl(net, op, none, pred, ts);
        (void)hipEventRecord(e1, ts);
        if (hipEventSynchronize(e1) != hipSuccess) st = fail(FCE_ERR_HIP, "fce_net_plan: autotune sync failed");
        float w = 0.f;
        (void)hipEventElapsedTime(&w, e0, e1);
        ms = std::min(ms, w);
      }
      if (st == FCE_OK) net->tune_log.push_back({int(&op - net->ops.data()), cand[i], ms / 3.f});
      if (st == FCE_OK && ms < best_ms) {
        best_ms = ms;
        best = cand[i];
      }
    }
    op.tile = best;
    if (st) break;
  }
  // alternative forms (fused C3k2 against its four tuned convs, fused Detect cls branch against its five tuned ops):
  // time both on the planned shapes, keep the faster (FCE_FUSE_C3K2=1 / FCE_FUSE_DCLS=1 keep the fused form without
  // timing).  Logged as codes 0xF01 (fused) / 0xF00 (the unfused ops).
  auto forced = [](const char* name) {
    const char* e = getenv(name);
    return e && strcmp(e, "1") == 0;
  };
  const bool force_c3k2 = forced("FCE_FUSE_C3K2"), force_dcls = forced("FCE_FUSE_DCLS"),
             force_stem = forced("FCE_FUSE_STEM"), force_bneck = forced("FCE_FUSE_BNECK"),
             force_pw2 = forced("FCE_FUSE_PW2");
  for (size_t i = 0; i < net->ops.size() && st == FCE_OK; ++i) {
    OpDesc& op = net->ops[i];
    if (op.alt_first < 0 || op.alt_locked || (op.kind == OP_C3K2 && force_c3k2) || (op.kind == OP_DCLS && force_dcls) ||
        (op.kind == OP_STEM2 && force_stem) || (op.kind == OP_BNECK && force_bneck) || (op.kind == OP_PW2 && force_pw2))
      continue;
    float t[2] = {1e30f, 1e30f};  // [convs, fused]
    for (int form = 0; form < 2 && st == FCE_OK; ++form) {
      auto run_form = [&]() {
        if (form == 1) return run_op_impl(net, op, input, pred, ts);
        for (int j = op.alt_first; j < op.alt_first + op.alt_n; ++j) {
          const int r = run_op_impl(net, net->ops[j], input, pred, ts);
          if (r) return r;
        }
        return FCE_OK;
      };
      for (int r = 0; r < 2 && st == FCE_OK; ++r) st = run_form();
      for (int w = 0; w < 2 && st == FCE_OK; ++w) {
        (void)hipEventRecord(e0, ts);
        for (int r = 0; r < 3 && st == FCE_OK; ++r) st = run_form();
        (void)hipEventRecord(e1, ts);
        if (hipEventSynchronize(e1) != hipSuccess) st = fail(FCE_ERR_HIP, "fce_net_plan: autotune sync failed");
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        t[form] = std::min(t[form], ms / 3.f);
      }
      if (st == FCE_OK) net->tune_log.push_back({int(i), 0xF00 | form, t[form]});
    }
    if (st == FCE_OK) set_alt_form(net, op, t[1] <= t[0]);
  }
  if (hipStreamSynchronize(ts) != hipSuccess && st == FCE_OK) st = fail(FCE_ERR_HIP, "fce_net_plan: autotune failed");
  cleanup();
  return st;
}

int fce_net_plan(fce_net* net, int batch, int h, int w) {
  const char* at = getenv("FCE_AUTOTUNE");
  return fce_net_plan_ex(net, batch, h, w, (at && atoi(at) == 0) ? FCE_PLAN_NO_AUTOTUNE : 0);
}

int fce_net_plan_ex(fce_net* net, int batch, int h, int w, int flags) {
  FCE_CHECK(net && batch > 0 && h > 0 && w > 0, "fce_net_plan: bad argument");
  FCE_CHECK((flags & ~FCE_PLAN_NO_AUTOTUNE) == 0, "fce_net_plan_ex: unknown flags");
  FCE_CHECK(h % 32 == 0 && w % 32 == 0, "fce_net_plan: H and W must be multiples of 32 (max stride)");
  FCE_GUARD({
    net->release();
    net->tune_log.clear();
    net->batch = batch;
    net->H = h;
    net->W = w;
    size_t off = 0;
    for (BufDesc& b : net->bufs) {
      b.offset = off;
      b.bytes = size_t(batch) * (h >> b.shift) * (w >> b.shift) * b.c * dtype_size(b.dtype);
      off += (b.bytes + 255) & ~size_t(255);
    }
    net->arena_bytes = off;
    size_t ws = 256;
    int A = 0;
    for (const OpDesc& op : net->ops) {
      if (op.kind == OP_COORD)
        ws = std::max(ws, coord_ws_bytes(op.coord, batch, h >> net->bufs[op.in].shift, w >> net->bufs[op.in].shift));
      if (op.kind == OP_DETECT)
        for (int i = 0; i < op.nl; ++i) A += (h >> net->bufs[op.box[i]].shift) * (w >> net->bufs[op.box[i]].shift);
    }
    // fused Detect levels: anchor blocks in level order (head.py:155 torch.cat over levels)
    int lv_hw[8] = {0, 0, 0, 0, 0, 0, 0, 0}, nlv = 0;
    for (const OpDesc& op : net->ops)
      if (op.kind == OP_CONV_DETECT && op.part == 0) {
        lv_hw[op.level] = (h >> net->bufs[op.in].shift) * (w >> net->bufs[op.in].shift);
        nlv = std::max(nlv, op.level + 1);
      }
    if (nlv) {
      A = 0;
      for (int i = 0; i < nlv; ++i) {
        net->level_off[i] = A;
        A += lv_hw[i];
      }
    }
    net->anchors = A;
    net->ws_bytes = ws;
    // a fused stem pair skips writing the stem's output: valid only when nothing but the second conv reads it, and
    // only for the input sizes its kernel is built for
    for (size_t i = 0; i < net->ops.size(); ++i) {
      OpDesc& op = net->ops[i];
      if (op.kind != OP_STEM2 || op.alt_first < 0) continue;
      op.alt_locked = !stem_fused_fits(op.stem2, h, w);
      const OpDesc& s0 = net->ops[op.alt_first];
      std::vector<Access> acc;
      for (size_t j = 0; j < net->ops.size() && !op.alt_locked; ++j) {
        if (int(j) == op.alt_first || int(j) == op.alt_first + 1 || j == i) continue;
        OpDesc probe = net->ops[j];
        probe.skip = false;
        op_accesses(net, probe, acc);
        for (const Access& x : acc)
          if (x.buf == s0.out && x.c0 < s0.out_coff + s0.conv.cout && s0.out_coff < x.c1) op.alt_locked = true;
      }
      if (op.alt_locked) set_alt_form(net, op, false);
    }
    // a fused 1x1 pair stores op 1's output only when some other op reads it (the ops of every form count)
    for (size_t i = 0; i < net->ops.size(); ++i) {
      OpDesc& op = net->ops[i];
      if (op.kind != OP_PW2 || op.alt_first < 0) continue;
      op.h_store = 0;
      std::vector<Access> acc;
      for (size_t j = 0; j < net->ops.size() && !op.h_store; ++j) {
        if (int(j) == op.alt_first || int(j) == op.alt_first + 1 || j == i) continue;
        OpDesc probe = net->ops[j];
        probe.skip = false;
        op_accesses(net, probe, acc);
        for (const Access& x : acc)
          if (!x.write && x.buf == op.out && x.c0 < op.out_coff + op.pw2.cout1 && op.out_coff < x.c1) op.h_store = 1;
      }
    }
    // a fused Bottleneck chain runs only where an instantiation covers its map width
    for (OpDesc& op : net->ops) {
      if (op.kind != OP_BNECK || op.alt_first < 0) continue;
      const int sh = net->bufs[op.in].shift;
      op.alt_locked = !bneck_fused_fits(op.bneck, h >> sh, w >> sh);
      if (op.alt_locked) set_alt_form(net, op, false);
      else if (const char* e = getenv("FCE_FUSE_BNECK"); e && strcmp(e, "1") == 0) set_alt_form(net, op, true);
    }
    FCE_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&net->arena), std::max<size_t>(off, 256)));
    FCE_HIP_CHECK(hipMalloc(&net->ws, ws));
    FCE_HIP_CHECK(hipMemset(net->arena, 0, std::max<size_t>(off, 256)));
    net->cur_best = nullptr;
    if (!(flags & FCE_PLAN_NO_AUTOTUNE)) return autotune(net);
    return FCE_OK;
  })
}

size_t fce_net_arena_bytes(const fce_net* net) { return net ? net->arena_bytes + net->ws_bytes : 0; }
int fce_net_num_anchors(const fce_net* net) { return net ? net->anchors : 0; }
int fce_net_num_ops(const fce_net* net) { return net ? int(net->ops.size()) : 0; }

static int check_input(const fce_net* net, const fce_tensor* in) {
  FCE_CHECK(net->arena, "fce_net: call fce_net_plan first");
  FCE_CHECK(in && in->layout == FCE_NCHW && in->n == net->batch && in->h == net->H && in->w == net->W,
            "fce_net: input must be NCHW with the planned batch/size");
  return FCE_OK;
}

int fce_net_forward(fce_net* net, const fce_tensor* input, float* pred, int graph, void* stream) {
  return fce_net_forward_best(net, input, pred, nullptr, graph, stream);
}

static int forward_best(fce_net* net, const fce_tensor* input, float* pred, unsigned long long* best, int graph,
                        void* stream);

int fce_net_forward_best(fce_net* net, const fce_tensor* input, float* pred, unsigned long long* best, int graph,
                         void* stream) {
  FCE_CHECK(net && pred, "fce_net_forward: null argument");
  // the Detect epilogues read cur_best while this call enqueues (captured graphs hold it by value); it is
  // cleared afterwards so a later profile / autotune pass can never write into a caller's key buffer
  net->cur_best = best;
  const int st = forward_best(net, input, pred, best, graph, stream);
  net->cur_best = nullptr;
  return st;
}

static int forward_best(fce_net* net, const fce_tensor* input, float* pred, unsigned long long* best, int graph,
                        void* stream) {
  int st = check_input(net, input);
  if (st) return st;
  hipStream_t caller = S(stream);
  FCE_GUARD({
    if (!graph) {
      // direct launches on the caller's stream (measured fastest: 1.865 ms vs 1.944 ms for the
      // captured graph and 2.24-2.30 ms for the DAG over 2-4 streams, n-fce 640 bs32); FCE_STREAMS > 1
      // spreads the op DAG over that many net-owned streams
      const char* ns = getenv("FCE_STREAMS");
      const int nstreams = std::max(1, std::min(8, ns ? atoi(ns) : 1));
      const bool mid = net->mid_ev && net->fork_op >= 0 && nstreams == 1;
      st = nstreams == 1 ? run_all(net, *input, pred, caller, mid) : run_all_streams(net, *input, pred, caller, nstreams);
      if (!st && net->mid_ev && !mid) FCE_HIP_CHECK(hipEventRecord(net->mid_ev, caller));
      return st;
    }
    // hipGraph: one linear capture (the legacy null stream cannot be captured, so the net then
    // captures and replays on a stream of its own, ordered against the caller's with events)
    hipStream_t s = caller;
    if (!net->join_ev[0]) {
      FCE_HIP_CHECK(hipEventCreateWithFlags(&net->join_ev[0], hipEventDisableTiming));
      FCE_HIP_CHECK(hipEventCreateWithFlags(&net->join_ev[1], hipEventDisableTiming));
    }
    if (s == nullptr) {
      if (!net->own) FCE_HIP_CHECK(hipStreamCreateWithFlags(&net->own, hipStreamNonBlocking));
      s = net->own;
      FCE_HIP_CHECK(hipEventRecord(net->join_ev[0], caller));
      FCE_HIP_CHECK(hipStreamWaitEvent(s, net->join_ev[0], 0));
    }
    fce_net::Captured* hit = nullptr;
    for (fce_net::Captured& c : net->graphs)
      if (c.in == input->data && c.out == pred && c.best == best && c.stream == s && c.dtype == input->dtype &&
          c.c == input->c)
        hit = &c;
    if (!hit) {
      if (int(net->graphs.size()) >= fce_net::kMaxGraphs) {  // evict the least recently replayed
        auto lru = std::min_element(net->graphs.begin(), net->graphs.end(),
                                    [](const fce_net::Captured& a, const fce_net::Captured& b) { return a.used < b.used; });
        fce_net::destroy(*lru);
        net->graphs.erase(lru);
      }
      FCE_HIP_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      st = run_all(net, *input, pred, s);
      hipGraph_t g = nullptr;
      hipError_t e = hipStreamEndCapture(s, &g);
      if (st) {
        if (g) (void)hipGraphDestroy(g);
        return st;
      }
      FCE_HIP_CHECK(e);
      hipGraphExec_t x = nullptr;
      if (hipGraphInstantiate(&x, g, nullptr, nullptr, 0) != hipSuccess) {
        (void)hipGraphDestroy(g);
        return fail(FCE_ERR_HIP, "fce_net_forward: hipGraphInstantiate failed");
      }
      net->graphs.push_back({g, x, input->data, pred, best, s, input->dtype, input->c, 0});
      hit = &net->graphs.back();
    }
    hit->used = ++net->graph_clock;
    FCE_HIP_CHECK(hipGraphLaunch(hit->exec, s));
    if (net->mid_ev) FCE_HIP_CHECK(hipEventRecord(net->mid_ev, s));
    if (s != caller) {
      FCE_HIP_CHECK(hipEventRecord(net->join_ev[1], s));
      FCE_HIP_CHECK(hipStreamWaitEvent(caller, net->join_ev[1], 0));
    }
    return FCE_OK;
  })
}

int fce_net_profile(fce_net* net, const fce_tensor* input, float* pred, float* ms, int* launches, int cap,
                    void* stream) {
  FCE_CHECK(net && pred && ms, "fce_net_profile: null argument");
  net->cur_best = nullptr;  // no best-class keys: the Detect epilogues write pred only
  int st = check_input(net, input);
  if (st) return st;
  hipStream_t s = S(stream);
  FCE_GUARD({
    // every kernel of every op carries its own (start, stop) event pair (hipExtLaunchKernelGGL): an
    // op's time is the sum of its kernels' execution intervals, the quantity rocprofv3 reports
    constexpr int kPerOp = 16;
    const int nops = int(net->ops.size());
    std::vector<hipEvent_t> ev(size_t(nops) * kPerOp * 2, nullptr);
    std::vector<int> used(nops, 0);
    auto destroy = [&]() {
      for (auto& e : ev)
        if (e) (void)hipEventDestroy(e);
    };
    for (auto& e : ev) {
      if (hipEventCreate(&e) != hipSuccess) {
        destroy();
        return fail(FCE_ERR_HIP, "fce_net_profile: hipEventCreate failed");
      }
    }
    for (int i = 0; i < nops && !st; ++i) {
      LaunchProbe probe{ev.data() + size_t(i) * kPerOp * 2, kPerOp, 0};
      g_probe = &probe;
      st = run_op(net, net->ops[i], *input, pred, s);
      g_probe = nullptr;
      used[i] = probe.n;
    }
    if (!st && hipStreamSynchronize(s) != hipSuccess) st = fail(FCE_ERR_HIP, "fce_net_profile: sync failed");
    for (int i = 0; i < nops && i < cap && !st; ++i) {
      float tot = 0.f;
      for (int k = 0; k < used[i]; ++k) {
        float t = 0.f;
        if (hipEventElapsedTime(&t, ev[(size_t(i) * kPerOp + k) * 2], ev[(size_t(i) * kPerOp + k) * 2 + 1]) !=
            hipSuccess) {
          st = fail(FCE_ERR_HIP, "fce_net_profile: hipEventElapsedTime failed");
          break;
        }
        tot += t;
      }
      ms[i] = tot;
      if (launches) launches[i] = used[i];
    }
    destroy();
    return st;
  })
}

int fce_net_op_info(const fce_net* net, int i, char* name, int cap, double* bytes, double* flops) {
  FCE_CHECK(net && i >= 0 && i < int(net->ops.size()) && bytes && flops, "fce_net_op_info: bad argument");
  std::string nm;
  op_cost(net, net->ops[i], &nm, bytes, flops);
  if (net->batch <= 0) *bytes = *flops = 0;  // before fce_net_plan: the op's name only (no sizes yet)
  if (name && cap > 0) {
    size_t n = std::min(nm.size(), size_t(cap - 1));
    nm.copy(name, n);
    name[n] = 0;
  }
  return FCE_OK;
}

int fce_net_op_variant(const fce_net* net, int i) {
  return net && i >= 0 && i < int(net->ops.size()) ? net->ops[i].tile : -1;
}

int fce_net_op_variants(const fce_net* net, int i, int* codes, int cap) {
  if (!net || i < 0 || i >= int(net->ops.size()) || !codes || cap <= 0 || net->batch <= 0) return 0;
  const OpDesc& op = net->ops[i];
  if (!(op.kind == OP_CONV && op.in >= 0) && op.kind != OP_CONV_DETECT) return 0;
  return conv_tile_candidates(op.conv, op.kind == OP_CONV_DETECT && op.part == 0, net->W >> net->bufs[op.in].shift,
                              codes, cap);
}

int fce_net_set_op_variant(fce_net* net, int i, int code) {
  FCE_CHECK(net && i >= 0 && i < int(net->ops.size()) && net->batch > 0, "fce_net_set_op_variant: bad argument");
  OpDesc& op = net->ops[i];
  FCE_CHECK((op.kind == OP_CONV && op.in >= 0) || op.kind == OP_CONV_DETECT, "fce_net_set_op_variant: not a conv op");
  if (code != -1) {
    int cand[128];
    const int nc = fce_net_op_variants(net, i, cand, 128);
    FCE_CHECK(std::find(cand, cand + nc, code) != cand + nc, "fce_net_set_op_variant: not a candidate of this op");
  }
  if (op.tile != code) net->drop_graph();  // captured forwards hold the old variant's launches
  op.tile = code;
  return FCE_OK;
}

int fce_net_tune_record(const fce_net* net, int k, int* op, int* code, float* ms) {
  if (!net || k < 0 || k >= int(net->tune_log.size())) return 0;
  if (op) *op = net->tune_log[k].op;
  if (code) *code = net->tune_log[k].code;
  if (ms) *ms = net->tune_log[k].ms;
  return 1;
}

int fce_net_buffer(const fce_net* net, int id, fce_tensor* out) {
  FCE_CHECK(net && out && id >= 0 && id < int(net->bufs.size()) && net->arena, "fce_net_buffer: bad argument");
  *out = net->view(id, 0, net->bufs[id].c);
  return FCE_OK;
}

}  // extern "C"
