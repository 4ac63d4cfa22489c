// Non-maximum suppression on the device (reference ultralytics/utils/nms.py:13-166 with the predict
// defaults multi_label=False, agnostic=False, classes=None; TorchNMS.nms :239-296; xywh2xyxy
// utils/ops.py:224-240).  nms_best_class_kernel (all CUs; skipped when the forward's Detect cls
// epilogue already produced the per-anchor best-class keys, fce_nms_best) + one 1024-thread workgroup
// per image:
//   1. candidates: best class per anchor (first maximum), keep conf > conf_thres, compacted in anchor
//      order with a block prefix sum; the class-offset xyxy box (cls * max_wh) and its area are
//      formed here, where the anchor-ordered loads coalesce;
//   2. order by (score desc, anchor asc): stable LDS radix sort (4 x 8-bit digits, ballot-matched
//      ranks) up to 8192 candidates, otherwise a bitonic sort of 64-bit keys in the workspace;
//      truncate to max_nms;
//   3. greedy suppression in sorted order, reproducing the reference's fp32 arithmetic (no FMA
//      contraction in this file) and stopping at max_det.  Fast path (all areas > 0, so no IoU is
//      NaN and the reference's "no overlap -> keep all" early exit changes nothing), by tiles of the
//      next 64 surviving candidates:
//        - the 64x64 suppression bit matrix of the tile is built by all 16 waves (one ballot per
//          row) and resolved in greedy order with 64-bit mask operations;
//        - later candidates are tested lazily: only those inside a frontier window
//          [tile end, F) are tested against each tile's kept boxes; a candidate entering the window
//          is tested once against every box kept so far.  The greedy typically stops (max_det) long
//          before the end of the sorted list, and nothing past its stop point is ever tested.
//      Degenerate boxes (or max_det > 1024) take the literal per-box loop with the early exit.
#include "common.h"

#pragma clang fp contract(off)

namespace fce {

static constexpr int NMS_THREADS = 1024;
static constexpr int NWAVES = NMS_THREADS / 64;
static constexpr int RADIX_CAP = 8192;   // LDS radix sort capacity (16 waves x 512)
static constexpr int REMOVED_CAP = 32768;
static constexpr int KEPT_CAP = 1024;    // kept boxes held in LDS by the tiled path
static constexpr int TILE = 64;
static constexpr int WIN = 256;  // frontier extension step (the multi-workgroup path)
// the one-workgroup kernel's frontier step: candidates entering the window are tested against every box kept so
// far, and those past the greedy's stop point are tested for nothing, so a short step wastes fewer tests at the
// price of more extension rounds (FCE_NMS_WIN overrides, a multiple of 64)
static int nms_win() {
  static const int w = [] {
    const char* e = getenv("FCE_NMS_WIN");
    const int v = e ? atoi(e) : 256;
    return v >= 64 && v % 64 == 0 ? v : 256;
  }();
  return w;
}
// small-set fast path: <= HEAD_CAP candidates sorted in LDS (1024 or 2048 slots instead of 8192).  Pool
// layout of that sort:
//   sort | keysA 8K | keysB 8K | valsA 4K | valsB 4K | wcnt (histogram) 16K |
// the greedy then uses the full layout's regions below valsA (removed | kept box | area | cand).
static constexpr int HEAD_CAP = 2048;
static constexpr int H_OFF_KA = 0, H_OFF_KB = 8 * 1024, H_OFF_VA = 16 * 1024, H_OFF_VB = 20 * 1024,
                     H_OFF_WC = 24 * 1024;

// LDS pool (bytes): sort phase  | keysA 32K | keysB 32K | valsA 16K | valsB 16K | wcnt 16K |
//                   greedy      | removed   | kept box+area | spos (= sorted valsA) |
static constexpr int POOL = 112 * 1024;
static constexpr int OFF_KB = 32 * 1024, OFF_VA = 64 * 1024, OFF_VB = 80 * 1024, OFF_WC = 96 * 1024;
static constexpr int OFF_KBOX = 32 * 1024, OFF_KAREA = 48 * 1024, OFF_KIDX = 52 * 1024;

// Candidate capacity C: A (best class per anchor), or A * nc with multi_label (one candidate per
// (anchor, class) above conf_thres).
struct NmsWs {
  float* aconf;    // per-anchor best score    [A]   (nms_best_class_kernel)
  int* acls;       // per-anchor best class    [A]
  int* cidx;       // candidate anchor index   [C]
  float* cscore;   // candidate score          [C]
  int* ccls;       // candidate class          [C]
  float4* cbox;    // candidate class-offset xyxy [C]
  float* carea;    // candidate area           [C]
  uint64_t* keys;  // global sort keys         [P2 = next_pow2(C)]  (> RADIX_CAP candidates)
  int* spos;       // sorted -> candidate pos  [M = min(C, max_nms)]   (> RADIX_CAP candidates)
};

// classes= filter (nms.py:128-132) as a bit mask over class ids < 1024; on == 0: every class
struct NmsClassMask {
  uint32_t w[32];
  int on;
};

static int next_pow2(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

static size_t nms2_ws_per_image(int A, int max_nms);

static size_t nms_ws_per_image(int A, int C, int max_nms) {
  const size_t M = std::min(C, max_nms);
  const size_t P2 = next_pow2(std::max(C, 1));
  auto al = [](size_t b) { return (b + 15) & ~size_t(15); };
  const size_t v1 = al(size_t(A) * 4) * 2 + al(size_t(C) * 4) * 4 + size_t(C) * 16 + P2 * 8 + al(M * 4);
  return (std::max(v1, nms2_ws_per_image(A, max_nms)) + 255) & ~size_t(255);  // either path fits (chosen per call)
}

static int nms_cap(int A, int nc, int multi) { return multi && nc > 1 ? A * nc : A; }

size_t nms_ws_bytes(int n, int A, int max_nms) { return size_t(n) * nms_ws_per_image(A, A, max_nms); }
size_t nms_ws_bytes_ex(int n, int nc, int A, int max_nms, int multi) {
  return size_t(n) * nms_ws_per_image(A, nms_cap(A, nc, multi), max_nms);
}

__device__ __forceinline__ int next_pow2_dev(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

__device__ NmsWs carve(char* p, int A, int C) {
  NmsWs w;
  const int P2 = next_pow2_dev(max(C, 1));
  auto al = [](size_t b) { return (b + 15) & ~size_t(15); };
  const size_t a4 = al(size_t(A) * 4), c4 = al(size_t(C) * 4);
  w.aconf = reinterpret_cast<float*>(p);
  w.acls = reinterpret_cast<int*>(p + a4);
  p += 2 * a4;
  w.cidx = reinterpret_cast<int*>(p);
  w.cscore = reinterpret_cast<float*>(p + c4);
  w.ccls = reinterpret_cast<int*>(p + 2 * c4);
  w.carea = reinterpret_cast<float*>(p + 3 * c4);
  p += 4 * c4;
  w.cbox = reinterpret_cast<float4*>(p);
  p += size_t(C) * 16;
  w.keys = reinterpret_cast<uint64_t*>(p);
  p += size_t(P2) * 8;
  w.spos = reinterpret_cast<int*>(p);
  return w;
}

// block-wide exclusive scan of 0/1 flags (1024 threads = 16 waves)
__device__ int block_scan(int flag, int* wsum, int* total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t m = __ballot(flag);
  const int before = __popcll(m & ((1ull << lane) - 1ull));
  if (lane == 0) wsum[wv] = __popcll(m);
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int i = 0; i < NWAVES; ++i) {
      const int v = wsum[i];
      wsum[i] = acc;
      acc += v;
    }
    *total = acc;
  }
  __syncthreads();
  return wsum[wv] + before;
}

// block-wide exclusive scan of non-negative counts
__device__ int block_scan_int(int v, int* wsum, int* total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[wv] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int i = 0; i < NWAVES; ++i) {
      const int t = wsum[i];
      wsum[i] = acc;
      acc += t;
    }
    *total = acc;
  }
  __syncthreads();
  return wsum[wv] + x - v;
}

__device__ void bitonic_desc(uint64_t* k, int n2) {
  for (int size = 2; size <= n2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = threadIdx.x; i < n2 / 2; i += blockDim.x) {
        const int lo = 2 * i - (i & (stride - 1));
        const int hi = lo + stride;
        const bool desc = ((lo & size) == 0);
        const uint64_t a = k[lo], b = k[hi];
        if ((a < b) == desc) {
          k[lo] = b;
          k[hi] = a;
        }
      }
      __syncthreads();
    }
  }
}

// Stable LSD radix sort of 1024 * IPL (key, index) pairs by ascending key, in LDS.  Wave w owns
// positions [64 IPL w, 64 IPL (w+1)) in lane-striped order (item j of lane l = 64 IPL w + 64j + l), so the
// ballot-matched running rank of a digit inside the wave is its stable rank; per-(digit, wave)
// counts are then scanned digit-major for the global offsets.
template <int IPL>
__device__ void radix_sort_lds(uint32_t* kA, uint32_t* kB, uint16_t* vA, uint16_t* vB, int* wcnt, int* wsum) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t lt = (1ull << lane) - 1ull;
  uint32_t* ks = kA;
  uint32_t* kd = kB;
  uint16_t* vs = vA;
  uint16_t* vd = vB;
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 8 * pass;
    for (int e = threadIdx.x; e < NWAVES * 256; e += NMS_THREADS) wcnt[e] = 0;
    __syncthreads();
    uint32_t k[IPL];
    uint16_t v[IPL];
    int d[IPL], rank[IPL];
#pragma unroll
    for (int j = 0; j < IPL; ++j) {
      const int idx = 64 * IPL * wv + 64 * j + lane;
      k[j] = ks[idx];
      v[j] = vs[idx];
      d[j] = int((k[j] >> shift) & 255u);
    }
    int* wc = wcnt + wv * 256;
#pragma unroll
    for (int j = 0; j < IPL; ++j) {
      uint64_t peer = ~0ull;
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        const bool bit = (d[j] >> b) & 1;
        const uint64_t bal = __ballot(bit);
        peer &= bit ? bal : ~bal;
      }
      const int pre = __popcll(peer & lt);
      const int base = wc[d[j]];
      rank[j] = base + pre;
      __builtin_amdgcn_wave_barrier();
      if (pre == 0) wc[d[j]] = base + __popcll(peer);
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    // exclusive scan over e = digit * 16 + wave
    int c[4], s = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = threadIdx.x * 4 + i;
      c[i] = wcnt[(e & 15) * 256 + (e >> 4)];
      s += c[i];
    }
    int inc = s;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int t = __shfl_up(inc, off);
      if (lane >= off) inc += t;
    }
    if (lane == 63) wsum[wv] = inc;
    __syncthreads();
    int excl = inc - s;
    for (int i = 0; i < wv; ++i) excl += wsum[i];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = threadIdx.x * 4 + i;
      wcnt[(e & 15) * 256 + (e >> 4)] = excl;
      excl += c[i];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < IPL; ++j) {
      const int pos = wc[d[j]] + rank[j];
      kd[pos] = k[j];
      vd[pos] = v[j];
    }
    __syncthreads();
    uint32_t* tk = ks;
    ks = kd;
    kd = tk;
    uint16_t* tv = vs;
    vs = vd;
    vd = tv;
  }
  // 4 passes: the result is back in (kA, vA)
}

// reference IoU (nms.py:276-291) in fp32, same operation order
__device__ __forceinline__ float iou_ref(float4 bi, float ai, float4 bj, float aj, float* inter_out) {
  const float ww = fmaxf(fminf(bi.z, bj.z) - fmaxf(bi.x, bj.x), 0.0f);
  const float hh = fmaxf(fminf(bi.w, bj.w) - fmaxf(bi.y, bj.y), 0.0f);
  const float inter = ww * hh;
  *inter_out = inter;
  return inter / ((ai + aj) - inter);
}

// iou_ref(...) > thr for positive areas: a zero intersection gives IoU 0 (thr >= 0), skip the division.  The IEEE
// division (~10 VALU ops) runs only when inter is within 2^-20 of thr * union: p = RN(thr * union) is within 2^-24 of
// the real product, so inter > p (1 + 2^-20) puts the real quotient above thr by far more than the half ulp RN(q)
// could lose (RN(q) > thr, as the reference computes it), and inter < p (1 - 2^-20) puts it below thr.  Exact.
// min / max of finite floats without the NaN-quieting canonicalisation fminf / fmaxf get in IEEE mode (two
// extra v_max per operand, re-done every iteration even for loop-invariant boxes): the same value for every
// finite input, and every box here is finite (degenerate boxes take the literal path)
__device__ __forceinline__ float vmin_(float a, float b) {
  float r;
  asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float vmax_(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

__device__ __forceinline__ bool suppresses(float4 bi, float ai, float4 bj, float aj, float thr) {
  const float ww = vmax_(vmin_(bi.z, bj.z) - vmax_(bi.x, bj.x), 0.0f);
  const float hh = vmax_(vmin_(bi.w, bj.w) - vmax_(bi.y, bj.y), 0.0f);
  const float inter = ww * hh;
  const float uni = (ai + aj) - inter;
  const float p = thr * uni;
  const bool hi = inter > p * 1.00000095367431640625f;  // 1 + 2^-20
  const bool lo = inter < p * 0.99999904632568359375f;  // 1 - 2^-20 (inter == 0 < p: lo, when thr > 0)
  bool r = hi;
  if (!(hi || lo)) r = inter / uni > thr;  // within 2^-20 of thr * union: the reference's quotient
  return r;
}

// best class per anchor (first maximum, like torch.max): one thread per (image, anchor), all CUs
__global__ __launch_bounds__(256) void nms_best_class_kernel(const float* pred, int nc, int A, int max_nms, char* ws,
                                                             size_t ws_per_image) {
  const int n = blockIdx.y;
  const int a = blockIdx.x * 256 + threadIdx.x;
  if (a >= A) return;
  const float* p = pred + (int64_t(n) * (4 + nc) + 4) * A + a;
  float best = -INFINITY;
  int bj = 0;
  int c = 0;
  for (; c + 8 <= nc; c += 8) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = p[int64_t(c + j) * A];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (v[j] > best) {
        best = v[j];
        bj = c + j;
      }
  }
  for (; c < nc; ++c) {
    const float v = p[int64_t(c) * A];
    if (v > best) {
      best = v;
      bj = c;
    }
  }
  NmsWs w = carve(ws + size_t(n) * ws_per_image, A, A);
  w.aconf[a] = best;
  w.acls[a] = bj;
}

__global__ __launch_bounds__(NMS_THREADS) void nms_kernel(const float* pred, const unsigned long long* bestk, int nc,
                                                          int A, float conf_thres,
                                                          float iou_thres, int max_det, int max_nms, float max_wh,
                                                          char* ws, size_t ws_per_image, float* dets, int64_t* keep,
                                                          int32_t* counts, int stop, int multi, int cap,
                                                          NmsClassMask cm, int win) {
  __shared__ __attribute__((aligned(16))) char pool[POOL];
  __shared__ int wsum[NWAVES];
  __shared__ int tile_idx[TILE];
  __shared__ float4 tile_box[TILE];
  __shared__ float tile_area[TILE];
  __shared__ uint64_t tile_sup[TILE];
  __shared__ int s_total, s_tile_n, s_need, s_next, s_nk, s_done, s_kept;

  const int n = blockIdx.x;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const float* P = pred + int64_t(n) * (4 + nc) * A;
  NmsWs w = carve(ws + size_t(n) * ws_per_image, A, cap);
  auto allowed = [&](int j) { return !cm.on || (j < 1024 && ((cm.w[j >> 5] >> (j & 31)) & 1u)); };

  // ---- 1. candidates in anchor order (+ their class-offset boxes)
  int base = 0, degenerate = 0;
  auto put = [&](int c, int a, float score, int j, float cx, float cy, float hw, float hh) {
    w.cidx[c] = a;
    w.cscore[c] = score;
    w.ccls[c] = j;
    const float off = (float)j * max_wh;
    const float bx1 = (cx - hw) + off, by1 = (cy - hh) + off, bx2 = (cx + hw) + off, by2 = (cy + hh) + off;
    w.cbox[c] = make_float4(bx1, by1, bx2, by2);
    const float ar = (bx2 - bx1) * (by2 - by1);
    w.carea[c] = ar;
    degenerate |= !(ar > 0.0f) || !isfinite(ar);
  };
  // multi_label (nms.py:116-120): torch.where(cls > conf_thres) in (anchor, class) order, then classes=
  for (int a0 = 0; multi && a0 < A; a0 += NMS_THREADS) {
    const int a = a0 + threadIdx.x;
    int cnt = 0;
    if (a < A)
      for (int j = 0; j < nc; ++j) cnt += (P[int64_t(4 + j) * A + a] > conf_thres) && allowed(j);
    int c = base + block_scan_int(cnt, wsum, &s_total);
    if (cnt) {
      const float cx = P[a], cy = P[int64_t(1) * A + a];
      const float hw = P[int64_t(2) * A + a] / 2.0f, hh = P[int64_t(3) * A + a] / 2.0f;
      for (int j = 0; j < nc; ++j) {
        const float v = P[int64_t(4 + j) * A + a];
        if (v > conf_thres && allowed(j)) put(c++, a, v, j, cx, cy, hw, hh);
      }
    }
    base += s_total;
    __syncthreads();
  }
  // best-class candidates: groups of CG chunks of 1024 anchors, ONE scan per group (two barriers) over the
  // per-(chunk, wave) counts, instead of a block scan (three barriers) per chunk; the candidates' box loads of
  // the whole group are issued before any of its workspace writes.  Same positions: anchor order.
  constexpr int CG = 9;
  __shared__ int gcnt[CG * NWAVES];
  const uint64_t lt = (1ull << lane) - 1ull;
  for (int g0 = 0; !multi && g0 < A; g0 += CG * NMS_THREADS) {
    float best[CG];
    int bj[CG];
    uint32_t fl = 0;
#pragma unroll
    for (int c = 0; c < CG; ++c) {
      const int a = g0 + c * NMS_THREADS + int(threadIdx.x);
      best[c] = -INFINITY;
      bj[c] = 0;
      if (a < A) {
        if (bestk) {  // fused into the Detect cls epilogue: score bits << 32 | ~class
          const unsigned long long k = bestk[int64_t(n) * A + a];
          best[c] = __uint_as_float(uint32_t(k >> 32));
          bj[c] = int(0xFFFFFFFFu - uint32_t(k));
        } else {
          best[c] = w.aconf[a];
          bj[c] = w.acls[a];
        }
      }
      const bool f = a < A && best[c] > conf_thres && allowed(bj[c]);
      fl |= uint32_t(f) << c;
      const uint64_t m = __ballot(f);
      if (lane == 0) gcnt[c * NWAVES + wv] = __popcll(m);
    }
    __syncthreads();
    if (wv == 0) {  // exclusive prefix over (chunk, wave) = anchor order, offset by the candidates so far
      constexpr int PER = (CG * NWAVES + 63) / 64;
      int v[PER], sum = 0;
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int idx = lane * PER + k;
        v[k] = idx < CG * NWAVES ? gcnt[idx] : 0;
        sum += v[k];
      }
      int inc = sum;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(inc, o);
        if (lane >= o) inc += y;
      }
      int ex = base + inc - sum;
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int idx = lane * PER + k;
        if (idx < CG * NWAVES) gcnt[idx] = ex;
        ex += v[k];
      }
      if (lane == 63) s_total = base + inc;
    }
    __syncthreads();
    float cx[CG], cy[CG], hw[CG], hh[CG];
#pragma unroll
    for (int c = 0; c < CG; ++c) {
      const int a = g0 + c * NMS_THREADS + int(threadIdx.x);
      if ((fl >> c) & 1u) {
        cx[c] = P[a];
        cy[c] = P[int64_t(1) * A + a];
        hw[c] = P[int64_t(2) * A + a] / 2.0f;
        hh[c] = P[int64_t(3) * A + a] / 2.0f;
      }
    }
#pragma unroll
    for (int c = 0; c < CG; ++c) {
      const bool f = (fl >> c) & 1u;
      const uint64_t m = __ballot(f);
      if (f) put(gcnt[c * NWAVES + wv] + __popcll(m & lt), g0 + c * NMS_THREADS + int(threadIdx.x), best[c], bj[c],
                 cx[c], cy[c], hw[c], hh[c]);
    }
    base = s_total;
    __syncthreads();  // gcnt / s_total are rewritten by the next group
  }
  const int ncand = base;
  degenerate = __syncthreads_or(degenerate);
  if (stop == 1) return;  // phase timing (FCE_NMS_STOP, diagnostics only)

  auto emit_det = [&](int c, int slot) {
    const int a = w.cidx[c];
    const float cx = P[a], cy = P[int64_t(1) * A + a];
    const float hw = P[int64_t(2) * A + a] / 2.0f, hh = P[int64_t(3) * A + a] / 2.0f;
    float* d = dets + (int64_t(n) * max_det + slot) * 6;
    d[0] = cx - hw;
    d[1] = cy - hh;
    d[2] = cx + hw;
    d[3] = cy + hh;
    d[4] = w.cscore[c];
    d[5] = (float)w.ccls[c];
    keep[int64_t(n) * max_det + slot] = a;
  };
  const int M = min(ncand, max_nms);
  const bool tiled = !degenerate && max_det <= KEPT_CAP;

  // ---- 2h. small candidate sets (<= HEAD_CAP, the usual case for a trained model) are sorted in 1024 or
  // 2048 LDS slots instead of RADIX_CAP (FCE_NMS_STOP=3, diagnostics: always the full sort)
  int hn = 0;
  bool head = false, prefix_only = false;
  if (tiled && stop != 3 && stop != 10) {
    hn = ncand;
    head = hn <= HEAD_CAP && hn > 0;
    if (hn > HEAD_CAP && hn <= RADIX_CAP) {  // empty and small sets never reach the select
      // ---- 2s. more than HEAD_CAP candidates: only the first HEAD_CAP entries of the sorted order (score desc,
      // position asc) are sorted.  A radix select (four 8-bit digit passes over the score bits held in registers,
      // wave-aggregated LDS atomics, three rotating histograms so each pass has one barrier, every wave finding
      // the digit itself) gives the HEAD_CAP-th largest score T and how many of the candidates scoring exactly T
      // the prefix takes (`need`: the first ones in position order, as the sort's tie order has it).  One ballot
      // scan over (chunk, wave) counts of the candidates above T and at T places the prefix in position order
      // and the 2048-slot sort orders it.  The greedy over the prefix is the full greedy's when max_det is reached
      // inside it; otherwise the full sort runs (attempt 1 below).
      constexpr int KPT = RADIX_CAP / NMS_THREADS;
      int* hist = reinterpret_cast<int*>(pool + H_OFF_WC);  // 3 x 256 bins, rotating over the passes
      int* gsel = hist + 3 * 256;                           // [KPT * NWAVES] above T, then [KPT * NWAVES] at T
      uint32_t key[KPT];
#pragma unroll
      for (int k = 0; k < KPT; ++k) {
        const int idx = k * NMS_THREADS + int(threadIdx.x);
        key[k] = idx < hn ? __float_as_uint(w.cscore[idx]) : 0u;  // scores > conf >= 0: valid keys > 0
      }
      if (threadIdx.x < 512) hist[threadIdx.x] = 0;
      __syncthreads();
      uint32_t pre = 0, pmask = 0;
      int need = HEAD_CAP;
#pragma unroll 1
      for (int pass = 0; pass < 4; ++pass) {
        const int shift = 24 - 8 * pass;
        int* h = hist + 256 * (pass % 3);
        // the histogram of pass + 1 was last read after the barrier of pass - 2: every wave is past that read
        if (pass > 0 && threadIdx.x < 256) hist[256 * ((pass + 1) % 3) + threadIdx.x] = 0;
#pragma unroll
        for (int k = 0; k < KPT; ++k) {
          // the lanes sharing the first active lane's digit add once (saturated scores put most keys in one
          // bin for the top digits; same-address LDS atomics would serialise)
          const bool in = k * NMS_THREADS + int(threadIdx.x) < hn && (key[k] & pmask) == pre;
          const int d = int(key[k] >> shift) & 255;
          const uint64_t act = __ballot(in);
          if (act) {
            const int first = __builtin_ctzll(act);
            const int d0 = __shfl(d, first);
            const uint64_t same = __ballot(in && d == d0);
            if (lane == first) atomicAdd(&h[d0], __popcll(same));
            if (in && d != d0) atomicAdd(&h[d], 1);
          }
        }
        __syncthreads();
        // every wave: lane l holds digits 4l .. 4l+3; the digit whose bin holds the need-th largest key
        int hv[4], s = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          hv[i] = h[4 * lane + i];
          s += hv[i];
        }
        int inc = s;  // suffix sum over lanes >= lane
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const int y = __shfl_down(inc, o);
          if (lane + o < 64) inc += y;
        }
        int above = inc - s, myd = 0, myab = 0;
        bool found = false;
#pragma unroll
        for (int i = 3; i >= 0; --i) {
          if (above < need && need <= above + hv[i]) {
            found = true;
            myd = 4 * lane + i;
            myab = above;
          }
          above += hv[i];
        }
        const int src = __builtin_ctzll(__ballot(found));
        pre |= uint32_t(__shfl(myd, src)) << shift;
        pmask |= 255u << shift;
        need -= __shfl(myab, src);
      }
      // pre = T; the prefix = every candidate above T and the first `need` at T in position order
#pragma unroll
      for (int k = 0; k < KPT; ++k) {
        const bool valid = k * NMS_THREADS + int(threadIdx.x) < hn;
        const uint64_t ma = __ballot(valid && key[k] > pre), mt = __ballot(valid && key[k] == pre);
        if (lane == 0) {
          gsel[k * NWAVES + wv] = __popcll(ma);
          gsel[KPT * NWAVES + k * NWAVES + wv] = __popcll(mt);
        }
      }
      __syncthreads();
      if (wv == 0) {  // two exclusive scans in (chunk, wave) = position order
        constexpr int PER = (KPT * NWAVES + 63) / 64;
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          int* g = gsel + half * KPT * NWAVES;
          int v[PER], sum = 0;
#pragma unroll
          for (int k = 0; k < PER; ++k) {
            v[k] = g[lane * PER + k];
            sum += v[k];
          }
          int inc = sum;
#pragma unroll
          for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(inc, o);
            if (lane >= o) inc += y;
          }
          int ex = inc - sum;
#pragma unroll
          for (int k = 0; k < PER; ++k) {
            g[lane * PER + k] = ex;
            ex += v[k];
          }
        }
      }
      __syncthreads();
      uint32_t* kA = reinterpret_cast<uint32_t*>(pool + H_OFF_KA);
      uint16_t* vA = reinterpret_cast<uint16_t*>(pool + H_OFF_VA);
#pragma unroll
      for (int k = 0; k < KPT; ++k) {
        const int idx = k * NMS_THREADS + int(threadIdx.x);
        const bool valid = idx < hn, ab = valid && key[k] > pre, at = valid && key[k] == pre;
        const uint64_t ma = __ballot(ab), mt = __ballot(at);
        const int nab = gsel[k * NWAVES + wv] + __popcll(ma & lt);               // above T before me
        const int nat = gsel[KPT * NWAVES + k * NWAVES + wv] + __popcll(mt & lt);  // at T before me
        if (ab || (at && nat < need)) {
          const int pos = nab + min(nat, need);
          kA[pos] = ~key[k];
          vA[pos] = uint16_t(idx);
        }
      }
      __syncthreads();
      radix_sort_lds<2>(kA, reinterpret_cast<uint32_t*>(pool + H_OFF_KB), vA,
                        reinterpret_cast<uint16_t*>(pool + H_OFF_VB), reinterpret_cast<int*>(pool + H_OFF_WC), wsum);
      __syncthreads();
      hn = HEAD_CAP;
      head = prefix_only = true;
    } else if (head) {
      uint32_t* kA = reinterpret_cast<uint32_t*>(pool + H_OFF_KA);
      uint16_t* vA = reinterpret_cast<uint16_t*>(pool + H_OFF_VA);
      const int cap = hn <= 1024 ? 1024 : 2048;
      for (int i = threadIdx.x; i < cap; i += NMS_THREADS) {
        kA[i] = i < hn ? ~__float_as_uint(w.cscore[i]) : 0xFFFFFFFFu;  // scores > conf >= 0
        vA[i] = uint16_t(i);
      }
      __syncthreads();
      if (cap == 1024)
        radix_sort_lds<1>(kA, reinterpret_cast<uint32_t*>(pool + H_OFF_KB), vA,
                          reinterpret_cast<uint16_t*>(pool + H_OFF_VB), reinterpret_cast<int*>(pool + H_OFF_WC), wsum);
      else
        radix_sort_lds<2>(kA, reinterpret_cast<uint32_t*>(pool + H_OFF_KB), vA,
                          reinterpret_cast<uint16_t*>(pool + H_OFF_VB), reinterpret_cast<int*>(pool + H_OFF_WC), wsum);
      __syncthreads();
    }
  }
  if (stop == 2) return;

  for (int attempt = head ? 0 : 1; attempt < 2; ++attempt) {  // the small (or prefix) sort, else the full sort
    const bool H = attempt == 0;
    int Mg = M;  // sorted positions this attempt covers
    bool lds_sorted = true;
    const uint16_t* spos16 = reinterpret_cast<const uint16_t*>(pool + (H ? H_OFF_VA : OFF_VA));
    if (H) {
      Mg = min(hn, M);
    } else {
      // ---- 2f. order the full candidate list (score desc, candidate position asc)
      lds_sorted = ncand <= RADIX_CAP;
      if (lds_sorted) {
        uint32_t* kA = reinterpret_cast<uint32_t*>(pool);
        uint16_t* vA = reinterpret_cast<uint16_t*>(pool + OFF_VA);
        for (int i = threadIdx.x; i < RADIX_CAP; i += NMS_THREADS) {
          kA[i] = i < ncand ? ~__float_as_uint(w.cscore[i]) : 0xFFFFFFFFu;  // scores > conf >= 0
          vA[i] = uint16_t(i);
        }
        __syncthreads();
        radix_sort_lds<8>(kA, reinterpret_cast<uint32_t*>(pool + OFF_KB), vA,
                          reinterpret_cast<uint16_t*>(pool + OFF_VB), reinterpret_cast<int*>(pool + OFF_WC), wsum);
      } else {
        const int n2 = next_pow2_dev(ncand);
        for (int i = threadIdx.x; i < n2; i += NMS_THREADS) {
          uint64_t k = 0;
          if (i < ncand) k = (uint64_t(__float_as_uint(w.cscore[i])) << 32) | uint64_t(0xFFFFFFFFu - uint32_t(i));
          w.keys[i] = k;
        }
        __syncthreads();
        bitonic_desc(w.keys, n2);
        for (int i = threadIdx.x; i < M; i += NMS_THREADS)
          w.spos[i] = int(0xFFFFFFFFu - uint32_t(w.keys[i] & 0xFFFFFFFFull));
        __syncthreads();
      }
      __syncthreads();
      if (stop == 10) return;  // phase timing (diagnostics only): the full sort's cost
    }
    auto sp = [&](int i) -> int { return lds_sorted ? int(spos16[i]) : w.spos[i]; };
    // greedy state over the dead sort keys (the sorted positions, spos16, stay live in either layout)
    uint8_t* lremoved = reinterpret_cast<uint8_t*>(pool);
    float4* kbox = reinterpret_cast<float4*>(pool + OFF_KBOX);
    float* karea = reinterpret_cast<float*>(pool + OFF_KAREA);
    int* kidx = reinterpret_cast<int*>(pool + OFF_KIDX);  // kept slot -> candidate
    if (threadIdx.x == 0) s_kept = 0;
    __syncthreads();

    if (!tiled) {
      // ---- 3b. literal per-box greedy (TorchNMS.nms with its early exit) for degenerate boxes
      for (int i = threadIdx.x; i < M; i += NMS_THREADS) lremoved[i] = 0;
      __syncthreads();
      int kept = 0;
      for (int i = 0; i < M && kept < max_det; ++i) {
        if (lremoved[i]) continue;
        const int ci = sp(i);
        if (threadIdx.x == 0) emit_det(ci, kept);
        ++kept;
        if (kept >= max_det) break;
        const float4 bi = w.cbox[ci];
        const float ai = w.carea[ci];
        int any = 0;
        for (int j = i + 1 + threadIdx.x; j < M; j += NMS_THREADS) {
          if (lremoved[j]) continue;
          const int cj = sp(j);
          float inter;
          iou_ref(bi, ai, w.cbox[cj], w.carea[cj], &inter);
          any |= inter != 0.0f;
        }
        any = __syncthreads_or(any);
        if (any) {
          for (int j = i + 1 + threadIdx.x; j < M; j += NMS_THREADS) {
            if (lremoved[j]) continue;
            const int cj = sp(j);
            float inter;
            const float iou = iou_ref(bi, ai, w.cbox[cj], w.carea[cj], &inter);
            if (!(iou <= iou_thres)) lremoved[j] = 1;
          }
        }
        __syncthreads();
      }
      if (threadIdx.x == 0) s_kept = kept;
      break;
    }

    // Candidates [jlo, jhi) (sorted positions, not yet removed) against kept boxes [klo, khi): all 1024
    // threads, thread = (candidate, split of the kept list).  Each wave holds 64 consecutive candidates
    // and one split, so every lane of a wave reads the same kept boxes (LDS broadcast), 4 per batch of
    // loads; a suppressed candidate's flag is set by whichever split finds it (all writers store 1).
    auto test_range = [&](int jlo, int jhi, int klo, int khi) {
      const int nj = jhi - jlo, nk = khi - klo;
      if (nj <= 0 || nk <= 0 || stop == 5) return;  // 5: diagnostics only (skips the tests)
      const int rj = (nj + 63) & ~63;
      const int S = max(1, min(nk, NMS_THREADS / rj));
      for (int idx = threadIdx.x; idx < rj * S; idx += NMS_THREADS) {
        const int j = jlo + idx % rj, sp0 = idx / rj;
        if (j >= jhi || lremoved[j]) continue;
        const int c = sp(j);
        const float4 bj = w.cbox[c];
        const float aj = w.carea[c];
        bool rem = false;
        int k = klo + sp0;
        for (; k + 3 * S < khi && !rem; k += 4 * S) {
          float4 kb[4];
          float ka[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            kb[u] = kbox[k + u * S];
            ka[u] = karea[k + u * S];
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) rem |= suppresses(kb[u], ka[u], bj, aj, iou_thres);
        }
        for (; k < khi && !rem; k += S) rem = suppresses(kbox[k], karea[k], bj, aj, iou_thres);
        if (rem) lremoved[j] = 1;
      }
    };

    // ---- 3a. tiled greedy with a lazy frontier (exact when every area > 0)
    uint64_t* colmask = tile_sup;  // colmask[u] = {t < u in the tile : IoU(t, u) > thr}
    int cursor = 0, F = 0;
    // diagnostics (FCE_NMS_STOP=9): s_memtime clocks per segment [select, colmask, resolve, window
    // test, tiles, extensions, extension tests, emit] written to dets[n][0..1][..] (8 floats)
    uint64_t tm[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tprev = stop == 9 ? __builtin_amdgcn_s_memtime() : 0;
    auto tick = [&](int slot) {
      if (stop == 9) {
        const uint64_t t = __builtin_amdgcn_s_memtime();
        tm[slot] += t - tprev;
        tprev = t;
      }
    };
    bool reached = false;  // max_det reached
    while (true) {
      // select the next <= 64 surviving candidates in [cursor, F), extending F while short
      while (true) {
        if (wv == 0) {
          int cnt = 0;
          for (int c = cursor; cnt < TILE && c < F; c += 64) {
            const int j = c + lane;
            const bool alive = j < F && !lremoved[j];
            const uint64_t bb = __ballot(alive);
            const int take = min(__popcll(bb), TILE - cnt);
            const int rank = __popcll(bb & ((1ull << lane) - 1ull));
            if (alive && rank < take) tile_idx[cnt + rank] = j;
            cnt += take;
          }
          __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's tile_idx writes have landed
          __builtin_amdgcn_wave_barrier();
          const bool need = cnt < TILE && F < Mg;
          if (!need && lane < cnt) {
            const int c = sp(tile_idx[lane]);
            tile_box[lane] = w.cbox[c];
            tile_area[lane] = w.carea[c];
          }
          if (lane == 0) {
            s_tile_n = cnt;
            s_need = need;
            s_next = cnt == TILE ? tile_idx[TILE - 1] + 1 : Mg;
          }
        }
        __syncthreads();
        tick(0);
        if (!s_need) break;
        // candidates entering the window: tested once against every box kept so far.  Near max_det the step
        // shrinks to what the survival rate so far (s_kept kept of F) says is still needed, +25 %, in multiples
        // of 64: candidates past the greedy's stop are tested for nothing (any schedule gives the same result)
        int step = win;
        if (s_kept > 0 && stop != 12) {  // 12: diagnostics only (fixed steps)
          const int64_t est = int64_t(max_det - s_kept) * F / s_kept;
          step = min(win, max(64, int(((est * 5) / 4 + 63) & ~int64_t(63))));
        }
        const int Fn = min(Mg, F + step);
        for (int j = F + threadIdx.x; j < Fn; j += NMS_THREADS) lremoved[j] = 0;
        __syncthreads();
        test_range(F, Fn, 0, s_kept);
        F = Fn;
        __syncthreads();
        tm[5] += 1;
        tick(6);
      }
      tm[4] += 1;
      const int cnt = s_tile_n;
      if (cnt == 0) break;
      // column masks of the tile's suppression relation: wave w owns columns u = w, w+16, ..; lane = row t
      for (int u = wv; u < TILE && stop != 6; u += NWAVES) {  // 6: diagnostics only
        bool sup = false;
        if (lane < u && u < cnt)
          sup = suppresses(tile_box[lane], tile_area[lane], tile_box[u], tile_area[u], iou_thres);
        const uint64_t bb = __ballot(sup);
        if (lane == 0) colmask[u] = bb;
      }
      __syncthreads();
      tick(1);
      if (wv == 0) {
        // greedy over the tile as a fixpoint (lane u = tile candidate u): u is kept once none of its
        // suppressors is kept or undecided, removed once one of them is kept.  Every round decides at
        // least the lowest undecided candidate, and each decision is the sequential greedy's.
        const int kept0 = s_kept;
        const uint64_t C = lane < cnt ? colmask[lane] : 0ull;
        uint64_t undecided = cnt == 64 ? ~0ull : ((1ull << cnt) - 1ull), kept = 0;
        while (undecided) {
          const bool me = (undecided >> lane) & 1ull;
          const uint64_t k = __ballot(me && (C & (kept | undecided)) == 0ull);
          const uint64_t r = __ballot(me && (C & kept) != 0ull);
          kept |= k;
          undecided &= ~(k | r);
        }
        // max_det: the greedy stops at the (max_det - kept0)-th kept candidate of the tile
        int nk = __popcll(kept);
        bool done = false;
        if (kept0 + nk >= max_det) {
          const int allow = max_det - kept0;
          uint64_t m = kept;
          for (int i = 0; i < allow - 1; ++i) m &= m - 1ull;  // drop the lowest allow-1 bits
          const uint64_t last = m & (~m + 1ull);               // the allow-th kept candidate
          kept &= (last << 1) - 1ull;
          nk = allow;
          done = true;
        }
        if ((kept >> lane) & 1ull) {
          const int r = __popcll(kept & ((1ull << lane) - 1ull));
          kbox[kept0 + r] = tile_box[lane];
          karea[kept0 + r] = tile_area[lane];
          kidx[kept0 + r] = sp(tile_idx[lane]);
        }
        if (lane == 0) {
          s_nk = nk;
          s_kept = kept0 + nk;
          s_done = done ? 2 : (s_next >= Mg ? 1 : 0);
        }
      }
      __syncthreads();
      tick(2);
      if (s_done) {
        reached = s_done == 2;
        break;
      }
      // the rest of the window against the tile's kept boxes
      const int start = s_next;
      test_range(start, F, s_kept - s_nk, s_kept);
      cursor = start;
      __syncthreads();
      tick(3);
    }
    __syncthreads();
    // the selected prefix ran out before max_det: its decisions are the full greedy's, but the greedy goes on
    // past it, so start again over the full sort
    if (H && prefix_only && !reached && Mg < M) continue;
    tick(7);
    for (int slot = threadIdx.x; slot < s_kept; slot += NMS_THREADS) emit_det(kidx[slot], slot);
    __syncthreads();
    tick(7);
    if (stop == 9 && threadIdx.x == 0)
      for (int i = 0; i < 8; ++i) dets[int64_t(n) * max_det * 6 + i] = float(tm[i]);
    break;
  }
  __syncthreads();
  if (threadIdx.x == 0) counts[n] = s_kept;
}


// ================================================================ multi-workgroup NMS (opt-in: FCE_NMS_V2=1)
// The one-workgroup kernel above needs a whole CU per image (1024 threads, 112 KB of LDS), so beside the
// forward of other batches it waits for CUs to drain, and its candidate and sort phases are serial over
// one workgroup.  Here the same computation is four launches:
//   K1 nms2_keys_kernel   (all CUs, one thread per anchor): best class (the Detect epilogue's key, or the
//                          arg-max over the class rows) and the sort key score bits << 32 | ~anchor (0 for
//                          a non-candidate).  Descending keys = (score desc, anchor asc) = the reference's
//                          order of candidates (they are formed in anchor order, nms.py:101-105, 150-153);
//   K2 nms2_sort_kernel   (one 256-thread workgroup per 2048-anchor chunk): bitonic sort of the chunk's
//                          keys in 16 KB of LDS, candidate count per chunk;
//   K3 nms2_rank_kernel   (one workgroup per chunk): a candidate's global rank = its rank in its chunk +
//                          the number of larger keys in every other chunk (binary searches); ranks <
//                          max_nms scatter the class-offset box, area, anchor, score and class into
//                          rank-ordered arrays (the truncation of nms.py:155-156), and flag degenerate boxes;
//   K4 nms2_greedy_kernel (one 256-thread workgroup per image, LDS = max_nms bytes + max_det kept boxes):
//                          the tiled greedy of the kernel above over the rank-ordered arrays (coalesced),
//                          or the literal loop when a box is degenerate.
// Same fp32 arithmetic, same order, same greedy: bitwise the results of nms_kernel.
static constexpr int NMS2_CH = 2048;
static constexpr int NMS2_SORT_THREADS = 256;
static constexpr int NMS2_G_THREADS = 256;
static constexpr int NMS2_G_WAVES = NMS2_G_THREADS / 64;

struct Nms2Ws {
  uint64_t* keys;  // [A2] per anchor, then sorted within each chunk (descending)
  int* acls;       // [A] best class per anchor
  int* ccount;     // [NCH] candidates per chunk
  int* flags;      // [4]: [0] = a degenerate box among the first M sorted candidates
  float4* sbox;    // [Mc] rank-ordered class-offset xyxy boxes
  float* sarea;    // [Mc]
  int* sanc;       // [Mc] anchor
  float* sscore;   // [Mc]
  int* scls;       // [Mc]
};

__host__ __device__ inline int nms2_a2(int A) { return (A + NMS2_CH - 1) / NMS2_CH * NMS2_CH; }

static size_t nms2_ws_per_image(int A, int max_nms) {
  auto al = [](size_t b) { return (b + 15) & ~size_t(15); };
  const size_t A2 = nms2_a2(A), NCH = A2 / NMS2_CH, Mc = std::min(A, max_nms);
  return A2 * 8 + al(size_t(A) * 4) + al(NCH * 4) + 16 + Mc * 16 + 4 * al(Mc * 4);
}

__device__ Nms2Ws carve2(char* p, int A, int Mc) {
  auto al = [](size_t b) { return (b + 15) & ~size_t(15); };
  const size_t A2 = nms2_a2(A), NCH = A2 / NMS2_CH;
  Nms2Ws w;
  w.keys = reinterpret_cast<uint64_t*>(p);
  p += A2 * 8;
  w.acls = reinterpret_cast<int*>(p);
  p += al(size_t(A) * 4);
  w.ccount = reinterpret_cast<int*>(p);
  p += al(NCH * 4);
  w.flags = reinterpret_cast<int*>(p);
  p += 16;
  w.sbox = reinterpret_cast<float4*>(p);
  p += size_t(Mc) * 16;
  w.sarea = reinterpret_cast<float*>(p);
  p += al(size_t(Mc) * 4);
  w.sanc = reinterpret_cast<int*>(p);
  p += al(size_t(Mc) * 4);
  w.sscore = reinterpret_cast<float*>(p);
  p += al(size_t(Mc) * 4);
  w.scls = reinterpret_cast<int*>(p);
  return w;
}

__global__ __launch_bounds__(256) void nms2_keys_kernel(const float* pred, const unsigned long long* bestk, int nc, int A,
                                                        int Mc, float conf_thres, char* ws, size_t per,
                                                        NmsClassMask cm) {
  const int n = blockIdx.y;
  const int a = blockIdx.x * 256 + threadIdx.x;
  Nms2Ws w = carve2(ws + size_t(n) * per, A, Mc);
  uint64_t key = 0;
  if (a < A) {
    float best = -INFINITY;
    int bj = 0;
    if (bestk) {  // fused into the Detect cls epilogue: score bits << 32 | ~class
      const unsigned long long k = bestk[int64_t(n) * A + a];
      best = __uint_as_float(uint32_t(k >> 32));
      bj = int(0xFFFFFFFFu - uint32_t(k));
    } else {  // first maximum over the class rows (torch.max, nms.py:101)
      const float* p = pred + (int64_t(n) * (4 + nc) + 4) * A + a;
      int c = 0;
      for (; c + 8 <= nc; c += 8) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = p[int64_t(c + j) * A];
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (v[j] > best) {
            best = v[j];
            bj = c + j;
          }
      }
      for (; c < nc; ++c) {
        const float v = p[int64_t(c) * A];
        if (v > best) {
          best = v;
          bj = c;
        }
      }
    }
    const bool allowed = !cm.on || (bj < 1024 && ((cm.w[bj >> 5] >> (bj & 31)) & 1u));
    if (best > conf_thres && allowed)  // a positive score: its bits order like the value
      key = (uint64_t(__float_as_uint(best)) << 32) | uint64_t(0xFFFFFFFFu - uint32_t(a));
    w.acls[a] = bj;
  }
  if (a < nms2_a2(A)) w.keys[a] = key;
}

__global__ __launch_bounds__(NMS2_SORT_THREADS) void nms2_sort_kernel(int A, int Mc, char* ws, size_t per) {
  __shared__ uint64_t sk[NMS2_CH];
  __shared__ int scount;
  const int n = blockIdx.y, chunk = blockIdx.x;
  Nms2Ws w = carve2(ws + size_t(n) * per, A, Mc);
  uint64_t* g = w.keys + size_t(chunk) * NMS2_CH;
  if (threadIdx.x == 0) scount = 0;
  __syncthreads();
  int cnt = 0;
  for (int i = threadIdx.x; i < NMS2_CH; i += NMS2_SORT_THREADS) {
    const uint64_t k = g[i];
    sk[i] = k;
    cnt += k != 0;
  }
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
  if ((threadIdx.x & 63) == 0) atomicAdd(&scount, cnt);
  __syncthreads();
  if (scount > 0) bitonic_desc(sk, NMS2_CH);  // ends with __syncthreads
  for (int i = threadIdx.x; i < NMS2_CH; i += NMS2_SORT_THREADS) g[i] = sk[i];
  if (threadIdx.x == 0) {
    w.ccount[chunk] = scount;
    if (chunk == 0) w.flags[0] = 0;
  }
}

// number of keys > k in a descending run of `cnt` distinct keys
__device__ __forceinline__ int count_greater(const uint64_t* run, int cnt, uint64_t k) {
  int lo = 0, hi = cnt;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (run[mid] > k)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

__global__ __launch_bounds__(256) void nms2_rank_kernel(const float* pred, int nc, int A, int Mc, int max_nms,
                                                        float max_wh, char* ws, size_t per) {
  const int n = blockIdx.y, chunk = blockIdx.x;
  Nms2Ws w = carve2(ws + size_t(n) * per, A, Mc);
  const int nch = nms2_a2(A) / NMS2_CH;
  int total = 0;
  for (int r = 0; r < nch; ++r) total += w.ccount[r];
  const int M = min(total, max_nms);
  const int mine = w.ccount[chunk];
  const uint64_t* run = w.keys + size_t(chunk) * NMS2_CH;
  const float* P = pred + int64_t(n) * (4 + nc) * A;
  int deg = 0;
  for (int i = threadIdx.x; i < mine; i += 256) {
    const uint64_t k = run[i];
    int rank = i;
    for (int r = 0; r < nch; ++r)
      if (r != chunk) rank += count_greater(w.keys + size_t(r) * NMS2_CH, w.ccount[r], k);
    if (rank >= M) continue;
    const int a = int(0xFFFFFFFFu - uint32_t(k));
    const int j = w.acls[a];
    const float cx = P[a], cy = P[int64_t(1) * A + a];
    const float hw = P[int64_t(2) * A + a] / 2.0f, hh = P[int64_t(3) * A + a] / 2.0f;
    const float off = (float)j * max_wh;
    const float bx1 = (cx - hw) + off, by1 = (cy - hh) + off, bx2 = (cx + hw) + off, by2 = (cy + hh) + off;
    const float ar = (bx2 - bx1) * (by2 - by1);
    w.sbox[rank] = make_float4(bx1, by1, bx2, by2);
    w.sarea[rank] = ar;
    w.sanc[rank] = a;
    w.sscore[rank] = __uint_as_float(uint32_t(k >> 32));
    w.scls[rank] = j;
    deg |= !(ar > 0.0f) || !isfinite(ar);
  }
  if (__any(deg) && (threadIdx.x & 63) == 0) atomicOr(w.flags, 1);
}

__global__ __launch_bounds__(NMS2_G_THREADS) void nms2_greedy_kernel(const float* pred, int nc, int A, int Mc,
                                                                     float iou_thres, int max_det, int max_nms,
                                                                     char* ws, size_t per, float* dets,
                                                                     int64_t* keep, int32_t* counts) {
  extern __shared__ __attribute__((aligned(16))) char g2pool[];  // removed [Mc] | kbox | karea | kidx
  __shared__ int tile_idx[TILE];
  __shared__ float4 tile_box[TILE];
  __shared__ float tile_area[TILE];
  __shared__ uint64_t colmask[TILE];
  __shared__ int s_tile_n, s_need, s_next, s_nk, s_done, s_kept;
  const int n = blockIdx.x;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  Nms2Ws w = carve2(ws + size_t(n) * per, A, Mc);
  const int nch = nms2_a2(A) / NMS2_CH;
  int total = 0;
  for (int r = 0; r < nch; ++r) total += w.ccount[r];
  const int M = min(total, max_nms);
  const bool degenerate = w.flags[0] != 0;
  const float* P = pred + int64_t(n) * (4 + nc) * A;
  uint8_t* lremoved = reinterpret_cast<uint8_t*>(g2pool);
  float4* kbox = reinterpret_cast<float4*>(g2pool + ((Mc + 15) & ~15));
  float* karea = reinterpret_cast<float*>(kbox + max_det);
  int* kidx = reinterpret_cast<int*>(karea + max_det);
  auto emit_det = [&](int pos, int slot) {
    const int a = w.sanc[pos];
    const float cx = P[a], cy = P[int64_t(1) * A + a];
    const float hw = P[int64_t(2) * A + a] / 2.0f, hh = P[int64_t(3) * A + a] / 2.0f;
    float* d = dets + (int64_t(n) * max_det + slot) * 6;
    d[0] = cx - hw;
    d[1] = cy - hh;
    d[2] = cx + hw;
    d[3] = cy + hh;
    d[4] = w.sscore[pos];
    d[5] = (float)w.scls[pos];
    keep[int64_t(n) * max_det + slot] = a;
  };
  if (threadIdx.x == 0) s_kept = 0;
  __syncthreads();

  if (degenerate) {
    // literal per-box greedy (TorchNMS.nms with its early exit, nms.py:276-296)
    for (int i = threadIdx.x; i < M; i += NMS2_G_THREADS) lremoved[i] = 0;
    __syncthreads();
    int kept = 0;
    for (int i = 0; i < M && kept < max_det; ++i) {
      if (lremoved[i]) continue;
      if (threadIdx.x == 0) emit_det(i, kept);
      ++kept;
      if (kept >= max_det) break;
      const float4 bi = w.sbox[i];
      const float ai = w.sarea[i];
      int any = 0;
      for (int j = i + 1 + threadIdx.x; j < M; j += NMS2_G_THREADS) {
        if (lremoved[j]) continue;
        float inter;
        iou_ref(bi, ai, w.sbox[j], w.sarea[j], &inter);
        any |= inter != 0.0f;
      }
      any = __syncthreads_or(any);
      if (any) {
        for (int j = i + 1 + threadIdx.x; j < M; j += NMS2_G_THREADS) {
          if (lremoved[j]) continue;
          float inter;
          const float iou = iou_ref(bi, ai, w.sbox[j], w.sarea[j], &inter);
          if (!(iou <= iou_thres)) lremoved[j] = 1;
        }
      }
      __syncthreads();
    }
    if (threadIdx.x == 0) counts[n] = kept;
    return;
  }

  // candidates [jlo, jhi) (not yet removed) against kept boxes [klo, khi): thread = (candidate, split of the
  // kept list); every lane of a wave reads the same kept boxes (LDS broadcast)
  auto test_range = [&](int jlo, int jhi, int klo, int khi) {
    const int nj = jhi - jlo, nk = khi - klo;
    if (nj <= 0 || nk <= 0) return;
    const int rj = (nj + 63) & ~63;
    const int S = max(1, min(nk, NMS2_G_THREADS / rj));
    for (int idx = threadIdx.x; idx < rj * S; idx += NMS2_G_THREADS) {
      const int j = jlo + idx % rj, sp0 = idx / rj;
      if (j >= jhi || lremoved[j]) continue;
      const float4 bj = w.sbox[j];
      const float aj = w.sarea[j];
      bool rem = false;
      int k = klo + sp0;
      for (; k + 3 * S < khi && !rem; k += 4 * S) {
        float4 kb[4];
        float ka[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          kb[u] = kbox[k + u * S];
          ka[u] = karea[k + u * S];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) rem |= suppresses(kb[u], ka[u], bj, aj, iou_thres);
      }
      for (; k < khi && !rem; k += S) rem = suppresses(kbox[k], karea[k], bj, aj, iou_thres);
      if (rem) lremoved[j] = 1;
    }
  };

  // tiled greedy with a lazy frontier (nms_kernel 3a): exact when every area > 0
  int cursor = 0, F = 0;
  while (true) {
    while (true) {
      if (wv == 0) {
        int cnt = 0;
        for (int c = cursor; cnt < TILE && c < F; c += 64) {
          const int j = c + lane;
          const bool alive = j < F && !lremoved[j];
          const uint64_t bb = __ballot(alive);
          const int take = min(__popcll(bb), TILE - cnt);
          const int rank = __popcll(bb & ((1ull << lane) - 1ull));
          if (alive && rank < take) tile_idx[cnt + rank] = j;
          cnt += take;
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        const bool need = cnt < TILE && F < M;
        if (!need && lane < cnt) {
          const int j = tile_idx[lane];
          tile_box[lane] = w.sbox[j];
          tile_area[lane] = w.sarea[j];
        }
        if (lane == 0) {
          s_tile_n = cnt;
          s_need = need;
          s_next = cnt == TILE ? tile_idx[TILE - 1] + 1 : M;
        }
      }
      __syncthreads();
      if (!s_need) break;
      const int Fn = min(M, F + WIN);
      for (int j = F + threadIdx.x; j < Fn; j += NMS2_G_THREADS) lremoved[j] = 0;
      __syncthreads();
      test_range(F, Fn, 0, s_kept);
      F = Fn;
      __syncthreads();
    }
    const int cnt = s_tile_n;
    if (cnt == 0) break;
    for (int u = wv; u < TILE; u += NMS2_G_WAVES) {
      bool sup = false;
      if (lane < u && u < cnt) sup = suppresses(tile_box[lane], tile_area[lane], tile_box[u], tile_area[u], iou_thres);
      const uint64_t bb = __ballot(sup);
      if (lane == 0) colmask[u] = bb;
    }
    __syncthreads();
    if (wv == 0) {
      const int kept0 = s_kept;
      const uint64_t Cm = lane < cnt ? colmask[lane] : 0ull;
      uint64_t undecided = cnt == 64 ? ~0ull : ((1ull << cnt) - 1ull), kept = 0;
      while (undecided) {
        const bool me = (undecided >> lane) & 1ull;
        const uint64_t k = __ballot(me && (Cm & (kept | undecided)) == 0ull);
        const uint64_t r = __ballot(me && (Cm & kept) != 0ull);
        kept |= k;
        undecided &= ~(k | r);
      }
      int nk = __popcll(kept);
      bool done = false;
      if (kept0 + nk >= max_det) {
        const int allow = max_det - kept0;
        uint64_t m = kept;
        for (int i = 0; i < allow - 1; ++i) m &= m - 1ull;
        const uint64_t last = m & (~m + 1ull);
        kept &= (last << 1) - 1ull;
        nk = allow;
        done = true;
      }
      if ((kept >> lane) & 1ull) {
        const int r = __popcll(kept & ((1ull << lane) - 1ull));
        kbox[kept0 + r] = tile_box[lane];
        karea[kept0 + r] = tile_area[lane];
        kidx[kept0 + r] = tile_idx[lane];
      }
      if (lane == 0) {
        s_nk = nk;
        s_kept = kept0 + nk;
        s_done = done ? 2 : (s_next >= M ? 1 : 0);
      }
    }
    __syncthreads();
    if (s_done) break;
    const int start = s_next;
    test_range(start, F, s_kept - s_nk, s_kept);
    cursor = start;
    __syncthreads();
  }
  for (int slot = threadIdx.x; slot < s_kept; slot += NMS2_G_THREADS) emit_det(kidx[slot], slot);
  if (threadIdx.x == 0) counts[n] = s_kept;
}

static int nms2(const float* pred, const unsigned long long* best, int n, int nc, int A, float conf, float iou,
                int max_det, int max_nms, float max_wh, char* ws, size_t per, float* dets, int64_t* keep,
                int32_t* counts, hipStream_t s, const NmsClassMask& cm) {
  const int Mc = std::min(A, max_nms);
  const int A2 = nms2_a2(A), nch = A2 / NMS2_CH;
  const size_t lds = size_t((Mc + 15) & ~15) + size_t(max_det) * 24;
  FCE_CHECK(lds <= 64 * 1024, "nms: greedy LDS over 64 KiB");
  FCE_LAUNCH(nms2_keys_kernel, dim3(A2 / 256, n), dim3(256), 0, s, pred, best, nc, A, Mc, conf, ws, per, cm);
  FCE_LAUNCH(nms2_sort_kernel, dim3(nch, n), dim3(NMS2_SORT_THREADS), 0, s, A, Mc, ws, per);
  FCE_LAUNCH(nms2_rank_kernel, dim3(nch, n), dim3(256), 0, s, pred, nc, A, Mc, max_nms, max_wh, ws, per);
  FCE_LAUNCH(nms2_greedy_kernel, dim3(n), dim3(NMS2_G_THREADS), lds, s, pred, nc, A, Mc, iou, max_det, max_nms, ws,
             per, dets, keep, counts);
  return launch_status("nms2_greedy_kernel");
}

int nms(const float* pred, const unsigned long long* best, int n, int nc, int A, float conf, float iou, int max_det,
        int max_nms, float max_wh, void* ws, size_t ws_bytes, float* dets, int64_t* keep, int32_t* counts,
        hipStream_t s, int multi, const int32_t* classes, int nclasses) {
  FCE_CHECK(nc >= 1 && nc <= 65535 && A >= 0 && max_det >= 1 && max_nms >= 1, "nms: bad sizes");
  FCE_CHECK(max_nms <= REMOVED_CAP, "nms: max_nms > 32768 unsupported");
  FCE_CHECK(conf >= 0.f && conf <= 1.f && iou >= 0.f && iou <= 1.f, "nms: thresholds must be in [0, 1]");
  FCE_CHECK(nclasses >= 0 && (nclasses == 0 || classes), "nms: classes list");
  multi = multi && nc > 1;  // nms.py:96 multi_label &= nc > 1
  FCE_CHECK(!multi || int64_t(A) * nc < (int64_t(1) << 30), "nms: multi_label candidate capacity too large");
  NmsClassMask cm{};
  cm.on = classes != nullptr;
  if (classes) {
    FCE_CHECK(nc <= 1024, "nms: classes filter supports nc <= 1024");
    for (int i = 0; i < nclasses; ++i)
      if (classes[i] >= 0 && classes[i] < nc) cm.w[classes[i] >> 5] |= 1u << (classes[i] & 31);
  }
  if (n == 0) return FCE_OK;
  const int cap = nms_cap(A, nc, multi);
  const size_t per = nms_ws_per_image(A, cap, max_nms);
  FCE_CHECK(ws && ws_bytes >= per * n, "nms: workspace too small");
  const char* stop_env = getenv("FCE_NMS_STOP");  // diagnostics: end the kernel after phase 1 / 2
  const int stop = stop_env ? atoi(stop_env) : 0;
  if (multi) best = nullptr;  // candidates come from every class row
  // FCE_NMS_V2=1: the multi-workgroup path (opt-in: measured slower on the bench batch)
  const char* v2e = getenv("FCE_NMS_V2");
  const bool v1 = !(v2e && atoi(v2e) != 0);
  // V2 only where its greedy workgroup's LDS (candidate flags + 24 B per kept box) fits 64 KiB; every other
  // configuration (multi_label, max_det > KEPT_CAP, a large max_det) takes the one-workgroup kernel
  const bool v2_lds = size_t((std::min(A, max_nms) + 15) & ~15) + size_t(max_det) * 24 <= 64 * 1024;
  if (!multi && A > 0 && max_det <= KEPT_CAP && !v1 && stop == 0 && v2_lds)
    return nms2(pred, best, n, nc, A, conf, iou, max_det, max_nms, max_wh, static_cast<char*>(ws), per, dets, keep,
                counts, s, cm);
  if (A > 0 && !best && !multi)  // else the keys came from the Detect cls epilogue (fce_nms_best)
    FCE_LAUNCH(nms_best_class_kernel, dim3((A + 255) / 256, n), dim3(256), 0, s, pred, nc, A, max_nms,
                       static_cast<char*>(ws), per);
  FCE_LAUNCH(nms_kernel, dim3(n), dim3(NMS_THREADS), 0, s, pred, best, nc, A, conf, iou, max_det, max_nms, max_wh,
                     static_cast<char*>(ws), per, dets, keep, counts, stop, multi, cap, cm, nms_win());
  return launch_status("nms_kernel");
}

}  // namespace fce
