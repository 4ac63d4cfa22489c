// Non-maximum suppression on the device (reference ultralytics/utils/nms.py:13-166 with the predict
// defaults multi_label=False, agnostic=False, classes=None; TorchNMS.nms :239-296; xywh2xyxy
// utils/ops.py:224-240).  One workgroup per image:
//   1. candidates: best class per anchor (first maximum), keep conf > conf_thres, compacted in anchor
//      order with a block prefix sum;
//   2. sort by (score desc, anchor asc) with a bitonic sort on 64-bit keys (LDS up to 8192
//      candidates, otherwise in the workspace); truncate to max_nms;
//   3. greedy suppression in sorted order over class-offset boxes (cls * max_wh), reproducing the
//      reference's fp32 arithmetic (no FMA contraction in this file) and its early exit when no
//      remaining box intersects the kept one; stop at max_det.
#include "common.h"

#pragma clang fp contract(off)

namespace fce {

static constexpr int NMS_THREADS = 1024;
static constexpr int LDS_SORT_CAP = 8192;

struct NmsWs {
  int* cidx;       // candidate anchor index   [A]
  float* cscore;   // candidate score          [A]
  int* ccls;       // candidate class          [A]
  uint64_t* keys;  // sort keys                [P2]
  float4* obox;    // class-offset xyxy        [M]
  float4* rbox;    // raw xyxy                 [M]
  float* area;     //                          [M]
  uint8_t* removed;//                          [M]
};

static int next_pow2(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

static size_t nms_ws_per_image(int A, int max_nms) {
  const size_t M = std::min(A, max_nms);
  const size_t P2 = next_pow2(std::max(A, 1));
  size_t b = 0;
  b += ((size_t(A) * 4 + 15) & ~size_t(15)) * 3;
  b += P2 * 8;
  b += M * 16 * 2;
  b += ((M * 4 + 15) & ~size_t(15));
  b += ((M + 15) & ~size_t(15));
  return b;
}

size_t nms_ws_bytes(int n, int A, int max_nms) { return size_t(n) * nms_ws_per_image(A, max_nms); }

__device__ __forceinline__ int next_pow2_dev(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

__device__ NmsWs carve(char* p, int A, int max_nms) {
  NmsWs w;
  const size_t M = min(A, max_nms);
  int P2 = 1;
  while (P2 < A) P2 <<= 1;
  const size_t a4 = (size_t(A) * 4 + 15) & ~size_t(15);
  w.cidx = reinterpret_cast<int*>(p);
  p += a4;
  w.cscore = reinterpret_cast<float*>(p);
  p += a4;
  w.ccls = reinterpret_cast<int*>(p);
  p += a4;
  w.keys = reinterpret_cast<uint64_t*>(p);
  p += size_t(P2) * 8;
  w.obox = reinterpret_cast<float4*>(p);
  p += M * 16;
  w.rbox = reinterpret_cast<float4*>(p);
  p += M * 16;
  w.area = reinterpret_cast<float*>(p);
  p += (M * 4 + 15) & ~size_t(15);
  w.removed = reinterpret_cast<uint8_t*>(p);
  return w;
}

// block-wide exclusive scan of 0/1 flags (1024 threads = 16 waves)
__device__ int block_scan(int flag, int* wsum, int* total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t m = __ballot(flag);
  const int before = __popcll(m & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))));
  if (lane == 0) wsum[wv] = __popcll(m);
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int i = 0; i < NMS_THREADS / 64; ++i) {
      const int v = wsum[i];
      wsum[i] = acc;
      acc += v;
    }
    *total = acc;
  }
  __syncthreads();
  const int r = wsum[wv] + before;
  return r;
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

__global__ __launch_bounds__(NMS_THREADS) void nms_kernel(const float* pred, int nc, int A, float conf_thres,
                                                          float iou_thres, int max_det, int max_nms, float max_wh,
                                                          char* ws, size_t ws_per_image, float* dets, int64_t* keep,
                                                          int32_t* counts) {
  __shared__ uint64_t lkeys[LDS_SORT_CAP];
  __shared__ int wsum[NMS_THREADS / 64];
  __shared__ int s_total, s_any, s_kept;
  const int n = blockIdx.x;
  const float* P = pred + int64_t(n) * (4 + nc) * A;
  NmsWs w = carve(ws + size_t(n) * ws_per_image, A, max_nms);

  // ---- 1. candidates in anchor order
  int base = 0;
  for (int a0 = 0; a0 < A; a0 += NMS_THREADS) {
    const int a = a0 + threadIdx.x;
    float best = -INFINITY;
    int bj = 0;
    if (a < A) {
      for (int c = 0; c < nc; ++c) {
        const float v = P[int64_t(4 + c) * A + a];
        if (v > best) {
          best = v;
          bj = c;
        }
      }
    }
    const int flag = (a < A) && (best > conf_thres);
    const int pos = block_scan(flag, wsum, &s_total);
    if (flag) {
      w.cidx[base + pos] = a;
      w.cscore[base + pos] = best;
      w.ccls[base + pos] = bj;
    }
    base += s_total;
    __syncthreads();
  }
  const int ncand = base;
  // ---- 2. sort (score desc, candidate position asc)
  const int n2 = next_pow2_dev(ncand);
  uint64_t* keys = n2 <= LDS_SORT_CAP ? lkeys : w.keys;
  __syncthreads();
  for (int i = threadIdx.x; i < n2; i += blockDim.x) {
    uint64_t k = 0;
    if (i < ncand) k = (uint64_t(__float_as_uint(w.cscore[i])) << 32) | uint64_t(0xFFFFFFFFu - uint32_t(i));
    keys[i] = k;
  }
  __syncthreads();
  if (ncand > 1) bitonic_desc(keys, n2);
  const int M = min(ncand, max_nms);
  for (int i = threadIdx.x; i < M; i += blockDim.x) {
    const int pos = int(0xFFFFFFFFu - uint32_t(keys[i] & 0xFFFFFFFFull));
    const int a = w.cidx[pos];
    const float cx = P[a], cy = P[int64_t(1) * A + a];
    const float hw = P[int64_t(2) * A + a] / 2.0f, hh = P[int64_t(3) * A + a] / 2.0f;
    const float x1 = cx - hw, y1 = cy - hh, x2 = cx + hw, y2 = cy + hh;
    const float off = (float)w.ccls[pos] * max_wh;
    const float bx1 = x1 + off, by1 = y1 + off, bx2 = x2 + off, by2 = y2 + off;
    w.rbox[i] = make_float4(x1, y1, x2, y2);
    w.obox[i] = make_float4(bx1, by1, bx2, by2);
    w.area[i] = (bx2 - bx1) * (by2 - by1);
    w.removed[i] = 0;
    keys[i] = (keys[i] & 0xFFFFFFFF00000000ull) | uint64_t(uint32_t(pos));  // keep score, store position
  }
  __syncthreads();
  // ---- 3. greedy
  int kept = 0;
  for (int i = 0; i < M && kept < max_det; ++i) {
    if (w.removed[i]) continue;  // uniform: all threads read the same byte after the last barrier
    if (threadIdx.x == 0) {
      const int pos = int(keys[i] & 0xFFFFFFFFull);
      const float4 r = w.rbox[i];
      float* d = dets + (int64_t(n) * max_det + kept) * 6;
      d[0] = r.x;
      d[1] = r.y;
      d[2] = r.z;
      d[3] = r.w;
      d[4] = w.cscore[pos];
      d[5] = (float)w.ccls[pos];
      keep[int64_t(n) * max_det + kept] = w.cidx[pos];
    }
    ++kept;
    if (kept >= max_det) break;
    const float4 bi = w.obox[i];
    const float ai = w.area[i];
    int any = 0;
    for (int j = i + 1 + threadIdx.x; j < M; j += blockDim.x) {
      if (w.removed[j]) continue;
      const float4 bj = w.obox[j];
      const float ww = fmaxf(fminf(bi.z, bj.z) - fmaxf(bi.x, bj.x), 0.0f);
      const float hh = fmaxf(fminf(bi.w, bj.w) - fmaxf(bi.y, bj.y), 0.0f);
      any |= (ww * hh) != 0.0f;
    }
    any = __syncthreads_or(any);
    if (any) {
      for (int j = i + 1 + threadIdx.x; j < M; j += blockDim.x) {
        if (w.removed[j]) continue;
        const float4 bj = w.obox[j];
        const float ww = fmaxf(fminf(bi.z, bj.z) - fmaxf(bi.x, bj.x), 0.0f);
        const float hh = fmaxf(fminf(bi.w, bj.w) - fmaxf(bi.y, bj.y), 0.0f);
        const float inter = ww * hh;
        const float iou = inter / ((ai + w.area[j]) - inter);
        if (!(iou <= iou_thres)) w.removed[j] = 1;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) counts[n] = kept;
}

int nms(const float* pred, int n, int nc, int A, float conf, float iou, int max_det, int max_nms, float max_wh,
        void* ws, size_t ws_bytes, float* dets, int64_t* keep, int32_t* counts, hipStream_t s) {
  FCE_CHECK(nc >= 1 && A >= 0 && max_det >= 1 && max_nms >= 1, "nms: bad sizes");
  FCE_CHECK(conf >= 0.f && conf <= 1.f && iou >= 0.f && iou <= 1.f, "nms: thresholds must be in [0, 1]");
  if (n == 0) return FCE_OK;
  const size_t per = nms_ws_per_image(A, max_nms);
  FCE_CHECK(ws && ws_bytes >= per * n, "nms: workspace too small");
  hipLaunchKernelGGL(nms_kernel, dim3(n), dim3(NMS_THREADS), 0, s, pred, nc, A, conf, iou, max_det, max_nms, max_wh,
                     static_cast<char*>(ws), per, dets, keep, counts);
  return launch_status("nms_kernel");
}

}  // namespace fce
