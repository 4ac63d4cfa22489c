// Non-maximum suppression on the device (reference ultralytics/utils/nms.py:13-166 with the predict
// defaults multi_label=False, agnostic=False, classes=None; TorchNMS.nms :239-296; xywh2xyxy
// utils/ops.py:224-240).  One 1024-thread workgroup per image:
//   1. candidates: best class per anchor (first maximum), keep conf > conf_thres, compacted in anchor
//      order with a block prefix sum;
//   2. sort by (score desc, anchor asc): bitonic sort of 64-bit keys (LDS up to 8192 candidates,
//      otherwise in the workspace); truncate to max_nms;
//   3. class-offset xyxy boxes (cls * max_wh) and areas, in LDS up to 4096 candidates;
//   4. greedy suppression in sorted order, reproducing the reference's fp32 arithmetic (no FMA
//      contraction in this file) and stopping at max_det.  Fast path (all areas > 0, so no IoU is
//      NaN and the reference's "no overlap -> keep all" early exit changes nothing): tiles of the
//      next 64 surviving candidates are resolved sequentially inside one wave (ballots + shuffles),
//      then every later candidate is tested against the tile's kept boxes in parallel — one
//      barrier round per tile instead of two per kept box.  Degenerate boxes take the literal
//      per-box loop (with the early exit) instead.
#include "common.h"

#pragma clang fp contract(off)

namespace fce {

static constexpr int NMS_THREADS = 1024;
static constexpr int LDS_SORT_CAP = 8192;
static constexpr int LDS_BOX_CAP = 4096;
static constexpr int REMOVED_CAP = 32768;
static constexpr int TILE = 64;

struct NmsWs {
  float* aconf;     // per-anchor best score    [A]   (nms_best_class_kernel)
  int* acls;        // per-anchor best class    [A]
  int* cidx;        // candidate anchor index   [A]
  float* cscore;    // candidate score          [A]
  int* ccls;        // candidate class          [A]
  uint64_t* keys;   // sort keys                [P2]
  float4* obox;     // class-offset xyxy        [M]
  float* area;      //                          [M]
  int* spos;        // sorted -> candidate pos  [M]
};

static int next_pow2(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

static size_t nms_ws_per_image(int A, int max_nms) {
  const size_t M = std::min(A, max_nms);
  const size_t P2 = next_pow2(std::max(A, 1));
  auto al = [](size_t b) { return (b + 15) & ~size_t(15); };
  return al(size_t(A) * 4) * 5 + P2 * 8 + M * 16 + al(M * 4) * 2;
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
  const int P2 = next_pow2_dev(max(A, 1));
  auto al = [](size_t b) { return (b + 15) & ~size_t(15); };
  w.aconf = reinterpret_cast<float*>(p);
  p += al(size_t(A) * 4);
  w.acls = reinterpret_cast<int*>(p);
  p += al(size_t(A) * 4);
  w.cidx = reinterpret_cast<int*>(p);
  p += al(size_t(A) * 4);
  w.cscore = reinterpret_cast<float*>(p);
  p += al(size_t(A) * 4);
  w.ccls = reinterpret_cast<int*>(p);
  p += al(size_t(A) * 4);
  w.keys = reinterpret_cast<uint64_t*>(p);
  p += size_t(P2) * 8;
  w.obox = reinterpret_cast<float4*>(p);
  p += M * 16;
  w.area = reinterpret_cast<float*>(p);
  p += al(M * 4);
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
    for (int i = 0; i < NMS_THREADS / 64; ++i) {
      const int v = wsum[i];
      wsum[i] = acc;
      acc += v;
    }
    *total = acc;
  }
  __syncthreads();
  return wsum[wv] + before;
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

// reference IoU (nms.py:276-291) in fp32, same operation order
__device__ __forceinline__ float iou_ref(float4 bi, float ai, float4 bj, float aj, float* inter_out) {
  const float ww = fmaxf(fminf(bi.z, bj.z) - fmaxf(bi.x, bj.x), 0.0f);
  const float hh = fmaxf(fminf(bi.w, bj.w) - fmaxf(bi.y, bj.y), 0.0f);
  const float inter = ww * hh;
  *inter_out = inter;
  return inter / ((ai + aj) - inter);
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
  NmsWs w = carve(ws + size_t(n) * ws_per_image, A, max_nms);
  w.aconf[a] = best;
  w.acls[a] = bj;
}

__global__ __launch_bounds__(NMS_THREADS) void nms_kernel(const float* pred, int nc, int A, float conf_thres,
                                                          float iou_thres, int max_det, int max_nms, float max_wh,
                                                          char* ws, size_t ws_per_image, float* dets, int64_t* keep,
                                                          int32_t* counts) {
  __shared__ __attribute__((aligned(16))) uint64_t lkeys[LDS_SORT_CAP];  // sort keys, then float4 boxes
  __shared__ float larea[LDS_BOX_CAP];
  __shared__ int lspos[LDS_BOX_CAP];
  __shared__ uint8_t lremoved[REMOVED_CAP];
  __shared__ int wsum[NMS_THREADS / 64];
  __shared__ int tile_idx[TILE];
  __shared__ float4 tile_box[TILE];
  __shared__ float tile_area[TILE];
  __shared__ uint64_t tile_sup[TILE];
  __shared__ float4 kept_box[TILE];
  __shared__ float kept_area[TILE];
  __shared__ int s_total, s_tile_n, s_next, s_nk, s_done, s_kept;

  const int n = blockIdx.x;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const float* P = pred + int64_t(n) * (4 + nc) * A;
  NmsWs w = carve(ws + size_t(n) * ws_per_image, A, max_nms);

  // ---- 1. candidates in anchor order (best class per anchor from nms_best_class_kernel)
  int base = 0;
  for (int a0 = 0; a0 < A; a0 += NMS_THREADS) {
    const int a = a0 + threadIdx.x;
    float best = -INFINITY;
    int bj = 0;
    if (a < A) {
      best = w.aconf[a];
      bj = w.acls[a];
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
  const int n2 = next_pow2_dev(max(ncand, 1));
  uint64_t* keys = n2 <= LDS_SORT_CAP ? lkeys : w.keys;
  for (int i = threadIdx.x; i < n2; i += blockDim.x) {
    uint64_t k = 0;
    if (i < ncand) k = (uint64_t(__float_as_uint(w.cscore[i])) << 32) | uint64_t(0xFFFFFFFFu - uint32_t(i));
    keys[i] = k;
  }
  __syncthreads();
  if (ncand > 1) bitonic_desc(keys, n2);
  const int M = min(ncand, max_nms);
  const bool lds_box = M <= LDS_BOX_CAP;
  int* spos = lds_box ? lspos : w.spos;
  float4* obox = lds_box ? reinterpret_cast<float4*>(lkeys) : w.obox;
  float* area = lds_box ? larea : w.area;
  for (int i = threadIdx.x; i < M; i += blockDim.x) spos[i] = int(0xFFFFFFFFu - uint32_t(keys[i] & 0xFFFFFFFFull));
  __syncthreads();  // keys are dead from here (the LDS key space becomes the box array)

  // ---- 3. class-offset boxes
  int degenerate = 0;
  for (int i = threadIdx.x; i < M; i += blockDim.x) {
    const int pos = spos[i];
    const int a = w.cidx[pos];
    const float cx = P[a], cy = P[int64_t(1) * A + a];
    const float hw = P[int64_t(2) * A + a] / 2.0f, hh = P[int64_t(3) * A + a] / 2.0f;
    const float off = (float)w.ccls[pos] * max_wh;
    const float bx1 = (cx - hw) + off, by1 = (cy - hh) + off, bx2 = (cx + hw) + off, by2 = (cy + hh) + off;
    obox[i] = make_float4(bx1, by1, bx2, by2);
    const float ar = (bx2 - bx1) * (by2 - by1);
    area[i] = ar;
    lremoved[i] = 0;
    degenerate |= !(ar > 0.0f) || !isfinite(ar);
  }
  if (threadIdx.x == 0) s_kept = 0;
  degenerate = __syncthreads_or(degenerate);

  auto emit_det = [&](int i, int slot) {
    const int pos = spos[i];
    const int a = w.cidx[pos];
    const float cx = P[a], cy = P[int64_t(1) * A + a];
    const float hw = P[int64_t(2) * A + a] / 2.0f, hh = P[int64_t(3) * A + a] / 2.0f;
    float* d = dets + (int64_t(n) * max_det + slot) * 6;
    d[0] = cx - hw;
    d[1] = cy - hh;
    d[2] = cx + hw;
    d[3] = cy + hh;
    d[4] = w.cscore[pos];
    d[5] = (float)w.ccls[pos];
    keep[int64_t(n) * max_det + slot] = a;
  };

  if (!degenerate) {
    // ---- 4a. tiled greedy (exact when every area > 0).  Per tile of the next 64 surviving
    // candidates: (i) wave 0 gathers them; (ii) all 16 waves build the tile's suppression rows
    // sup[t] = {u > t : IoU(t, u) > thr} with one ballot each; (iii) wave 0 resolves the greedy
    // order with 64-bit mask operations; (iv) every later candidate is tested against the kept
    // members in parallel.
    int cursor = 0;
    while (true) {
      if (wv == 0) {
        int cnt = 0, c = cursor;
        while (cnt < TILE && c < M) {
          const int j = c + lane;
          const bool alive = j < M && !lremoved[j];
          const uint64_t b = __ballot(alive);
          const int avail = __popcll(b);
          const int take = min(avail, TILE - cnt);
          const int rank = __popcll(b & ((1ull << lane) - 1ull));
          if (alive && rank < take) tile_idx[cnt + rank] = j;
          cnt += take;
          c += 64;
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's tile_idx writes have landed
        __builtin_amdgcn_wave_barrier();
        if (lane < cnt) {
          const int my = tile_idx[lane];
          tile_box[lane] = obox[my];
          tile_area[lane] = area[my];
        }
        if (lane == 0) {
          s_tile_n = cnt;
          s_next = cnt == TILE ? tile_idx[TILE - 1] + 1 : M;  // resume right after the last member
        }
      }
      __syncthreads();
      const int cnt = s_tile_n;
      if (cnt == 0) break;
      for (int t = wv; t < cnt; t += NMS_THREADS / 64) {
        bool sup = false;
        if (lane > t && lane < cnt) {
          float inter;
          sup = iou_ref(tile_box[t], tile_area[t], tile_box[lane], tile_area[lane], &inter) > iou_thres;
        }
        const uint64_t b = __ballot(sup);
        if (lane == 0) tile_sup[t] = b;
      }
      __syncthreads();
      if (wv == 0) {
        const int kept0 = s_kept;
        const uint64_t mysup = lane < cnt ? tile_sup[lane] : 0ull;
        const uint32_t sup_lo = uint32_t(mysup), sup_hi = uint32_t(mysup >> 32);
        uint64_t removed = 0, keptm = 0;
        int nk = 0;
        bool done = false;
        for (int t = 0; t < cnt; ++t) {  // wave-uniform: SALU bit ops + v_readlane
          if ((removed >> t) & 1ull) continue;
          keptm |= 1ull << t;
          ++nk;
          if (kept0 + nk >= max_det) {
            done = true;
            break;
          }
          removed |= uint64_t(__builtin_amdgcn_readlane(sup_lo, t)) |
                     (uint64_t(__builtin_amdgcn_readlane(sup_hi, t)) << 32);
        }
        if ((keptm >> lane) & 1ull) {
          const int r = __popcll(keptm & ((1ull << lane) - 1ull));
          kept_box[r] = tile_box[lane];
          kept_area[r] = tile_area[lane];
          emit_det(tile_idx[lane], kept0 + r);
        }
        if (lane == 0) {
          s_nk = nk;
          s_kept = kept0 + nk;
          s_done = done || s_next >= M;
        }
      }
      __syncthreads();
      if (s_done) break;
      // suppress everything after the tile against the tile's kept boxes
      const int nk = s_nk, start = s_next;
      for (int j = start + threadIdx.x; j < M; j += blockDim.x) {
        if (lremoved[j]) continue;
        const float4 bj = obox[j];
        const float aj = area[j];
        for (int k = 0; k < nk; ++k) {
          float inter;
          if (iou_ref(kept_box[k], kept_area[k], bj, aj, &inter) > iou_thres) {
            lremoved[j] = 1;
            break;
          }
        }
      }
      cursor = start;
      __syncthreads();
    }
  } else {
    // ---- 4b. literal per-box greedy (TorchNMS.nms with its early exit) for degenerate boxes
    int kept = 0;
    for (int i = 0; i < M && kept < max_det; ++i) {
      if (lremoved[i]) continue;
      if (threadIdx.x == 0) emit_det(i, kept);
      ++kept;
      if (kept >= max_det) break;
      const float4 bi = obox[i];
      const float ai = area[i];
      int any = 0;
      for (int j = i + 1 + threadIdx.x; j < M; j += blockDim.x) {
        if (lremoved[j]) continue;
        float inter;
        iou_ref(bi, ai, obox[j], area[j], &inter);
        any |= inter != 0.0f;
      }
      any = __syncthreads_or(any);
      if (any) {
        for (int j = i + 1 + threadIdx.x; j < M; j += blockDim.x) {
          if (lremoved[j]) continue;
          float inter;
          const float iou = iou_ref(bi, ai, obox[j], area[j], &inter);
          if (!(iou <= iou_thres)) lremoved[j] = 1;
        }
      }
      __syncthreads();
    }
    if (threadIdx.x == 0) s_kept = kept;
  }
  __syncthreads();
  if (threadIdx.x == 0) counts[n] = s_kept;
}

int nms(const float* pred, int n, int nc, int A, float conf, float iou, int max_det, int max_nms, float max_wh,
        void* ws, size_t ws_bytes, float* dets, int64_t* keep, int32_t* counts, hipStream_t s) {
  FCE_CHECK(nc >= 1 && A >= 0 && max_det >= 1 && max_nms >= 1, "nms: bad sizes");
  FCE_CHECK(max_nms <= REMOVED_CAP, "nms: max_nms > 32768 unsupported");
  FCE_CHECK(conf >= 0.f && conf <= 1.f && iou >= 0.f && iou <= 1.f, "nms: thresholds must be in [0, 1]");
  if (n == 0) return FCE_OK;
  const size_t per = nms_ws_per_image(A, max_nms);
  FCE_CHECK(ws && ws_bytes >= per * n, "nms: workspace too small");
  if (A > 0)
    hipLaunchKernelGGL(nms_best_class_kernel, dim3((A + 255) / 256, n), dim3(256), 0, s, pred, nc, A, max_nms,
                       static_cast<char*>(ws), per);
  hipLaunchKernelGGL(nms_kernel, dim3(n), dim3(NMS_THREADS), 0, s, pred, nc, A, conf, iou, max_det, max_nms, max_wh,
                     static_cast<char*>(ws), per, dets, keep, counts);
  return launch_status("nms_kernel");
}

}  // namespace fce
