// Shared by the dense conv translation units (conv.hip, conv3x3_big.hip): the kernel argument block,
// the output kinds, the zero line, and the 3x3 halo-tile helpers (image layout, block order, epilogue).
#pragma once
#include "common.h"

namespace fce {

// 16 zero bytes: the source of every out-of-image / padded-K B fragment (static device memory is
// zero-initialised)
static __device__ __attribute__((aligned(16))) _Float16 g_zero_line[8];

struct ConvArgs {
  const _Float16* x;  // input view base (already offset by coff)
  int N, Hs, Ws, xcs;  // source buffer spatial size, channel stride
  int Hin, Win;        // logical input size (Hs << up)
  int up;
  int cin, cout, stride;
  int Ho, Wo, P;  // output spatial, pixels total
  const _Float16* w;
  const float* bias;
  const _Float16* res;  // residual view base or null
  int rcs;
  void* y;  // output view base
  int ycs;
  int act;
  const float* fw;
  int fn, fi;
  int cpt, nchunk, nsteps;  // K-steps of 32
  int nalloc;               // fragments stored per cout tile (see dense_geom)
  unsigned cmagic;          // ceil(2^32 / cpt) for c / cpt = umulhi(c, cmagic)
  int gx, gy;               // logical grid: pixel tiles x cout tiles (launched 1-D, see kernel)
  int vec_ok;
  int stg;                  // LDS-tile 1x1 kernels: fp16 output staged through LDS, 16-byte stores
  // fused Detect tail (OUT_DFL / OUT_CLS): pred (N, 4+nc, A) fp32
  float* pred;
  int det_A, det_a0, det_nc, det_hw, det_w;
  float det_stride;
  unsigned long long* det_best;  // per-anchor best-class key [N][A] (fce_detect_epi::best), or null
  // duplicate store (1x1, plain fp16 output): output channels [duplo, duplo + dupn) are also written to the
  // dense view dup (dupcs channels per pixel), e.g. the half of a C2f cv1 output that the bottleneck reads,
  // so it reads whole cache lines instead of a slice of the concat record; null = off
  _Float16* dup;
  int dupcs, duplo, dupn;
};

enum { OUT_F16 = 0, OUT_F32 = 1, OUT_WSTORE = 2, OUT_ACCUM = 3, OUT_DFL = 4, OUT_CLS = 5 };

// LDS image of a staged tile: pixel (r, c) at position u = r * CI + tile_col(c), its four 16-byte
// channel pieces q at slot q ^ ((u >> 1) & 3).  For stride 2 the even input columns come first, then
// the odd ones, so the 16 lanes of a B fragment (output columns col * 2 + kx) read 16 consecutive
// positions for every tap; with the XOR every ds_read_b128 lane group then meets 16 distinct 16-byte
// slots of the bank row (was 2-way at stride 1 and 4-way at stride 2).
template <int S, int CI>
__device__ __forceinline__ int tile_col(int c) {
  if (S == 1) return c;
  return (c & 1) ? (CI + 1) / 2 + (c >> 1) : (c >> 1);
}

// XCD-aware block order of the 3x3 tile kernels: the grid is 1-D (tiles x cout groups); block b runs on
// XCD b % 8, so each XCD gets a contiguous range of logical blocks, cout groups innermost: the blocks that
// stage the same input tile, and the neighbouring tiles that share its halo rows, hit one L2.
__device__ __forceinline__ void tile_block(int gy, int& tile, int& cog) {
  const int total = int(gridDim.x), b = int(blockIdx.x), per = total >> 3, body = per << 3;
  const int L = b < body ? (b & 7) * per + (b >> 3) : b;
  tile = L / gy;
  cog = L - tile * gy;
}

// Epilogue of the 3x3 tile kernels: acc[r][p] = cout tile cot0 + r x output row oy0 + p (16 columns
// from ox0, lane col); bias, SiLU, optional residual, fp16 NHWC store.
template <int RC, int RP>
__device__ __forceinline__ void tile3_store(const ConvArgs& a, f4 (&acc)[RC][RP], int n, int oy0, int ox0, int cot0,
                                            int col, int grp) {
  const int cotiles = (a.cout + 15) >> 4;
  const int ox = ox0 + col;
  if (ox >= a.Wo) return;
  // residuals of RG cout tiles x RP rows loaded before their first store (see conv_epilogue)
  constexpr int RG = RC * RP <= 8 ? RC : 1;
  const bool vres = a.res && a.vec_ok && a.cout >= 4;
#pragma unroll
  for (int r0 = 0; r0 < RC; r0 += RG) {
    h4 rpre[RG][RP];
    if (vres) {
#pragma unroll
      for (int g = 0; g < RG; ++g) {
        const int co0 = min((cot0 + r0 + g) * 16 + grp * 4, (a.cout - 4) & ~3);
#pragma unroll
        for (int p = 0; p < RP; ++p) {
          const int64_t pix = (int64_t(n) * a.Ho + min(oy0 + p, a.Ho - 1)) * a.Wo + ox;
          rpre[g][p] = *reinterpret_cast<const h4*>(a.res + pix * a.rcs + co0);
        }
      }
      // all of them landed before the first store: hipcc otherwise waits vmcnt(0) at every join of the store loop
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    }
#pragma unroll
  for (int g = 0; g < RG; ++g) {
    const int r = r0 + g;
    const int co0 = (cot0 + r) * 16 + grp * 4;
    if (cot0 + r >= cotiles || co0 >= a.cout) continue;
    float bz[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bz[j] = bias_or0(a.bias, co0 + j, a.cout);
    // landed before the stores: with a load still pending at the joins of the loop below hipcc waits vmcnt(0),
    // i.e. also for the previous row's store, at every row
    __builtin_amdgcn_s_waitcnt(0x0F70);
#pragma unroll
    for (int p = 0; p < RP; ++p) {
      const int oy = oy0 + p;
      if (oy >= a.Ho) continue;
      const int64_t pix = (int64_t(n) * a.Ho + oy) * a.Wo + ox;
      float v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float tt = acc[r][p][j] + bz[j];
        v[j] = a.act ? silu(tt) : tt;
      }
      _Float16* yo = static_cast<_Float16*>(a.y) + pix * a.ycs + co0;
      const bool vec = a.vec_ok && co0 + 3 < a.cout;
      if (a.res) {
        if (vec) {
          const h4 rv = rpre[g][p];
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = fpin(v[j] + (float)rv[j]);
        } else {
          const _Float16* ro = a.res + pix * a.rcs + co0;
          for (int j = 0; j < 4; ++j)
            if (co0 + j < a.cout) v[j] = fpin(v[j] + (float)ro[j]);
        }
      }
      if (vec) {
        *reinterpret_cast<h4*>(yo) = h4{(_Float16)fpin(v[0]), (_Float16)fpin(v[1]), (_Float16)fpin(v[2]), (_Float16)fpin(v[3])};
      } else {
        for (int j = 0; j < 4; ++j)
          if (co0 + j < a.cout) yo[j] = (_Float16)fpin(v[j]);
      }
    }
  }
  }
}

// The same epilogue split in two for the persistent 3x3 ring (one cout tile per wave): tile3_pre loads the
// residuals and biases of the wave's tile (clamped, unconditional) BEFORE the next tile's staging loads are issued,
// so tile3_post needs no vmcnt(0): vmcnt retires in issue order, and a wait for a residual issued after the
// prefetch waited for the whole prefetch (the ring's look-ahead was lost at every epilogue).
template <int RP>
struct Tile3Pre {
  h4 r[RP];
  float bz[4];
};

template <int RP>
__device__ __forceinline__ void tile3_pre(const ConvArgs& a, int n, int oy0, int ox0, int cot0, int grp, int col,
                                          Tile3Pre<RP>& pre) {
  const int co0 = min(cot0 * 16 + grp * 4, (a.cout - 4) & ~3);
  const int ox = min(ox0 + col, a.Wo - 1);
  if (a.res && a.vec_ok && a.cout >= 4) {
#pragma unroll
    for (int p = 0; p < RP; ++p) {
      const int64_t pix = (int64_t(n) * a.Ho + min(oy0 + p, a.Ho - 1)) * a.Wo + ox;
      pre.r[p] = *reinterpret_cast<const h4*>(a.res + pix * a.rcs + co0);
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) pre.bz[j] = bias_or0(a.bias, cot0 * 16 + grp * 4 + j, a.cout);
}

template <int RP>
__device__ __forceinline__ void tile3_post(const ConvArgs& a, f4 (&acc)[RP], const Tile3Pre<RP>& pre, int n, int oy0,
                                           int ox0, int cot0, int col, int grp) {
  const int ox = ox0 + col;
  const int co0 = cot0 * 16 + grp * 4;
  if (ox >= a.Wo || cot0 >= ((a.cout + 15) >> 4) || co0 >= a.cout) return;
  const bool vec = a.vec_ok && co0 + 3 < a.cout;
#pragma unroll
  for (int p = 0; p < RP; ++p) {
    const int oy = oy0 + p;
    if (oy >= a.Ho) continue;
    const int64_t pix = (int64_t(n) * a.Ho + oy) * a.Wo + ox;
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float tt = acc[p][j] + pre.bz[j];
      v[j] = a.act ? silu(tt) : tt;
    }
    _Float16* yo = static_cast<_Float16*>(a.y) + pix * a.ycs + co0;
    if (a.res) {
      if (vec && a.cout >= 4) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = fpin(v[j] + (float)pre.r[p][j]);
      } else {
        const _Float16* ro = a.res + pix * a.rcs + co0;
        for (int j = 0; j < 4; ++j)
          if (co0 + j < a.cout) v[j] = fpin(v[j] + (float)ro[j]);
      }
    }
    if (vec) {
      *reinterpret_cast<h4*>(yo) = h4{(_Float16)fpin(v[0]), (_Float16)fpin(v[1]), (_Float16)fpin(v[2]), (_Float16)fpin(v[3])};
    } else {
      for (int j = 0; j < 4; ++j)
        if (co0 + j < a.cout) yo[j] = (_Float16)fpin(v[j]);
    }
  }
}

// Epilogue of the dense MFMA kernels: acc[r][p] = 16 couts (cout tile cot0 + r) x 16 pixels
// (pix_base + 16 p ..) of this wave; lane = (col = pixel, grp = 4-cout group).  Bias, SiLU, residual,
// BiFPN weighted store / accumulate, or the fused Detect DFL / cls-sigmoid tails.
template <int RC, int RP, int OUT>
__device__ __forceinline__ void conv_epilogue(const ConvArgs& a, f4 (&acc)[RC][RP], int pix_base, int cot0, int col,
                                              int grp) {
  const int cotiles = (a.cout + 15) >> 4;
  if (OUT == OUT_DFL) {
    // Detect box branch (head.py:161-162, block.py:76-79, tal.py:367-376): the 4 x 16 logits of a
    // pixel live in tiles r = side, lanes {p, p+16, p+32, p+48} x 4 registers -> softmax expectation
    // with two xor-shuffles, then xywh * stride into pred rows 0..3 (fp32 throughout).
    float bz[4][4];  // loaded once, not per pixel
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < 4; ++j) bz[r][j] = a.bias[r * 16 + grp * 4 + j];
#pragma unroll
    for (int p = 0; p < RP; ++p) {
      float dist[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v[4], mx = -INFINITY;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[j] = acc[r < RC ? r : 0][p][j] + bz[r][j];
          mx = fmaxf(mx, v[j]);
        }
        mx = fmaxf(mx, __shfl_xor(mx, 16));
        mx = fmaxf(mx, __shfl_xor(mx, 32));
        float den = 0.f, num = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float e = __expf(v[j] - mx);  // v_exp_f32 (as detect_decode)
          den += e;
          num = __fadd_rn(num, __fmul_rn(e, (float)(grp * 4 + j)));  // no FMA: match detect_decode
        }
        den += __shfl_xor(den, 16);
        den += __shfl_xor(den, 32);
        num += __shfl_xor(num, 16);
        num += __shfl_xor(num, 32);
        dist[r] = num / den;
      }
      const int pix = pix_base + p * 16 + col;
      if (grp == 0 && pix < a.P) {
        const int n = pix / a.det_hw, q = pix - n * a.det_hw;
        const float ax = (float)(q % a.det_w) + 0.5f, ay = (float)(q / a.det_w) + 0.5f;
        const float x1 = ax - dist[0], y1 = ay - dist[1], x2 = ax + dist[2], y2 = ay + dist[3];
        float* o = a.pred + int64_t(n) * (4 + a.det_nc) * a.det_A + a.det_a0 + q;
        if (a.det_best) a.det_best[int64_t(n) * a.det_A + a.det_a0 + q] = 0ull;  // the cls epilogue maxes into it
        o[0] = (x1 + x2) / 2.0f * a.det_stride;
        o[a.det_A] = (y1 + y2) / 2.0f * a.det_stride;
        o[int64_t(2) * a.det_A] = (x2 - x1) * a.det_stride;
        o[int64_t(3) * a.det_A] = (y2 - y1) * a.det_stride;
      }
    }
    return;
  }
  if (OUT == OUT_CLS) {  // Detect cls branch: sigmoid(logit) into pred rows 4..
    // with det_best: the pixel's best class over this wave's couts (first maximum, like torch.max in
    // utils/nms.py) as one key = score bits << 32 | ~class (scores >= 0: integer order = float order;
    // ties -> the lower class), merged over the 4 cout groups by xor-shuffles, one atomic max per pixel.
    // The biases are loaded once per cout tile and the pixel's pred column once per pixel: loaded per element
    // (as before) every score waited for its own bias load, and the epilogue was the kernel's bound.
    unsigned long long bk[RP];
    float* orow[RP];  // pred[n][4][a0 + q] of this lane's pixels (nullptr: past the end)
#pragma unroll
    for (int p = 0; p < RP; ++p) {
      bk[p] = 0ull;
      const int pix = pix_base + p * 16 + col;
      const int n = pix / a.det_hw, q = pix - n * a.det_hw;
      orow[p] = pix < a.P ? a.pred + (int64_t(n) * (4 + a.det_nc) + 4) * a.det_A + a.det_a0 + q : nullptr;
    }
    // every bias of the wave's couts loaded (unconditionally: clamped) and landed before the first score store:
    // a load issued after a store, or pending at a join, is waited for with vmcnt(0), i.e. with every store
    float bzr[RC][4];
#pragma unroll
    for (int r = 0; r < RC; ++r)
#pragma unroll
      for (int j = 0; j < 4; ++j) bzr[r][j] = a.bias[min((cot0 + r) * 16 + grp * 4 + j, a.cout - 1)];
    __builtin_amdgcn_s_waitcnt(0x0F70);
#pragma unroll
    for (int r = 0; r < RC; ++r) {
      const int co0 = (cot0 + r) * 16 + grp * 4;
      const float* bz = bzr[r];
      const int64_t rofs = int64_t(co0) * a.det_A;
      const int nv = min(4, a.cout - co0);  // valid couts of this lane group (<= 0: none)
#pragma unroll
      for (int p = 0; p < RP; ++p) {
        if (!orow[p]) continue;
        float* o = orow[p] + rofs;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (j < nv) {
            const float sc = sigmoidf_(acc[r][p][j] + bz[j]);
            o[int64_t(j) * a.det_A] = sc;
            const unsigned long long key =
                (uint64_t(__float_as_uint(sc)) << 32) | uint64_t(0xFFFFFFFFu - uint32_t(co0 + j));
            bk[p] = key > bk[p] ? key : bk[p];
          }
      }
    }
    if (a.det_best) {
#pragma unroll
      for (int p = 0; p < RP; ++p) {
        unsigned long long k = bk[p];
        const unsigned long long k16 = __shfl_xor(k, 16);
        k = k16 > k ? k16 : k;
        const unsigned long long k32 = __shfl_xor(k, 32);
        k = k32 > k ? k32 : k;
        const int pix = pix_base + p * 16 + col;
        if (grp == 0 && pix < a.P && k) {
          const int n = pix / a.det_hw, q = pix - n * a.det_hw;
          atomicMax(a.det_best + int64_t(n) * a.det_A + a.det_a0 + q, k);
        }
      }
    }
    return;
  }
  float alpha = 1.f;
  if (OUT == OUT_WSTORE || OUT == OUT_ACCUM) alpha = fusion_alpha(a.fw, a.fn, a.fi);
  // The vector path's residual (and the ACCUM target) of RG cout tiles x RP pixels are loaded before the first of
  // their stores: a load issued after a store is waited for together with that store (CDNA4 vmcnt counts stores),
  // which serialised every (tile, pixel) of the epilogue on a store round trip.  Clamped addresses: the loads are
  // unconditional inside one uniform branch; lanes past the edge use the scalar path below, as before.
  constexpr int RG = RC * RP <= 8 ? RC : 1;
  const bool vres = a.res && a.vec_ok && a.cout >= 4, vacc = OUT == OUT_ACCUM && a.vec_ok && a.cout >= 4;
#pragma unroll
  for (int r0 = 0; r0 < RC; r0 += RG) {
    h4 rpre[RG][RP], apre[RG][RP];
    if (OUT != OUT_F32 && (vres || vacc)) {
#pragma unroll
      for (int g = 0; g < RG; ++g) {
        const int co0 = min((cot0 + r0 + g) * 16 + grp * 4, (a.cout - 4) & ~3);  // 8-byte aligned, in range
#pragma unroll
        for (int p = 0; p < RP; ++p) {
          const int pix = min(pix_base + p * 16 + col, a.P - 1);
          if (vres) rpre[g][p] = *reinterpret_cast<const h4*>(a.res + int64_t(pix) * a.rcs + co0);
          if (vacc) apre[g][p] = *reinterpret_cast<const h4*>(static_cast<const _Float16*>(a.y) + int64_t(pix) * a.ycs + co0);
        }
      }
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): all landed before the first store (tile3_store)
    }
#pragma unroll
  for (int g = 0; g < RG; ++g) {
    const int r = r0 + g;
    const int co0 = (cot0 + r) * 16 + grp * 4;
    if (cot0 + r >= cotiles || co0 >= a.cout) continue;
    float bz[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bz[j] = bias_or0(a.bias, co0 + j, a.cout);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) before the stores (tile3_store)
#pragma unroll
    for (int p = 0; p < RP; ++p) {
      const int pix = pix_base + p * 16 + col;
      if (pix >= a.P) continue;
      float v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float t = acc[r][p][j] + bz[j];
        v[j] = a.act ? silu(t) : t;
      }
      if (OUT == OUT_F32) {
        float* yo = static_cast<float*>(a.y) + int64_t(pix) * a.ycs + co0;
        if (a.vec_ok && co0 + 3 < a.cout) {
          *reinterpret_cast<f4*>(yo) = f4{v[0], v[1], v[2], v[3]};
        } else {
          for (int j = 0; j < 4; ++j)
            if (co0 + j < a.cout) yo[j] = v[j];
        }
        continue;
      }
      _Float16* yo = static_cast<_Float16*>(a.y) + int64_t(pix) * a.ycs + co0;
      const bool vec = a.vec_ok && co0 + 3 < a.cout;
      if (a.res) {
        if (vec) {
          const h4 rv = rpre[g][p];
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = fpin(v[j] + (float)rv[j]);
        } else {
          const _Float16* ro = a.res + int64_t(pix) * a.rcs + co0;
          for (int j = 0; j < 4; ++j)
            if (co0 + j < a.cout) v[j] = fpin(v[j] + (float)ro[j]);
        }
      }
      if (OUT == OUT_WSTORE) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = fpin(v[j] * alpha);
      }
      if (vec) {
        if (OUT == OUT_ACCUM) {
          const h4 pv4 = apre[g][p];
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = fpin((float)pv4[j] + fpin(alpha * v[j]));
        }
        const h4 hv = h4{(_Float16)fpin(v[0]), (_Float16)fpin(v[1]), (_Float16)fpin(v[2]), (_Float16)fpin(v[3])};
        *reinterpret_cast<h4*>(yo) = hv;
        if (OUT == OUT_F16 && a.dup && co0 >= a.duplo && co0 < a.duplo + a.dupn)  // dupn % 8 == 0 (host)
          *reinterpret_cast<h4*>(a.dup + int64_t(pix) * a.dupcs + (co0 - a.duplo)) = hv;
      } else {
        for (int j = 0; j < 4; ++j) {
          if (co0 + j >= a.cout) continue;
          float t = v[j];
          if (OUT == OUT_ACCUM) t = fpin((float)yo[j] + fpin(alpha * t));
          yo[j] = (_Float16)fpin(t);
          if (OUT == OUT_F16 && a.dup && co0 + j >= a.duplo && co0 + j < a.duplo + a.dupn)
            a.dup[int64_t(pix) * a.dupcs + (co0 + j - a.duplo)] = (_Float16)fpin(t);
        }
      }
    }
  }
  }
}

// NHWC source offset of output pixel `pix` of a 1x1 stride-1 conv (through the nearest x2^up upsampling)
__device__ __forceinline__ int64_t conv1x1_src(const ConvArgs& a, int pix) {
  if (!a.up) return int64_t(pix) * a.xcs;
  const int hw = a.Ho * a.Wo;
  const int n = pix / hw, r = pix - n * hw;
  const int oy = r / a.Wo, ox = r - oy * a.Wo;
  return nhwc_off(n, oy >> a.up, ox >> a.up, a.Hs, a.Ws, a.xcs);
}

// Big-tile LDS-DMA 3x3 configurations (conv3x3_big.hip), coded 0x800 | wm << 4 | (ab - 2) << 12: wm waves along
// the couts, ab weight-stage buffers, 4 waves per block (8-wave blocks were measured and dropped);
// stride 2 needs wm 2 (LDS)
static constexpr bool big3_ok(int s, int wm, int ab, int nw = 4) {
  return nw == 4 && (ab == 2 || ab == 3) && (s == 1 ? (wm == 1 || wm == 2) : wm == 2);
}
int launch_big3(const ConvArgs& a, int wm, int ab, int nw, int stride, int n, hipStream_t s);
// Persistent 3x3 ring fed by LDS-DMA (conv3x3_dring.hip), coded 0xD00 | rp << 4 | (cpw - 1) << 3 | (sub - 1) << 2 |
// (nbuf - 2): cin 32 / 64 / 128, cpw cout tiles per wave (1: 4 waves along the couts; 2: 2 x 2 waves), sub x rp rows x
// 16 columns per wave and tile (sub sub-tiles of rp rows, one after the other, per barrier), nbuf LDS tile buffers
// (nbuf - 1 tiles of input in flight)
template <int S, int RP, int NCH, int WRW = 1>
struct Dring3Geom {
  static constexpr int TW = 16, TH = WRW * RP;  // WRW waves along the rows (2 when each wave owns 2 cout tiles)
  static constexpr int RI = (TH - 1) * S + 3, CI = (TW - 1) * S + 3;
  static constexpr int NQ = 4 * NCH, NE = RI * CI * NQ;
  static constexpr int NINS = (NE + 63) / 64;  // 1 KiB copy instructions per tile
  static constexpr int DPW = (NINS + 3) / 4;   // per wave (4 waves), padded
  static constexpr int BUF = DPW * 4 * 64;     // pieces per tile buffer
};

static constexpr bool dring3_fits(int s, int rp, int nch, int nbuf, int cpw = 1, int sub = 1) {
  return size_t(nbuf) * ((((((cpw * rp * sub - 1) * s + 3) * (15 * s + 3) * 4 * nch + 63) / 64 + 3) / 4) * 4 * 64) * 16 <=
             80 * 1024 &&       // two blocks per CU
         // two cout tiles of 64-channel A fragments: 1- and 2-row tiles with three buffers only (253 VGPRs at 2 rows;
         // more rows or buffers spill at two waves per SIMD)
         (cpw == 1 || nch == 1 || (nch == 2 && rp <= 2 && nbuf == 3 && sub == 1)) &&
         (rp < 8 || (nch == 1 && nbuf == 3)) &&  // 8-row tiles of 64-channel fragments spill too (or with four buffers)
         // 128 channels (36 A fragments in registers): stride-2 one-row tiles only; the two-row stride-1 ones spilled
         // (31.2 against 24.3 us, r06al)
         (nch < 4 || (s == 2 && rp == 1)) &&
         (sub == 1 || (sub == 2 && rp * sub <= 8));  // sub-tiles: 8 rows of held residuals at most
}
// the candidates offered: two buffers or one-row tiles only for the 128-channel tiles, which need them to fit (at 32 /
// 64 channels the two-buffer ones are the big stride-2 tiles, which spill), and for the 64-channel two-cout-tile ones
// (0xd19: 2 x 1 rows per block; 0xd29 25.6 against 25.9-26.3 us for 0xd41 at 64 -> 64 80 x 80, its MFMA phase 1.97k
// against 2.16k clocks per tile at half the LDS reads, r06av); two sub-tiles only for the 32-channel
// stride-1 convs, the one place they measured ahead (48.4 against 49.9 us at 160 x 160; 64 -> 64 at 80 x 80 and the
// stride-2 ones slower, the 64-channel 8-row tiles spilling: profiles/r06_dring_probe.txt)
static constexpr bool dring3_offer(int s, int rp, int nch, int nbuf, int cpw = 1, int sub = 1) {
  return dring3_fits(s, rp, nch, nbuf, cpw, sub) && (nch == 4 || (nbuf > 2 && (rp > 1 || (cpw == 2 && nch == 2)))) &&
         (nbuf > 2 || !dring3_fits(s, rp, nch, 3, cpw, sub)) && (sub == 1 || (nbuf > 2 && rp >= 2 && nch == 1 && s == 1));
}
int launch_dring3(const ConvArgs& a, int rp, int nbuf, int cpw, int sub, int stride, hipStream_t s);
// Wide-tile 3x3 (conv3x3_wide.hip), coded 0xA00 | log2(cw) << 4: 64 cw couts x 16 (4 / cw) rows per block
bool wide3_ok(int stride, int cw);
int launch_wide3(const ConvArgs& a, int cw, int stride, int n, hipStream_t s);
// Big-tile implicit GEMM (conv_big.hip): 16 wr wc couts x 64 (nw / wc) pixels per nw-wave block (nw 8: one block per
// CU; nw 4: two; wr = cout tiles per wave, 8, or 4 with nw 4); 1x1 coded 0xB00 | log2(wc) << 4 | (nw == 4) << 6 |
// (wr == 4) << 7, 3x3 (cin % 32 == 0, stride 1 / 2, plain fp16 output) 0xC00 | the same bits
bool big1_ok(int wc);
bool big1_split_ok(int wc, int nw, int wr);
int launch_big1(const ConvArgs& a, int out_kind, int wc, int nw, int wr, bool split, hipStream_t s);  // split: | 0x20
int launch_big3g(const ConvArgs& a, int wc, int nw, int wr, int stride, bool split, hipStream_t s);

}  // namespace fce
