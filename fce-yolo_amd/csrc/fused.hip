// Fused C3k2 block (reference ultralytics/nn/modules/block.py C2f.forward :303-307 with C3k2's
// Bottleneck branch :1064-1084, Bottleneck.forward :474-476): for c3k = False and one repeat,
//
//   t = SiLU(cv1(x))            1x1, cin -> 2c          t = [a | b]
//   h = SiLU(m.cv1(b))          3x3, c -> c_mid
//   m = SiLU(m.cv2(h)) + b      3x3, c_mid -> c   (shortcut)
//   y = SiLU(cv2([a | b | m]))  1x1, 3c -> cout
//
// in ONE persistent kernel.  A block owns a contiguous run of TH x TW output tiles and keeps the four
// convs' packed A fragments resident in LDS for its whole life (copied once); per tile
//   stage 1: cv1 over the tile + 2-pixel halo, its B operands (x) loaded straight from HBM into registers
//            while the PREVIOUS tile's stages 2-4 run (one read of x per tile, latency off the critical path),
//   stage 2: m.cv1 over the tile + 1-pixel halo, from the t image in LDS,
//   stage 3: m.cv2 + the residual b over the tile, into the m image in LDS,
//   stage 4: cv2 over [a | b | m] from LDS, y to HBM.
// t / h / m never leave LDS: the block is one read of x and one write of y (the four separate convs move
// x, t twice, h twice, m twice and [a | b | m] through HBM, n32's L2 block alone ~390 MB against ~157 MB).
//
// Bitwise identical to the four unfused convs (conv_mfma_kernel and its variants): every stage walks
// the same K-steps of the same packed A fragments (conv_pack: chunk-major for cin % 32 == 0, else
// tap-major 8-channel chunks c = 4 s + lane / 16) with v_mfma_f32_16x16x32_f16 from zero, the B data
// are the same fp16 values (intermediates rounded to fp16 exactly where the unfused path stores them,
// zeros where it zero-pads), and the epilogue arithmetic is conv_epilogue's (bias, SiLU, residual add,
// fpin before every fp16 conversion).
#include <algorithm>

#include "common.h"

namespace fce {

static __device__ __attribute__((aligned(16))) _Float16 g_c3_zero[8];

struct C3Stage {
  const h8* w;     // packed A fragments in HBM (conv_pack layout: [cout tile][nalloc][64 lanes])
  const float* b;  // bias (BN folded)
  int cout, cotiles, nsteps, nalloc, fast, cpt, taps;
  int wl;  // 16-byte offset of the stage's fragments in LDS: [cout tile][step][64 lanes]
  int bl;  // float offset of the stage's bias in the LDS bias block (cotiles * 16, zero past cout)
};

struct C3k2Args {
  const _Float16* x;
  int xcs;
  _Float16* y;
  int ycs;
  int N, H, W, c;
  C3Stage st[4];
  int TH, TW, tiles_x, tiles_y, ntiles;
  int R2W, R2, R1W, R1, NC;  // cv1 region (tile + 2-pixel halo), m.cv1 region (+ 1 pixel), tile positions
  int sT, sH, sM;            // LDS strides of the t, h, m images in 16-byte units (odd: conflict-free B reads)
  int oT, oH, oM;            // their 16-byte offsets
  int wtotal;                // 16-byte units of resident fragments
  int ob, nbias;             // 16-byte offset of the bias block, its floats
  int diag;                  // FCE_C3K2_DIAG: block 0 prints its per-stage clocks
};

__device__ __forceinline__ h4 c3_h4(const float (&v)[4]) {
  return h4{(_Float16)fpin(v[0]), (_Float16)fpin(v[1]), (_Float16)fpin(v[2]), (_Float16)fpin(v[3])};
}

// The wave's MF 16-position fragments f0, f0 + NW, ... (nf of them valid) x cout tiles [c0, c0 + MCT) of one
// stage, every K-step; A from the stage's LDS fragments, B from bl(i, step) (base[] precomputed by the caller),
// the next step's operands read while this step's MFMAs run.  epi(i, ct, acc) per valid (fragment, tile).
template <int MF, int MCT, typename BL, typename EPI>
__device__ __forceinline__ void c3_mma(const h8* wl, int ns, int cot, int c0, int nf, BL bl, EPI epi) {
  f4 acc[MF][MCT];
#pragma unroll
  for (int i = 0; i < MF; ++i)
#pragma unroll
    for (int ct = 0; ct < MCT; ++ct) acc[i][ct] = f4{0.f, 0.f, 0.f, 0.f};
  h8 av[MCT], bv[MF];
#pragma unroll
  for (int ct = 0; ct < MCT; ++ct)
    if (c0 + ct < cot) av[ct] = wl[((c0 + ct) * ns) * 64];
#pragma unroll
  for (int i = 0; i < MF; ++i)
    if (i < nf) bv[i] = bl(i, 0);
  for (int st = 0; st < ns; ++st) {
    h8 an[MCT], bn[MF];
    const int sn = st + 1 < ns ? st + 1 : st;
#pragma unroll
    for (int ct = 0; ct < MCT; ++ct)
      if (c0 + ct < cot) an[ct] = wl[((c0 + ct) * ns + sn) * 64];
#pragma unroll
    for (int i = 0; i < MF; ++i)
      if (i < nf) bn[i] = bl(i, sn);
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
      for (int ct = 0; ct < MCT; ++ct)
        if (i < nf && c0 + ct < cot) acc[i][ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[ct], bv[i], acc[i][ct], 0, 0, 0);
#pragma unroll
    for (int ct = 0; ct < MCT; ++ct) av[ct] = an[ct];
#pragma unroll
    for (int i = 0; i < MF; ++i) bv[i] = bn[i];
  }
#pragma unroll
  for (int i = 0; i < MF; ++i)
#pragma unroll
    for (int ct = 0; ct < MCT; ++ct)
      if (i < nf && c0 + ct < cot) epi(i, c0 + ct, acc[i][ct]);
}

// SiLU(acc + bias) of lane group grp's 4 couts of tile ct; the bias from the block's LDS copy (a global load
// here would make the epilogue wait for the next tile's x prefetch: vmcnt retires in issue order)
__device__ __forceinline__ void c3_act(const C3Stage& s, const float* bias, int ct, int grp, const f4& acc,
                                       float (&v)[4]) {
  const int co0 = ct * 16 + grp * 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = silu(acc[j] + bias[s.bl + co0 + j]);
}

// decode tile t of the block's run -> image n, output origin (y0, x0)
__device__ __forceinline__ void c3_tile(const C3k2Args& a, int t, int& n, int& y0, int& x0) {
  const int tx = t % a.tiles_x;
  t /= a.tiles_x;
  const int ty = t % a.tiles_y;
  n = t / a.tiles_y;
  y0 = ty * a.TH;
  x0 = tx * a.TW;
}

// stage-1 B operands of tile t: x at the cv1 region's positions (zero line outside the image)
template <int NW, int MF1, int NS1>
__device__ __forceinline__ void c3_load_x(const C3k2Args& a, int t, h8 (&xb)[MF1][NS1]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, col = lane & 15, grp = lane >> 4;
  int n, y0, x0;
  c3_tile(a, t, n, y0, x0);
  const _Float16* zl = g_c3_zero;
#pragma unroll
  for (int i = 0; i < MF1; ++i) {
    const int q = (wave + NW * i) * 16 + col;
    const int r = q / a.R2W, cc = q - r * a.R2W;
    const int iy = y0 - 2 + r, ix = x0 - 2 + cc;
    const bool in = q < a.R2 && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
    const _Float16* src = a.x + (in ? nhwc_off(n, iy, ix, a.H, a.W, a.xcs) + grp * 8 : 0);
#pragma unroll
    for (int s = 0; s < NS1; ++s) xb[i][s] = *reinterpret_cast<const h8*>(in ? src + s * 32 : zl);
  }
}

template <int NW, int MF1, int NS1>
__global__ __launch_bounds__(NW * 64, 2) void c3k2_fused_kernel(C3k2Args a) {
  extern __shared__ __attribute__((aligned(16))) h8 sm[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, col = lane & 15, grp = lane >> 4;
  const int G = gridDim.x, bi = blockIdx.x;
  const int t_begin = int(int64_t(bi) * a.ntiles / G), t_end = int(int64_t(bi + 1) * a.ntiles / G);
  if (t_begin >= t_end) return;  // block-uniform

  h8 xb[MF1][NS1];
  c3_load_x<NW, MF1, NS1>(a, t_begin, xb);
  // the four convs' fragments -> LDS, once per block (batches of 4 loads in flight per thread)
#pragma unroll 1
  for (int s = 0; s < 4; ++s) {
    const C3Stage& S = a.st[s];
    const int nfr = S.cotiles * S.nsteps * 64;
    for (int e0 = int(threadIdx.x); e0 < nfr; e0 += 4 * NW * 64) {
      h8 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = e0 + u * NW * 64;
        const int k = e >> 6, ct = k / S.nsteps, stp = k - ct * S.nsteps;
        if (e < nfr) v[u] = S.w[(size_t(ct) * S.nalloc + stp) * 64 + (e & 63)];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = e0 + u * NW * 64;
        if (e < nfr) sm[S.wl + e] = v[u];
      }
    }
  }
  // biases -> LDS (zero past each conv's cout)
  float* bias = reinterpret_cast<float*>(sm + a.ob);
#pragma unroll 1
  for (int s = 0; s < 4; ++s) {
    const C3Stage& S = a.st[s];
    for (int e = int(threadIdx.x); e < S.cotiles * 16; e += NW * 64) bias[S.bl + e] = e < S.cout ? S.b[e] : 0.f;
  }
  __syncthreads();

  const int c8 = a.c / 8;
  const int nfr1 = (a.R2 + 15) >> 4, nfr2 = (a.R1 + 15) >> 4, nfr4 = (a.NC + 15) >> 4;
  // diagnostics (FCE_C3K2_DIAG=1): block 0, wave 0 sums s_memtime clocks per stage over its tiles and prints them
  uint64_t clk[6] = {0, 0, 0, 0, 0, 0}, tprev = a.diag ? __builtin_amdgcn_s_memtime() : 0;
  auto tick = [&](int k) {
    if (a.diag) {
      const uint64_t tn = __builtin_amdgcn_s_memtime();
      clk[k] += tn - tprev;
      tprev = tn;
    }
  };
  _Float16* T = reinterpret_cast<_Float16*>(sm + a.oT);
  _Float16* Hh = reinterpret_cast<_Float16*>(sm + a.oH);
  _Float16* Mm = reinterpret_cast<_Float16*>(sm + a.oM);
  constexpr int MF = 4, MCT = 4;

  for (int t = t_begin; t < t_end; ++t) {
    int n, y0, x0;
    c3_tile(a, t, n, y0, x0);
    // ---------------- stage 1: t = cv1(x) over the cv1 region (B operands already in registers)
    {
      const C3Stage& S = a.st[0];
      const h8* wl = sm + S.wl + lane;
      const int nf = wave < nfr1 ? min(MF1, (nfr1 - wave + NW - 1) / NW) : 0;
      if (nf > 0) {
        for (int c0 = 0; c0 < S.cotiles; c0 += MCT) {
          f4 acc[MF1][MCT];
#pragma unroll
          for (int i = 0; i < MF1; ++i)
#pragma unroll
            for (int ct = 0; ct < MCT; ++ct) acc[i][ct] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int s = 0; s < NS1; ++s) {
            h8 av[MCT];
#pragma unroll
            for (int ct = 0; ct < MCT; ++ct)
              if (c0 + ct < S.cotiles) av[ct] = wl[((c0 + ct) * NS1 + s) * 64];
#pragma unroll
            for (int i = 0; i < MF1; ++i)
#pragma unroll
              for (int ct = 0; ct < MCT; ++ct)
                if (i < nf && c0 + ct < S.cotiles)
                  acc[i][ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[ct], xb[i][s], acc[i][ct], 0, 0, 0);
          }
#pragma unroll
          for (int i = 0; i < MF1; ++i) {
            const int q = (wave + NW * i) * 16 + col;
            if (i >= nf || q >= a.R2) continue;
            const int r = q / a.R2W, cq = q - r * a.R2W;
            const int iy = y0 - 2 + r, ix = x0 - 2 + cq;
            const bool in = iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
#pragma unroll
            for (int ct = 0; ct < MCT; ++ct) {
              if (c0 + ct >= S.cotiles || (c0 + ct) * 16 + grp * 4 >= S.cout) continue;
              float v[4];
              c3_act(S, bias, c0 + ct, grp, acc[i][ct], v);
              h4 o = c3_h4(v);
              if (!in) o = h4{0, 0, 0, 0};  // the 3x3 convs' zero padding of b
              *reinterpret_cast<h4*>(T + (q * a.sT) * 8 + (c0 + ct) * 16 + grp * 4) = o;
            }
          }
        }
      }
    }
    tick(0);
    if (t + 1 < t_end) c3_load_x<NW, MF1, NS1>(a, t + 1, xb);  // in flight during stages 2-4
    tick(1);
    __syncthreads();
    // ---------------- stage 2: h = m.cv1(b) over the m.cv1 region (3x3 from the t image)
    {
      const C3Stage& S = a.st[1];
      const h8* wl = sm + S.wl + lane;
      const h8* Tin = sm + a.oT;
      for (int f0 = wave; f0 < nfr2; f0 += NW * MF) {
        const int nf = min(MF, (nfr2 - f0 + NW - 1) / NW);
        int pb[MF];
#pragma unroll
        for (int i = 0; i < MF; ++i) {
          const int q = min((f0 + NW * i) * 16 + col, a.R1 - 1);
          const int r = q / a.R1W, cq = q - r * a.R1W;
          pb[i] = r * a.R2W + cq;  // tap (0, 0) of output (r, cq): R2 position (r + 1 - 1, cq + 1 - 1)
        }
        auto bl = [&](int i, int st) -> h8 {
          int tap, cc;
          bool ok = true;
          if (S.fast) {
            const int ch = st / 9;
            tap = st - ch * 9;
            cc = ch * 4 + grp;
          } else {
            const int k = st * 4 + grp;
            tap = k / S.cpt;
            cc = k - tap * S.cpt;
            ok = tap < 9;
          }
          const int ky = (tap * 11) >> 5, kx = tap - ky * 3;
          return ok ? Tin[(pb[i] + ky * a.R2W + kx) * a.sT + c8 + cc] : h8{0, 0, 0, 0, 0, 0, 0, 0};
        };
        auto epi = [&](int i, int ct, const f4& acc) {
          const int q = (f0 + NW * i) * 16 + col;
          if (q >= a.R1) return;
          const int r = q / a.R1W, cq = q - r * a.R1W;
          const int iy = y0 - 1 + r, ix = x0 - 1 + cq;
          if (ct * 16 + grp * 4 >= S.cout) return;  // partial cout tile (c_mid % 16 == 8)
          float v[4];
          c3_act(S, bias, ct, grp, acc, v);
          h4 o = c3_h4(v);
          if (!(iy >= 0 && iy < a.H && ix >= 0 && ix < a.W)) o = h4{0, 0, 0, 0};
          *reinterpret_cast<h4*>(Hh + (q * a.sH) * 8 + ct * 16 + grp * 4) = o;
        };
        for (int c0 = 0; c0 < S.cotiles; c0 += MCT) c3_mma<MF, MCT>(wl, S.nsteps, S.cotiles, c0, nf, bl, epi);
      }
    }
    tick(2);
    __syncthreads();
    // ---------------- stage 3: m = m.cv2(h) + b over the tile (3x3 from the h image)
    {
      const C3Stage& S = a.st[2];
      const h8* wl = sm + S.wl + lane;
      const h8* Hin = sm + a.oH;
      for (int f0 = wave; f0 < nfr4; f0 += NW * MF) {
        const int nf = min(MF, (nfr4 - f0 + NW - 1) / NW);
        int pb[MF];
#pragma unroll
        for (int i = 0; i < MF; ++i) {
          const int q = min((f0 + NW * i) * 16 + col, a.NC - 1);
          const int r = q / a.TW, cq = q - r * a.TW;
          pb[i] = r * a.R1W + cq;
        }
        auto bl = [&](int i, int st) -> h8 {
          int tap, cc;
          bool ok = true;
          if (S.fast) {
            const int ch = st / 9;
            tap = st - ch * 9;
            cc = ch * 4 + grp;
          } else {
            const int k = st * 4 + grp;
            tap = k / S.cpt;
            cc = k - tap * S.cpt;
            ok = tap < 9;
          }
          const int ky = (tap * 11) >> 5, kx = tap - ky * 3;
          return ok ? Hin[(pb[i] + ky * a.R1W + kx) * a.sH + cc] : h8{0, 0, 0, 0, 0, 0, 0, 0};
        };
        auto epi = [&](int i, int ct, const f4& acc) {
          const int q = (f0 + NW * i) * 16 + col;
          if (q >= a.NC) return;
          const int r = q / a.TW, cq = q - r * a.TW;
          const int co0 = ct * 16 + grp * 4;
          if (co0 >= S.cout) return;  // partial cout tile (c % 16 == 8)
          float v[4];
          c3_act(S, bias, ct, grp, acc, v);
          const h4 rv = *reinterpret_cast<const h4*>(T + (((r + 2) * a.R2W + cq + 2) * a.sT) * 8 + a.c + co0);
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = fpin(v[j] + (float)rv[j]);
          *reinterpret_cast<h4*>(Mm + (q * a.sM) * 8 + co0) = c3_h4(v);
        };
        for (int c0 = 0; c0 < S.cotiles; c0 += MCT) c3_mma<MF, MCT>(wl, S.nsteps, S.cotiles, c0, nf, bl, epi);
      }
    }
    tick(3);
    __syncthreads();
    // ---------------- stage 4: y = cv2([a | b | m]) over the tile, to HBM
    {
      const C3Stage& S = a.st[3];
      const h8* wl = sm + S.wl + lane;
      const h8* Tin = sm + a.oT;
      const h8* Min = sm + a.oM;
      const int c2 = 2 * c8, c3 = 3 * c8;
      for (int f0 = wave; f0 < nfr4; f0 += NW * MF) {
        const int nf = min(MF, (nfr4 - f0 + NW - 1) / NW);
        int pt[MF], pm[MF];
#pragma unroll
        for (int i = 0; i < MF; ++i) {
          const int q = min((f0 + NW * i) * 16 + col, a.NC - 1);
          const int r = q / a.TW, cq = q - r * a.TW;
          pt[i] = ((r + 2) * a.R2W + cq + 2) * a.sT;
          pm[i] = q * a.sM - c2;
        }
        auto bl = [&](int i, int st) -> h8 {
          const int cc = st * 4 + grp;  // 1x1 (either K order): the 8-channel chunk of [a | b | m]
          if (cc >= c3) return h8{0, 0, 0, 0, 0, 0, 0, 0};
          return cc < c2 ? Tin[pt[i] + cc] : Min[pm[i] + cc];
        };
        auto epi = [&](int i, int ct, const f4& acc) {
          const int q = (f0 + NW * i) * 16 + col;
          if (q >= a.NC) return;
          const int r = q / a.TW, cq = q - r * a.TW;
          const int iy = y0 + r, ix = x0 + cq;
          if (iy >= a.H || ix >= a.W || ct * 16 + grp * 4 >= S.cout) return;
          float v[4];
          c3_act(S, bias, ct, grp, acc, v);
          *reinterpret_cast<h4*>(a.y + nhwc_off(n, iy, ix, a.H, a.W, a.ycs) + ct * 16 + grp * 4) = c3_h4(v);
        };
        for (int c0 = 0; c0 < S.cotiles; c0 += MCT) c3_mma<MF, MCT>(wl, S.nsteps, S.cotiles, c0, nf, bl, epi);
      }
    }
    tick(4);
    __syncthreads();  // stage 4's reads of t / m before the next tile's stage 1 overwrites them
    tick(5);
  }
  if (a.diag && blockIdx.x == 0 && threadIdx.x == 0)
    printf("c3k2 fused diag: %d tiles, clocks per tile: stage1 %llu, x-issue %llu, stage2 %llu, stage3 %llu, stage4 %llu, "
           "last barrier %llu\n", t_end - t_begin, (unsigned long long)(clk[0] / (t_end - t_begin)),
           (unsigned long long)(clk[1] / (t_end - t_begin)), (unsigned long long)(clk[2] / (t_end - t_begin)),
           (unsigned long long)(clk[3] / (t_end - t_begin)), (unsigned long long)(clk[4] / (t_end - t_begin)),
           (unsigned long long)(clk[5] / (t_end - t_begin)));
}

// ============================================================================ host
static C3Stage make_stage(const fce_conv_desc& d, const void* w, const float* b) {
  C3Stage s{};
  s.w = static_cast<const h8*>(w);
  s.b = b;
  s.cout = d.cout;
  s.taps = d.k * d.k;
  s.fast = d.cin % 32 == 0;
  s.cpt = d.cin / 8;
  const int nchunk = s.taps * s.cpt;
  s.nsteps = (nchunk + 3) / 4;
  s.nalloc = ((s.nsteps + 7) & ~7) + 8;
  s.cotiles = (d.cout + 15) / 16;
  return s;
}

struct C3Plan {
  int TH, TW, NW, MF1;
  size_t lds;
};

static int c3_weights16(const fce_c3k2_desc& d, C3Stage (&st)[4]) {
  const fce_conv_desc c1{d.cin, 2 * d.c, 1, 1, 1, FCE_ACT_SILU, 0, FCE_EPI_STORE, nullptr, 0, 0};
  const fce_conv_desc m1{d.c, d.c_mid, 3, 1, 1, FCE_ACT_SILU, 0, FCE_EPI_STORE, nullptr, 0, 0};
  const fce_conv_desc m2{d.c_mid, d.c, 3, 1, 1, FCE_ACT_SILU, 0, FCE_EPI_STORE, nullptr, 0, 0};
  const fce_conv_desc c2{3 * d.c, d.cout, 1, 1, 1, FCE_ACT_SILU, 0, FCE_EPI_STORE, nullptr, 0, 0};
  const fce_conv_desc* cd[4] = {&c1, &m1, &m2, &c2};
  int off = 0, boff = 0;
  for (int i = 0; i < 4; ++i) {
    st[i] = make_stage(*cd[i], d.w[i], d.b[i]);
    st[i].wl = off;
    off += st[i].cotiles * st[i].nsteps * 64;
    st[i].bl = boff;
    boff += st[i].cotiles * 16;
  }
  return off + boff / 4;  // fragments, then the bias block (16 floats per cout tile = 4 units)
}

// LDS image of a (TH, TW) tile: t = [a | b] over the cv1 region, h over the m.cv1 region, m over the tile
static size_t c3_lds(const fce_c3k2_desc& d, int w16, int TH, int TW) {
  const int R2 = (TH + 4) * (TW + 4), R1 = (TH + 2) * (TW + 2), NC = TH * TW;
  const int sT = (2 * d.c / 8) | 1, sH = (d.c_mid / 8) | 1, sM = (d.c / 8) | 1;
  return size_t(w16 + R2 * sT + R1 * sH + NC * sM) * 16;  // w16: fragments + biases
}

// tile / waves for a map: 4 waves with two blocks per CU on wide maps, 8 waves and one block per CU
// (the larger weight sets) otherwise; FCE_C3K2_TILE="TH,TW,NW" overrides (tuning)
static bool c3_plan(const fce_c3k2_desc& d, int H, int W, int w16, C3Plan* p) {
  const char* env = getenv("FCE_C3K2_TILE");  // read per plan: tests switch it within one process
  int cand[6][3] = {{8, 16, 4}, {4, 40, 8}, {4, 32, 8}, {4, 16, 8}, {2, 40, 8}, {2, 16, 8}};
  int nc = 6, first = W >= 128 ? 0 : 1;
  if (env && *env) {
    int th, tw, nw;
    if (sscanf(env, "%d,%d,%d", &th, &tw, &nw) == 3 && th > 0 && tw > 0 && (nw == 4 || nw == 8)) {
      cand[0][0] = th;
      cand[0][1] = tw;
      cand[0][2] = nw;
      nc = 1;
      first = 0;
    }
  }
  for (int i = first; i < nc || (nc == 1 && i < 7); ++i) {  // a forced shape that does not fit: the defaults
    if (nc == 1 && i == 1) {
      const int dflt[6][3] = {{8, 16, 4}, {4, 40, 8}, {4, 32, 8}, {4, 16, 8}, {2, 40, 8}, {2, 16, 8}};
      for (int k = 0; k < 6; ++k)
        for (int j = 0; j < 3; ++j) cand[k][j] = dflt[k][j];
      i = W >= 128 ? 0 : 1;
      nc = 6;
    }
    const int TH = std::min(cand[i][0], H), TW = std::min(cand[i][1], W), NW = cand[i][2];
    const int nfr1 = ((TH + 4) * (TW + 4) + 15) / 16;
    const int mf1 = (nfr1 + NW - 1) / NW;
    const size_t lds = c3_lds(d, w16, TH, TW);
    if (mf1 > 4 || lds > 160 * 1024) continue;
    *p = C3Plan{TH, TW, NW, mf1 <= 2 ? 2 : 4, lds};
    return true;
  }
  return false;
}

bool c3k2_fused_ok(const fce_c3k2_desc& d) {
  if (!(d.cin % 32 == 0 && d.cin <= 64 && d.c % 8 == 0 && d.c_mid % 8 == 0 && d.cout % 8 == 0 && 2 * d.c <= 128 &&
        d.c_mid <= 128 && d.cout <= 128))
    return false;
  C3Stage st[4];
  const int w16 = c3_weights16(d, st);
  C3Plan p;  // the candidates end with (2, 16): if some tile fits a 16-wide map, one fits every map
  return c3_plan(d, 16, 16, w16, &p);
}

template <int NW, int MF1, int NS1>
static int c3_launch(const C3k2Args& a, const C3Plan& p, hipStream_t s) {
  auto k = c3k2_fused_kernel<NW, MF1, NS1>;
  static const bool big = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
  if (!big && p.lds > 64 * 1024) return fail(FCE_ERR_HIP, "c3k2 fused: cannot opt in to >64 KiB LDS");
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
  }
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k, NW * 64, p.lds) != hipSuccess || occ < 1) occ = 1;
  const int grid = int(std::min<int64_t>(a.ntiles, int64_t(cus) * occ));
  FCE_LAUNCH(k, dim3(unsigned(grid)), dim3(NW * 64), p.lds, s, a);
  return launch_status("c3k2_fused_kernel");
}

int c3k2_fused(const fce_c3k2_desc& d, const fce_tensor& x, const fce_tensor& y, hipStream_t s) {
  FCE_CHECK(c3k2_fused_ok(d), "c3k2 fused: unsupported channel configuration");
  FCE_CHECK(x.layout == FCE_NHWC && y.layout == FCE_NHWC && x.dtype == FCE_F16 && y.dtype == FCE_F16,
            "c3k2 fused: NHWC f16 views");
  FCE_CHECK(x.c == d.cin && y.c == d.cout && x.n == y.n && x.h == y.h && x.w == y.w, "c3k2 fused: shape mismatch");
  FCE_CHECK(x.cstride % 8 == 0 && x.coff % 8 == 0 && y.cstride % 4 == 0 && y.coff % 4 == 0,
            "c3k2 fused: aligned channel slices");
  for (int i = 0; i < 4; ++i) FCE_CHECK(d.w[i] && d.b[i], "c3k2 fused: null weights");
  C3k2Args a{};
  const int w16 = c3_weights16(d, a.st);
  C3Plan p;
  FCE_CHECK(c3_plan(d, x.h, x.w, w16, &p), "c3k2 fused: no tile fits the LDS");
  a.x = static_cast<const _Float16*>(x.data) + x.coff;
  a.xcs = x.cstride;
  a.y = static_cast<_Float16*>(y.data) + y.coff;
  a.ycs = y.cstride;
  a.N = x.n;
  a.H = x.h;
  a.W = x.w;
  a.c = d.c;
  a.TH = p.TH;
  a.TW = p.TW;
  a.tiles_x = (x.w + p.TW - 1) / p.TW;
  a.tiles_y = (x.h + p.TH - 1) / p.TH;
  const int64_t tiles = int64_t(a.tiles_x) * a.tiles_y * x.n;
  if (tiles == 0) return FCE_OK;
  FCE_CHECK(tiles < (int64_t(1) << 30), "c3k2 fused: grid too large");
  a.ntiles = int(tiles);
  a.R2W = p.TW + 4;
  a.R2 = (p.TH + 4) * a.R2W;
  a.R1W = p.TW + 2;
  a.R1 = (p.TH + 2) * a.R1W;
  a.NC = p.TH * p.TW;
  a.sT = (2 * d.c / 8) | 1;
  a.sH = (d.c_mid / 8) | 1;
  a.sM = (d.c / 8) | 1;
  a.wtotal = w16;
  a.ob = a.st[3].wl + a.st[3].cotiles * a.st[3].nsteps * 64;  // the bias block follows the fragments
  a.nbias = (w16 - a.ob) * 4;
  {
    const char* de = getenv("FCE_C3K2_DIAG");
    a.diag = de && atoi(de) != 0;
  }
  a.oT = w16;
  a.oH = a.oT + a.R2 * a.sT;
  a.oM = a.oH + a.R1 * a.sH;
  const int ns1 = d.cin / 32;
  // host-side shape checks of what the kernel's indexing assumes
  FCE_CHECK(a.st[0].nsteps == ns1 && a.st[0].fast, "c3k2 fused: cv1 K-steps");
  FCE_CHECK((a.R2 + 15) / 16 <= p.NW * p.MF1, "c3k2 fused: cv1 region exceeds the wave fragments");
  FCE_CHECK(size_t(a.oM + a.NC * a.sM) * 16 == p.lds, "c3k2 fused: LDS layout");
#define C3L(NW_, MF_)                                                      \
  do {                                                                     \
    if (ns1 == 1) return c3_launch<NW_, MF_, 1>(a, p, s);                  \
    return c3_launch<NW_, MF_, 2>(a, p, s);                                \
  } while (0)
  if (p.NW == 4) {
    if (p.MF1 == 2) C3L(4, 2);
    C3L(4, 4);
  }
  if (p.MF1 == 2) C3L(8, 2);
  C3L(8, 4);
#undef C3L
}

}  // namespace fce
