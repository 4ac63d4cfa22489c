// Fused Detect cls branch (reference ultralytics/nn/modules/head.py:86-107, legacy = False:
//   cv3[i] = DWConv(x, x, 3) -> Conv(x, c3, 1) -> DWConv(c3, c3, 3) -> Conv(c3, c3, 1) -> nn.Conv2d(c3, nc, 1),
// DWConv / Conv = conv.py:39-89, 185-200 with the BN folded, and the sigmoid of head.py:149-167) in ONE persistent
// kernel:
//
//   t1 = SiLU(dw1(x))    depthwise 3x3 over the tile + 1-pixel halo, from x staged with a 2-pixel halo
//   t2 = SiLU(pw1(t1))   1x1 c0 -> c3 over the tile + 1-pixel halo (zero outside the image: dw2's padding)
//   t3 = SiLU(dw2(t2))   depthwise 3x3 over the tile
//   t4 = SiLU(pw2(t3))   1x1 c3 -> c3 over the tile
//   pred[n][4 + k][a0 + p] = sigmoid(cls(t4))   1x1 c3 -> nc, plus the per-anchor best-class key (OUT_CLS)
//
// A block owns a contiguous run of TH x TW tiles.  The three 1x1s' packed A fragments, both depthwise tables and
// every bias are copied into LDS once; t1..t4 never leave LDS (two images, P: t1 / t3, Q: x / t2 / t4), and the next
// tile's x is loaded into registers while the current tile's five stages run.  The five separate launches move x,
// t1, t2, t3 and t4 through HBM (each written once and read once): n32's P3 branch ~360 MB against ~92 MB here (x
// read once, the fp32 scores written once).
//
// Bitwise identical to the five unfused ops (tests/test_gpu.py::test_fused_detect_cls_bitwise_equal_to_five_ops):
// the depthwise stages are dwconv_kernel's arithmetic (acc = bias, taps in (ky, kx) order, rows outside the image
// skipped, columns outside it multiplied as zeros, v_fma_mix with fp32 weights, SiLU, fpin, fp16); the 1x1 stages
// walk the same K-steps of the same packed fragments with v_mfma_f32_16x16x32_f16 from zero (mfma_stage.h) and
// round to fp16 where the unfused ops store; the cls tail is conv_epilogue's OUT_CLS (sigmoidf_, the same key, one
// atomic max per pixel).
#include <algorithm>

#include "mfma_stage.h"

namespace fce {

static __device__ __attribute__((aligned(16))) _Float16 g_dc_zero[8];

constexpr int dc_max(int a, int b) { return a > b ? a : b; }

// compile-time geometry of one instantiation (LDS offsets in 16-byte units)
template <int C0, int C3, int NCLS, int TH, int TW, int NW>
struct DcG {
  static constexpr int NT = NW * 64;
  static constexpr int K0 = C0 / 8, K3 = C3 / 8;           // 8-channel chunks
  static constexpr int XW = TW + 4, XR = (TH + 4) * XW;    // x region: tile + 2-pixel halo
  static constexpr int RW = TW + 2, R1 = (TH + 2) * RW;    // t1 / t2 region: tile + 1-pixel halo
  static constexpr int NC = TH * TW;
  // units per position: x is read by the depthwise stage only (lane = chunk fastest: conflict-free unpadded); t1..t4
  // are MFMA B operands (16 lanes = 16 positions of one chunk: odd strides)
  static constexpr int sX = K0, s1 = K0 | 1, s3 = K3 | 1;
  static constexpr int NF1 = (R1 + 15) / 16, NF2 = (NC + 15) / 16;
  static constexpr int MF1 = (NF1 + NW - 1) / NW, MF2 = (NF2 + NW - 1) / NW;
  static constexpr int CT3 = (C3 + 15) / 16, CTN = (NCLS + 15) / 16;
  static constexpr int NS1 = (K0 + 3) / 4, NS2 = (K3 + 3) / 4;  // 1x1 K-steps as dense_geom counts them
  static constexpr int W1 = CT3 * NS1 * 64, W2 = CT3 * NS2 * 64, W3 = CTN * NS2 * 64;
  static constexpr int OW2 = W1, OW3 = W1 + W2, OD = W1 + W2 + W3;
  static constexpr int ND = 9 * (C0 + C3);  // floats: dw1 [9][C0], dw2 [9][C3]
  // biases (floats): dw1, pw1 (CT3 x 16), dw2, pw2 (CT3 x 16), cls (CTN x 16)
  static constexpr int BD1 = 0, BP1 = C0, BD2 = BP1 + CT3 * 16, BP2 = BD2 + C3, BC = BP2 + CT3 * 16, NB = BC + CTN * 16;
  static constexpr int OB = OD + ND / 4;
  static constexpr int OP = OB + (NB + 3) / 4;
  static constexpr int PSZ = dc_max(R1 * s1, NC * s3);
  static constexpr int OQ = OP + PSZ;
  // x and t2 are the depthwise stages' inputs: staged as fp32 (the fp16 values, converted once) in two planes, the
  // low and high 4 channels of each 8-channel chunk, so a thread's 8 channels are two conflict-free 16-byte reads and
  // the taps run as v_pk_fma_f32 (two exact fmas per instruction, the same values as v_fma_mix)
  static constexpr int QX = XR * K0, QT = R1 * K3;  // units per plane
  static constexpr int QSZ = dc_max(dc_max(2 * QX, 2 * QT), NC * s3);
  static constexpr int TOTAL = OQ + QSZ;
  static constexpr size_t LDS = size_t(TOTAL) * 16;
  static constexpr int NXE = (XR * K0 + NT - 1) / NT;  // x chunks per thread
  static constexpr int NPG3 = NT / K3;                // dw2 position groups (threads >= NPG3 * K3 idle there)
  // blocks per CU the LDS allows (two only under 80 KiB): the register budget follows (one 4-wave block: 512)
  static constexpr int MINB = (LDS <= 80 * 1024 && NW == 4) ? 2 : 1;
  static_assert(C0 % 8 == 0 && C3 % 8 == 0 && NT % K0 == 0 && NPG3 > 0, "detect cls fused: channel alignment");
};

struct DclsArgs {
  const _Float16* x;
  int xcs;
  int H, W, tiles_x, tiles_y, ntiles;
  const float* dw[2];  // depthwise tables [9][c] fp32 (conv_pack of the depthwise desc)
  const h8* pw[3];     // pw1, pw2, cls packed A fragments (conv_pack layout [cout tile][nalloc][64 lanes])
  int nalloc[3];
  const float* b[5];   // dw1, pw1, dw2, pw2, cls biases (BN folded)
  float* pred;
  unsigned long long* best;
  int A, a0;
  int diag;  // FCE_DCLS_DIAG: block 0 prints its per-stage clocks
};

__device__ __forceinline__ void dc_tile(const DclsArgs& a, int TH, int TW, int t, int& n, int& y0, int& x0) {
  const int tx = t % a.tiles_x;
  t /= a.tiles_x;
  const int ty = t % a.tiles_y;
  n = t / a.tiles_y;
  y0 = ty * TH;
  x0 = tx * TW;
}

// depthwise 3x3 (stride 1) of one 8-channel chunk at one output position from an fp32 LDS image (planes lo / hi of
// `plane` units each, position stride k chunks): dwconv_kernel's order (acc = bias, (ky, kx) order, rows outside the
// image skipped, every column of a kept row fused, zeros outside), each tap as four v_pk_fma_f32 -- fma(x, w, acc)
// with the exactly converted fp16 x, as v_fma_mix computes it -- then SiLU and fp16.  (A taps-outermost form over
// several positions per thread, which let a 16-wave block fit 128 VGPRs, measured slower: 86.6 against 81.7 us on
// n32's P3, 132 us with 16 waves, DESIGN.md.)
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ h8 dc_dw(const f4* img, int plane, int p00, int rw, int k, int ch, int iy, int H,
                                    const float (&wk)[9][8], const float (&bz)[8]) {
  f2 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = f2{bz[2 * j], bz[2 * j + 1]};
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
    const int yy = iy - 1 + ky;
    if (yy < 0 || yy >= H) continue;
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      const int u = (p00 + ky * rw + kx) * k + ch;
      const f4 lo = img[u], hi = img[plane + u];
      const float* w = wk[ky * 3 + kx];
      acc[0] = __builtin_elementwise_fma(f2{lo[0], lo[1]}, f2{w[0], w[1]}, acc[0]);
      acc[1] = __builtin_elementwise_fma(f2{lo[2], lo[3]}, f2{w[2], w[3]}, acc[1]);
      acc[2] = __builtin_elementwise_fma(f2{hi[0], hi[1]}, f2{w[4], w[5]}, acc[2]);
      acc[3] = __builtin_elementwise_fma(f2{hi[2], hi[3]}, f2{w[6], w[7]}, acc[3]);
    }
  }
  h8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (_Float16)fpin(silu(acc[j >> 1][j & 1]));
  return o;
}

// the 9 x 8 depthwise weights and 8 biases of chunk ch from the LDS tables ([9][c] fp32)
__device__ __forceinline__ void dc_weights(const float* tab, int c, int ch, const float* bias, float (&wk)[9][8],
                                           float (&bz)[8]) {
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const f4 w0 = *reinterpret_cast<const f4*>(tab + t * c + ch * 8);
    const f4 w1 = *reinterpret_cast<const f4*>(tab + t * c + ch * 8 + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      wk[t][j] = w0[j];
      wk[t][j + 4] = w1[j];
    }
  }
  const f4 b0 = *reinterpret_cast<const f4*>(bias + ch * 8);
  const f4 b1 = *reinterpret_cast<const f4*>(bias + ch * 8 + 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    bz[j] = b0[j];
    bz[j + 4] = b1[j];
  }
}

template <int C0, int C3, int NCLS, int TH, int TW, int NW>
__global__ __launch_bounds__(NW * 64, (DcG<C0, C3, NCLS, TH, TW, NW>::MINB)) void detect_cls_fused_kernel(DclsArgs a) {
  using G = DcG<C0, C3, NCLS, TH, TW, NW>;
  extern __shared__ __attribute__((aligned(16))) h8 sm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, col = lane & 15, grp = lane >> 4;
  const int NG = gridDim.x, bi = blockIdx.x;
  const int t_begin = int(int64_t(bi) * a.ntiles / NG), t_end = int(int64_t(bi + 1) * a.ntiles / NG);
  if (t_begin >= t_end) return;  // block-uniform

  // x of tile t at the x region's positions, 8 channels per element (zeros outside the image / region)
  h8 xr[G::NXE];
  auto load_x = [&](int t) {
    int n, y0, x0;
    dc_tile(a, TH, TW, t, n, y0, x0);
#pragma unroll
    for (int k = 0; k < G::NXE; ++k) {
      const int e = tid + k * G::NT, pos = e / G::K0, ch = e - pos * G::K0;
      const int r = pos / G::XW, c = pos - r * G::XW;
      const int iy = y0 - 2 + r, ix = x0 - 2 + c;
      const bool in = pos < G::XR && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
      const _Float16* src = in ? a.x + nhwc_off(n, iy, ix, a.H, a.W, a.xcs) + ch * 8 : g_dc_zero;
      xr[k] = *reinterpret_cast<const h8*>(src);
    }
  };
  load_x(t_begin);
  // fragments, depthwise tables and biases -> LDS, once per block
  {
    stage_copy_frags(sm, a.pw[0], G::CT3, G::NS1, a.nalloc[0], G::NT);
    stage_copy_frags(sm + G::OW2, a.pw[1], G::CT3, G::NS2, a.nalloc[1], G::NT);
    stage_copy_frags(sm + G::OW3, a.pw[2], G::CTN, G::NS2, a.nalloc[2], G::NT);
    float* d = reinterpret_cast<float*>(sm + G::OD);
    for (int e = tid; e < 9 * C0; e += G::NT) d[e] = a.dw[0][e];
    for (int e = tid; e < 9 * C3; e += G::NT) d[9 * C0 + e] = a.dw[1][e];
    float* bs = reinterpret_cast<float*>(sm + G::OB);
    for (int e = tid; e < G::NB; e += G::NT) {
      float v;
      if (e < G::BP1) v = a.b[0][e];
      else if (e < G::BD2) v = e - G::BP1 < C3 ? a.b[1][e - G::BP1] : 0.f;
      else if (e < G::BP2) v = a.b[2][e - G::BD2];
      else if (e < G::BC) v = e - G::BP2 < C3 ? a.b[3][e - G::BP2] : 0.f;
      else v = e - G::BC < NCLS ? a.b[4][e - G::BC] : 0.f;
      bs[e] = v;
    }
  }
  __syncthreads();

  const float* dwt = reinterpret_cast<const float*>(sm + G::OD);
  const float* bias = reinterpret_cast<const float*>(sm + G::OB);
  h8* P = sm + G::OP;
  h8* Q = sm + G::OQ;
  _Float16* Qh = reinterpret_cast<_Float16*>(Q);
  f4* Qf = reinterpret_cast<f4*>(Q);
  const h8 zero8 = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t clk[7] = {0, 0, 0, 0, 0, 0, 0}, tprev = a.diag ? __builtin_amdgcn_s_memtime() : 0;
  auto tick = [&](int k) {
    if (a.diag) {
      const uint64_t tn = __builtin_amdgcn_s_memtime();
      clk[k] += tn - tprev;
      tprev = tn;
    }
  };

  for (int t = t_begin; t < t_end; ++t) {
    int n, y0, x0;
    dc_tile(a, TH, TW, t, n, y0, x0);
    // x(t) -> Q, then the next tile's x in flight during the five stages
#pragma unroll
    for (int k = 0; k < G::NXE; ++k) {
      const int e = tid + k * G::NT, pos = e / G::K0;
      if (pos < G::XR) {
        const h8 v = xr[k];
        Qf[e] = f4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
        Qf[G::QX + e] = f4{(float)v[4], (float)v[5], (float)v[6], (float)v[7]};
      }
    }
    tick(0);
    if (t + 1 < t_end) load_x(t + 1);
    stage_barrier();
    tick(1);
    // ---------------- t1 = SiLU(dw1(x)) over the tile + 1-pixel halo -> P
    {
      const int ch = tid % G::K0;
      float wk[9][8], bz[8];
      dc_weights(dwt, C0, ch, bias + G::BD1, wk, bz);
      for (int pos = tid / G::K0; pos < G::R1; pos += G::NT / G::K0) {
        const int r = pos / G::RW, c = pos - r * G::RW;
        const int iy = y0 - 1 + r, ix = x0 - 1 + c;
        h8 o = zero8;  // outside the image: unused (pw1 zeroes t2 there)
        if (iy >= 0 && iy < a.H && ix >= 0 && ix < a.W) o = dc_dw(Qf, G::QX, r * G::XW + c, G::XW, G::K0, ch, iy, a.H, wk, bz);
        P[pos * G::s1 + ch] = o;
      }
    }
    stage_barrier();
    tick(2);
    // ---------------- t2 = SiLU(pw1(t1)) over the tile + 1-pixel halo -> Q (zero outside the image)
    {
      int pq[G::MF1];
#pragma unroll
      for (int i = 0; i < G::MF1; ++i) pq[i] = min((wave + NW * i) * 16 + col, G::R1 - 1) * G::s1;
      auto bl = [&](int i, int st) -> h8 {
        const int cc = st * 4 + grp;
        return cc < G::K0 ? P[pq[i] + cc] : zero8;
      };
      auto epi = [&](int i, int ct, const f4& acc) {
        const int q = (wave + NW * i) * 16 + col, co0 = ct * 16 + grp * 4;
        if (q >= G::R1 || co0 >= C3) return;
        const int r = q / G::RW, c = q - r * G::RW;
        const int iy = y0 - 1 + r, ix = x0 - 1 + c;
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = silu(acc[j] + bias[G::BP1 + co0 + j]);
        const h4 o = h4_of(v);  // t2 is stored as the fp32 values of its fp16 rounding (zero outside the image)
        const bool in = iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
        Qf[(co0 & 4 ? G::QT : 0) + q * G::K3 + (co0 >> 3)] =
            in ? f4{(float)o[0], (float)o[1], (float)o[2], (float)o[3]} : f4{0.f, 0.f, 0.f, 0.f};
      };
      mfma_stage<G::MF1, G::CT3, G::NS1>(sm + lane, bl, epi);
    }
    stage_barrier();
    tick(3);
    // ---------------- t3 = SiLU(dw2(t2)) over the tile -> P
    if (tid < G::NPG3 * G::K3) {
      const int ch = tid % G::K3;
      float wk[9][8], bz[8];
      dc_weights(dwt + 9 * C0, C3, ch, bias + G::BD2, wk, bz);
      for (int pos = tid / G::K3; pos < G::NC; pos += G::NPG3) {
        const int r = pos / TW, c = pos - r * TW;
        const int iy = y0 + r, ix = x0 + c;
        h8 o = zero8;  // outside the image: never stored
        if (iy < a.H && ix < a.W) o = dc_dw(Qf, G::QT, r * G::RW + c, G::RW, G::K3, ch, iy, a.H, wk, bz);
        P[pos * G::s3 + ch] = o;
      }
    }
    stage_barrier();
    tick(4);
    // ---------------- t4 = SiLU(pw2(t3)) over the tile -> Q
    {
      int pq[G::MF2];
#pragma unroll
      for (int i = 0; i < G::MF2; ++i) pq[i] = min((wave + NW * i) * 16 + col, G::NC - 1) * G::s3;
      auto bl = [&](int i, int st) -> h8 {
        const int cc = st * 4 + grp;
        return cc < G::K3 ? P[pq[i] + cc] : zero8;
      };
      auto epi = [&](int i, int ct, const f4& acc) {
        const int q = (wave + NW * i) * 16 + col, co0 = ct * 16 + grp * 4;
        if (q >= G::NC || co0 >= C3) return;
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = silu(acc[j] + bias[G::BP2 + co0 + j]);
        *reinterpret_cast<h4*>(Qh + (q * G::s3) * 8 + co0) = h4_of(v);
      };
      mfma_stage<G::MF2, G::CT3, G::NS2>(sm + G::OW2 + lane, bl, epi);
    }
    stage_barrier();
    tick(5);
    // ---------------- pred rows 4.. = sigmoid(cls(t4)) over the tile, + the best-class key
    {
      int pq[G::MF2];
#pragma unroll
      for (int i = 0; i < G::MF2; ++i) pq[i] = min((wave + NW * i) * 16 + col, G::NC - 1) * G::s3;
      unsigned long long bk[G::MF2];
#pragma unroll
      for (int i = 0; i < G::MF2; ++i) bk[i] = 0ull;
      auto bl = [&](int i, int st) -> h8 {
        const int cc = st * 4 + grp;
        return cc < G::K3 ? Q[pq[i] + cc] : zero8;
      };
      auto epi = [&](int i, int ct, const f4& acc) {
        const int q = (wave + NW * i) * 16 + col, co0 = ct * 16 + grp * 4;
        if (q >= G::NC) return;
        const int r = q / TW, c = q - r * TW;
        const int iy = y0 + r, ix = x0 + c;
        if (iy >= a.H || ix >= a.W) return;
        float* o = a.pred + (int64_t(n) * (4 + NCLS) + 4 + co0) * a.A + a.a0 + iy * a.W + ix;
        const int nv = min(4, NCLS - co0);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (j < nv) {
            const float sc = sigmoidf_(acc[j] + bias[G::BC + co0 + j]);
            o[int64_t(j) * a.A] = sc;
            const unsigned long long key =
                (uint64_t(__float_as_uint(sc)) << 32) | uint64_t(0xFFFFFFFFu - uint32_t(co0 + j));
            bk[i] = key > bk[i] ? key : bk[i];
          }
      };
      mfma_stage<G::MF2, G::CTN, G::NS2>(sm + G::OW3 + lane, bl, epi);
      if (a.best) {
#pragma unroll
        for (int i = 0; i < G::MF2; ++i) {
          unsigned long long k = bk[i];
          const unsigned long long k16 = __shfl_xor(k, 16);
          k = k16 > k ? k16 : k;
          const unsigned long long k32 = __shfl_xor(k, 32);
          k = k32 > k ? k32 : k;
          const int q = (wave + NW * i) * 16 + col;
          const int r = q / TW, c = q - r * TW;
          if (grp == 0 && q < G::NC && y0 + r < a.H && x0 + c < a.W && k)
            atomicMax(a.best + int64_t(n) * a.A + a.a0 + (y0 + r) * a.W + x0 + c, k);
        }
      }
    }
    stage_barrier();  // the cls stage's reads of t4 before the next tile's x overwrites Q
    tick(6);
  }
  if (a.diag && blockIdx.x == 0 && threadIdx.x == 0) {
    const unsigned long long nt = (unsigned long long)(t_end - t_begin);
    printf("detect cls fused diag: %llu tiles, clocks per tile: x->lds %llu, x-issue+barrier %llu, dw1 %llu, pw1 %llu, "
           "dw2 %llu, pw2 %llu, cls %llu\n", nt, (unsigned long long)clk[0] / nt, (unsigned long long)clk[1] / nt,
           (unsigned long long)clk[2] / nt, (unsigned long long)clk[3] / nt, (unsigned long long)clk[4] / nt,
           (unsigned long long)clk[5] / nt, (unsigned long long)clk[6] / nt);
  }
}

// ============================================================================ host
// instantiated (c0, c3, nc): the n scale's P3 / P4 levels (c3 = max(c0_P3, min(nc, 100)) = 80, nc 80).  P3 runs
// 8 x 16 tiles with 8 waves (~103 KiB LDS, one block per CU), P4 8 x 8 with 8 waves (~122 KiB); P5 (c0 256) needs
// > 160 KiB at any tile of 64 positions and keeps the five ops.  The kernel is bound by its VALU (the depthwise
// FMAs and the SiLU / sigmoid of every stage, recomputed over the 1-pixel halo for dw1 / pw1) at two waves per SIMD
// (FCE_DCLS_DIAG stage clocks).
struct DcInst {
  int c0, c3, nc;
};
static constexpr DcInst kDcInsts[] = {{64, 80, 80}, {128, 80, 80}};

template <int C0, int C3, int NCLS, int TH, int TW, int NW>
static int dc_launch(const DclsArgs& a0, int N, hipStream_t s) {
  using G = DcG<C0, C3, NCLS, TH, TW, NW>;
  static_assert(G::LDS <= 160 * 1024, "detect cls fused: LDS over 160 KiB");
  auto k = detect_cls_fused_kernel<C0, C3, NCLS, TH, TW, NW>;
  static const bool big = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
  if (!big && G::LDS > 64 * 1024) return fail(FCE_ERR_HIP, "detect cls fused: cannot opt in to >64 KiB LDS");
  DclsArgs a = a0;
  a.tiles_x = (a.W + TW - 1) / TW;
  a.tiles_y = (a.H + TH - 1) / TH;
  const int64_t tiles = int64_t(a.tiles_x) * a.tiles_y * N;
  if (tiles == 0) return FCE_OK;
  FCE_CHECK(tiles < (int64_t(1) << 30), "detect cls fused: grid too large");
  a.ntiles = int(tiles);
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
  }
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k, G::NT, G::LDS) != hipSuccess || occ < 1) occ = 1;
  const int grid = int(std::min<int64_t>(a.ntiles, int64_t(cus) * occ));
  FCE_LAUNCH(k, dim3(unsigned(grid)), dim3(G::NT), G::LDS, s, a);
  return launch_status("detect_cls_fused_kernel");
}

// FCE_DCLS_TILE_64 = "8,16,8" (default) / "8,16,4" / "8,8,4" and FCE_DCLS_TILE_128 = "8,8,8" (default) / "8,8,4"
// (experiments, tests) force a tile of that c0's instantiation; any other value is an error.  n32 (five ops 109 / 50
// us): P3 8,16,8 82 us, 8,8,4 97, 8,16,4 125; P4 8,8,8 44 us, 8,8,4 56 (profiles/r05_detect_cls_probe.txt)
static bool dc_tile_env(const char* name, const char* v) {
  const char* e = getenv(name);  // read per call: tests switch it within one process
  return e && strcmp(e, v) == 0;
}

static int dc_dispatch(int inst, const DclsArgs& a, int N, hipStream_t s) {
  const char* name = inst == 0 ? "FCE_DCLS_TILE_64" : "FCE_DCLS_TILE_128";
  const char* env = getenv(name);
  const bool set = env && *env;
  if (inst == 0) {
    if (!set || dc_tile_env(name, "8,16,8")) return dc_launch<64, 80, 80, 8, 16, 8>(a, N, s);
    if (dc_tile_env(name, "8,16,4")) return dc_launch<64, 80, 80, 8, 16, 4>(a, N, s);
    if (dc_tile_env(name, "8,8,4")) return dc_launch<64, 80, 80, 8, 8, 4>(a, N, s);
  } else {
    if (!set || dc_tile_env(name, "8,8,8")) return dc_launch<128, 80, 80, 8, 8, 8>(a, N, s);
    if (dc_tile_env(name, "8,8,4")) return dc_launch<128, 80, 80, 8, 8, 4>(a, N, s);
  }
  return fail(FCE_ERR_INVALID, std::string(name) + ": not a tile of this instantiation");
}

static int dc_inst(const fce_dcls_desc& d) {
  for (int i = 0; i < int(sizeof(kDcInsts) / sizeof(kDcInsts[0])); ++i)
    if (kDcInsts[i].c0 == d.c0 && kDcInsts[i].c3 == d.c3 && kDcInsts[i].nc == d.nc) return i;
  return -1;
}

bool detect_cls_fused_ok(const fce_dcls_desc& d) { return dc_inst(d) >= 0; }

int detect_cls_fused(const fce_dcls_desc& d, const fce_tensor& x, const fce_detect_epi& e, hipStream_t s) {
  const int inst = dc_inst(d);
  FCE_CHECK(inst >= 0, "detect cls fused: unsupported channel configuration");
  FCE_CHECK(x.layout == FCE_NHWC && x.dtype == FCE_F16 && x.c == d.c0, "detect cls fused: NHWC f16 view of c0 channels");
  FCE_CHECK(x.cstride % 8 == 0 && x.coff % 8 == 0, "detect cls fused: aligned channel slice");
  FCE_CHECK(e.pred && e.part == 1 && e.nc == d.nc && e.anchor_offset >= 0 &&
                int64_t(e.anchor_offset) + int64_t(x.h) * x.w <= e.anchors,
            "detect cls fused: the cls epilogue of this level (part 1, nc, anchors)");
  for (int i = 0; i < 5; ++i) FCE_CHECK(d.w[i] && d.b[i], "detect cls fused: null weights");
  DclsArgs a{};
  a.x = static_cast<const _Float16*>(x.data) + x.coff;
  a.xcs = x.cstride;
  a.H = x.h;
  a.W = x.w;
  a.dw[0] = static_cast<const float*>(d.w[0]);
  a.dw[1] = static_cast<const float*>(d.w[2]);
  a.pw[0] = static_cast<const h8*>(d.w[1]);
  a.pw[1] = static_cast<const h8*>(d.w[3]);
  a.pw[2] = static_cast<const h8*>(d.w[4]);
  a.nalloc[0] = stage_nalloc(d.c0, 1);
  a.nalloc[1] = stage_nalloc(d.c3, 1);
  a.nalloc[2] = stage_nalloc(d.c3, 1);
  for (int i = 0; i < 5; ++i) a.b[i] = d.b[i];
  a.pred = e.pred;
  a.best = e.best;
  a.A = e.anchors;
  a.a0 = e.anchor_offset;
  {
    const char* de = getenv("FCE_DCLS_DIAG");
    a.diag = de && atoi(de) != 0;
  }
  return dc_dispatch(inst, a, x.n, s);
}

}  // namespace fce
