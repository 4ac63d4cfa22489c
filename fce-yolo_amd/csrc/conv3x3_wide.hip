// Wide-tile 3x3 convolution with per-K-step weight staging; the m/l-scale dense 3x3 convs.
// Replaces (reference, ultralytics/): nn/modules/conv.py:39-89 Conv.forward_fuse (3x3, BN folded by
// utils/torch_utils.py:237-267) for cin % 32 == 0.  Variant code 0xA00 | log2(cw) << 4 of fce_conv2d_variant.
//
// Every wave owns 64 couts x 64 output pixels (4 cout tiles x 4 output rows of 16 columns: 16 MFMAs per 4 A +
// 4 B fragment reads from LDS); the block is CW x (4 / CW) such waves, i.e. 64 CW couts x 16 (4 / CW) rows of
// 16 pixels.  The K loop runs over single K-steps s = (32-channel chunk c, tap) in the implicit-GEMM order:
//   * the block's A fragments of step s (CW * 4 cout tiles, 1 KiB each, contiguous per tile in the packed
//     weights) sit in one of three LDS slots: each thread loads its CW pieces of step s + 2 into registers at
//     step s and stores the pieces of step s + 1 after step s's MFMAs, so a global load has a whole step to
//     land and the weights cross L2 -> LDS once per block instead of once per wave;
//   * the chunk's input halo tile (the tile kernels' swizzled image) is double-buffered: the pieces of chunk
//     c + 1 are loaded in 8 batches during taps 0..7 of chunk c and stored one tap later;
//   * one barrier per K-step; two blocks (or one 8-wave pair of blocks) per CU keep a block's MFMAs running
//     while the other waits at its barrier.
// Plain global loads + ds_write instead of LDS-DMA: the DMA copies' issue cost (60-185 clocks each, stage
// clocks of conv3x3_big.hip) is what held that kernel's matrix core idle.  Same K order and fragments as
// every other variant: bitwise identical.
#include "conv_args.h"

namespace fce {

template <int S, int CW>
struct WideGeom {
  static constexpr int RW = 4 / CW, RC = 4, RP = 4;
  static constexpr int TW = 16, TH = RW * RP;
  static constexpr int RI = (TH - 1) * S + 3, CI = (TW - 1) * S + 3;
  static constexpr int NE = RI * CI * 4;          // 16-byte pieces of one chunk's halo image
  static constexpr int NL = (NE + 255) / 256;     // pieces per thread per chunk
  static constexpr int NB = NL * 256;             // padded image: the last round stores unconditionally
  static constexpr int PB = (NL + 7) / 8;         // pieces per thread per tap batch (8 batches per chunk)
  static constexpr int AT = CW * RC;              // cout tiles of the block
  static constexpr int NLA = AT * 64 / 256;       // A pieces per thread per K-step (= CW)
  static constexpr int AS = 3;                    // A slots
  static constexpr size_t lds = size_t(2 * NB + AS * AT * 64) * 16;
};

template <int S, int CW>
__global__ __launch_bounds__(256, 2) void conv3x3_wide_kernel(ConvArgs a) {
  using G = WideGeom<S, CW>;
  constexpr int RW = G::RW, TW = G::TW, TH = G::TH, CI = G::CI, NE = G::NE, NL = G::NL, NB = G::NB, PB = G::PB;
  constexpr int AT = G::AT, NLA = G::NLA;
  extern __shared__ __attribute__((aligned(16))) h8 wide_smem[];  // [halo 0 | halo 1 | A0 | A1 | A2]
  h8* const halo = wide_smem;
  h8* const aslot = wide_smem + 2 * NB;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 15, grp = lane >> 4;
  const int wc = wave / RW, wr = wave - wc * RW;
  const int tiles_x = (a.Wo + TW - 1) / TW, tiles_y = (a.Ho + TH - 1) / TH;
  int t, cog;
  tile_block(a.gy, t, cog);
  const int tx = t % tiles_x;
  t /= tiles_x;
  const int ty = t % tiles_y;
  const int n = t / tiles_y;
  const int ox0 = tx * TW, oy0 = ty * TH;
  const int cotiles = (a.cout + 15) >> 4;
  const int ct_blk = cog * AT;
  const int spt = a.cin >> 5;
  const int nst = spt * 9;
  const _Float16* xn = a.x + int64_t(n) * a.Hs * a.Ws * a.xcs;
  const h8* wts = reinterpret_cast<const h8*>(a.w);
  const h8* zero = reinterpret_cast<const h8*>(g_zero_line);
  const int iy0 = oy0 * S - 1, ix0 = ox0 * S - 1;

  // this thread's halo pieces (fixed over chunks): source element offset (-1: zero line) and LDS slot
  int hoff[NL], hslot[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int e = tid + 256 * i;
    const int pc = e >> 2, q = e & 3;
    const int r = pc / CI, c = pc - r * CI;
    const int iy = iy0 + r, ix = ix0 + c;
    const int u = r * CI + tile_col<S, CI>(c);
    hslot[i] = e < NE ? u * 4 + (q ^ ((u >> 1) & 3)) : e;
    hoff[i] = (e < NE && iy >= 0 && iy < a.Hs && ix >= 0 && ix < a.Ws) ? (iy * a.Ws + ix) * a.xcs + q * 8 : -1;
  }
  auto hsrc = [&](int i, int c) -> const h8* {
    return hoff[i] >= 0 ? reinterpret_cast<const h8*>(xn + hoff[i] + c * 32) : zero;
  };
  // this thread's A pieces: piece p = tid + 256 j -> block cout tile p >> 6 (clamped), lane p & 63
  const h8* asrc[NLA];
#pragma unroll
  for (int j = 0; j < NLA; ++j) {
    const int p = tid + 256 * j;
    const int ct = min(ct_blk + (p >> 6), cotiles - 1);
    asrc[j] = wts + size_t(ct) * a.nalloc * 64 + (p & 63);
  }

  f4 acc[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int p = 0; p < 4; ++p) acc[r][p] = f4{0.f, 0.f, 0.f, 0.f};

  // prologue: A(0) -> slot 0, A(1) in registers, chunk 0's halo -> buffer 0
  h8 ra[3][NLA];
#pragma unroll
  for (int j = 0; j < NLA; ++j) {
    ra[0][j] = asrc[j][0];
    ra[1][j] = asrc[j][64];
  }
  {
    h8 hv[NL];
#pragma unroll
    for (int i = 0; i < NL; ++i) hv[i] = *hsrc(i, 0);
#pragma unroll
    for (int i = 0; i < NL; ++i) halo[hslot[i]] = hv[i];
  }
#pragma unroll
  for (int j = 0; j < NLA; ++j) aslot[tid + 256 * j] = ra[0][j];
  __syncthreads();

  h8 hb[2][PB];  // halo batch registers (loaded at tap t, stored at tap t + 1)
  for (int c = 0; c < spt; ++c) {
    const h8* hcur = halo + (c & 1) * NB;
    h8* const hnext = halo + ((c + 1) & 1) * NB;
    const bool more = c + 1 < spt;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int s = c * 9 + tap;
      const int ky = tap / 3, kx = tap - ky * 3;
      // A(s + 2) -> registers (the packed weights carry >= 8 zero steps past the last: no guard)
#pragma unroll
      for (int j = 0; j < NLA; ++j) ra[(tap + 2) % 3][j] = asrc[j][size_t(s + 2) * 64];
      // next chunk's halo: batch `tap` issued now, stored at tap + 1
      if (more && tap < 8) {
#pragma unroll
        for (int b = 0; b < PB; ++b) {
          const int i = tap * PB + b;
          if (i < NL) hb[tap & 1][b] = *hsrc(i, c + 1);
        }
      }
      // this step's fragments and MFMAs
      const h8* as = aslot + (tap % 3) * (AT * 64) + (wc * 4) * 64 + lane;
      h8 af[4], bf[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) af[r] = as[r * 64];
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const int ry = (wr * 4 + p) * S + ky;
        const int u = ry * CI + tile_col<S, CI>(col * S + kx);
        bf[p] = hcur[u * 4 + (grp ^ ((u >> 1) & 3))];
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int p = 0; p < 4; ++p)
          acc[r][p] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[r], bf[p], acc[r][p], 0, 0, 0);
      // A(s + 1) -> its slot (last read at step s - 2), the previous halo batch -> the other buffer
      if (s + 1 < nst) {
#pragma unroll
        for (int j = 0; j < NLA; ++j) aslot[((tap + 1) % 3) * (AT * 64) + tid + 256 * j] = ra[(tap + 1) % 3][j];
      }
      if (more && tap > 0) {
#pragma unroll
        for (int b = 0; b < PB; ++b) {
          const int i = (tap - 1) * PB + b;
          if (i < NL) hnext[hslot[i]] = hb[(tap - 1) & 1][b];
        }
      }
      __syncthreads();
    }
  }
  tile3_store<4, 4>(a, acc, n, oy0 + wr * 4, ox0, ct_blk + wc * 4, col, grp);
}

template <int S, int CW>
static int launch_wide_k(const ConvArgs& a, dim3 grid, hipStream_t s) {
  constexpr size_t lds = WideGeom<S, CW>::lds;
  static_assert(lds <= 160 * 1024, "wide 3x3 tile: LDS over 160 KiB");
  static const bool big = hipFuncSetAttribute(reinterpret_cast<const void*>(&conv3x3_wide_kernel<S, CW>),
                                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
  if (!big) return fail(FCE_ERR_HIP, "conv 3x3 wide tile: cannot opt in to >64 KiB LDS");
  FCE_LAUNCH((conv3x3_wide_kernel<S, CW>), grid, dim3(256), lds, s, a);
  return FCE_OK;
}

bool wide3_ok(int stride, int cw) { return stride == 1 ? (cw == 1 || cw == 2 || cw == 4) : stride == 2 && cw == 2; }

int launch_wide3(const ConvArgs& a, int cw, int stride, int n, hipStream_t s) {
  FCE_CHECK(wide3_ok(stride, cw) && a.cin % 32 == 0 && a.up == 0, "conv 3x3 wide tile: bad configuration");
  const int th = (4 / cw) * 4;
  const int64_t tiles = int64_t((a.Wo + 15) / 16) * ((a.Ho + th - 1) / th) * n;
  ConvArgs b = a;
  b.gy = ((a.cout + 15) / 16 + cw * 4 - 1) / (cw * 4);
  FCE_CHECK(tiles * b.gy < (int64_t(1) << 31), "conv 3x3 wide tile: grid too large");
  FCE_CHECK(a.Hs * a.Ws * int64_t(a.xcs) < (int64_t(1) << 31), "conv 3x3 wide tile: image too large");
  const dim3 grid(unsigned(tiles * b.gy));
  int rc;
  if (stride == 1)
    rc = cw == 1 ? launch_wide_k<1, 1>(b, grid, s) : cw == 2 ? launch_wide_k<1, 2>(b, grid, s) : launch_wide_k<1, 4>(b, grid, s);
  else  // stride 2: cw 2 only (cw 1 / 4 spill: 18 halo pieces per thread / 3 x 4 A pieces in registers)
    rc = launch_wide_k<2, 2>(b, grid, s);
  if (rc != FCE_OK) return rc;
  return launch_status("conv3x3_wide_kernel");
}

}  // namespace fce
