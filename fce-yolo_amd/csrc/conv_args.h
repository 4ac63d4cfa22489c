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
#pragma unroll
  for (int r = 0; r < RC; ++r) {
    const int co0 = (cot0 + r) * 16 + grp * 4;
    if (cot0 + r >= cotiles || co0 >= a.cout) continue;
    float bz[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bz[j] = (co0 + j < a.cout) ? a.bias[co0 + j] : 0.f;
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
      if (a.res) {
        const _Float16* ro = a.res + pix * a.rcs + co0;
        if (a.vec_ok && co0 + 3 < a.cout) {
          const h4 rv = *reinterpret_cast<const h4*>(ro);
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = fpin(v[j] + (float)rv[j]);
        } else {
          for (int j = 0; j < 4; ++j)
            if (co0 + j < a.cout) v[j] = fpin(v[j] + (float)ro[j]);
        }
      }
      if (a.vec_ok && co0 + 3 < a.cout) {
        *reinterpret_cast<h4*>(yo) = h4{(_Float16)fpin(v[0]), (_Float16)fpin(v[1]), (_Float16)fpin(v[2]), (_Float16)fpin(v[3])};
      } else {
        for (int j = 0; j < 4; ++j)
          if (co0 + j < a.cout) yo[j] = (_Float16)fpin(v[j]);
      }
    }
  }
}

// Big-tile LDS-DMA 3x3 configurations (conv3x3_big.hip), coded 0x800 | wm << 4 | (ab - 2) << 12: wm waves along
// the couts, ab weight-stage buffers, 4 waves per block (8-wave blocks were measured and dropped);
// stride 2 needs wm 2 (LDS)
static constexpr bool big3_ok(int s, int wm, int ab, int nw = 4) {
  return nw == 4 && (ab == 2 || ab == 3) && (s == 1 ? (wm == 1 || wm == 2) : wm == 2);
}
int launch_big3(const ConvArgs& a, int wm, int ab, int nw, int stride, int n, hipStream_t s);
// Wide-tile 3x3 (conv3x3_wide.hip), coded 0xA00 | log2(cw) << 4: 64 cw couts x 16 (4 / cw) rows per block
bool wide3_ok(int stride, int cw);
int launch_wide3(const ConvArgs& a, int cw, int stride, int n, hipStream_t s);

}  // namespace fce
