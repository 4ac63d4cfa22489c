// Fused C3k2 block (reference ultralytics/nn/modules/block.py C2f.forward :303-307 with C3k2's
// Bottleneck branch :1064-1084, Bottleneck.forward :474-476): for c3k = False and one repeat,
//
//   t = SiLU(cv1(x))            1x1, cin -> 2c          t = [a | b]
//   h = SiLU(m.cv1(b))          3x3, c -> c_mid
//   m = SiLU(m.cv2(h)) + b      3x3, c_mid -> c   (shortcut)
//   y = SiLU(cv2([a | b | m]))  1x1, 3c -> cout
//
// in ONE kernel per 8 x 16 output tile (8 waves): x is read once (with a 2-pixel halo), t / h / m never leave
// LDS, y is written once.  At the n scale (C3k2 at 160^2 and 80^2, 16-64 channels) the four separate
// convs are HBM round trips of small tensors plus four launch tails; fused, the block is one read of x
// and one write of y.
//
// Bitwise identical to the four unfused convs (conv_mfma_kernel and its variants): every stage walks
// the same K-steps of the same packed A fragments (conv_pack: chunk-major for cin % 32 == 0, else
// tap-major 8-channel chunks c = 4 s + lane / 16) with v_mfma_f32_16x16x32_f16 from zero, the B data
// are the same fp16 values (intermediates rounded to fp16 exactly where the unfused path stores them,
// zeros where it zero-pads), and the epilogue arithmetic is conv_epilogue's (bias, SiLU, residual add,
// fpin before every fp16 conversion).
#include "common.h"

namespace fce {

struct FStage {
  const h8* w;      // packed A fragments (conv_pack layout)
  const float* b;   // bias (BN folded)
  int cin, cout, taps, fast, cpt, nsteps, nalloc, cotiles;
};

struct C3k2Args {
  const _Float16* x;
  int xcs;
  _Float16* y;
  int ycs;
  int N, H, W;
  int c, c2;
  FStage st[4];
  int tiles_x, tiles_y;
  int sx, sy, sh;  // LDS row strides (16-byte units) of the x, t|m and h images: odd, so 16 consecutive
                   // positions meet 16 distinct 16-byte slots of a bank row (conflict-free B gathers)
  int xh_off;      // 16-byte offset of the x / h image (h reuses x's space: x is dead after stage 1)
};

constexpr int FT_H = 8, FT_W = 16;
constexpr int R2H = FT_H + 4, R2W = FT_W + 4;  // cv1 output region: tile + 2-pixel halo (two 3x3 convs)
constexpr int R1H = FT_H + 2, R1W = FT_W + 2;  // m.cv1 output region: tile + 1-pixel halo
constexpr int NR2 = R2H * R2W, NR1 = R1H * R1W, NCORE = FT_H * FT_W;

constexpr int FNW = 4;  // waves per block (several blocks per CU overlap each other's stage barriers)

// One stage: outputs at `npos` positions of a region OW wide, read from the LDS image `in` (row stride
// sin, first channel chunk coff8) of a region IW wide (3x3: output (r, c) reads input (r + ky, c + kx);
// 1x1: input (r + off, c + off)).  Wave w owns the 16-position fragments w, w + FNW (<= MAXF of them)
// and all cout tiles; the K loop walks the packed steps with the A fragments of step s + 1 in flight
// while step s's MFMAs run (one L2 latency per stage, not one per step and fragment).
// epi(q, co0, v[4]) gets the 4 SiLU'd fp32 outputs of lane group grp.
template <int MAXCT, int MAXF, typename Epi>
__device__ __forceinline__ void fstage(const FStage& s, const h8* in, int sin, int coff8, int IW, int npos, int OW,
                                       int off, Epi epi) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, col = lane & 15, grp = lane >> 4;
  const int nfr = (npos + 15) >> 4;
  if (wave >= nfr) return;  // wave-uniform
  int base[MAXF];
#pragma unroll
  for (int i = 0; i < MAXF; ++i) {
    const int q = min((wave + FNW * i) * 16 + col, npos - 1);
    const int qr = q / OW, qc = q - qr * OW;
    base[i] = s.taps == 9 ? qr * IW + qc : (qr + off) * IW + (qc + off);
  }
  f4 acc[MAXF][MAXCT];
#pragma unroll
  for (int i = 0; i < MAXF; ++i)
#pragma unroll
    for (int ct = 0; ct < MAXCT; ++ct) acc[i][ct] = f4{0.f, 0.f, 0.f, 0.f};
  const h8* wl = s.w + lane;
  h8 ac[MAXCT], an[MAXCT];
#pragma unroll
  for (int ct = 0; ct < MAXCT; ++ct)
    if (ct < s.cotiles) ac[ct] = wl[(size_t(ct) * s.nalloc) * 64];
  for (int st = 0; st < s.nsteps; ++st) {
    const int sn = st + 1 < s.nsteps ? st + 1 : st;
#pragma unroll
    for (int ct = 0; ct < MAXCT; ++ct)
      if (ct < s.cotiles) an[ct] = wl[(size_t(ct) * s.nalloc + sn) * 64];
    int tap, c8;
    bool ok;
    if (s.fast) {  // step = 32-channel chunk * taps + tap
      const int ch = st / s.taps;
      tap = st - ch * s.taps;
      c8 = ch * 4 + grp;
      ok = true;
    } else {  // 8-channel chunk c = 4 step + lane group, tap-major
      const int cc = st * 4 + grp;
      tap = cc / s.cpt;
      c8 = cc - tap * s.cpt;
      ok = tap < s.taps;
    }
    const int ky = (tap * 11) >> 5, kx = tap - ky * 3;  // tap / 3 for tap < 9
    const int toff = s.taps == 9 ? ky * IW + kx : 0;
#pragma unroll
    for (int i = 0; i < MAXF; ++i) {
      if (wave + FNW * i >= nfr) break;
      const h8 bf = ok ? in[(base[i] + toff) * sin + coff8 + c8] : h8{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int ct = 0; ct < MAXCT; ++ct)
        if (ct < s.cotiles) acc[i][ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ac[ct], bf, acc[i][ct], 0, 0, 0);
    }
#pragma unroll
    for (int ct = 0; ct < MAXCT; ++ct) ac[ct] = an[ct];
  }
#pragma unroll
  for (int i = 0; i < MAXF; ++i) {
    const int qq = (wave + FNW * i) * 16 + col;
    if (wave + FNW * i >= nfr || qq >= npos) continue;
#pragma unroll
    for (int ct = 0; ct < MAXCT; ++ct) {
      const int co0 = ct * 16 + grp * 4;
      if (ct >= s.cotiles || co0 >= s.cout) continue;
      float v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float t = acc[i][ct][j] + s.b[co0 + j];
        v[j] = silu(t);
      }
      epi(qq, co0, v);
    }
  }
}

__device__ __forceinline__ h4 to_h4(const float (&v)[4]) {
  return h4{(_Float16)fpin(v[0]), (_Float16)fpin(v[1]), (_Float16)fpin(v[2]), (_Float16)fpin(v[3])};
}

template <int MAXCT>
__global__ __launch_bounds__(FNW * 64) void c3k2_fused_kernel(C3k2Args a) {
  extern __shared__ __attribute__((aligned(16))) h8 fsm[];
  h8* Y = fsm;              // [NR2][sy]: a | b | m (m at the core positions only)
  h8* XH = fsm + a.xh_off;  // [NR2][sx] x, then [NR1][sh] h
  int t = blockIdx.x;
  const int tx = t % a.tiles_x;
  t /= a.tiles_x;
  const int ty = t % a.tiles_y;
  const int n = t / a.tiles_y;
  const int y0 = ty * FT_H, x0 = tx * FT_W;
  const int c8 = a.c / 8;

  // stage 0: x over the 2-pixel-halo region, zeros outside the image
  {
    const int cpt = a.st[0].cpt, np = NR2 * cpt;
    for (int e = threadIdx.x; e < np; e += FNW * 64) {
      const int p = e / cpt, cc = e - p * cpt;
      const int r = p / R2W, q = p - r * R2W;
      const int iy = y0 - 2 + r, ix = x0 - 2 + q;
      h8 v = h8{0, 0, 0, 0, 0, 0, 0, 0};
      if (iy >= 0 && iy < a.H && ix >= 0 && ix < a.W)
        v = *reinterpret_cast<const h8*>(a.x + nhwc_off(n, iy, ix, a.H, a.W, a.xcs) + cc * 8);
      XH[p * a.sx + cc] = v;
    }
  }
  __syncthreads();
  // stage 1: t = cv1(x) over the region; 0 outside the image (the 3x3 convs' zero padding of b)
  fstage<MAXCT, (NR2 + 16 * FNW - 1) / (16 * FNW)>(a.st[0], XH, a.sx, 0, R2W, NR2, R2W, 0, [&](int q, int co0, float (&v)[4]) {
    const int r = q / R2W, cq = q - r * R2W;
    const int iy = y0 - 2 + r, ix = x0 - 2 + cq;
    const bool in = iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
    h4 o = to_h4(v);
    if (!in) o = h4{0, 0, 0, 0};
    *reinterpret_cast<h4*>(reinterpret_cast<_Float16*>(Y + q * a.sy) + co0) = o;
  });
  __syncthreads();
  // stage 2: h = m.cv1(b) over the 1-pixel-halo region; 0 outside the image
  fstage<MAXCT, (NR2 + 16 * FNW - 1) / (16 * FNW)>(a.st[1], Y, a.sy, c8, R2W, NR1, R1W, 0, [&](int q, int co0, float (&v)[4]) {
    const int r = q / R1W, cq = q - r * R1W;
    const int iy = y0 - 1 + r, ix = x0 - 1 + cq;
    const bool in = iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
    h4 o = to_h4(v);
    if (!in) o = h4{0, 0, 0, 0};
    *reinterpret_cast<h4*>(reinterpret_cast<_Float16*>(XH + q * a.sh) + co0) = o;
  });
  __syncthreads();
  // stage 3: m = m.cv2(h) + b over the tile, into t's third channel block
  fstage<MAXCT, (NR2 + 16 * FNW - 1) / (16 * FNW)>(a.st[2], XH, a.sh, 0, R1W, NCORE, FT_W, 0, [&](int q, int co0, float (&v)[4]) {
    const int r = q / FT_W, cq = q - r * FT_W;
    _Float16* yp = reinterpret_cast<_Float16*>(Y + ((r + 2) * R2W + cq + 2) * a.sy);
    const h4 rv = *reinterpret_cast<const h4*>(yp + a.c + co0);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = fpin(v[j] + (float)rv[j]);
    *reinterpret_cast<h4*>(yp + 2 * a.c + co0) = to_h4(v);
  });
  __syncthreads();
  // stage 4: y = cv2([a | b | m]) over the tile, to global
  fstage<MAXCT, (NR2 + 16 * FNW - 1) / (16 * FNW)>(a.st[3], Y, a.sy, 0, R2W, NCORE, FT_W, 2, [&](int q, int co0, float (&v)[4]) {
    const int r = q / FT_W, cq = q - r * FT_W;
    const int iy = y0 + r, ix = x0 + cq;
    if (iy < a.H && ix < a.W)
      *reinterpret_cast<h4*>(a.y + nhwc_off(n, iy, ix, a.H, a.W, a.ycs) + co0) = to_h4(v);
  });
}

static FStage make_stage(const fce_conv_desc& d, const void* w, const float* b) {
  FStage s;
  s.w = static_cast<const h8*>(w);
  s.b = b;
  s.cin = d.cin;
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

static size_t c3k2_lds_bytes(int cin, int c, int cm, int* sx, int* sy, int* sh, int* xh_off) {
  *sx = (cin / 8) | 1;
  *sy = (3 * c / 8) | 1;
  *sh = (cm / 8) | 1;
  *xh_off = NR2 * *sy;
  const int xh = std::max(NR2 * *sx, NR1 * *sh);
  return size_t(*xh_off + xh) * 16;
}

bool c3k2_fused_ok(const fce_c3k2_desc& d) {
  int sx, sy, sh, xo;
  return d.cin % 8 == 0 && d.c % 8 == 0 && d.c_mid % 8 == 0 && d.cout % 4 == 0 && 2 * d.c <= 128 &&
         d.c_mid <= 128 && d.c <= 128 && d.cout <= 128 && c3k2_lds_bytes(d.cin, d.c, d.c_mid, &sx, &sy, &sh, &xo) <= 160 * 1024;
}

int c3k2_fused(const fce_c3k2_desc& d, const fce_tensor& x, const fce_tensor& y, hipStream_t s) {
  FCE_CHECK(c3k2_fused_ok(d), "c3k2 fused: unsupported channel configuration");
  FCE_CHECK(x.layout == FCE_NHWC && y.layout == FCE_NHWC && x.dtype == FCE_F16 && y.dtype == FCE_F16,
            "c3k2 fused: NHWC f16 views");
  FCE_CHECK(x.c == d.cin && y.c == d.cout && x.n == y.n && x.h == y.h && x.w == y.w, "c3k2 fused: shape mismatch");
  FCE_CHECK(x.cstride % 8 == 0 && x.coff % 8 == 0 && y.cstride % 4 == 0 && y.coff % 4 == 0,
            "c3k2 fused: aligned channel slices");
  for (int i = 0; i < 4; ++i) FCE_CHECK(d.w[i] && d.b[i], "c3k2 fused: null weights");
  const fce_conv_desc c1{d.cin, 2 * d.c, 1, 1, 1, FCE_ACT_SILU, 0, FCE_EPI_STORE, nullptr, 0, 0};
  const fce_conv_desc m1{d.c, d.c_mid, 3, 1, 1, FCE_ACT_SILU, 0, FCE_EPI_STORE, nullptr, 0, 0};
  const fce_conv_desc m2{d.c_mid, d.c, 3, 1, 1, FCE_ACT_SILU, 0, FCE_EPI_STORE, nullptr, 0, 0};
  const fce_conv_desc c2{3 * d.c, d.cout, 1, 1, 1, FCE_ACT_SILU, 0, FCE_EPI_STORE, nullptr, 0, 0};
  C3k2Args a;
  a.x = static_cast<const _Float16*>(x.data) + x.coff;
  a.xcs = x.cstride;
  a.y = static_cast<_Float16*>(y.data) + y.coff;
  a.ycs = y.cstride;
  a.N = x.n;
  a.H = x.h;
  a.W = x.w;
  a.c = d.c;
  a.c2 = d.cout;
  a.st[0] = make_stage(c1, d.w[0], d.b[0]);
  a.st[1] = make_stage(m1, d.w[1], d.b[1]);
  a.st[2] = make_stage(m2, d.w[2], d.b[2]);
  a.st[3] = make_stage(c2, d.w[3], d.b[3]);
  a.tiles_x = (x.w + FT_W - 1) / FT_W;
  a.tiles_y = (x.h + FT_H - 1) / FT_H;
  const size_t lds = c3k2_lds_bytes(d.cin, d.c, d.c_mid, &a.sx, &a.sy, &a.sh, &a.xh_off);
  const int64_t blocks = int64_t(a.tiles_x) * a.tiles_y * x.n;
  if (blocks == 0) return FCE_OK;
  FCE_CHECK(blocks < (int64_t(1) << 31), "c3k2 fused: grid too large");
  int maxct = 0;
  for (const FStage& st : a.st) maxct = std::max(maxct, st.cotiles);
  if (maxct <= 4) {  // fewer accumulator / fragment registers: more blocks per CU
    static const bool big = hipFuncSetAttribute(reinterpret_cast<const void*>(&c3k2_fused_kernel<4>),
                                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
    if (!big && lds > 64 * 1024) return fail(FCE_ERR_HIP, "c3k2 fused: cannot opt in to >64 KiB LDS");
    FCE_LAUNCH(c3k2_fused_kernel<4>, dim3(unsigned(blocks)), dim3(FNW * 64), lds, s, a);
  } else {
    static const bool big = hipFuncSetAttribute(reinterpret_cast<const void*>(&c3k2_fused_kernel<8>),
                                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
    if (!big && lds > 64 * 1024) return fail(FCE_ERR_HIP, "c3k2 fused: cannot opt in to >64 KiB LDS");
    FCE_LAUNCH(c3k2_fused_kernel<8>, dim3(unsigned(blocks)), dim3(FNW * 64), lds, s, a);
  }
  return launch_status("c3k2_fused_kernel");
}

}  // namespace fce
