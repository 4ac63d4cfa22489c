// Convolutions for gfx950: MFMA implicit GEMM (dense 1x1 / 3x3), depthwise 3x3, and the
// Cin<=4 stem that reads the NCHW network input directly.
//
// Replaces (reference, ultralytics/): nn/modules/conv.py:39-89 Conv.forward_fuse with the BN
// folded by utils/torch_utils.py:237-267; conv.py:185-200 DWConv; the Detect 1x1 nn.Conv2d
// (head.py:86-107); Bottleneck's residual add (block.py:474-476); torch.cat / chunk of
// C2f / C3 / SPPF / C2PSA (block.py:303-307, 338-340, 228-232, 1453-1464) through channel-offset
// reads and writes; nn.Upsample(x2, nearest) feeding a 1x1 conv through `up`.
//
// Data layout: activations NHWC fp16, any view may be a channel slice of a wider buffer.
// Dense conv as GEMM  D[cout][pixel] = sum_k W[cout][k] * X[k][pixel],  k = (tap, cin):
//   v_mfma_f32_16x16x32_f16 with A = weights (16 couts x 32 k), B = activations (32 k x 16 px).
//   Lane l owns A[co = l&15][k = 8(l>>4)+j] and B[k = 8(l>>4)+j][px = l&15]: one 16-byte load
//   of 8 consecutive input channels of one pixel (coalesced along NHWC) per fragment; the
//   weight fragments are pre-packed in exactly this lane order (1 KiB per fragment).
//   D: lane l holds px = l&15, couts 4(l>>4)+0..3  -> 8-byte NHWC stores.
#include <type_traits>

#include "conv_args.h"

namespace fce {

// ============================================================================ packing (host)
// nsteps K-steps of 32 (4 chunks of 8 input channels); each cout tile stores nalloc >= nsteps
// fragments: rounded up to a multiple of 8 (the main loop consumes steps in groups of its pipeline
// depth D <= 8) + 8 zero fragments, so the branch-free prefetch D steps ahead never reads past the
// image.
struct DenseGeom {
  int cpt, taps, nchunk, nsteps, nalloc, cotiles;
};
static DenseGeom dense_geom(const fce_conv_desc& d) {
  DenseGeom g;
  g.cpt = d.cin / 8;
  g.taps = d.k * d.k;
  g.nchunk = g.taps * g.cpt;
  g.nsteps = (g.nchunk + 3) / 4;
  g.nalloc = ((g.nsteps + 7) & ~7) + 8;
  g.cotiles = (d.cout + 15) / 16;
  return g;
}

static bool is_stem(const fce_conv_desc& d) { return d.groups == 1 && d.cin <= 4; }
static bool is_dw(const fce_conv_desc& d) { return d.groups > 1; }

// 3x3 stems with cin * 9 <= 32 also carry one MFMA K-step of fp16 fragments (k = ci * 9 + tap, zero
// padded to 32) per 16-cout tile after the fp32 table: the stem_mfma_kernel's A operand
static bool stem_mfma_ok(const fce_conv_desc& d) { return d.k == 3 && d.cin * 9 <= 32 && d.cout <= 64; }
static size_t stem_fp32_bytes(const fce_conv_desc& d) { return size_t(d.cin) * d.k * d.k * d.cout * sizeof(float); }

size_t conv_weight_bytes(const fce_conv_desc& d) {
  if (is_stem(d))  // [cin*k*k][cout] fp32 (+ MFMA fragments)
    return stem_fp32_bytes(d) + (stem_mfma_ok(d) ? size_t((d.cout + 15) / 16) * 64 * 8 * sizeof(_Float16) : 0);
  if (is_dw(d)) return size_t(d.k) * d.k * d.cin * sizeof(float);             // [k*k][c] fp32
  DenseGeom g = dense_geom(d);
  return size_t(g.cotiles) * g.nalloc * 64 * 8 * sizeof(_Float16);
}

int conv_pack(const fce_conv_desc& d, const float* w, void* out) {
  const int k = d.k, kk = k * k;
  if (is_stem(d)) {  // [ci][ky][kx][co]
    float* o = static_cast<float*>(out);
    for (int co = 0; co < d.cout; ++co)
      for (int ci = 0; ci < d.cin; ++ci)
        for (int t = 0; t < kk; ++t) o[(ci * kk + t) * d.cout + co] = w[(co * d.cin + ci) * kk + t];
    if (stem_mfma_ok(d)) {  // lane l of tile ct: cout ct*16 + (l & 15), k = 8 (l >> 4) + j
      _Float16* f = reinterpret_cast<_Float16*>(static_cast<char*>(out) + stem_fp32_bytes(d));
      for (int ct = 0; ct < (d.cout + 15) / 16; ++ct)
        for (int l = 0; l < 64; ++l)
          for (int j = 0; j < 8; ++j) {
            const int co = ct * 16 + (l & 15), kq = 8 * (l >> 4) + j;
            f[(ct * 64 + l) * 8 + j] = (_Float16)((co < d.cout && kq < d.cin * 9) ? w[co * d.cin * 9 + kq] : 0.f);
          }
    }
    return FCE_OK;
  }
  if (is_dw(d)) {  // [t][c]
    float* o = static_cast<float*>(out);
    for (int c = 0; c < d.cin; ++c)
      for (int t = 0; t < kk; ++t) o[t * d.cin + c] = w[c * kk + t];
    return FCE_OK;
  }
  // K-step order: cin % 32 == 0 -> chunk-major, step s = (32-channel chunk) * k*k + tap (the order
  // of the LDS-tile 3x3 kernel, so both kernels sum every output in the same order); otherwise
  // 8-channel chunks c = 4s + lane/16 in tap-major order (tap = c / (cin/8)).
  DenseGeom g = dense_geom(d);
  const bool chunk_major = d.cin % 32 == 0;
  _Float16* o = static_cast<_Float16*>(out);
  for (int ct = 0; ct < g.cotiles; ++ct)
    for (int s = 0; s < g.nalloc; ++s)
      for (int l = 0; l < 64; ++l) {
        const int co = ct * 16 + (l & 15);
        _Float16* dst = o + ((size_t(ct) * g.nalloc + s) * 64 + l) * 8;
        int tap, ci0;
        bool in;
        if (chunk_major) {
          tap = s % kk;
          ci0 = (s / kk) * 32 + (l >> 4) * 8;
          in = s < g.nsteps;
        } else {
          const int c = s * 4 + (l >> 4);
          tap = c / g.cpt;
          ci0 = (c % g.cpt) * 8;
          in = c < g.nchunk;
        }
        for (int j = 0; j < 8; ++j) {
          float v = 0.f;
          if (co < d.cout && in) v = w[(size_t(co) * d.cin + ci0 + j) * kk + tap];
          dst[j] = (_Float16)v;
        }
      }
  return FCE_OK;
}

// ============================================================================ dense MFMA kernel
// Software-pipeline depth: K-steps of fragments in flight per wave.  Small register tiles have little
// MFMA work per step to cover a load's latency, so they keep more steps in flight (the summation
// order over K is the same for every depth).
template <int RC, int RP>
struct ConvDepth {
  static constexpr int D = RC * RP == 1 ? 8 : RC * RP == 2 ? 4 : 2;
};

// conv_epilogue (the dense MFMA kernels' epilogue) lives in conv_args.h, shared with conv_big.hip

template <int KS, int RC, int RP, int OUT, bool FAST>
__global__ __launch_bounds__(256) void conv_mfma_kernel(ConvArgs a) {
  constexpr int D = ConvDepth<RC, RP>::D;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int col = lane & 15;
  const int grp = lane >> 4;
  // XCD-aware block order.  The grid is 1-D (gx pixel tiles x gy cout tiles); the hardware deals
  // block b to XCD b % 8.  Remap so each XCD owns one contiguous range of logical tiles
  // (pixel-tile major, cout tile minor): the cout tiles that re-read a pixel tile's input, and the
  // neighbouring pixel tiles sharing its 3x3 halo rows, run on the same XCD and hit its L2.
  int bx, by;
  {
    const int total = a.gx * a.gy, b = blockIdx.x;
    const int per = total >> 3, body = per << 3;
    const int L = b < body ? (b & 7) * per + (b >> 3) : b;
    bx = L / a.gy;
    by = L - bx * a.gy;
  }
  const int pix_base = (bx * 4 + wave) * (RP * 16);
  const int cot0 = by * RC;
  const int cotiles = (a.cout + 15) >> 4;

  // Per pixel-rep (this lane's B column): element offset of the tap-(0,0) source pixel, and a
  // bit mask of the taps that fall inside the image (zero padding = the other taps).  Computed
  // once, so a B load in the K loop costs a bit test, a 64-bit add and a pointer select.
  int64_t pbase[RP];
  unsigned vmask[RP];
#pragma unroll
  for (int p = 0; p < RP; ++p) {
    int pix = pix_base + p * 16 + col;
    const bool pv = pix < a.P;
    pix = pv ? pix : 0;
    const int hw = a.Ho * a.Wo;
    const int n = pix / hw;
    const int r = pix - n * hw;
    const int iy0 = (r / a.Wo) * a.stride - (KS / 2);
    const int ix0 = (r % a.Wo) * a.stride - (KS / 2);
    unsigned m = 0;
#pragma unroll
    for (int t = 0; t < KS * KS; ++t) {
      const int iy = iy0 + t / KS, ix = ix0 + t % KS;
      m |= unsigned(pv && iy >= 0 && iy < a.Hin && ix >= 0 && ix < a.Win) << t;
    }
    vmask[p] = m;
    // KS == 3 requires up == 0 (host materialises upsampled inputs first)
    pbase[p] = KS == 1 ? nhwc_off(n, iy0 >> a.up, ix0 >> a.up, a.Hs, a.Ws, a.xcs)
                       : (int64_t(n) * a.Hs + iy0) * a.Ws * int64_t(a.xcs) + int64_t(ix0) * a.xcs;
  }

  f4 acc[RC][RP];
#pragma unroll
  for (int r = 0; r < RC; ++r)
#pragma unroll
    for (int p = 0; p < RP; ++p) acc[r][p] = f4{0.f, 0.f, 0.f, 0.f};

  // Branch-free K loop: an out-of-image tap or padded K chunk loads a 16-byte zero line (address
  // select, never a value mask), so no load is conditional and hipcc places counted vmcnt waits;
  // D K-steps of fragments stay in flight (a ring of D register sets, unrolled: static indices).
  // FAST (cin % 32 == 0): a K-step is 32 channels of ONE tap, ordered chunk-major (step =
  // chunk * taps + tap, see conv_pack), so the (chunk, tap) cursor is wave-uniform (scalar).
  // Otherwise each lane decodes its chunk c = 4s+grp with a magic divide.
  const h8* wfrag[RC];
#pragma unroll
  for (int r = 0; r < RC; ++r) {
    const int ct = min(cot0 + r, cotiles - 1);
    wfrag[r] = reinterpret_cast<const h8*>(a.w) + (size_t(ct) * a.nalloc) * 64 + lane;
  }
  const h8* zline = reinterpret_cast<const h8*>(g_zero_line);
  const int spt = a.cpt >> 2;  // 32-channel chunks (FAST)
  int lt = 0, ls = 0;          // load cursor: tap, chunk (FAST)
  auto tap_off = [&](int t) -> int64_t {
    const int ky = (t * 11) >> 5;  // t / 3 for t < 9
    return KS == 1 ? 0 : (int64_t(ky) * a.Ws + (t - ky * 3)) * a.xcs;
  };
  auto load_b = [&](int s, h8 (&b)[RP]) {
    int t, ce;  // tap and element offset within the pixel's channels
    bool tin;   // a real K-step (padded steps past the end load the zero line)
    if (FAST) {
      t = lt;
      ce = ls * 32 + grp * 8;
      tin = ls < spt;
      if (++lt == KS * KS) {
        lt = 0;
        ++ls;
      }
    } else {
      const unsigned c = unsigned(s * 4 + grp);
      t = a.cpt == 1 ? int(c) : int(__umulhi(c, a.cmagic));
      ce = (int(c) - t * a.cpt) * 8;
      tin = t < KS * KS;
    }
    const int64_t toff = tap_off(t) + ce;
#pragma unroll
    for (int p = 0; p < RP; ++p) {
      const bool ok = tin && ((vmask[p] >> (t & 31)) & 1u);
      const h8* src = ok ? reinterpret_cast<const h8*>(a.x + pbase[p] + toff) : zline;
      b[p] = *src;
    }
  };
  auto load_a = [&](int s, h8 (&w)[RC]) {  // past the last step: one broadcast zero line, not a 1 KiB fragment
    const bool in = s < a.nsteps;
#pragma unroll
    for (int r = 0; r < RC; ++r) w[r] = *(in ? wfrag[r] + s * 64 : zline);
  };
  h8 bq[D][RP], aq[D][RC];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    load_b(d, bq[d]);
    load_a(d, aq[d]);
  }
  const int full = a.nsteps - a.nsteps % D;
  for (int s = 0; s < full; s += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
#pragma unroll
      for (int r = 0; r < RC; ++r)
#pragma unroll
        for (int p = 0; p < RP; ++p)
          acc[r][p] = __builtin_amdgcn_mfma_f32_16x16x32_f16(aq[d][r], bq[d][p], acc[r][p], 0, 0, 0);
      load_b(s + D + d, bq[d]);  // reads at most step nsteps + D - 1 < nalloc (zero padded)
      load_a(s + D + d, aq[d]);
    }
  }
  // tail: steps full .. nsteps-1 already sit in ring slots 0 .. rem-1
#pragma unroll
  for (int d = 0; d < D; ++d) {
    if (d < a.nsteps - full) {
#pragma unroll
      for (int r = 0; r < RC; ++r)
#pragma unroll
        for (int p = 0; p < RP; ++p)
          acc[r][p] = __builtin_amdgcn_mfma_f32_16x16x32_f16(aq[d][r], bq[d][p], acc[r][p], 0, 0, 0);
    }
  }

  // ---------------------------------------------------------------- epilogue
  conv_epilogue<RC, RP, OUT>(a, acc, pix_base, cot0, col, grp);
}

// ============================================================================ 1x1, streaming waves
// For 1x1 convs with cin % 32 == 0 and few K-steps (cin <= 32 * NSM): in the implicit-GEMM kernel a
// wave then does a handful of MFMAs behind one load latency and exits.  Here a wave keeps the weight
// fragments of its RC cout tiles for ALL K-steps in registers (loaded once) and walks a strided
// sequence of pixel tiles (RP x 16 pixels), the next tile's B fragments in flight while the current
// tile's MFMAs and epilogue run.  Waves gw of a launch: cout group gw % gy, tile sequence
// gw / gy, + W, + 2W, ...  (adjacent waves = the cout groups of the same pixels, on one CU).  Per
// output the K order is the implicit-GEMM kernel's (steps 0..nsteps-1): bitwise-identical results.
template <int RC, int RP, int NSM, int OUT>
__global__ __launch_bounds__(256) void conv1x1_stream_kernel(ConvArgs a, int W) {
  const int lane = threadIdx.x & 63, col = lane & 15, grp = lane >> 4;
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int g = gw % a.gy, i0 = gw / a.gy;
  const int ns = a.nsteps;
  const int cot0 = g * RC;
  const int cotiles = (a.cout + 15) >> 4;
  const int ntiles = (a.P + 16 * RP - 1) / (16 * RP);
  h8 aw[NSM][RC];
#pragma unroll
  for (int r = 0; r < RC; ++r) {
    const h8* wf = reinterpret_cast<const h8*>(a.w) + (size_t(min(cot0 + r, cotiles - 1)) * a.nalloc) * 64 + lane;
#pragma unroll
    for (int st = 0; st < NSM; ++st) aw[st][r] = st < ns ? wf[st * 64] : h8{0, 0, 0, 0, 0, 0, 0, 0};
  }
  const int hw = a.Ho * a.Wo;
  auto load_tile = [&](int t, h8 (&b)[NSM][RP]) {
#pragma unroll
    for (int p = 0; p < RP; ++p) {
      int pix = t * 16 * RP + p * 16 + col;
      pix = pix < a.P ? pix : 0;  // past the end: any valid pixel (the epilogue skips it)
      const int n = pix / hw, r = pix - n * hw;
      const int oy = r / a.Wo, ox = r - oy * a.Wo;
      const _Float16* src = a.x + nhwc_off(n, oy >> a.up, ox >> a.up, a.Hs, a.Ws, a.xcs) + grp * 8;
#pragma unroll
      for (int st = 0; st < NSM; ++st)
        if (st < ns) b[st][p] = *reinterpret_cast<const h8*>(src + st * 32);
    }
  };
  h8 bq[NSM][RP];
  if (i0 < ntiles) load_tile(i0, bq);
  for (int t = i0; t < ntiles; t += W) {
    h8 bc[NSM][RP];
#pragma unroll
    for (int st = 0; st < NSM; ++st)
#pragma unroll
      for (int p = 0; p < RP; ++p) bc[st][p] = bq[st][p];
    if (t + W < ntiles) load_tile(t + W, bq);
    f4 acc[RC][RP];
#pragma unroll
    for (int r = 0; r < RC; ++r)
#pragma unroll
      for (int p = 0; p < RP; ++p) acc[r][p] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int st = 0; st < NSM; ++st) {
      if (st < ns) {
#pragma unroll
        for (int r = 0; r < RC; ++r)
#pragma unroll
          for (int p = 0; p < RP; ++p)
            acc[r][p] = __builtin_amdgcn_mfma_f32_16x16x32_f16(aw[st][r], bc[st][p], acc[r][p], 0, 0, 0);
      }
    }
    conv_epilogue<RC, RP, OUT>(a, acc, t * 16 * RP, cot0, col, grp);
  }
}

static bool stream_ok(int nsm, int rc, int rp) { return nsm * (rc + 2 * rp) <= 40; }

template <int RC, int RP, int NSM>
static void launch_stream_o(const ConvArgs& a, int out_kind, dim3 grid, int W, hipStream_t s) {
#define STREAM_L(O) FCE_LAUNCH((conv1x1_stream_kernel<RC, RP, NSM, O>), grid, dim3(256), 0, s, a, W)
  switch (out_kind) {
    case OUT_F16: STREAM_L(OUT_F16); break;
    case OUT_F32: STREAM_L(OUT_F32); break;
    case OUT_WSTORE: STREAM_L(OUT_WSTORE); break;
    case OUT_DFL: STREAM_L(OUT_DFL); break;
    case OUT_CLS: STREAM_L(OUT_CLS); break;
    default: STREAM_L(OUT_ACCUM); break;
  }
#undef STREAM_L
}

template <int NSM>
static void launch_stream_n(const ConvArgs& a, int out_kind, int rc, int rp, dim3 grid, int W, hipStream_t s) {
  if constexpr (NSM <= 4) {
    if (rc == 4 && rp == 2) return launch_stream_o<4, 2, NSM>(a, out_kind, grid, W, s);
    if (rc == 2 && rp == 2) return launch_stream_o<2, 2, NSM>(a, out_kind, grid, W, s);
    if (rc == 4 && rp == 1) return launch_stream_o<4, 1, NSM>(a, out_kind, grid, W, s);
  }
  if (rc == 1 && rp == 2) return launch_stream_o<1, 2, NSM>(a, out_kind, grid, W, s);
  if (rc == 2 && rp == 1) return launch_stream_o<2, 1, NSM>(a, out_kind, grid, W, s);
  launch_stream_o<1, 1, NSM>(a, out_kind, grid, W, s);
}

static int stream_nsm(int nsteps) { return nsteps <= 2 ? 2 : nsteps <= 4 ? 4 : nsteps <= 8 ? 8 : 0; }

// waves per cout group: enough pixel-tile streams to fill the GPU (about 8 waves per SIMD in all),
// but every wave gets at least 2 tiles so the prefetch has something to overlap
static int launch_stream(const ConvArgs& a0, int out_kind, int rc, int rp, hipStream_t s) {
  const int nsm = stream_nsm(a0.nsteps);
  FCE_CHECK(nsm > 0 && stream_ok(nsm, rc, rp), "conv 1x1 stream: K too deep for the register budget");
  ConvArgs a = a0;
  const int cotiles = (a.cout + 15) / 16;
  a.gy = (cotiles + rc - 1) / rc;
  const int ntiles = (a.P + 16 * rp - 1) / (16 * rp);
  int W = std::max(1, std::min((ntiles + 1) / 2, 8192 / a.gy));
  while ((int64_t(W) * a.gy) % 4) ++W;  // whole blocks of 4 waves
  const dim3 grid(unsigned(int64_t(W) * a.gy / 4));
  if (nsm == 2)
    launch_stream_n<2>(a, out_kind, rc, rp, grid, W, s);
  else if (nsm == 4)
    launch_stream_n<4>(a, out_kind, rc, rp, grid, W, s);
  else
    launch_stream_n<8>(a, out_kind, rc, rp, grid, W, s);
  return launch_status("conv1x1_stream_kernel");
}

// Staged fp16 store for the LDS-tile 1x1 kernels (OUT_F16 / OUT_WSTORE with a.stg): the block's output
// tile (TPB pixels x CB*16 couts) is assembled in LDS (`ot`, rows of CB*16 halves, 16-byte slot sl of
// pixel px at sl ^ (px & (2 CB - 1))) and written with 16-byte lane stores, whole pixel rows per 2 CB
// lanes, instead of 8-byte stores scattered over 16 pixels.  Values are computed exactly as in
// conv_epilogue (bias, SiLU, residual, BiFPN alpha, then one fp16 rounding): bitwise the same.
// Caller: every thread of the block, after the last B read of `ot`'s memory (barrier inside).
template <int RC, int RP, int CB, int TPB, int OUT>
__device__ __forceinline__ void conv_store_staged(const ConvArgs& a, f4 (&acc)[RC][RP], int pix0, int pw, int cbl0,
                                                  int wc, int col, int grp, _Float16* ot) {
  constexpr int ROW = CB * 16, NSL = 2 * CB;
  const int cotiles = (a.cout + 15) >> 4;
  float alpha = 1.f;
  if (OUT == OUT_WSTORE) alpha = fusion_alpha(a.fw, a.fn, a.fi);
#pragma unroll
  for (int r = 0; r < RC; ++r) {
    const int ctl = wc * RC + r;  // local cout tile
    const int co0 = (cbl0 + ctl) * 16 + grp * 4;
    if (cbl0 + ctl >= cotiles) continue;
    float bz[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bz[j] = bias_or0(a.bias, co0 + j, a.cout);
#pragma unroll
    for (int p = 0; p < RP; ++p) {
      const int px = pw + p * 16 + col, pix = pix0 + px;
      float v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float t = acc[r][p][j] + bz[j];
        v[j] = a.act ? silu(t) : t;
      }
      if (a.res && pix < a.P) {
        const _Float16* ro = a.res + int64_t(pix) * a.rcs + co0;
        if (a.vec_ok && co0 + 3 < a.cout) {
          const h4 rv = *reinterpret_cast<const h4*>(ro);
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = fpin(v[j] + (float)rv[j]);
        } else {
          for (int j = 0; j < 4; ++j)
            if (co0 + j < a.cout) v[j] = fpin(v[j] + (float)ro[j]);
        }
      }
      if (OUT == OUT_WSTORE) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = fpin(v[j] * alpha);
      }
      const int sl = ctl * 2 + (grp >> 1);
      *reinterpret_cast<h4*>(ot + px * ROW + ((sl ^ (px & (NSL - 1))) * 8) + (grp & 1) * 4) =
          h4{(_Float16)fpin(v[0]), (_Float16)fpin(v[1]), (_Float16)fpin(v[2]), (_Float16)fpin(v[3])};
    }
  }
  __syncthreads();
  constexpr int NP = TPB * NSL;  // 16-byte pieces of the tile
#pragma unroll
  for (int e0 = 0; e0 < NP; e0 += 256) {
    const int e = e0 + int(threadIdx.x);
    if (NP % 256 != 0 && e >= NP) break;
    const int px = e / NSL, sl = e - px * NSL;
    const int pix = pix0 + px, co = cbl0 * 16 + sl * 8;
    if (pix < a.P && co < a.cout) {
      const h8 hv = *reinterpret_cast<const h8*>(ot + px * ROW + (sl ^ (px & (NSL - 1))) * 8);
      *reinterpret_cast<h8*>(static_cast<_Float16*>(a.y) + int64_t(pix) * a.ycs + co) = hv;
      if (OUT == OUT_F16 && a.dup && co >= a.duplo && co < a.duplo + a.dupn)  // duplo, dupn % 8 == 0 (host)
        *reinterpret_cast<h8*>(a.dup + int64_t(pix) * a.dupcs + (co - a.duplo)) = hv;
    }
  }
}

// ============================================================================ 1x1, LDS-staged pixel tiles
// For 1x1 stride-1 convs (any cin % 8 == 0, optional fused nearest upsampling).  A block (4 waves)
// owns TPB = WP*RP*16 consecutive output pixels and CB = (4/WP)*RC cout tiles; wave (wc, wp) computes
// RC cout tiles x RP 16-pixel groups.  Per K chunk of NSC 32-channel steps the block stages its
// pixels' input rows in LDS with full-line loads (8 lanes = one pixel's 128-byte pair of steps) and
// every wave reads its B fragments from there, instead of each wave issuing fragment-shaped
// (16 pixels x 64 B) loads that re-read the input once per cout group.
// LDS image per pair of steps: [pixel][8 x 16 B]; piece j of pixel p sits in slot j ^ ((p >> 1) & 7).
// That is conflict-free for the staging ds_write_b128 (8 lanes = the 8 slots of one 128-B row) and
// for the B-fragment ds_read_b128 (each 16-lane group meets 16 distinct 16-B slots of the bank row).
// Channels past cin are staged as zeros.  A fragments, K-step contents and the per-output summation
// order are the implicit-GEMM kernel's, so the results are bitwise identical.
template <int RC, int RP, int WP, int NSC, int OUT>
__global__ __launch_bounds__(256) void conv1x1_lds_kernel(ConvArgs a) {
  constexpr int TPB = WP * RP * 16;
  constexpr int NPAIR = (NSC + 1) / 2;
  constexpr int NPC = TPB * NPAIR * 8;  // 16-byte pieces staged per chunk
  static_assert(NPC % 256 == 0, "whole staging rounds");
  constexpr int IT = NPC / 256;
  extern __shared__ __attribute__((aligned(16))) h8 xt[];  // [NPAIR][TPB][8]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = lane & 15, grp = lane >> 4;
  const int wc = wave / WP, wp = wave - wc * WP;
  int bx, by;  // XCD-aware order, as conv_mfma_kernel: a pixel tile's cout groups share an XCD's L2
  {
    const int total = a.gx * a.gy, b = blockIdx.x;
    const int per = total >> 3, body = per << 3;
    const int L = b < body ? (b & 7) * per + (b >> 3) : b;
    bx = L / a.gy;
    by = L - bx * a.gy;
  }
  const int pix0 = bx * TPB;
  const int cot0 = (by * (4 / WP) + wc) * RC;
  const int cotiles = (a.cout + 15) >> 4;
  const h8* wfrag[RC];
#pragma unroll
  for (int r = 0; r < RC; ++r) {
    const int ct = min(cot0 + r, cotiles - 1);
    wfrag[r] = reinterpret_cast<const h8*>(a.w) + (size_t(ct) * a.nalloc) * 64 + lane;
  }
  // staging: piece e = threadIdx.x + 256 i -> (pixel p = e / (8 NPAIR), pair q, piece j): a pixel's
  // chunk is contiguous in global memory, so consecutive lanes read consecutive 16-byte pieces
  int64_t soff[IT];
  int spos[IT], sch[IT];
  bool spv[IT];
  const int hw = a.Ho * a.Wo;
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int e = threadIdx.x + 256 * i;
    const int j = e & 7, rest = e >> 3;
    const int p = rest / NPAIR, q = rest - p * NPAIR;
    const int pix = pix0 + p;
    spv[i] = pix < a.P;
    const int pc = spv[i] ? pix : 0;
    if (a.up) {
      const int n = pc / hw, r = pc - n * hw;
      const int oy = r / a.Wo, ox = r - oy * a.Wo;
      soff[i] = nhwc_off(n, oy >> a.up, ox >> a.up, a.Hs, a.Ws, a.xcs);
    } else {
      soff[i] = int64_t(pc) * a.xcs;
    }
    sch[i] = q * 64 + j * 8;
    spos[i] = (q * TPB + p) * 8 + (j ^ ((p >> 1) & 7));
  }
  f4 acc[RC][RP];
#pragma unroll
  for (int r = 0; r < RC; ++r)
#pragma unroll
    for (int p = 0; p < RP; ++p) acc[r][p] = f4{0.f, 0.f, 0.f, 0.f};
  const int pw = wp * RP * 16;  // this wave's first pixel within the tile
  for (int k0 = 0; k0 < a.nsteps; k0 += NSC) {
    if (k0) __syncthreads();  // previous chunk's B reads done
    h8 af[NSC][RC];           // packed A is zero-padded past nsteps: always in bounds
#pragma unroll
    for (int s = 0; s < NSC; ++s)
#pragma unroll
      for (int r = 0; r < RC; ++r) af[s][r] = wfrag[r][(k0 + s) * 64];
    h8 v[IT];
    const int cbase = k0 * 32;
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int c = cbase + sch[i];
      const bool ok = spv[i] && c < a.cin;
      v[i] = *(ok ? reinterpret_cast<const h8*>(a.x + soff[i] + c) : reinterpret_cast<const h8*>(g_zero_line));
    }
#pragma unroll
    for (int i = 0; i < IT; ++i) xt[spos[i]] = v[i];
    __syncthreads();
    const int nsc = min(NSC, a.nsteps - k0);
#pragma unroll
    for (int s = 0; s < NSC; ++s) {
      if (s < nsc) {
        h8 bf[RP];
#pragma unroll
        for (int p = 0; p < RP; ++p) {
          const int px = pw + p * 16 + col;
          const int j = (s & 1) * 4 + grp;
          bf[p] = xt[((s >> 1) * TPB + px) * 8 + (j ^ ((px >> 1) & 7))];
        }
#pragma unroll
        for (int r = 0; r < RC; ++r)
#pragma unroll
          for (int p = 0; p < RP; ++p)
            acc[r][p] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[s][r], bf[p], acc[r][p], 0, 0, 0);
      }
    }
  }
  if constexpr (OUT == OUT_F16 || OUT == OUT_WSTORE) {
    if (a.stg) {
      __syncthreads();  // every wave's last B read done: the staging image becomes the output tile
      conv_store_staged<RC, RP, (4 / WP) * RC, TPB, OUT>(a, acc, pix0, pw, by * (4 / WP) * RC, wc, col, grp,
                                                         reinterpret_cast<_Float16*>(xt));
      return;
    }
  }
  conv_epilogue<RC, RP, OUT>(a, acc, pix0 + pw, cot0, col, grp);
}

// Source element offset of output pixel pix of a stride-1 1x1 conv (nearest upsampling folded in).

// 1x1 with the whole K (nsteps <= NSC <= 8) in one LDS image, as a persistent double-buffered ring:
// the same tile geometry, LDS image and fragment reads as conv1x1_lds_kernel, but each block walks a
// sequence of pixel tiles and issues the global loads of tile i+1 into registers before it computes
// and stores tile i, so HBM reads stay in flight through the MFMA and epilogue phases (one barrier per
// tile).  Block b: XCD b % 8, cout group by, slot; pixel tiles bx = xcd + 8 (slot + k nslot): the gy
// blocks that read the same pixel tiles sit on one XCD and walk them in step (L2 hits), and a block's
// cout group never changes, so its A fragments are loaded once.  Bitwise identical to the others.
template <int RC, int RP, int WP, int NSC, int OUT>
__global__ __launch_bounds__(256) void conv1x1_ring_kernel(ConvArgs a, int nslot) {
  constexpr int TPB = WP * RP * 16;
  constexpr int NPAIR = (NSC + 1) / 2;
  constexpr int BUF = NPAIR * TPB * 8;  // h8 per LDS buffer
  static_assert(BUF % 256 == 0, "whole staging rounds");
  constexpr int IT = BUF / 256;
  extern __shared__ __attribute__((aligned(16))) h8 xr[];  // [2][NPAIR][TPB][8]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = lane & 15, grp = lane >> 4;
  const int wc = wave / WP, wp = wave - wc * WP;
  const int xcd = blockIdx.x & 7, loc = blockIdx.x >> 3;
  const int by = loc % a.gy, slot = loc / a.gy;
  int bx = xcd + 8 * slot;
  if (bx >= a.gx) return;  // block-uniform
  const int cot0 = (by * (4 / WP) + wc) * RC;
  const int cotiles = (a.cout + 15) >> 4;
  h8 af[NSC][RC];
#pragma unroll
  for (int r = 0; r < RC; ++r) {
    const h8* wf = reinterpret_cast<const h8*>(a.w) + (size_t(min(cot0 + r, cotiles - 1)) * a.nalloc) * 64 + lane;
#pragma unroll
    for (int s = 0; s < NSC; ++s) af[s][r] = wf[s * 64];  // zero-padded past nsteps
  }
  // (the upsampling branch is hoisted out of the unrolled loads: per-piece branches make hipcc wrap
  // every load in its own exec branch)
  auto stage_load_t = [&](auto up_tag, int tile, h8 (&v)[IT]) {
    constexpr bool UP = decltype(up_tag)::value;
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int e = threadIdx.x + 256 * i;
      const int j = e & 7, rest = e >> 3;
      const int p = rest / NPAIR, q = rest - p * NPAIR;
      const int pix = tile * TPB + p, c = q * 64 + j * 8;
      const bool ok = pix < a.P && c < a.cin;
      const int64_t off = UP ? conv1x1_src(a, ok ? pix : 0) : int64_t(ok ? pix : 0) * a.xcs;
      v[i] = *(ok ? reinterpret_cast<const h8*>(a.x + off + c) : reinterpret_cast<const h8*>(g_zero_line));
    }
  };
  auto stage_load = [&](int tile, h8 (&v)[IT]) {
    if (a.up)
      stage_load_t(std::true_type{}, tile, v);
    else
      stage_load_t(std::false_type{}, tile, v);
  };
  auto stage_store = [&](int buf, const h8 (&v)[IT]) {
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int e = threadIdx.x + 256 * i;
      const int j = e & 7, rest = e >> 3;
      const int p = rest / NPAIR, q = rest - p * NPAIR;
      xr[buf * BUF + (q * TPB + p) * 8 + (j ^ ((p >> 1) & 7))] = v[i];
    }
  };
  const int pw = wp * RP * 16;
  const int step = 8 * nslot;
  h8 v[IT];
  stage_load(bx, v);
  for (int cur = 0; bx < a.gx; cur ^= 1) {
    stage_store(cur, v);
    __syncthreads();
    const int nbx = bx + step;
    if (nbx < a.gx) stage_load(nbx, v);
    f4 acc[RC][RP];
#pragma unroll
    for (int r = 0; r < RC; ++r)
#pragma unroll
      for (int p = 0; p < RP; ++p) acc[r][p] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NSC; ++s) {
      if (s < a.nsteps) {
        h8 bf[RP];
#pragma unroll
        for (int p = 0; p < RP; ++p) {
          const int px = pw + p * 16 + col;
          const int j = (s & 1) * 4 + grp;
          bf[p] = xr[cur * BUF + ((s >> 1) * TPB + px) * 8 + (j ^ ((px >> 1) & 7))];
        }
#pragma unroll
        for (int r = 0; r < RC; ++r)
#pragma unroll
          for (int p = 0; p < RP; ++p)
            acc[r][p] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[s][r], bf[p], acc[r][p], 0, 0, 0);
      }
    }
    conv_epilogue<RC, RP, OUT>(a, acc, bx * TPB + pw, cot0, col, grp);
    bx = nbx;
  }
}

// LDS-staged 1x1 configurations, coded 0x400 | rc | rp << 4 | log2(wp) << 12 (0x500 | ..: the ring)
static bool lds1_cfg_ok(int rc, int rp, int wp) {
  return (rc == 1 && rp == 4 && wp == 1) || (rc == 2 && rp == 4 && wp == 1) || (rc == 2 && rp == 2 && wp == 2) ||
         (rc == 1 && rp == 4 && wp == 2) || (rc == 1 && rp == 2 && wp == 4) || (rc == 4 && rp == 1 && wp == 4) ||
         (rc == 4 && rp == 2 && wp == 4);
}
static int lds1_nsc(int nsteps, int rc) {
  const int cap = rc == 4 ? 4 : 8;
  return nsteps <= 2 ? 2 : nsteps <= 4 || cap == 4 ? 4 : 8;
}
static size_t lds1_bytes(int rp, int wp, int nsc) { return size_t(wp) * rp * 16 * ((nsc + 1) / 2) * 128; }
static size_t lds1_out_bytes(int rc, int rp, int wp) { return size_t(wp) * rp * 16 * (4 / wp) * rc * 16 * 2; }

template <int RC, int RP, int WP, int NSC>
static void launch_lds1_o(const ConvArgs& a, int out_kind, dim3 grid, size_t lds, hipStream_t s) {
#define LDS1_L(O) FCE_LAUNCH((conv1x1_lds_kernel<RC, RP, WP, NSC, O>), grid, dim3(256), lds, s, a)
  switch (out_kind) {
    case OUT_F16: LDS1_L(OUT_F16); break;
    case OUT_F32: LDS1_L(OUT_F32); break;
    case OUT_WSTORE: LDS1_L(OUT_WSTORE); break;
    case OUT_CLS: LDS1_L(OUT_CLS); break;
    case OUT_DFL:
      if constexpr (RC == 4) LDS1_L(OUT_DFL);
      break;
    default: LDS1_L(OUT_ACCUM); break;
  }
#undef LDS1_L
}

template <int RC, int RP, int WP>
static void launch_lds1_n(const ConvArgs& a, int out_kind, int nsc, dim3 grid, size_t lds, hipStream_t s) {
  if (nsc == 2)
    launch_lds1_o<RC, RP, WP, 2>(a, out_kind, grid, lds, s);
  else if (nsc == 4 || RC == 4)
    launch_lds1_o<RC, RP, WP, 4>(a, out_kind, grid, lds, s);
  else
    launch_lds1_o<RC, RP, WP, (RC == 4 ? 4 : 8)>(a, out_kind, grid, lds, s);
}

// Persistent launches size their grid from the kernel's real occupancy (registers and LDS), queried
// once per instantiation: blocks beyond one resident wave would start only when a first-wave block
// finishes its whole tile sequence.
static int cus_per_xcd() {
  static const int v = [] {
    int d = 0, n = 0;
    if (hipGetDevice(&d) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess) {
      (void)hipGetLastError();
      n = 256;
    }
    return std::max(1, n / 8);
  }();
  return v;
}
template <typename K>
static int blocks_per_cu(K kernel, size_t lds) {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kernel, 256, lds) != hipSuccess) {
    (void)hipGetLastError();
    n = 1;
  }
  return std::max(1, n);
}
// FCE_PERSIST_OCC=k (experiment): at most k resident blocks per CU for the persistent grids, leaving the rest of
// each CU to the other lanes' kernels
static int persist_cap(int occ) {
  static const int cap = [] {
    const char* e = getenv("FCE_PERSIST_OCC");
    return e ? atoi(e) : 0;
  }();
  return cap > 0 ? std::min(occ, cap) : occ;
}
static int ring_slots(int units, int gy, int occ) {
  return std::max(1, std::min((units + 7) / 8, cus_per_xcd() * persist_cap(occ) / std::max(1, gy)));
}

static int ring_nsc(int nsteps) { return nsteps <= 2 ? 2 : nsteps <= 4 ? 4 : nsteps <= 6 ? 6 : nsteps <= 8 ? 8 : 0; }
static bool ring_ok(int nsteps, int rc, int rp, int wp) {
  const int nsc = ring_nsc(nsteps);
  return nsc > 0 && lds1_cfg_ok(rc, rp, wp) && nsc * rc <= 16 && 2 * lds1_bytes(rp, wp, nsc) <= 64 * 1024;
}

template <int RC, int RP, int WP, int NSC>
static void launch_ring_o(const ConvArgs& a, int out_kind, dim3, size_t lds, int, hipStream_t s) {
#define RING_L(O)                                                                                  \
  {                                                                                                \
    static const int occ = blocks_per_cu(conv1x1_ring_kernel<RC, RP, WP, NSC, O>, lds);            \
    const int nslot = ring_slots(a.gx, a.gy, occ);                                                 \
    FCE_LAUNCH((conv1x1_ring_kernel<RC, RP, WP, NSC, O>), dim3(unsigned(8 * a.gy * nslot)), dim3(256), lds, s, a, \
               nslot);                                                                             \
  }
  switch (out_kind) {
    case OUT_F16: RING_L(OUT_F16); break;
    case OUT_F32: RING_L(OUT_F32); break;
    case OUT_WSTORE: RING_L(OUT_WSTORE); break;
    case OUT_CLS: RING_L(OUT_CLS); break;
    case OUT_DFL:
      if constexpr (RC == 4) RING_L(OUT_DFL);
      break;
    default: RING_L(OUT_ACCUM); break;
  }
#undef RING_L
}

template <int RC, int RP, int WP>
static bool launch_ring_n(const ConvArgs& a, int out_kind, int nsc, dim3 grid, size_t lds, int nslot, hipStream_t s) {
  if constexpr (RC * 4 <= 16)
    if (nsc == 4) return launch_ring_o<RC, RP, WP, 4>(a, out_kind, grid, lds, nslot, s), true;
  if constexpr (RC * 6 <= 16 && 2 * WP * RP * 16 * 3 * 128 <= 64 * 1024)
    if (nsc == 6) return launch_ring_o<RC, RP, WP, 6>(a, out_kind, grid, lds, nslot, s), true;
  if constexpr (RC * 8 <= 16 && 2 * WP * RP * 16 * 4 * 128 <= 64 * 1024)
    if (nsc == 8) return launch_ring_o<RC, RP, WP, 8>(a, out_kind, grid, lds, nslot, s), true;
  if (nsc != 2) return false;
  launch_ring_o<RC, RP, WP, 2>(a, out_kind, grid, lds, nslot, s);
  return true;
}

static int launch_ring(const ConvArgs& a0, int out_kind, int rc, int rp, int wp, hipStream_t s) {
  FCE_CHECK(ring_ok(a0.nsteps, rc, rp, wp), "conv 1x1 ring: bad configuration");
  ConvArgs a = a0;
  const int cotiles = (a.cout + 15) / 16, cb = (4 / wp) * rc, tpb = wp * rp * 16;
  a.gx = (a.P + tpb - 1) / tpb;
  a.gy = (cotiles + cb - 1) / cb;
  const int nsc = ring_nsc(a.nsteps);
  const size_t lds = 2 * lds1_bytes(rp, wp, nsc);
  FCE_CHECK(int64_t(8) * a.gy * cus_per_xcd() * 8 < (int64_t(1) << 31), "conv 1x1 ring: grid too large");
  const int nslot = 0;  // per instantiation, from its occupancy (launch_ring_o)
  const dim3 grid(1);
  bool ok;
  if (rc == 1 && rp == 4 && wp == 1) ok = launch_ring_n<1, 4, 1>(a, out_kind, nsc, grid, lds, nslot, s);
  else if (rc == 2 && rp == 4 && wp == 1) ok = launch_ring_n<2, 4, 1>(a, out_kind, nsc, grid, lds, nslot, s);
  else if (rc == 2 && rp == 2 && wp == 2) ok = launch_ring_n<2, 2, 2>(a, out_kind, nsc, grid, lds, nslot, s);
  else if (rc == 1 && rp == 4 && wp == 2) ok = launch_ring_n<1, 4, 2>(a, out_kind, nsc, grid, lds, nslot, s);
  else if (rc == 1 && rp == 2 && wp == 4) ok = launch_ring_n<1, 2, 4>(a, out_kind, nsc, grid, lds, nslot, s);
  else if (rc == 4 && rp == 1 && wp == 4) ok = launch_ring_n<4, 1, 4>(a, out_kind, nsc, grid, lds, nslot, s);
  else ok = launch_ring_n<4, 2, 4>(a, out_kind, nsc, grid, lds, nslot, s);
  FCE_CHECK(ok, "conv 1x1 ring: no instantiation for this K depth");
  return launch_status("conv1x1_ring_kernel");
}

static int launch_lds1(const ConvArgs& a0, int out_kind, int rc, int rp, int wp, hipStream_t s) {
  FCE_CHECK(lds1_cfg_ok(rc, rp, wp), "conv 1x1 LDS tile: bad configuration");
  ConvArgs a = a0;
  const int cotiles = (a.cout + 15) / 16, cb = (4 / wp) * rc, tpb = wp * rp * 16;
  a.gx = (a.P + tpb - 1) / tpb;
  a.gy = (cotiles + cb - 1) / cb;
  FCE_CHECK(int64_t(a.gx) * a.gy < (int64_t(1) << 31), "conv 1x1 LDS tile: grid too large");
  const int nsc = lds1_nsc(a.nsteps, rc);
  const size_t lds = std::max(lds1_bytes(rp, wp, nsc), a.stg ? lds1_out_bytes(rc, rp, wp) : size_t(0));
  const dim3 grid(unsigned(a.gx * a.gy));
  if (rc == 1 && rp == 4 && wp == 1) launch_lds1_n<1, 4, 1>(a, out_kind, nsc, grid, lds, s);
  else if (rc == 2 && rp == 4 && wp == 1) launch_lds1_n<2, 4, 1>(a, out_kind, nsc, grid, lds, s);
  else if (rc == 2 && rp == 2 && wp == 2) launch_lds1_n<2, 2, 2>(a, out_kind, nsc, grid, lds, s);
  else if (rc == 1 && rp == 4 && wp == 2) launch_lds1_n<1, 4, 2>(a, out_kind, nsc, grid, lds, s);
  else if (rc == 1 && rp == 2 && wp == 4) launch_lds1_n<1, 2, 4>(a, out_kind, nsc, grid, lds, s);
  else if (rc == 4 && rp == 1 && wp == 4) launch_lds1_n<4, 1, 4>(a, out_kind, nsc, grid, lds, s);
  else launch_lds1_n<4, 2, 4>(a, out_kind, nsc, grid, lds, s);
  return launch_status("conv1x1_lds_kernel");
}

// ============================================================================ 1x1, big tiles, K-pipelined
// For the wide 1x1 convs of the m/l scales (cin, cout >= 64: up to tens of K-steps per output), where
// conv1x1_lds_kernel's 64-cout blocks re-stage each pixel tile once per cout group and wait on every
// chunk's loads.  Each wave owns RC=4 cout tiles x RP=4 pixel groups (64 x 64 outputs: 16 MFMAs per
// K-step per 4 A + 4 B fragment reads); the block (4 waves, WP of them along pixels) owns TPB = WP*64
// pixels x CBT = (4/WP)*4 cout tiles.  The K loop walks pairs of steps (64 channels): per pair the block
// stages its B rows (TPB x 128 B, the swizzled image of conv1x1_lds_kernel) and its A fragments (CBT x
// 2 x 1 KiB, packed order) in one of two LDS buffers with coalesced 16-byte loads, 8 per thread.  Two
// pairs are in flight in registers: the loads of pair k+2 are issued before pair k's MFMAs, pair k+1's
// registers are stored to the other buffer after them, one barrier per pair, so each load has two
// compute phases to land.  Per-output K order (steps 0..nsteps-1) is the implicit-GEMM kernel's:
// bitwise identical to every other variant.
template <int WP, int OUT>
__global__ __launch_bounds__(256, 2) void conv1x1_pipe_kernel(ConvArgs a) {
  constexpr int RC = 4, RP = 4;
  constexpr int TPB = WP * RP * 16;
  constexpr int CBT = (4 / WP) * RC;
  constexpr int BB = TPB * 8;        // h8 of B per buffer (one pair of steps)
  constexpr int AB = CBT * 2 * 64;   // h8 of A per buffer
  constexpr int BUF = BB + AB;
  constexpr int ITB = BB / 256, ITA = AB / 256, IT = ITB + ITA;
  static_assert(BB % 256 == 0 && AB % 256 == 0, "whole staging rounds");
  extern __shared__ __attribute__((aligned(16))) h8 xp[];  // [2][B image | A fragments]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = lane & 15, grp = lane >> 4;
  const int wc = wave / WP, wp = wave - wc * WP;
  int bx, by;  // XCD-aware order: a pixel tile's cout groups share an XCD's L2
  {
    const int total = a.gx * a.gy, b = blockIdx.x;
    const int per = total >> 3, body = per << 3;
    const int L = b < body ? (b & 7) * per + (b >> 3) : b;
    bx = L / a.gy;
    by = L - bx * a.gy;
  }
  const int pix0 = bx * TPB;
  const int cbl0 = by * CBT;
  const int cotiles = (a.cout + 15) >> 4;
  // staging pieces: B piece e = threadIdx.x + 256 i -> pixel e >> 3, 16-byte piece j = e & 7 of its
  // 128-byte pair; A piece e -> cout tile e >> 7, step (e >> 6) & 1, lane e & 63 (2 KiB per tile)
  const h8* sptr[IT];
  int spos[IT], sch[ITB];
  bool spv[ITB];
#pragma unroll
  for (int i = 0; i < ITB; ++i) {
    const int e = threadIdx.x + 256 * i;
    const int j = e & 7, p = e >> 3;
    const int pix = pix0 + p;
    spv[i] = pix < a.P;
    sptr[i] = reinterpret_cast<const h8*>(a.x + conv1x1_src(a, spv[i] ? pix : 0) + j * 8);
    sch[i] = j * 8;
    spos[i] = p * 8 + (j ^ ((p >> 1) & 7));
  }
#pragma unroll
  for (int i = 0; i < ITA; ++i) {
    const int e = threadIdx.x + 256 * i;
    const int t = e >> 7, sl = e & 127;  // sl = step * 64 + lane
    sptr[ITB + i] = reinterpret_cast<const h8*>(a.w) + size_t(min(cbl0 + t, cotiles - 1)) * a.nalloc * 64 + sl;
    spos[ITB + i] = BB + e;
  }
  auto load = [&](int k0, h8 (&v)[IT]) {  // packed A is zero-padded past nsteps: in bounds
    const int cbase = k0 * 32;
#pragma unroll
    for (int i = 0; i < ITB; ++i) {
      const bool ok = spv[i] && cbase + sch[i] < a.cin;
      v[i] = *(ok ? sptr[i] + cbase / 8 : reinterpret_cast<const h8*>(g_zero_line));
    }
#pragma unroll
    for (int i = 0; i < ITA; ++i) v[ITB + i] = sptr[ITB + i][size_t(k0) * 64];
  };
  auto store = [&](int buf, const h8 (&v)[IT]) {
#pragma unroll
    for (int i = 0; i < IT; ++i) xp[buf * BUF + spos[i]] = v[i];
  };
  f4 acc[RC][RP];
#pragma unroll
  for (int r = 0; r < RC; ++r)
#pragma unroll
    for (int p = 0; p < RP; ++p) acc[r][p] = f4{0.f, 0.f, 0.f, 0.f};
  const int pw = wp * RP * 16;
  const int npair = (a.nsteps + 1) >> 1;
  h8 v0[IT], v1[IT];
  load(0, v0);
  if (npair > 1) load(2, v1);
  store(0, v0);
  __syncthreads();
  for (int k = 0; k < npair; ++k) {
    const int cur = k & 1;
    if (k + 2 < npair) load(2 * (k + 2), v0);  // v0 was stored last iteration
    const int nsc = min(2, a.nsteps - 2 * k);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (s < nsc) {
        h8 af[RC], bf[RP];
#pragma unroll
        for (int r = 0; r < RC; ++r) af[r] = xp[cur * BUF + BB + ((wc * RC + r) * 2 + s) * 64 + lane];
#pragma unroll
        for (int p = 0; p < RP; ++p) {
          const int px = pw + p * 16 + col;
          const int j = s * 4 + grp;
          bf[p] = xp[cur * BUF + px * 8 + (j ^ ((px >> 1) & 7))];
        }
#pragma unroll
        for (int r = 0; r < RC; ++r)
#pragma unroll
          for (int p = 0; p < RP; ++p)
            acc[r][p] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[r], bf[p], acc[r][p], 0, 0, 0);
      }
    }
    if (k + 1 < npair) store(cur ^ 1, v1);
    __syncthreads();  // pair k's reads and pair k+1's stores done
#pragma unroll
    for (int i = 0; i < IT; ++i) v1[i] = v0[i];
  }
  if constexpr (OUT == OUT_F16 || OUT == OUT_WSTORE) {
    if (a.stg) {  // launch_pipe1 sizes the LDS for the output tile too (TPB x CBT*16 couts x 2 bytes)
      conv_store_staged<RC, RP, CBT, TPB, OUT>(a, acc, pix0, pw, cbl0, wc, col, grp, reinterpret_cast<_Float16*>(xp));
      return;
    }
  }
  conv_epilogue<RC, RP, OUT>(a, acc, pix0 + pw, cbl0 + wc * RC, col, grp);
}

// big-tile configurations, coded 0x700 | log2(wp) << 12 (rc = rp = 4)
static bool pipe1_ok(const fce_conv_desc& d, int det_box) {
  return d.k == 1 && d.stride == 1 && !det_box && d.cout >= 64 && d.cin >= 64;
}

template <int WP>
static int launch_pipe1_w(const ConvArgs& a, int out_kind, dim3 grid, size_t lds, hipStream_t s) {
#define PIPE1_L(O)                                                                                      \
  {                                                                                                     \
    static const bool lds_ok = hipFuncSetAttribute(reinterpret_cast<const void*>(&conv1x1_pipe_kernel<WP, O>), \
                                                    hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024) == hipSuccess; \
    FCE_CHECK(lds_ok || lds <= 64 * 1024, "conv 1x1 big tile: cannot opt in to >64 KiB LDS");          \
    FCE_LAUNCH((conv1x1_pipe_kernel<WP, O>), grid, dim3(256), lds, s, a);                               \
  }
  switch (out_kind) {
    case OUT_F16: PIPE1_L(OUT_F16); break;
    case OUT_F32: PIPE1_L(OUT_F32); break;
    case OUT_WSTORE: PIPE1_L(OUT_WSTORE); break;
    case OUT_CLS: PIPE1_L(OUT_CLS); break;
    default: PIPE1_L(OUT_ACCUM); break;
  }
#undef PIPE1_L
  return FCE_OK;
}

static int launch_pipe1(const ConvArgs& a0, int out_kind, int wp, hipStream_t s) {
  FCE_CHECK(out_kind != OUT_DFL && (wp == 1 || wp == 2 || wp == 4), "conv 1x1 big tile: bad configuration");
  ConvArgs a = a0;
  const int cotiles = (a.cout + 15) / 16, cb = (4 / wp) * 4, tpb = wp * 64;
  a.gx = (a.P + tpb - 1) / tpb;
  a.gy = (cotiles + cb - 1) / cb;
  FCE_CHECK(int64_t(a.gx) * a.gy < (int64_t(1) << 31), "conv 1x1 big tile: grid too large");
  const size_t lds = std::max(size_t(2) * (tpb * 128 + cb * 2048), a.stg ? size_t(tpb) * cb * 16 * 2 : size_t(0));
  const dim3 grid(unsigned(a.gx * a.gy));
  const int st = wp == 1 ? launch_pipe1_w<1>(a, out_kind, grid, lds, s)
                 : wp == 2 ? launch_pipe1_w<2>(a, out_kind, grid, lds, s)
                           : launch_pipe1_w<4>(a, out_kind, grid, lds, s);
  if (st != FCE_OK) return st;
  return launch_status("conv1x1_pipe_kernel");
}

// ============================================================================ 3x3, LDS halo tiles
// For cin % 32 == 0.  A block (4 waves) owns a 2-D output tile of TW = 16 columns x TH = 4*RP rows
// of one image and RC*16 couts; wave w owns rows [w*RP, w*RP+RP) (one 16-pixel B fragment per row).
// Per 32-channel chunk the input tile + halo ((TH-1)*S+3 x (TW-1)*S+3 pixels x 64 B) is staged in
// LDS once with coalesced 16-byte loads, and all 9 taps read their B fragments from it (a wave
// reads 16 consecutive pixels x 64 B = 1 KiB contiguous per fragment), instead of every tap
// re-fetching the pixels from L2 as the implicit-GEMM kernel does.  A fragments: the same packed
// layout (K-step = chunk * 9 + tap).  Per output element the K order (chunk-major, tap, channel)
// is the implicit-GEMM kernel's, so both kernels give bitwise-identical results.
// Tile-kernel geometry (template): CW waves split the block's cout tiles (CW*RC of them), the other
// 4/CW split its rows (RP rows each, TH = (4/CW)*RP); KP 32-channel chunks are staged per barrier
// (KP = 2: 128 bytes per pixel, full-line loads, half the barriers).  Slot swizzle of the 4*KP pieces
// of position u: q ^ ((u >> 1) & 3) for KP = 1, q ^ (u & 6) for KP = 2 (both conflict-free for the
// B-fragment reads at any alignment; checked exhaustively over the ds_read_b128 lane groups).
template <int KP>
__device__ __forceinline__ int tile_slot(int u, int q) {
  return KP == 1 ? (q ^ ((u >> 1) & 3)) : (q ^ (u & 6));
}

// AL = true: the block's weight fragments (CW * RC cout tiles x 9 taps x KP chunks, 1 KiB each) are
// staged in LDS next to the input tile, once per block per chunk group, and every wave reads its A
// fragments with ds_read_b128 (conflict-free: lane order).  Without it each wave streams its own A
// fragments from L2 for every K-step, and at the m/l scales (rc * rp MFMAs per fragment load) the
// per-CU vector-memory path, not the MFMA, sets the rate.  Same K order: bitwise identical.
template <int S, int RC, int RP, int CW, int KP, bool AL>
struct Tile3Geom {
  static constexpr int TW = 16, RW = 4 / CW, TH = RW * RP;
  static constexpr int RI = (TH - 1) * S + 3, CI = (TW - 1) * S + 3;
  static constexpr int NQ = 4 * KP;
  static constexpr int NE = RI * CI * NQ, NL = (NE + 255) / 256;
  static constexpr int NA = AL ? CW * RC * 9 * KP * 64 : 0, NLA = (NA + 255) / 256;
  // register prefetch of the next stage (rc 1 has the registers for 10 pieces: stride-2 rp 8 tiles)
  static constexpr bool PF = AL ? NL + NLA <= 16 : NL <= (RC == 1 ? 10 : 8);
  static constexpr size_t lds = size_t(PF ? NL * 256 : NE) * 16 + size_t(AL ? (PF ? NLA * 256 : NA) : 0) * 16;
};

template <int S, int RC, int RP, int CW, int KP, bool AL>
__global__ __launch_bounds__(256) void conv3x3_tile_kernel(ConvArgs a) {
  using G = Tile3Geom<S, RC, RP, CW, KP, AL>;
  constexpr int TW = 16, RW = 4 / CW, TH = RW * RP;
  constexpr int RI = (TH - 1) * S + 3, CI = (TW - 1) * S + 3;  // staged input rows / cols
  constexpr int NQ = 4 * KP;                                    // 16-byte pieces per staged pixel
  constexpr int NL0 = G::NL;
  // with the register prefetch the image is padded to NL0 * 256 pieces so that the last staging round
  // stores unconditionally (see conv3x3_ring_kernel)
  __shared__ __attribute__((aligned(16))) h8 tile[G::PF ? NL0 * 256 : G::NE];
  __shared__ __attribute__((aligned(16))) h8 atile[AL ? (G::PF ? G::NLA * 256 : G::NA) : 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
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
  const int cot0 = (cog * CW + wc) * RC;
  const int cotiles = (a.cout + 15) >> 4;
  const int spt = a.cin >> 5;  // 32-channel chunks = K-steps per tap
  const h8* wfrag[RC];
#pragma unroll
  for (int r = 0; r < RC; ++r) {
    const int ct = min(cot0 + r, cotiles - 1);
    wfrag[r] = reinterpret_cast<const h8*>(a.w) + (size_t(ct) * a.nalloc) * 64 + lane;
  }
  f4 acc[RC][RP];
#pragma unroll
  for (int r = 0; r < RC; ++r)
#pragma unroll
    for (int p = 0; p < RP; ++p) acc[r][p] = f4{0.f, 0.f, 0.f, 0.f};
  h8 af[RC];  // A fragments of the current K-step (prefetched one step ahead in the tap loop)
  if constexpr (!AL) {
#pragma unroll
    for (int r = 0; r < RC; ++r) af[r] = wfrag[r][0];
  }
  const _Float16* xn = a.x + int64_t(n) * a.Hs * a.Ws * a.xcs;
  const int iy0 = oy0 * S - 1, ix0 = ox0 * S - 1;
  // Staging: NL pieces per thread.  When they fit in registers (NL <= 8) the next stage's global
  // loads are issued right after this stage's LDS image is complete, so they are in flight during
  // this stage's MFMAs (register double buffer; one LDS image).
  constexpr int NE = G::NE, NL = G::NL, NA = G::NA, NLA = G::NLA;
  constexpr bool PF = G::PF;
  // A piece e of chunk group c0: fragment f = (block cout tile, k, tap) in that order, lane e & 63
  const h8* wblk = reinterpret_cast<const h8*>(a.w);
  const int ct_blk = cog * CW * RC;
  auto apiece = [&](int e, int c0) -> h8 {
    const int f = e >> 6, l = e & 63;
    const int rb = f / (9 * KP), rem = f - rb * (9 * KP);
    const int ct = min(ct_blk + rb, cotiles - 1);
    // select the address, not the loaded value: a select of two h8 values is done per 16-bit half and
    // makes the prefetch wait for its own loads right after issuing them
    return *(e < NA ? wblk + (size_t(ct) * a.nalloc + c0 * 9 + rem) * 64 + l : reinterpret_cast<const h8*>(g_zero_line));
  };
  auto piece = [&](int e, int c0, int& u, int& slot) -> h8 {
    const int pc = e / NQ, q = e - pc * NQ;
    const int r = pc / CI, c = pc - r * CI;
    const int iy = iy0 + r, ix = ix0 + c;
    u = r * CI + tile_col<S, CI>(c);
    slot = e < NE ? u * NQ + tile_slot<KP>(u, q) : e;
    const bool ok = e < NE && iy >= 0 && iy < a.Hs && ix >= 0 && ix < a.Ws && (KP == 1 || c0 + (q >> 2) < spt);
    return *(ok ? reinterpret_cast<const h8*>(xn + (int64_t(iy) * a.Ws + ix) * a.xcs + c0 * 32 + q * 8)
                : reinterpret_cast<const h8*>(g_zero_line));
  };
  h8 pv[PF ? NL : 1];
  int ps[PF ? NL : 1];
  h8 pa[PF && AL ? NLA : 1];
  if constexpr (PF) {
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      int u;
      pv[i] = piece(threadIdx.x + 256 * i, 0, u, ps[i]);
    }
    if constexpr (AL) {
#pragma unroll
      for (int i = 0; i < NLA; ++i) pa[i] = apiece(threadIdx.x + 256 * i, 0);
    }
  }
  for (int c0 = 0; c0 < spt; c0 += KP) {
    __syncthreads();  // previous stage's reads done
    if constexpr (PF) {
#pragma unroll
      for (int i = 0; i < NL; ++i) tile[ps[i]] = pv[i];
      if constexpr (AL) {
#pragma unroll
        for (int i = 0; i < NLA; ++i) atile[threadIdx.x + 256 * i] = pa[i];
      }
    } else {
      for (int e = threadIdx.x; e < NE; e += 256) {
        int u, sl;
        const h8 v = piece(e, c0, u, sl);
        tile[sl] = v;
      }
      if constexpr (AL)
        for (int e = threadIdx.x; e < NA; e += 256) atile[e] = apiece(e, c0);
    }
    __syncthreads();
    if constexpr (PF) {
      if (c0 + KP < spt) {
#pragma unroll
        for (int i = 0; i < NL; ++i) {
          int u;
          pv[i] = piece(threadIdx.x + 256 * i, c0 + KP, u, ps[i]);
        }
        if constexpr (AL) {
#pragma unroll
          for (int i = 0; i < NLA; ++i) pa[i] = apiece(threadIdx.x + 256 * i, c0 + KP);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < KP; ++k) {
      if (KP > 1 && c0 + k >= spt) break;
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int ky = tap / 3, kx = tap - ky * 3;
        h8 bf[RP];
        // A fragments one K-step ahead (the last step of the last chunk re-reads its own; weights only,
        // no LDS hazard across the staging barrier): the L2 latency hides under this step's MFMAs
        const int ks = (c0 + k) * 9 + tap + 1;
        const int ksn = ks < spt * 9 ? ks : ks - 1;
        h8 an[RC];
        if constexpr (AL) {
#pragma unroll
          for (int r = 0; r < RC; ++r) af[r] = atile[(((wc * RC + r) * KP + k) * 9 + tap) * 64 + lane];
        } else {
#pragma unroll
          for (int r = 0; r < RC; ++r) an[r] = wfrag[r][ksn * 64];
        }
#pragma unroll
        for (int p = 0; p < RP; ++p) {
          const int ry = (wr * RP + p) * S + ky;
          const int u = ry * CI + tile_col<S, CI>(col * S + kx);
          bf[p] = tile[u * NQ + tile_slot<KP>(u, k * 4 + grp)];
        }
#pragma unroll
        for (int r = 0; r < RC; ++r)
#pragma unroll
          for (int p = 0; p < RP; ++p)
            acc[r][p] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[r], bf[p], acc[r][p], 0, 0, 0);
        if constexpr (!AL) {
#pragma unroll
          for (int r = 0; r < RC; ++r) af[r] = an[r];
        }
      }
    }
  }
  tile3_store<RC, RP>(a, acc, n, oy0 + wr * RP, ox0, cot0, col, grp);
}

// ============================================================================ 3x3, persistent, A in registers
// For cin = 32 * NCH (NCH = 1, 2: the 32/64-channel 3x3 convs of the n/s scales, which the tile kernels
// run far below the MFMA rate because every wave re-reads its weight fragments from L2 for each
// 64-pixel tile).  Each wave owns ONE cout tile and keeps its 9 * NCH A fragments in registers for the
// whole launch; the block (4 cout tiles) walks a sequence of TH = RP row x 16 column output tiles,
// staging each tile's input (+ halo, all cin, 64 * NCH bytes per pixel, the swizzled image of the tile
// kernels) in one of two LDS buffers while the previous tile computes (the next tile's global loads are
// issued before this tile's MFMAs).  Block b: XCD b % 8, cout group, slot; XCD x owns the contiguous tile
// range [x chunk, (x + 1) chunk) and its slot-th blocks take tiles x chunk + slot + k nslot, so the tiles
// whose halos overlap are in flight on one XCD's L2 at the same time.
// K order (chunk, tap) is the implicit-GEMM kernel's: bitwise identical.
// PD = 2 (round 4): two register sets of staged input, the loop unrolled by two so each set's loads are issued two
// tiles ahead of their LDS store (two compute phases to land instead of one).
template <int S, int RP, int NCH, int PD = 1>
__global__ __launch_bounds__(256) void conv3x3_ring_kernel(ConvArgs a, int nslot) {
  constexpr int TW = 16, TH = RP;
  constexpr int RI = (TH - 1) * S + 3, CI = (TW - 1) * S + 3;
  // BUF = NL * 256 >= NE: slots past NE absorb the dummy pieces of the last staging round, so every
  // staging load and LDS store is unconditional (a guarded store lets hipcc sink the load under a
  // branch and serialise the loads with vmcnt waits)
  constexpr int NQ = 4 * NCH, NE = RI * CI * NQ, NL = (NE + 255) / 256, BUF = NL * 256;
  constexpr int KP = NCH;  // slot swizzle of the tile kernels for 4 * NCH pieces per pixel
  __shared__ __attribute__((aligned(16))) h8 tile[2 * BUF];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = lane & 15, grp = lane >> 4;
  const int xcd = blockIdx.x & 7, loc = blockIdx.x >> 3;
  const int by = loc % a.gy, slot = loc / a.gy;
  const int tiles_x = (a.Wo + TW - 1) / TW, tiles_y = (a.Ho + TH - 1) / TH;
  const int ntiles = tiles_x * tiles_y * a.N;
  const int chunk = (ntiles + 7) >> 3, tend = min(ntiles, (xcd + 1) * chunk);
  int t = xcd * chunk + slot;
  if (t >= tend) return;  // block-uniform
  const int cot0 = by * 4 + wave;
  const int cotiles = (a.cout + 15) >> 4;
  h8 af[NCH * 9];
  {
    const h8* wf = reinterpret_cast<const h8*>(a.w) + (size_t(min(cot0, cotiles - 1)) * a.nalloc) * 64 + lane;
#pragma unroll
    for (int k = 0; k < NCH * 9; ++k) af[k] = wf[k * 64];
  }
  auto stage_load = [&](int tt, h8 (&v)[NL], int (&sl)[NL]) {
    const int tx = tt % tiles_x, r0 = tt / tiles_x, ty = r0 % tiles_y, n = r0 / tiles_y;
    const int iy0 = ty * TH * S - 1, ix0 = tx * TW * S - 1;
    const _Float16* xn = a.x + int64_t(n) * a.Hs * a.Ws * a.xcs;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int e = threadIdx.x + 256 * i;
      const int pc = e / NQ, q = e - pc * NQ;
      const int r = pc / CI, c = pc - r * CI;
      const int iy = iy0 + r, ix = ix0 + c;
      const int u = r * CI + tile_col<S, CI>(c);
      sl[i] = e < NE ? u * NQ + tile_slot<KP>(u, q) : e;
      const bool ok = e < NE && iy >= 0 && iy < a.Hs && ix >= 0 && ix < a.Ws;
      v[i] = *(ok ? reinterpret_cast<const h8*>(xn + (int64_t(iy) * a.Ws + ix) * a.xcs + q * 8)
                  : reinterpret_cast<const h8*>(g_zero_line));
    }
  };
  h8 v[NL], v2[NL];
  int sl[NL], sl2[NL];
  const int step = nslot;
  // one tile: vv holds its staged input; vv is then reloaded with the tile PD steps on
  auto iter = [&](h8 (&vv)[NL], int (&ss)[NL], int cur) {
#pragma unroll
    for (int i = 0; i < NL; ++i) tile[cur * BUF + ss[i]] = vv[i];
    __syncthreads();
    const int tx = t % tiles_x, r0 = t / tiles_x, ty = r0 % tiles_y, n = r0 / tiles_y;
    Tile3Pre<RP> pre;  // residual + bias, issued before the prefetch (see tile3_pre)
    tile3_pre<RP>(a, n, ty * TH, tx * TW, cot0, grp, col, pre);
    // unconditional (clamped to the last tile, whose loads are then unused): a prefetch under a branch leaves the
    // waitcnt pass a join with nothing in flight on one side, and it waits vmcnt(0) for the residual there
    stage_load(min(t + PD * step, tend - 1), vv, ss);
    f4 acc[RP];
#pragma unroll
    for (int p = 0; p < RP; ++p) acc[p] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < NCH; ++k)
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int ky = tap / 3, kx = tap - ky * 3;
#pragma unroll
        for (int p = 0; p < RP; ++p) {
          const int u = (p * S + ky) * CI + tile_col<S, CI>(col * S + kx);
          const h8 bf = tile[cur * BUF + u * NQ + tile_slot<KP>(u, k * 4 + grp)];
          acc[p] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[k * 9 + tap], bf, acc[p], 0, 0, 0);
        }
      }
    tile3_post<RP>(a, acc, pre, n, ty * TH, tx * TW, cot0, col, grp);
    t += step;
  };
  stage_load(t, v, sl);
  if (PD == 1) {
    for (int cur = 0; t < tend; cur ^= 1) iter(v, sl, cur);
  } else {
    if (t + step < tend) stage_load(t + step, v2, sl2);
    for (int cur = 0; t < tend;) {
      iter(v, sl, cur);
      cur ^= 1;
      if (t >= tend) break;
      iter(v2, sl2, cur);
      cur ^= 1;
    }
  }
}

// ============================================================================ 3x3, persistent, 32x32x16 MFMA
// The ring above on v_mfma_f32_32x32x16_f16: a wave owns 32 couts x 32 pixels (2 rows x 16 columns) per MFMA, so each
// B fragment read from LDS (1 KiB: 16 k x 32 pixels) feeds 32 x 32 x 16 MACs instead of 16 x 16 x 32 -- half the LDS
// bytes per MAC, the ring's bound on the 64 -> 64 convs.  Bitwise identical to the 16x16x32 variants:
// each 32-deep K-step runs as two 32x32x16 MFMAs over its chunks (4s, 4s+1) then (4s+2, 4s+3), which is how
// v_mfma_f32_16x16x32_f16 sums a step (profiles/r05_mfma_order.txt: 0 of 200 000 random steps differ).
// Block: WC waves along the couts (32 each) x WR = 4 / WC along the rows, RPW 2-row pixel tiles per wave: a tile is
// TH = 2 RPW WR rows x 16 columns, staged like the ring's (swizzled halo image, double-buffered LDS, the next tile's
// loads issued before this tile's MFMAs).  A: lane l holds cout cb + (l & 31) and chunk 4 s + 2 h + (l >> 5) of
// K-step s, i.e. lane (l & 15) + 16 (l >> 5) + 32 h of the packed 16x16x32 fragment of cout tile (cb + (l & 31)) / 16.
// D: register r of lane l is cout cb + 8 (r / 4) + 4 (l >> 5) + r % 4, pixel l & 31.
typedef float f16v __attribute__((ext_vector_type(16)));

// the double-buffered staged tile of a ring32 configuration fits the 64 KiB of static LDS
static constexpr bool ring32_fits(int s, int nch, int wc, int rpw) {
  return wc >= 1 && 2 * ((((2 * rpw * (4 / wc) - 1) * s + 3) * (15 * s + 3) * 4 * nch + 255) / 256) * 256 * 16 <= 64 * 1024;
}

template <int S, int NCH, int WC, int RPW>
__global__ __launch_bounds__(256) void conv3x3_ring32_kernel(ConvArgs a, int nslot) {
  constexpr int WR = 4 / WC, TW = 16, TH = 2 * RPW * WR;
  constexpr int RI = (TH - 1) * S + 3, CI = (TW - 1) * S + 3;
  constexpr int NQ = 4 * NCH, NE = RI * CI * NQ, NL = (NE + 255) / 256, BUF = NL * 256;
  constexpr int KP = NCH;
  __shared__ __attribute__((aligned(16))) h8 tile[2 * BUF];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wc = wave % WC, wr = wave / WC, hi = lane >> 5;
  const int xcd = blockIdx.x & 7, loc = blockIdx.x >> 3;
  const int by = loc % a.gy, slot = loc / a.gy;
  const int tiles_x = (a.Wo + TW - 1) / TW, tiles_y = (a.Ho + TH - 1) / TH;
  const int ntiles = tiles_x * tiles_y * a.N;
  const int chunk = (ntiles + 7) >> 3, tend = min(ntiles, (xcd + 1) * chunk);
  int t = xcd * chunk + slot;
  if (t >= tend) return;  // block-uniform
  const int cb = (by * WC + wc) * 32;  // the wave's first cout
  const int cotiles = (a.cout + 15) >> 4;
  h8 af[NCH * 9][2];
  {
    const int ct = min((cb + (lane & 31)) >> 4, cotiles - 1);
    const h8* wf = reinterpret_cast<const h8*>(a.w) + size_t(ct) * a.nalloc * 64 + (lane & 15) + 16 * hi;
#pragma unroll
    for (int k = 0; k < NCH * 9; ++k) {
      af[k][0] = wf[k * 64];
      af[k][1] = wf[k * 64 + 32];
    }
  }
  float bz[4][4];  // the wave's biases: couts cb + 8 g + 4 hi + j
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int j = 0; j < 4; ++j) bz[g][j] = bias_or0(a.bias, cb + 8 * g + 4 * hi + j, a.cout);
  const bool vres = a.res && a.vec_ok;
  auto stage_load = [&](int tt, h8 (&v)[NL], int (&sl)[NL]) {
    const int tx = tt % tiles_x, r0 = tt / tiles_x, ty = r0 % tiles_y, n = r0 / tiles_y;
    const int iy0 = ty * TH * S - 1, ix0 = tx * TW * S - 1;
    const _Float16* xn = a.x + int64_t(n) * a.Hs * a.Ws * a.xcs;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int e = threadIdx.x + 256 * i;
      const int pc = e / NQ, q = e - pc * NQ;
      const int r = pc / CI, c = pc - r * CI;
      const int iy = iy0 + r, ix = ix0 + c;
      const int u = r * CI + tile_col<S, CI>(c);
      sl[i] = e < NE ? u * NQ + tile_slot<KP>(u, q) : e;
      const bool ok = e < NE && iy >= 0 && iy < a.Hs && ix >= 0 && ix < a.Ws;
      v[i] = *(ok ? reinterpret_cast<const h8*>(xn + (int64_t(iy) * a.Ws + ix) * a.xcs + q * 8)
                  : reinterpret_cast<const h8*>(g_zero_line));
    }
  };
  h8 v[NL];
  int sl[NL];
  const int step = nslot;
  stage_load(t, v, sl);
  for (int cur = 0; t < tend; cur ^= 1) {
#pragma unroll
    for (int i = 0; i < NL; ++i) tile[cur * BUF + sl[i]] = v[i];
    __syncthreads();
    const int tx = t % tiles_x, r0 = t / tiles_x, ty = r0 % tiles_y, n = r0 / tiles_y;
    // residuals of the wave's outputs (clamped, unconditional), issued before the prefetch: vmcnt retires in order
    h4 rres[RPW][4];
    if (vres) {
#pragma unroll
      for (int p = 0; p < RPW; ++p) {
        const int px = lane & 31;
        const int oy = min(ty * TH + (wr * RPW + p) * 2 + (px >> 4), a.Ho - 1), ox = min(tx * TW + (px & 15), a.Wo - 1);
        const int64_t pix = (int64_t(n) * a.Ho + oy) * a.Wo + ox;
#pragma unroll
        for (int g = 0; g < 4; ++g)
          rres[p][g] = *reinterpret_cast<const h4*>(a.res + pix * a.rcs + min(cb + 8 * g + 4 * hi, (a.cout - 4) & ~3));
      }
    }
    stage_load(min(t + step, tend - 1), v, sl);  // unconditional (clamped): see conv3x3_ring_kernel
    f16v acc[RPW];
#pragma unroll
    for (int p = 0; p < RPW; ++p)
#pragma unroll
      for (int j = 0; j < 16; ++j) acc[p][j] = 0.f;
#pragma unroll
    for (int k = 0; k < NCH; ++k)
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int ky = tap / 3, kx = tap - ky * 3;
#pragma unroll
        for (int p = 0; p < RPW; ++p) {
          const int px = lane & 31, rr = (wr * RPW + p) * 2 + (px >> 4);
          const int u = (rr * S + ky) * CI + tile_col<S, CI>((px & 15) * S + kx);
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const h8 bf = tile[cur * BUF + u * NQ + tile_slot<KP>(u, k * 4 + 2 * h + hi)];
            acc[p] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[k * 9 + tap][h], bf, acc[p], 0, 0, 0);
          }
        }
      }
    // epilogue: tile3_post's arithmetic (bias, SiLU, residual, fp16)
#pragma unroll
    for (int p = 0; p < RPW; ++p) {
      const int px = lane & 31;
      const int oy = ty * TH + (wr * RPW + p) * 2 + (px >> 4), ox = tx * TW + (px & 15);
      if (oy >= a.Ho || ox >= a.Wo) continue;
      const int64_t pix = (int64_t(n) * a.Ho + oy) * a.Wo + ox;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int co0 = cb + 8 * g + 4 * hi;
        if (co0 >= a.cout) continue;
        float vv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float tt = acc[p][4 * g + j] + bz[g][j];
          vv[j] = a.act ? silu(tt) : tt;
        }
        _Float16* yo = static_cast<_Float16*>(a.y) + pix * a.ycs + co0;
        const bool vec = a.vec_ok && co0 + 3 < a.cout;
        if (a.res) {
          if (vec && vres) {
#pragma unroll
            for (int j = 0; j < 4; ++j) vv[j] = fpin(vv[j] + (float)rres[p][g][j]);
          } else {
            const _Float16* ro = a.res + pix * a.rcs + co0;
            for (int j = 0; j < 4; ++j)
              if (co0 + j < a.cout) vv[j] = fpin(vv[j] + (float)ro[j]);
          }
        }
        if (vec) {
          *reinterpret_cast<h4*>(yo) = h4{(_Float16)fpin(vv[0]), (_Float16)fpin(vv[1]), (_Float16)fpin(vv[2]), (_Float16)fpin(vv[3])};
        } else {
          for (int j = 0; j < 4; ++j)
            if (co0 + j < a.cout) yo[j] = (_Float16)fpin(vv[j]);
        }
      }
    }
    t += step;
  }
}

// ============================================================================ 3x3, small cin, LDS tiles
// For cin % 8 == 0 and cin % 32 != 0 (cin <= 64: the C3k2 bottlenecks and early convs of small models,
// e.g. 8 -> 8 at 160 x 160).  Same block / wave geometry as conv3x3_tile_kernel, but the whole input
// tile + halo with ALL cin channels ((TH-1)*S+3 x (TW-1)*S+3 pixels x cin*2 B) is staged in LDS once,
// and the K loop walks the implicit-GEMM kernel's tap-major 8-channel chunks (c = 4 s + lane/16,
// tap = c / cpt): the same A fragments and the same per-output summation order as conv_mfma_kernel, so
// the two give bitwise-identical results.  Input pixels are read from HBM once (plus halo) instead of
// once per tap from L2.
// CPT > 0: cin = 8 CPT at compile time (the staging's index divisions, the K loop's tap / chunk arithmetic and
// its trip count become constants: the loop unrolls, every B read is base + a constant); 0: runtime cin.
template <int S, int RC, int RP, int CPT = 0>
__global__ __launch_bounds__(256) void conv3x3_tile_small_kernel(ConvArgs a) {
  constexpr int TW = 16, TH = 4 * RP;
  constexpr int RI = (TH - 1) * S + 3, CI = (TW - 1) * S + 3;
  extern __shared__ __attribute__((aligned(16))) h8 stile[];  // [RI][CI][cpt]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = lane & 15, grp = lane >> 4;
  const int cpt = CPT ? CPT : a.cpt;
  const int nsteps = CPT ? (9 * CPT + 3) / 4 : a.nsteps;
  const int tiles_x = (a.Wo + TW - 1) / TW, tiles_y = (a.Ho + TH - 1) / TH;
  int t, cog;
  tile_block(a.gy, t, cog);
  const int tx = t % tiles_x;
  t /= tiles_x;
  const int ty = t % tiles_y;
  const int n = t / tiles_y;
  const int ox0 = tx * TW, oy0 = ty * TH;
  const int cot0 = cog * RC;
  const int cotiles = (a.cout + 15) >> 4;
  const h8* wfrag[RC];
#pragma unroll
  for (int r = 0; r < RC; ++r) {
    const int ct = min(cot0 + r, cotiles - 1);
    wfrag[r] = reinterpret_cast<const h8*>(a.w) + (size_t(ct) * a.nalloc) * 64 + lane;
  }
  // A fragments of step 0 in flight while the tile is staged
  h8 an[RC];
#pragma unroll
  for (int r = 0; r < RC; ++r) an[r] = wfrag[r][0];
  const _Float16* xn = a.x + int64_t(n) * a.Hs * a.Ws * a.xcs;
  const int iy0 = oy0 * S - 1, ix0 = ox0 * S - 1;
  const int ne = RI * CI * cpt;
  for (int e = threadIdx.x; e < ne; e += 256) {
    const int pc = e / cpt, q = e - pc * cpt;
    const int r = pc / CI, c = pc - r * CI;
    const int iy = iy0 + r, ix = ix0 + c;
    h8 v = h8{0, 0, 0, 0, 0, 0, 0, 0};
    if (iy >= 0 && iy < a.Hs && ix >= 0 && ix < a.Ws)
      v = *reinterpret_cast<const h8*>(xn + (int64_t(iy) * a.Ws + ix) * a.xcs + q * 8);
    stile[e] = v;
  }
  __syncthreads();
  f4 acc[RC][RP];
#pragma unroll
  for (int r = 0; r < RC; ++r)
#pragma unroll
    for (int p = 0; p < RP; ++p) acc[r][p] = f4{0.f, 0.f, 0.f, 0.f};
  const h8 zero = h8{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int st = 0; st < nsteps; ++st) {
    h8 af[RC];
#pragma unroll
    for (int r = 0; r < RC; ++r) af[r] = an[r];
    if (st + 1 < nsteps) {
#pragma unroll
      for (int r = 0; r < RC; ++r) an[r] = wfrag[r][(st + 1) * 64];
    }
    const unsigned c = unsigned(st * 4 + grp);
    const int tap = CPT ? int(c) / CPT : cpt == 1 ? int(c) : int(__umulhi(c, a.cmagic));
    const int ch = int(c) - tap * cpt;
    const bool tin = tap < 9;
    const int ky = (tap * 11) >> 5, kx = tap - ky * 3;  // tap / 3 for tap < 9
    h8 bf[RP];
#pragma unroll
    for (int p = 0; p < RP; ++p) {
      const int ry = (wave * RP + p) * S + ky, cx = col * S + kx;
      bf[p] = tin ? stile[(ry * CI + cx) * cpt + ch] : zero;
    }
#pragma unroll
    for (int r = 0; r < RC; ++r)
#pragma unroll
      for (int p = 0; p < RP; ++p) acc[r][p] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[r], bf[p], acc[r][p], 0, 0, 0);
  }
  tile3_store<RC, RP>(a, acc, n, oy0 + wave * RP, ox0, cot0, col, grp);  // bias, SiLU, residual, fp16 store
}

static size_t small_tile_lds(int stride, int rp, int cin) {
  const int th = 4 * rp, ri = (th - 1) * stride + 3, ci = 15 * stride + 3;
  return size_t(ri) * ci * (cin / 8) * 16;
}

// ============================================================================ depthwise 3x3
// HBM-bound (each input pixel read once from HBM, 9x from L2): grid = (row chunks, N*Ho), one
// thread per (output pixel, 8 channels) with 32-bit index math; taps unrolled, weights [9][wcs].
struct DwArgs {
  const _Float16* x;
  int N, H, W, xcs;
  int C, stride;
  int Ho, Wo;
  const float* w;  // [9][wcs] (wcs >= C: a channel slice of a wider packed table)
  int wcs;
  const float* bias;
  _Float16* y;
  int ycs;
  int act;
};

// XCD-aware 2-D block order: block b runs on XCD b % 8; logical block L = (b % 8) * per + b / 8 gives each
// XCD a contiguous run of (x fastest, then y) blocks, so the row bands that share halo rows meet in one L2
__device__ __forceinline__ void xcd_block2(int& bx, int& by) {
  const int gx = int(gridDim.x), total = gx * int(gridDim.y), b = int(blockIdx.y) * gx + int(blockIdx.x);
  const int per = total >> 3, body = per << 3;
  const int L = b < body ? (b & 7) * per + (b >> 3) : b;
  by = L / gx;
  bx = L - by * gx;
}

// One thread = PX adjacent output pixels x 8 channels: the 9 tap weights are loaded once and the
// S*(PX-1)+3 input columns of each row are shared by the PX outputs.
template <int S, int PX>
__global__ __launch_bounds__(256) void dwconv_kernel(DwArgs a) {
  constexpr int NCOL = S * (PX - 1) + 3;
  const int cg8 = a.C >> 3;
  const int Q = (a.Wo + PX - 1) / PX;
  int bx, by;
  xcd_block2(bx, by);  // the rows that share input rows run on one XCD's L2
  const int idx = bx * 256 + threadIdx.x;
  if (idx >= Q * cg8) return;
  const int q = idx / cg8, c0 = (idx - q * cg8) * 8;
  const int row = by, n = row / a.Ho, oy = row - n * a.Ho;
  const int ox0 = q * PX, ix0 = ox0 * S - 1;
  float wk[9][8];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const f4 w0 = *reinterpret_cast<const f4*>(a.w + t * a.wcs + c0);
    const f4 w1 = *reinterpret_cast<const f4*>(a.w + t * a.wcs + c0 + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      wk[t][j] = w0[j];
      wk[t][j + 4] = w1[j];
    }
  }
  float acc[PX][8];
  {
    const f4 b0 = *reinterpret_cast<const f4*>(a.bias + c0);
    const f4 b1 = *reinterpret_cast<const f4*>(a.bias + c0 + 4);
#pragma unroll
    for (int p = 0; p < PX; ++p)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[p][j] = b0[j];
        acc[p][j + 4] = b1[j];
      }
  }
  const _Float16* xn = a.x + int64_t(n) * a.H * a.W * a.xcs + c0;
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
    const int iy = oy * S - 1 + ky;
    if (iy < 0 || iy >= a.H) continue;
    const _Float16* xr = xn + int64_t(iy) * a.W * a.xcs;
    h8 v[NCOL];
#pragma unroll
    for (int c = 0; c < NCOL; ++c) {
      const int ix = ix0 + c;
      v[c] = (ix >= 0 && ix < a.W) ? *reinterpret_cast<const h8*>(xr + int64_t(ix) * a.xcs)
                                   : h8{0, 0, 0, 0, 0, 0, 0, 0};
    }
#pragma unroll
    for (int p = 0; p < PX; ++p)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx)
        fma8_mix(v[p * S + kx], wk[ky * 3 + kx], acc[p]);
  }
#pragma unroll
  for (int p = 0; p < PX; ++p) {
    if (ox0 + p >= a.Wo) break;
    h8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (_Float16)fpin(a.act ? silu(acc[p][j]) : acc[p][j]);
    *reinterpret_cast<h8*>(a.y + (int64_t(row) * a.Wo + ox0 + p) * a.ycs + c0) = o;
  }
}

// Row-staged variant: one block = (channel slab of CS <= 64 channels, output row).  The 3 input rows
// of the slab are staged in LDS with coalesced 16-byte loads; thread e then owns output
// (pixel e / cg, 8-channel group e % cg), so consecutive lanes store consecutive 16-byte chunks
// (no partial-line writes).  Per pixel the (ky, kx) order and skipped padding taps match dwconv_kernel.
template <int S>
__global__ __launch_bounds__(256) void dwconv_rows_kernel(DwArgs a, int CS) {
  extern __shared__ __attribute__((aligned(16))) float dsm[];
  int bx, by;
  xcd_block2(bx, by);
  const int c0 = bx * CS;
  const int cs = min(CS, a.C - c0), cg = cs >> 3;
  const int row = by, n = row / a.Ho, oy = row - n * a.Ho;
  float* wl = dsm;              // [9][CS]
  float* bl = wl + 9 * CS;      // [CS]
  h8* rows = reinterpret_cast<h8*>(bl + CS);  // [3][W][CS/8]
  for (int e = threadIdx.x; e < 9 * cs; e += 256) {
    const int t = e / cs, c = e - t * cs;
    wl[t * CS + c] = a.w[t * a.wcs + c0 + c];
  }
  for (int c = threadIdx.x; c < cs; c += 256) bl[c] = a.bias[c0 + c];
  const _Float16* xn = a.x + int64_t(n) * a.H * a.W * a.xcs + c0;
  const int RW = a.W * (CS >> 3);
  for (int r = 0; r < 3; ++r) {
    const int iy = oy * S - 1 + r;
    const bool rin = iy >= 0 && iy < a.H;
    for (int e = threadIdx.x; e < a.W * cg; e += 256) {
      const int xx = e / cg, g = e - xx * cg;
      h8 v = h8{0, 0, 0, 0, 0, 0, 0, 0};
      if (rin) v = *reinterpret_cast<const h8*>(xn + (int64_t(iy) * a.W + xx) * a.xcs + 8 * g);
      rows[r * RW + xx * (CS >> 3) + g] = v;
    }
  }
  __syncthreads();
  _Float16* yr = a.y + int64_t(row) * a.Wo * a.ycs + c0;
  for (int e = threadIdx.x; e < a.Wo * cg; e += 256) {
    const int ox = e / cg, g = e - ox * cg;
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = bl[8 * g + j];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int iy = oy * S - 1 + ky;
      if (iy < 0 || iy >= a.H) continue;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int ix = ox * S - 1 + kx;
        if (ix < 0 || ix >= a.W) continue;
        const h8 v = rows[ky * RW + ix * (CS >> 3) + g];
        const float* wt = wl + (ky * 3 + kx) * CS + 8 * g;
        fma8_mix(v, wt, acc);
      }
    }
    h8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (_Float16)fpin(a.act ? silu(acc[j]) : acc[j]);
    *reinterpret_cast<h8*>(yr + int64_t(ox) * a.ycs + 8 * g) = o;
  }
}

// depthwise 3x3 (pad 1) on NHWC f16 slices; w = [9][wcs] fp32 taps (BN folded), bias fp32 [C]
// Lane-contiguous variant: a block owns one output row; thread t = (pixel slot t / cg, group t % cg)
// with blockDim a multiple of cg, so a thread keeps one channel group (its 9 x 8 weights stay in
// registers) while striding over the row, and every load / store instruction covers consecutive
// 16-byte chunks across lanes.
template <int S>
__global__ __launch_bounds__(256) void dwconv_lanes_kernel(DwArgs a) {
  const int cg = a.C >> 3;
  const int tpx = blockDim.x / cg;  // pixels per sweep
  const int t = threadIdx.x, g = t % cg, px = t / cg;
  const int row = blockIdx.x, n = row / a.Ho, oy = row - n * a.Ho;
  const int c0 = g * 8;
  float wk[9][8], bz[8];
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const f4 w0 = *reinterpret_cast<const f4*>(a.w + k * a.wcs + c0);
    const f4 w1 = *reinterpret_cast<const f4*>(a.w + k * a.wcs + c0 + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      wk[k][j] = w0[j];
      wk[k][j + 4] = w1[j];
    }
  }
  {
    const f4 b0 = *reinterpret_cast<const f4*>(a.bias + c0), b1 = *reinterpret_cast<const f4*>(a.bias + c0 + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bz[j] = b0[j];
      bz[j + 4] = b1[j];
    }
  }
  const _Float16* xn = a.x + int64_t(n) * a.H * a.W * a.xcs + c0;
  _Float16* yr = a.y + int64_t(row) * a.Wo * a.ycs + c0;
  for (int ox = px; ox < a.Wo; ox += tpx) {
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = bz[j];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int iy = oy * S - 1 + ky;
      if (iy < 0 || iy >= a.H) continue;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int ix = ox * S - 1 + kx;
        if (ix < 0 || ix >= a.W) continue;
        const h8 v = *reinterpret_cast<const h8*>(xn + (int64_t(iy) * a.W + ix) * a.xcs);
        fma8_mix(v, wk[ky * 3 + kx], acc);
      }
    }
    h8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (_Float16)fpin(a.act ? silu(acc[j]) : acc[j]);
    *reinterpret_cast<h8*>(yr + int64_t(ox) * a.ycs) = o;
  }
}

// Column-run variant: thread = (output column ox, 8-channel group), consecutive lanes = consecutive
// channel groups then columns, so every load / store instruction covers contiguous pixels (full
// lines); each thread computes PY outputs down its column from (PY-1)*S+3 input rows, every loaded
// row feeding all the outputs that use it.  Out-of-image taps load the zero line and add fmaf(0, w, acc) == acc,
// the value the other variants get by skipping them; each output accumulates its taps in (ky, kx) order with fmaf.
template <int S, int PY>
__global__ __launch_bounds__(256) void dwconv_cols_kernel(DwArgs a) {
  const int cg = a.C >> 3;
  int bx, by;
  xcd_block2(bx, by);
  const int e = bx * 256 + threadIdx.x;
  if (e >= a.Wo * cg) return;
  const int ox = e / cg, g = e - ox * cg, c0 = g * 8;
  const int bands = (a.Ho + PY - 1) / PY;
  const int n = by / bands, oy0 = (by - n * bands) * PY;
  float wk[9][8], acc[PY][8];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const f4 w0 = *reinterpret_cast<const f4*>(a.w + t * a.wcs + c0);
    const f4 w1 = *reinterpret_cast<const f4*>(a.w + t * a.wcs + c0 + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      wk[t][j] = w0[j];
      wk[t][j + 4] = w1[j];
    }
  }
  {
    const f4 b0 = *reinterpret_cast<const f4*>(a.bias + c0), b1 = *reinterpret_cast<const f4*>(a.bias + c0 + 4);
#pragma unroll
    for (int p = 0; p < PY; ++p)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[p][j] = b0[j];
        acc[p][j + 4] = b1[j];
      }
  }
  const _Float16* xn = a.x + int64_t(n) * a.H * a.W * a.xcs + c0;
  const int iy0 = oy0 * S - 1, ix0 = ox * S - 1;
  bool cok[3];
#pragma unroll
  for (int kx = 0; kx < 3; ++kx) cok[kx] = ix0 + kx >= 0 && ix0 + kx < a.W;
  constexpr int NR = (PY - 1) * S + 3;
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const int iy = iy0 + r;
    const bool rin = iy >= 0 && iy < a.H;
    h8 v[3];
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      const bool ok = rin && cok[kx];
      v[kx] = *(ok ? reinterpret_cast<const h8*>(xn + (int64_t(iy) * a.W + ix0 + kx) * a.xcs)
                   : reinterpret_cast<const h8*>(g_zero_line));
    }
#pragma unroll
    for (int p = 0; p < PY; ++p) {
      const int ky = r - p * S;
      if (ky < 0 || ky > 2) continue;  // compile-time after unrolling
      // an out-of-image tap loaded the zero line: fmaf(0, w, acc) == acc (the skipped tap of the other variants;
      // a select per FMA here was a third of the kernel's VALU work)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const u4 pk = __builtin_bit_cast(u4, v[kx]);
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          acc[p][2 * jj] = fma_mix_lo(pk[jj], wk[ky * 3 + kx][2 * jj], acc[p][2 * jj]);
          acc[p][2 * jj + 1] = fma_mix_hi(pk[jj], wk[ky * 3 + kx][2 * jj + 1], acc[p][2 * jj + 1]);
        }
      }
    }
  }
#pragma unroll
  for (int p = 0; p < PY; ++p) {
    if (oy0 + p >= a.Ho) break;
    h8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (_Float16)fpin(a.act ? silu(acc[p][j]) : acc[p][j]);
    *reinterpret_cast<h8*>(a.y + ((int64_t(n) * a.Ho + oy0 + p) * a.Wo + ox) * a.ycs + c0) = o;
  }
}

// Variants (bitwise-identical results; the executor autotunes `variant` per layer, -1 = default).  All
// three accumulate with explicit fmaf in (ky, kx) order and pin the result before the fp16 conversion,
// so hipcc cannot contract them differently.
//   0 pixel-quad (dwconv_kernel<S,4>)   1 row-staged LDS (dwconv_rows_kernel)   2 lane-contiguous
//   3 / 4 column runs of 2 / 4 outputs (dwconv_cols_kernel<S,PY>; runs of 8 measured slower on every n32 op)
int dwconv_variants(int c, int w, int* out, int cap) {
  int n = 0;
  if (n < cap) out[n++] = 0;
  if (n < cap && size_t(10) * 8 * sizeof(float) + size_t(3) * w * 8 * sizeof(_Float16) <= 64 * 1024) out[n++] = 1;
  if (n < cap && c / 8 <= 256) out[n++] = 2;
  if (n < cap) out[n++] = 3;  // column runs of 2
  if (n < cap) out[n++] = 4;  // column runs of 4
  return n;
}

// depthwise 3x3 (pad 1) on NHWC f16 slices; w = [9][wcs] fp32 taps (BN folded), bias fp32 [C]
int dwconv3x3(const fce_tensor& x, int stride, const float* w, int wcs, const float* bias, int act,
              const fce_tensor& y, hipStream_t s, int variant) {
  FCE_CHECK(x.c == y.c && x.c % 8 == 0 && wcs >= x.c && wcs % 4 == 0, "dwconv: channel mismatch");
  FCE_CHECK(x.layout == FCE_NHWC && y.layout == FCE_NHWC && x.dtype == FCE_F16 && y.dtype == FCE_F16,
            "dwconv: NHWC f16 views");
  FCE_CHECK(x.cstride % 8 == 0 && x.coff % 8 == 0 && y.cstride % 8 == 0 && y.coff % 8 == 0,
            "dwconv: slices must be 8-aligned");
  const int Ho = (x.h - 1) / stride + 1, Wo = (x.w - 1) / stride + 1;
  FCE_CHECK(y.n == x.n && y.h == Ho && y.w == Wo, "dwconv: output size mismatch");
  if (int64_t(y.n) * Ho * Wo == 0) return FCE_OK;
  FCE_CHECK(int64_t(y.n) * Ho < 65536 * 1024, "dwconv: too many output rows");
  DwArgs a{static_cast<const _Float16*>(x.data) + x.coff, x.n, x.h, x.w, x.cstride, x.c, stride, Ho, Wo,
           w, wcs, bias, static_cast<_Float16*>(y.data) + y.coff, y.cstride, act};
  if (variant < 0) variant = 0;
  if (variant == 1) {
    for (int CS = std::min(64, x.c); CS >= 8; CS /= 2) {  // row-staged kernel while its LDS fits 64 KiB
      if (CS % 8) continue;
      const size_t lds = size_t(10) * CS * sizeof(float) + size_t(3) * x.w * CS * sizeof(_Float16);
      if (lds > 64 * 1024) continue;
      dim3 g((x.c + CS - 1) / CS, y.n * Ho);
      if (stride == 1)
        FCE_LAUNCH((dwconv_rows_kernel<1>), g, dim3(256), lds, s, a, CS);
      else
        FCE_LAUNCH((dwconv_rows_kernel<2>), g, dim3(256), lds, s, a, CS);
      return launch_status("dwconv_rows_kernel");
    }
  }
  if (variant == 2 && x.c / 8 <= 256) {
    const int cg = x.c / 8;
    const int threads = (256 / cg) * cg;
    if (stride == 1)
      FCE_LAUNCH((dwconv_lanes_kernel<1>), dim3(y.n * Ho), dim3(threads), 0, s, a);
    else
      FCE_LAUNCH((dwconv_lanes_kernel<2>), dim3(y.n * Ho), dim3(threads), 0, s, a);
    return launch_status("dwconv_lanes_kernel");
  }
  if (variant == 3 || variant == 4) {
    const int py = variant == 3 ? 2 : 4;
    const int64_t rows = int64_t(y.n) * ((Ho + py - 1) / py);
    FCE_CHECK(rows < 65536, "dwconv: too many row bands");
    const dim3 g((Wo * (x.c / 8) + 255) / 256, unsigned(rows));
    if (stride == 1 && py == 2)
      FCE_LAUNCH((dwconv_cols_kernel<1, 2>), g, dim3(256), 0, s, a);
    else if (stride == 1)
      FCE_LAUNCH((dwconv_cols_kernel<1, 4>), g, dim3(256), 0, s, a);
    else if (py == 2)
      FCE_LAUNCH((dwconv_cols_kernel<2, 2>), g, dim3(256), 0, s, a);
    else
      FCE_LAUNCH((dwconv_cols_kernel<2, 4>), g, dim3(256), 0, s, a);
    return launch_status("dwconv_cols_kernel");
  }
  constexpr int PX = 4;
  dim3 grid(((Wo + PX - 1) / PX * (x.c / 8) + 255) / 256, y.n * Ho);
  if (stride == 1)
    FCE_LAUNCH((dwconv_kernel<1, PX>), grid, dim3(256), 0, s, a);
  else
    FCE_LAUNCH((dwconv_kernel<2, PX>), grid, dim3(256), 0, s, a);
  return launch_status("dwconv_kernel");
}

// ============================================================================ stem (NCHW input, cin <= 4)
struct StemArgs {
  const void* x;
  int dtype;
  int N, C, H, W;
  int stride, k;
  int Ho, Wo, cout;
  const float* w;  // [ci][ky][kx][co]
  const float* bias;
  _Float16* y;
  int ycs;
  int act;
};

template <typename T>
__device__ __forceinline__ float ld_in(const T* p, int64_t i);
template <>
__device__ __forceinline__ float ld_in<_Float16>(const _Float16* p, int64_t i) {
  return (float)p[i];
}
template <>
__device__ __forceinline__ float ld_in<float>(const float* p, int64_t i) {
  return p[i];
}
// uint8 network input: the reference preprocess (predictor.py:151-173) computes `im.half() / 255`, i.e.
// the fp16 rounding of v / 255 — the value the fp16 model sees for every pixel
__device__ __forceinline__ float u8_to_unit(unsigned v) { return (float)(_Float16)((float)v / 255.0f); }
template <>
__device__ __forceinline__ float ld_in<uint8_t>(const uint8_t* p, int64_t i) {
  return u8_to_unit(p[i]);
}

template <int COUT, typename T>
__global__ __launch_bounds__(256) void stem_kernel(StemArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int nw = a.C * a.k * a.k * COUT;
  for (int i = threadIdx.x; i < nw; i += blockDim.x) {
    const int co = i % COUT, r = i / COUT;
    smem[i] = co < a.cout ? a.w[r * a.cout + co] : 0.f;
  }
  __syncthreads();
  const T* x = static_cast<const T*>(a.x);
  const int64_t P = int64_t(a.N) * a.Ho * a.Wo;
  const int pad = a.k / 2;
  for (int64_t pix = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; pix < P; pix += int64_t(gridDim.x) * blockDim.x) {
    const int ox = int(pix % a.Wo);
    const int oy = int((pix / a.Wo) % a.Ho);
    const int n = int(pix / (int64_t(a.Wo) * a.Ho));
    float acc[COUT];
#pragma unroll
    for (int co = 0; co < COUT; ++co) acc[co] = 0.f;
    for (int ci = 0; ci < a.C; ++ci) {
      const int64_t plane = (int64_t(n) * a.C + ci) * a.H * a.W;
      for (int ky = 0; ky < a.k; ++ky) {
        const int iy = oy * a.stride - pad + ky;
        if (iy < 0 || iy >= a.H) continue;
        for (int kx = 0; kx < a.k; ++kx) {
          const int ix = ox * a.stride - pad + kx;
          if (ix < 0 || ix >= a.W) continue;
          const float v = ld_in<T>(x, plane + int64_t(iy) * a.W + ix);
          const float* wt = smem + ((ci * a.k + ky) * a.k + kx) * COUT;
#pragma unroll
          for (int co = 0; co < COUT; ++co) acc[co] += v * wt[co];
        }
      }
    }
    _Float16* yo = a.y + pix * a.ycs;
#pragma unroll
    for (int co0 = 0; co0 < COUT; co0 += 8) {
      if (co0 >= a.cout) break;
      h8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int co = co0 + j;
        const float t = acc[co] + bias_or0(a.bias, co, a.cout);
        o[j] = (_Float16)(a.act ? silu(t) : t);
      }
      *reinterpret_cast<h8*>(yo + co0) = o;
    }
  }
}

// 3x3 stride-2 stem (the network's first Conv, 640 -> 320): one thread = PX adjacent output pixels
// of one row.  Their receptive columns are the aligned run x[2*PX*q .. 2*PX*q + 2PX-1] plus the
// element before it, so each (ci, ky) costs one vector load + one scalar load instead of 3*PX.
// Weights [ci][ky][kx][co] broadcast from LDS; same per-pixel summation order as stem_kernel.
// NE consecutive input elements held as raw 32-bit words (one aligned vector load)
template <typename T, int NE>
struct RawRun {
  static constexpr int NW = (int(sizeof(T)) * NE + 3) / 4;
  uint32_t w[NW];
  __device__ __forceinline__ void load(const T* p) {
    if constexpr (NW == 8) {
      const uint4 lo = reinterpret_cast<const uint4*>(p)[0], hi = reinterpret_cast<const uint4*>(p)[1];
      w[0] = lo.x; w[1] = lo.y; w[2] = lo.z; w[3] = lo.w; w[4] = hi.x; w[5] = hi.y; w[6] = hi.z; w[7] = hi.w;
    } else if constexpr (NW == 4) {
      const uint4 v = *reinterpret_cast<const uint4*>(p);
      w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
    } else if constexpr (NW == 2) {
      const uint2 v = *reinterpret_cast<const uint2*>(p);
      w[0] = v.x; w[1] = v.y;
    } else {
      static_assert(NW == 1, "run size");
      w[0] = *reinterpret_cast<const uint32_t*>(p);
    }
  }
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int i = 0; i < NW; ++i) w[i] = 0u;
  }
  __device__ __forceinline__ float get(int e) const {
    if constexpr (sizeof(T) == 4) {
      return __uint_as_float(w[e]);
    } else if constexpr (sizeof(T) == 2) {
      const unsigned short h = (unsigned short)(w[e >> 1] >> ((e & 1) * 16));
      return (float)__ushort_as_half(h);
    } else {
      return u8_to_unit((w[e >> 2] >> ((e & 3) * 8)) & 255u);
    }
  }
};

template <int COUT, int PX, typename T>
__global__ __launch_bounds__(256) void stem_s2_kernel(StemArgs a) {
  // RGB input (CIN = 3).  Output: when the view is a dense [pixel][COUT] buffer the block stages its
  // results in LDS and each store instruction writes 64 x 16 contiguous bytes (direct per-thread
  // stores at a 32*PX-byte lane stride reach HBM as partial lines: 2.4x the output bytes measured).
  constexpr int CIN = 3, NE = 2 * PX, CPT = PX * COUT / 8;  // 16-byte chunks per thread
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int nw = CIN * 9 * COUT;
  for (int i = threadIdx.x; i < nw; i += blockDim.x) {
    const int co = i % COUT, r = i / COUT;
    smem[i] = co < a.cout ? a.w[r * a.cout + co] : 0.f;
  }
  __syncthreads();
  const int Q = (a.Wo + PX - 1) / PX;
  const int nthreads = a.N * a.Ho * Q;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  const bool valid = idx < nthreads;
  const int row = valid ? idx / Q : 0, q = valid ? idx - row * Q : 0;
  const int n = row / a.Ho, oy = row - n * a.Ho;
  const int ix0 = 2 * PX * q;
  const bool interior = ix0 + NE <= a.W;
  const T* x = static_cast<const T*>(a.x);
  float acc[PX][COUT];
#pragma unroll
  for (int j = 0; j < PX; ++j)
#pragma unroll
    for (int co = 0; co < COUT; ++co) acc[j][co] = 0.f;
#pragma unroll 1
  for (int ci = 0; ci < CIN; ++ci) {
    RawRun<T, NE> run[3];
    float pre[3];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {  // the three row loads of a channel are issued together
      const int iy = 2 * oy - 1 + ky;
      const bool rin = valid && iy >= 0 && iy < a.H;
      const T* rp = x + ((int64_t(n) * CIN + ci) * a.H + (rin ? iy : 0)) * a.W;
      pre[ky] = (rin && ix0 > 0) ? ld_in<T>(rp, ix0 - 1) : 0.f;
      if (rin && interior)
        run[ky].load(rp + ix0);
      else  // rows outside the image (the dispatcher only launches this kernel for W % 2PX == 0)
        run[ky].zero();
    }
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      float v[NE + 1];
      v[0] = pre[ky];
#pragma unroll
      for (int e = 0; e < NE; ++e) v[1 + e] = run[ky].get(e);
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const float* wt = smem + ((ci * 3 + ky) * 3 + kx) * COUT;
#pragma unroll
        for (int co = 0; co < COUT; co += 4) {
          const f4 w4 = *reinterpret_cast<const f4*>(wt + co);
#pragma unroll
          for (int j = 0; j < PX; ++j) {
            const float xv = v[2 * j + kx];
            acc[j][co] += xv * w4[0];
            acc[j][co + 1] += xv * w4[1];
            acc[j][co + 2] += xv * w4[2];
            acc[j][co + 3] += xv * w4[3];
          }
        }
      }
    }
  }
  h8 o[PX][COUT / 8];
#pragma unroll
  for (int j = 0; j < PX; ++j)
#pragma unroll
    for (int c8 = 0; c8 < COUT / 8; ++c8)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int co = c8 * 8 + e;
        const float t = acc[j][co] + bias_or0(a.bias, co, a.cout);
        o[j][c8][e] = (_Float16)(a.act ? silu(t) : t);
      }
  if (a.cout == COUT && a.ycs == COUT) {
    h8* st = reinterpret_cast<h8*>(smem + nw);  // [256][CPT]
#pragma unroll
    for (int j = 0; j < PX; ++j)
#pragma unroll
      for (int c8 = 0; c8 < COUT / 8; ++c8) st[threadIdx.x * CPT + j * (COUT / 8) + c8] = o[j][c8];
    __syncthreads();
    const int lane = threadIdx.x & 63, t0 = threadIdx.x - lane;  // this wave's first thread
    const int idx0 = blockIdx.x * 256 + t0;
    if (idx0 >= nthreads) return;
    const int row0 = idx0 / Q, q0 = idx0 - row0 * Q;
    // consecutive threads own consecutive output pixels (Wo % PX == 0), so the wave's output is one
    // contiguous run of 64 * PX pixels
    _Float16* y0 = a.y + (int64_t(row0) * a.Wo + PX * q0) * COUT;
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int c = k * 64 + lane, tt = c / CPT;
      if (idx0 + tt < nthreads) reinterpret_cast<h8*>(y0)[c] = st[(t0 + tt) * CPT + (c - tt * CPT)];
    }
    return;
  }
  if (!valid) return;
#pragma unroll
  for (int j = 0; j < PX; ++j) {
    const int ox = PX * q + j;
    if (ox >= a.Wo) break;
    _Float16* yo = a.y + (int64_t(row) * a.Wo + ox) * a.ycs;
#pragma unroll
    for (int c8 = 0; c8 < COUT / 8; ++c8)
      if (c8 * 8 < a.cout) *reinterpret_cast<h8*>(yo + c8 * 8) = o[j][c8];
  }
}

// 3x3 stride-2 stem on MFMA (3 -> <= 64 channels; k = ci * 9 + tap fits one 32-deep K-step).  A block
// takes SR output rows of one image: the 2 SR + 1 input rows of all channels are staged in LDS as fp16
// (the network's input type; f32 inputs are rounded, u8 inputs become fp16(v / 255) as im.half() / 255
// does) with 16-byte loads and a 16-byte zero pad each side; each wave then builds, per 16-pixel fragment, its B operand by
// gathering the 8 (ci, ky, kx) values of its lane group from LDS and runs RC MFMAs (16 couts each).
// Lane (col, grp) of D holds couts 4 grp .. of pixel col: 8-byte stores, a fragment's 16 pixels x
// RC*16 couts contiguous in NHWC.  fp16 weights, fp32 accumulation, like every other conv here.
template <typename T, int RC, int SR>
__global__ __launch_bounds__(256) void stem_mfma_kernel(StemArgs a, const _Float16* wfr) {
  // SR output rows per block
  constexpr int IR = 2 * SR + 1;        // staged input rows
  extern __shared__ __attribute__((aligned(16))) _Float16 ssm[];  // [C][IR][8 + W + 8]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = lane & 15, grp = lane >> 4;
  const int rows = (a.Ho + SR - 1) / SR;
  const int n = blockIdx.x / rows, oy0 = (blockIdx.x - n * rows) * SR;
  const int WP = a.W + 16;  // 16-byte zero pads left and right keep every staged chunk aligned
  const int CW = WP / 8;    // 16-byte chunks per staged row
  const T* x = static_cast<const T*>(a.x);
  const int ne = a.C * IR * CW;
  if constexpr (std::is_same<T, _Float16>::value) {
    // fp16 input: up to 12 staging chunks per thread issued back to back (address select onto a zero
    // line, unconditional LDS stores), instead of one dependent load -> store round trip per chunk
    constexpr int NLS = 12;
    if (ne <= NLS * 256) {
      h8 v[NLS];
      int dst[NLS];
      // (staged row, chunk) of e = threadIdx.x + 256 i, stepped without a division per chunk
      const int dq = 256 % CW, dcr = 256 / CW;
      int cr = int(threadIdx.x) / CW, q = int(threadIdx.x) - cr * CW;
#pragma unroll
      for (int i = 0; i < NLS; ++i) {
        const int e = threadIdx.x + 256 * i;
        if (i > 0) {
          q += dq;
          cr += dcr;
          if (q >= CW) {
            q -= CW;
            ++cr;
          }
        }
        const int ci = cr / IR, r = cr - ci * IR;
        const int iy = 2 * oy0 - 1 + r, ix0 = (q - 1) * 8;
        const bool ok = e < ne && iy >= 0 && iy < a.H && q >= 1 && ix0 < a.W;
        dst[i] = e < ne ? cr * WP + q * 8 : a.C * IR * WP;  // one 16-byte dummy slot past the image
        v[i] = *(ok ? reinterpret_cast<const h8*>(x + ((int64_t(n) * a.C + ci) * a.H + iy) * a.W + ix0)
                    : reinterpret_cast<const h8*>(g_zero_line));
      }
#pragma unroll
      for (int i = 0; i < NLS; ++i) *reinterpret_cast<h8*>(ssm + dst[i]) = v[i];
    } else {
      for (int e = threadIdx.x; e < ne; e += 256) {
        const int cr = e / CW, q = e - cr * CW;
        const int ci = cr / IR, r = cr - ci * IR;
        const int iy = 2 * oy0 - 1 + r, ix0 = (q - 1) * 8;
        const bool ok = iy >= 0 && iy < a.H && q >= 1 && ix0 < a.W;
        *reinterpret_cast<h8*>(ssm + cr * WP + q * 8) =
            *(ok ? reinterpret_cast<const h8*>(x + ((int64_t(n) * a.C + ci) * a.H + iy) * a.W + ix0)
                 : reinterpret_cast<const h8*>(g_zero_line));
      }
    }
  } else {
    for (int e = threadIdx.x; e < ne; e += 256) {
      const int cr = e / CW, q = e - cr * CW;
      const int ci = cr / IR, r = cr - ci * IR;
      const int iy = 2 * oy0 - 1 + r, ix0 = (q - 1) * 8;
      h8 v = h8{0, 0, 0, 0, 0, 0, 0, 0};
      if (iy >= 0 && iy < a.H && q >= 1 && ix0 < a.W) {
        const T* src = x + ((int64_t(n) * a.C + ci) * a.H + iy) * a.W + ix0;
        RawRun<T, 8> run;
        run.load(src);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (_Float16)run.get(j);
      }
      *reinterpret_cast<h8*>(ssm + cr * WP + q * 8) = v;
    }
  }
  // this lane's 8 k values: (ci, ky, kx) -> LDS offset relative to the pixel's window origin.  k >= cin * 9 (the
  // zero-padded tail of the K-step) reads tap (0, 0, 0) again: its weights are zero and the value finite
  // (that tap is also a real tap of the same output), so the gather needs no per-element select or exec mask
  int koff[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int kq = 8 * grp + j, ci = kq / 9, t = kq - ci * 9;
    koff[j] = kq < a.C * 9 ? (ci * IR + t / 3) * WP + (t % 3) : 0;  // staged col of ix = 2 ox - 1 + kx is 2 ox + 7 + kx
  }
  h8 af[RC];
#pragma unroll
  for (int r = 0; r < RC; ++r) af[r] = reinterpret_cast<const h8*>(wfr)[r * 64 + lane];
  float bz[RC][4];
#pragma unroll
  for (int r = 0; r < RC; ++r)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int co = r * 16 + grp * 4 + j;
      bz[r][j] = bias_or0(a.bias, co, a.cout);
    }
  __syncthreads();
  // the block's outputs: rows oy0 .. oy0 + SR - 1 of image n; 32-bit offsets from the block's first pixel
  _Float16* yb = a.y + (int64_t(n) * a.Ho + oy0) * a.Wo * a.ycs;
  const int fpr = (a.Wo + 15) / 16;  // fragments per output row
#pragma unroll
  for (int rr = 0; rr < SR; ++rr) {
    if (oy0 + rr >= a.Ho) break;
    for (int fx = wave; fx < fpr; fx += 4) {
      const int ox = fx * 16 + col;
      const int base = (2 * rr) * WP + 2 * min(ox, a.Wo - 1) + 7;  // window origin: staged row 2 rr, col 2 ox + 7
      h8 b;
#pragma unroll
      for (int j = 0; j < 8; ++j) b[j] = ssm[base + koff[j]];
      _Float16* yo = yb + (rr * a.Wo + ox) * a.ycs;
#pragma unroll
      for (int r = 0; r < RC; ++r) {
        const f4 d = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[r], b, f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        const int co0 = r * 16 + grp * 4;
        if (ox < a.Wo && co0 < a.cout) {
          h4 o;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float t = d[j] + bz[r][j];
            o[j] = (_Float16)(a.act ? silu(t) : t);
          }
          *reinterpret_cast<h4*>(yo + co0) = o;
        }
      }
    }
  }
}

// ============================================================================ dispatch
static int grid_cap(int64_t blocks) { return int(blocks < 65535 * 16 ? blocks : 65535 * 16); }

template <int KS, int RC, int RP>
static void launch_dense(const ConvArgs& a, int out_kind, bool fast, dim3 grid, hipStream_t s) {
#define CONV_L(O, F) FCE_LAUNCH((conv_mfma_kernel<KS, RC, RP, O, F>), grid, dim3(256), 0, s, a)
#define CONV_O(O)  \
  if (fast)        \
    CONV_L(O, true); \
  else             \
    CONV_L(O, false);
  if (KS == 3) {  // 3x3 convs always store fp16 (Conv + BN + SiLU [+ residual])
    CONV_O(OUT_F16);
    return;
  }
  switch (out_kind) {
    case OUT_F16:
      CONV_O(OUT_F16);
      break;
    case OUT_F32:
      CONV_O(OUT_F32);
      break;
    case OUT_WSTORE:
      CONV_O(OUT_WSTORE);
      break;
    case OUT_DFL:
      CONV_O(OUT_DFL);
      break;
    case OUT_CLS:
      CONV_O(OUT_CLS);
      break;
    default:
      CONV_O(OUT_ACCUM);
      break;
  }
#undef CONV_O
#undef CONV_L
}

template <int KS, int RP>
static void launch_dense_rp(const ConvArgs& a, int out_kind, bool fast, int rc, hipStream_t s) {
  const int cotiles = (a.cout + 15) / 16;
  ConvArgs b = a;
  b.gx = (a.P + 64 * RP - 1) / (64 * RP);
  b.gy = (cotiles + rc - 1) / rc;
  dim3 grid(unsigned(b.gx * b.gy));
  if (rc == 1)
    launch_dense<KS, 1, RP>(b, out_kind, fast, grid, s);
  else if (rc == 2)
    launch_dense<KS, 2, RP>(b, out_kind, fast, grid, s);
  else
    launch_dense<KS, 4, RP>(b, out_kind, fast, grid, s);
}

// Tile choice: a wave owns (16*RC couts) x (16*RP pixels).  Big tiles reuse each loaded fragment
// more; small layers (20x20, 40x40 maps) need more waves in flight to hide load latency, so the
// tile shrinks until the launch has >= ~4 waves per SIMD (4096 waves on 256 CUs) or hits 1x1.
static void pick_tile(int P, int cotiles, bool need_rc4, int* rc, int* rp) {
  constexpr int64_t kTargetWaves = 4096;
  int c = cotiles >= 4 ? 4 : cotiles >= 2 ? 2 : 1;
  int p = 4;
  auto waves = [&](int c_, int p_) { return int64_t((P + 16 * p_ - 1) / (16 * p_)) * ((cotiles + c_ - 1) / c_); };
  while (waves(c, p) < kTargetWaves) {
    if (p > 1) {
      p /= 2;
    } else if (c > 1 && !need_rc4) {
      c /= 2;
    } else {
      break;
    }
  }
  *rc = c;
  *rp = p;
}

template <int KS>
static void launch_dense_rc(const ConvArgs& a, int out_kind, bool fast, int rc, int rp, hipStream_t s) {
  if (rp == 1)
    launch_dense_rp<KS, 1>(a, out_kind, fast, rc, s);
  else if (rp == 2)
    launch_dense_rp<KS, 2>(a, out_kind, fast, rc, s);
  else
    launch_dense_rp<KS, 4>(a, out_kind, fast, rc, s);
}

// Tile-kernel configurations, coded 0x100 | rc | rp << 4 | log2(cw) << 12 | (kp - 1) << 14 | al << 15
static constexpr size_t tile3_lds(int s, int rp, int cw, int kp) {
  return size_t(((4 / cw) * rp - 1) * s + 3) * (15 * s + 3) * 4 * kp * 16;
}
// A-in-LDS variants: rc 2 / 4, rc * rp <= 16 (registers: the accumulators plus up to 16 staged pieces
// per thread), input tile + weight stage within 96 KiB
static constexpr bool tile3al_ok(int s, int rc, int rp, int cw, int kp) {
  return (rc == 2 || rc == 4) && (rp == 2 || rp == 4 || rp == 8) && (cw == 1 || cw == 2 || cw == 4) &&
         (kp == 1 || kp == 2) && rc * rp <= 16 &&
         tile3_lds(s, rp, cw, kp) + size_t(cw) * rc * 9 * kp * 1024 <= 96 * 1024;
}
// rp = 8 (8 output rows per wave: every A fragment read from L2 feeds 8 MFMAs, the m/l-scale 3x3 convs
// are L2-bound at rp <= 4) with rc 1 (any cw: the weight stream per output pixel halves at 32 accumulator
// registers) or with the couts split over 2 / 4 waves
static bool tile3_ok(int s, int rc, int rp, int cw, int kp) {
  return (rc == 1 || rc == 2 || rc == 4) && (rp == 1 || rp == 2 || rp == 4 || (rp == 8 && (rc == 1 || cw >= 2))) &&
         (cw == 1 || cw == 2 || cw == 4) && (kp == 1 || kp == 2) && rc * rp <= 32 &&
         tile3_lds(s, rp, cw, kp) <= 80 * 1024;
}

// Register tiles a dense conv may run with, encoded rc | rp << 4, or depthwise kernel variants,
// encoded 100 + variant (the executor times them at plan time and keeps the fastest; neither
// changes the per-output summation order, so results are bitwise the same for every choice).
// Returns the count; 0 for the stem.
static bool tile3al_on() {  // FCE_TILE3AL=1 adds the A-in-LDS 3x3 variants (they lose on every l / m layer
                             // measured, so the planner does not spend autotune time on them by default)
  const char* e = getenv("FCE_TILE3AL");
  return e && atoi(e) != 0;
}
static bool no_ring() {  // diagnostics: FCE_NO_RING=1 drops the persistent (ring) variants
  static const bool v = [] {
    const char* e = getenv("FCE_NO_RING");
    return e && atoi(e) != 0;
  }();
  return v;
}

// the 32x32x16 ring 3x3 candidates (0x900) are opt-in, FCE_RING32=1: on every shape they apply to in the BASELINE
// models (the 64 -> 64 Detect box 3x3s, the 32 / 64-channel bottlenecks) they ran slower than the 16x16x32 ring,
// e.g. 33.4 against 23.8 us on n32's P3 box convs (256 VGPRs: one wave per SIMD), profiles/r05_ring32_tune.txt
static bool no_ring32() {  // read per call, like FCE_WIDE3 (the variant tests switch it on mid-process)
  const char* e = getenv("FCE_RING32");
  return !(e && atoi(e) != 0);
}
static bool no_gemm3() {  // diagnostics / A-B runs: FCE_NO_GEMM3=1 drops the implicit-GEMM 3x3 candidates (0xC00)
  const char* e = getenv("FCE_NO_GEMM3");
  return e && atoi(e) != 0;
}

static bool no_dring() {  // A/B runs: FCE_NO_DRING=1 drops the LDS-DMA ring 3x3 candidates (0xD00)
  const char* e = getenv("FCE_NO_DRING");
  return e && atoi(e) != 0;
}

static bool wide3_on() {  // read per call, like FCE_TILE3AL (the variant tests switch it on mid-process)
  const char* e = getenv("FCE_WIDE3");
  return e && atoi(e) != 0;
}

int conv_tile_candidates(const fce_conv_desc& d, int det_box, int in_w, int* out, int cap) {
  if (is_stem(d)) return 0;
  if (is_dw(d)) {  // depthwise kernel variants, coded 100 + variant
    int v[8];  // every variant dwconv_variants lists (a cap of 4 used to drop the 4-row column runs)
    const int nv = d.k == 3 ? dwconv_variants(d.cin, in_w, v, 8) : 0;
    for (int i = 0; i < nv && i < cap; ++i) out[i] = 100 + v[i];
    return std::min(nv, cap);
  }
  const int cotiles = (d.cout + 15) / 16;
  int n = 0;
  for (int rc : {1, 2, 4}) {
    if (det_box ? rc != 4 : (rc > 1 && (rc >> 1) >= cotiles)) continue;
    for (int rp : {1, 2, 4})
      if (n < cap) out[n++] = rc | (rp << 4);
  }
  if (d.k == 1 && d.cin % 32 == 0 && stream_nsm(d.cin / 32) > 0)  // streaming 1x1: 0x300 | rc | rp << 4
    for (int rc : {1, 2, 4}) {
      if (det_box ? rc != 4 : (rc > 1 && (rc >> 1) >= cotiles)) continue;
      for (int rp : {1, 2})
        if (n < cap && stream_ok(stream_nsm(d.cin / 32), rc, rp)) out[n++] = 0x300 | rc | (rp << 4);
    }
  if (d.k == 1 && d.stride == 1)  // LDS-staged 1x1: 0x400 | rc | rp << 4 | log2(wp) << 12
    for (int wl = 0; wl < 3; ++wl)
      for (int rc : {1, 2, 4})
        for (int rp : {1, 2, 4}) {
          const int wp = 1 << wl, cb = (4 / wp) * rc;
          if (!lds1_cfg_ok(rc, rp, wp)) continue;
          if (det_box ? (rc != 4 || wp != 4) : (cb > 1 && (cb >> 1) >= cotiles)) continue;
          if (n < cap) out[n++] = 0x400 | rc | (rp << 4) | (wl << 12);
        }
  if (d.k == 1 && d.stride == 1 && !no_ring())  // persistent LDS ring 1x1: 0x500 | rc | rp << 4 | log2(wp) << 12
    for (int wl = 0; wl < 3; ++wl)
      for (int rc : {1, 2, 4})
        for (int rp : {1, 2, 4}) {
          const int wp = 1 << wl, cb = (4 / wp) * rc;
          if (!ring_ok((d.cin / 8 + 3) / 4, rc, rp, wp)) continue;
          if (det_box ? (rc != 4 || wp != 4) : (cb > 1 && (cb >> 1) >= cotiles)) continue;
          if (n < cap) out[n++] = 0x500 | rc | (rp << 4) | (wl << 12);
        }
  if (d.k == 1 && d.stride == 1 && !det_box && d.cin >= 64 && d.cout >= 64)  // big tiles: 0xB00 | wcl << 4 | nw4 | wr4
    for (int split : {0, 1})   // one ring, or split rings with a deep pixel ring (0x20)
      for (int nwc : {0, 1, 2})  // 8 waves x 8 cout tiles, 4 x 8, 4 x 4
        for (int wcl = 0; wcl < 2; ++wcl)
          if (n < cap && (((nwc == 2 ? 4 : 8) << wcl) >> 1) < cotiles &&
              (!split || big1_split_ok(1 << wcl, nwc ? 4 : 8, nwc == 2 ? 4 : 8)))
            out[n++] = 0xB00 | (wcl << 4) | (split << 5) | ((nwc > 0) << 6) | ((nwc == 2) << 7);
  if (pipe1_ok(d, det_box))  // big-tile K-pipelined 1x1: 0x700 | log2(wp) << 12
    for (int wl = 0; wl < 3; ++wl) {
      const int cb = (4 >> wl) * 4;
      if ((cb >> 1) >= cotiles) continue;
      if (n < cap) out[n++] = 0x700 | (wl << 12);
    }
  if (d.k == 3 && d.cin % 32 != 0 && d.cin <= 64 && d.up == 0 && !det_box)  // small-cin LDS tile: 0x200 | ..
    for (int rc : {1, 2, 4}) {
      if (rc > 1 && (rc >> 1) >= cotiles) continue;
      for (int rp : {1, 2, 4})
        if (n < cap && small_tile_lds(d.stride, rp, d.cin) <= 64 * 1024) out[n++] = 0x200 | rc | (rp << 4);
    }
  if (d.k == 3 && (d.cin == 32 || d.cin == 64) && d.up == 0 && !det_box && !no_ring())  // persistent: 0x600 | rp << 4
    for (int rp : {1, 2, 4})
      for (int pd : {1, 2})
        if (n < cap) out[n++] = 0x600 | (rp << 4) | (pd - 1);
  if (d.k == 3 && (d.cin == 32 || d.cin == 64 || d.cin == 128) && d.cout % 16 == 0 && d.up == 0 && !det_box &&
      !no_ring() && !no_dring())
    for (int cpw : {1, 2})  // persistent LDS-DMA ring: 0xD00 | rp << 4 | (cpw - 1) << 3 | (sub - 1) << 2 | (nbuf - 2)
      for (int rp : {1, 2, 4, 8})
        for (int sub : {1, 2})
          for (int nbuf : {2, 3, 4})
            if (n < cap && d.cout % (16 * cpw) == 0 && (rp < 8 || cpw == 1) &&
                dring3_offer(d.stride, rp, d.cin / 32, nbuf, cpw, sub))
              out[n++] = 0xD00 | (rp << 4) | ((cpw - 1) << 3) | ((sub - 1) << 2) | (nbuf - 2);
  if (d.k == 3 && (d.cin == 32 || d.cin == 64) && d.cout % 32 == 0 && d.up == 0 && !det_box && !no_ring() &&
      !no_ring32())  // persistent 32x32x16 ring: 0x900 | rpw << 4 | log2(wc) << 12
    for (int wcl = 0; wcl < 3; ++wcl)
      for (int rpw : {1, 2})
        if (n < cap && ((32 << wcl) >> 1) < d.cout && ring32_fits(d.stride, d.cin / 32, 1 << wcl, rpw))
          out[n++] = 0x900 | (rpw << 4) | (wcl << 12);
  if (d.k == 3 && d.cin % 32 == 0 && d.up == 0)  // LDS halo-tile kernel: 0x100 | rc | rp << 4 | cw, kp bits
    for (int kp : {1, 2}) {
      if (kp == 2 && d.cin % 64 != 0) continue;
      for (int cwl = 0; cwl < 3; ++cwl)
        for (int rc : {1, 2, 4}) {
          const int cb = (1 << cwl) * rc;
          if (cb > 1 && (cb >> 1) >= cotiles) continue;
          for (int rp : {1, 2, 4, 8})
            if (n < cap && tile3_ok(d.stride, rc, rp, 1 << cwl, kp))
              out[n++] = 0x100 | rc | (rp << 4) | (cwl << 12) | ((kp - 1) << 14);
        }
    }
  if (d.k == 3 && d.cin % 32 == 0 && d.up == 0 && d.cin >= 64 && d.cout >= 64 && !det_box)  // big tile: 0x800 | wm << 4
    for (int ab : {2, 3})
      for (int wm : {1, 2})
        if (n < cap && big3_ok(d.stride, wm, ab) && (wm == 1 || d.cout >= 128)) out[n++] = 0x800 | (wm << 4) | ((ab - 2) << 12);
  if (d.k == 3 && d.cin % 32 == 0 && d.up == 0 && d.cin >= 64 && d.cout >= 64 && !det_box && !no_gemm3())  // 0xC00
    for (int split : {0, 1})  // split rings (0x20): wc 2 only
      for (int nwc : {0, 1, 2})
        for (int wcl = split; wcl < 2; ++wcl)
          if (n < cap && (((nwc == 2 ? 4 : 8) << wcl) >> 1) < cotiles &&
              (!split || big1_split_ok(1 << wcl, nwc ? 4 : 8, nwc == 2 ? 4 : 8)))
            out[n++] = 0xC00 | (wcl << 4) | (split << 5) | ((nwc > 0) << 6) | ((nwc == 2) << 7);
  // wide tile (opt-in, FCE_WIDE3=1: measured at parity or slower on every m/l shape): 0xA00 | cwl << 4
  if (d.k == 3 && d.cin % 32 == 0 && d.up == 0 && d.cin >= 64 && d.cout >= 64 && !det_box && wide3_on())
    for (int cwl = 0; cwl < 3; ++cwl)
      if (n < cap && wide3_ok(d.stride, 1 << cwl) && ((4 << cwl) >> 1) < cotiles) out[n++] = 0xA00 | (cwl << 4);
  if (d.k == 3 && d.cin % 32 == 0 && d.up == 0 && d.cin >= 128 && tile3al_on())  // A in LDS: | 1 << 15
    for (int kp : {1, 2}) {
      if (kp == 2 && d.cin % 64 != 0) continue;
      for (int cwl = 0; cwl < 3; ++cwl)
        for (int rc : {2, 4}) {
          const int cb = (1 << cwl) * rc;
          if ((cb >> 1) >= cotiles) continue;
          for (int rp : {2, 4, 8})
            if (n < cap && tile3al_ok(d.stride, rc, rp, 1 << cwl, kp))
              out[n++] = 0x100 | rc | (rp << 4) | (cwl << 12) | ((kp - 1) << 14) | (1 << 15);
        }
    }
  return n;
}

template <int S, int RC, int RP, int CW, int KP>
static void launch_tile3_k(const ConvArgs& a, bool al, dim3 grid, hipStream_t s) {
  if (al) {
    if constexpr (tile3al_ok(S, RC, RP, CW, KP)) {
      static_assert(Tile3Geom<S, RC, RP, CW, KP, true>::lds <= 160 * 1024, "A-in-LDS tile too large");
      FCE_LAUNCH((conv3x3_tile_kernel<S, RC, RP, CW, KP, true>), grid, dim3(256), 0, s, a);
    }
  } else if constexpr (tile3_lds(S, RP, CW, KP) <= 80 * 1024) {
    FCE_LAUNCH((conv3x3_tile_kernel<S, RC, RP, CW, KP, false>), grid, dim3(256), 0, s, a);
  }
}

template <int S, int RC, int RP>
static void launch_tile3_w(const ConvArgs& a, int cw, int kp, bool al, dim3 grid, hipStream_t s) {
  if (cw == 1)
    kp == 1 ? launch_tile3_k<S, RC, RP, 1, 1>(a, al, grid, s) : launch_tile3_k<S, RC, RP, 1, 2>(a, al, grid, s);
  else if (cw == 2)
    kp == 1 ? launch_tile3_k<S, RC, RP, 2, 1>(a, al, grid, s) : launch_tile3_k<S, RC, RP, 2, 2>(a, al, grid, s);
  else
    kp == 1 ? launch_tile3_k<S, RC, RP, 4, 1>(a, al, grid, s) : launch_tile3_k<S, RC, RP, 4, 2>(a, al, grid, s);
}

template <int S, int RC>
static void launch_tile3_rc(const ConvArgs& a, int rp, int cw, int kp, bool al, dim3 grid, hipStream_t s) {
  if (rp == 1)
    launch_tile3_w<S, RC, 1>(a, cw, kp, al, grid, s);
  else if (rp == 2)
    launch_tile3_w<S, RC, 2>(a, cw, kp, al, grid, s);
  else if (rp == 4)
    launch_tile3_w<S, RC, 4>(a, cw, kp, al, grid, s);
  else {  // rp == 8: rc 1 or cw 2 / 4 (tile3_ok), any cw with A in LDS (tile3al_ok)
    if (cw == 1)
      kp == 1 ? launch_tile3_k<S, RC, 8, 1, 1>(a, al, grid, s) : launch_tile3_k<S, RC, 8, 1, 2>(a, al, grid, s);
    else if (cw == 2)
      kp == 1 ? launch_tile3_k<S, RC, 8, 2, 1>(a, al, grid, s) : launch_tile3_k<S, RC, 8, 2, 2>(a, al, grid, s);
    else
      kp == 1 ? launch_tile3_k<S, RC, 8, 4, 1>(a, al, grid, s) : launch_tile3_k<S, RC, 8, 4, 2>(a, al, grid, s);
  }
}

template <int S>
static void launch_tile3_s(const ConvArgs& a, int rc, int rp, int cw, int kp, bool al, dim3 grid, hipStream_t s) {
  if (rc == 1)
    launch_tile3_rc<S, 1>(a, rp, cw, kp, al, grid, s);
  else if (rc == 2)
    launch_tile3_rc<S, 2>(a, rp, cw, kp, al, grid, s);
  else
    launch_tile3_rc<S, 4>(a, rp, cw, kp, al, grid, s);
}

template <int S, int RC>
static void launch_small3_rc(const ConvArgs& a, int rp, dim3 grid, size_t lds, hipStream_t s) {
  // compile-time cin for 8 and 16 channels (the n / s scales' small-cin 3x3s), runtime otherwise
#define SMALL3(RPV)                                                                                     \
  do {                                                                                                  \
    if (a.cpt == 1)                                                                                     \
      FCE_LAUNCH((conv3x3_tile_small_kernel<S, RC, RPV, 1>), grid, dim3(256), lds, s, a);               \
    else if (a.cpt == 2)                                                                                \
      FCE_LAUNCH((conv3x3_tile_small_kernel<S, RC, RPV, 2>), grid, dim3(256), lds, s, a);               \
    else                                                                                                \
      FCE_LAUNCH((conv3x3_tile_small_kernel<S, RC, RPV, 0>), grid, dim3(256), lds, s, a);               \
  } while (0)
  if (rp == 1)
    SMALL3(1);
  else if (rp == 2)
    SMALL3(2);
  else
    SMALL3(4);
#undef SMALL3
}

template <int S>
static void launch_small3_s(const ConvArgs& a, int rc, int rp, dim3 grid, size_t lds, hipStream_t s) {
  if (rc == 1)
    launch_small3_rc<S, 1>(a, rp, grid, lds, s);
  else if (rc == 2)
    launch_small3_rc<S, 2>(a, rp, grid, lds, s);
  else
    launch_small3_rc<S, 4>(a, rp, grid, lds, s);
}

static int launch_small3(const ConvArgs& a, int rc, int rp, int stride, int n, hipStream_t s) {
  const int th = 4 * rp;
  const int64_t tiles = int64_t((a.Wo + 15) / 16) * ((a.Ho + th - 1) / th) * n;
  FCE_CHECK(tiles < (int64_t(1) << 31), "conv 3x3 small tile: grid too large");
  const size_t lds = small_tile_lds(stride, rp, a.cin);
  FCE_CHECK(lds <= 64 * 1024, "conv 3x3 small tile: LDS tile too large");
  ConvArgs b = a;
  b.gy = ((a.cout + 15) / 16 + rc - 1) / rc;
  FCE_CHECK(tiles * b.gy < (int64_t(1) << 31), "conv 3x3 small tile: grid too large");
  const dim3 grid(unsigned(tiles * b.gy));
  if (stride == 1)
    launch_small3_s<1>(b, rc, rp, grid, lds, s);
  else
    launch_small3_s<2>(b, rc, rp, grid, lds, s);
  return launch_status("conv3x3_tile_small_kernel");
}

static int launch_tile3(const ConvArgs& a, int rc, int rp, int cw, int kp, bool al, int stride, int n, hipStream_t s) {
  FCE_CHECK(al ? tile3al_ok(stride, rc, rp, cw, kp) : tile3_ok(stride, rc, rp, cw, kp), "conv 3x3 tile: bad configuration");
  const int th = (4 / cw) * rp;
  const int64_t tiles = int64_t((a.Wo + 15) / 16) * ((a.Ho + th - 1) / th) * n;
  FCE_CHECK(tiles < (int64_t(1) << 31), "conv 3x3 tile: grid too large");
  ConvArgs b = a;
  b.gy = ((a.cout + 15) / 16 + cw * rc - 1) / (cw * rc);
  FCE_CHECK(tiles * b.gy < (int64_t(1) << 31), "conv 3x3 tile: grid too large");
  const dim3 grid(unsigned(tiles * b.gy));
  if (stride == 1)
    launch_tile3_s<1>(b, rc, rp, cw, kp, al, grid, s);
  else
    launch_tile3_s<2>(b, rc, rp, cw, kp, al, grid, s);
  return launch_status("conv3x3_tile_kernel");
}

template <int S, int RP, int NCH, int PD>
static void launch_ring3_k(const ConvArgs& a, dim3, int ntiles, hipStream_t s) {
  static const int occ = blocks_per_cu(conv3x3_ring_kernel<S, RP, NCH, PD>, 0);
  const int nslot = ring_slots(ntiles, a.gy, occ);
  FCE_LAUNCH((conv3x3_ring_kernel<S, RP, NCH, PD>), dim3(unsigned(8 * a.gy * nslot)), dim3(256), 0, s, a, nslot);
}

template <int S, int NCH>
static void launch_ring3_s(const ConvArgs& a, int rp, int pd, dim3 grid, int nslot, hipStream_t s) {
  if (pd == 2) {
    if (rp == 1)
      launch_ring3_k<S, 1, NCH, 2>(a, grid, nslot, s);
    else if (rp == 2)
      launch_ring3_k<S, 2, NCH, 2>(a, grid, nslot, s);
    else
      launch_ring3_k<S, 4, NCH, 2>(a, grid, nslot, s);
  } else if (rp == 1) {
    launch_ring3_k<S, 1, NCH, 1>(a, grid, nslot, s);
  } else if (rp == 2) {
    launch_ring3_k<S, 2, NCH, 1>(a, grid, nslot, s);
  } else {
    launch_ring3_k<S, 4, NCH, 1>(a, grid, nslot, s);
  }
}


template <int S, int NCH, int WC, int RPW>
static void launch_ring32_k(const ConvArgs& a, int ntiles, hipStream_t s) {
  if constexpr (!ring32_fits(S, NCH, WC, RPW)) {
    return;  // not a candidate (conv_tile_candidates checks ring32_fits)
  } else {
  static const int occ = blocks_per_cu(conv3x3_ring32_kernel<S, NCH, WC, RPW>, 0);
  const int nslot = ring_slots(ntiles, a.gy, occ);
  FCE_LAUNCH((conv3x3_ring32_kernel<S, NCH, WC, RPW>), dim3(unsigned(8 * a.gy * nslot)), dim3(256), 0, s, a, nslot);
  }
}

template <int S, int NCH>
static void launch_ring32_s(const ConvArgs& a, int wc, int rpw, int ntiles, hipStream_t s) {
  if (wc == 1)
    rpw == 1 ? launch_ring32_k<S, NCH, 1, 1>(a, ntiles, s) : launch_ring32_k<S, NCH, 1, 2>(a, ntiles, s);
  else if (wc == 2)
    rpw == 1 ? launch_ring32_k<S, NCH, 2, 1>(a, ntiles, s) : launch_ring32_k<S, NCH, 2, 2>(a, ntiles, s);
  else
    rpw == 1 ? launch_ring32_k<S, NCH, 4, 1>(a, ntiles, s) : launch_ring32_k<S, NCH, 4, 2>(a, ntiles, s);
}

static int launch_ring32(const ConvArgs& a0, int wc, int rpw, int stride, hipStream_t s) {
  FCE_CHECK((a0.cin == 32 || a0.cin == 64) && a0.cout % 32 == 0 && (wc == 1 || wc == 2 || wc == 4) &&
                (rpw == 1 || rpw == 2) && (stride == 1 || stride == 2) && ring32_fits(stride, a0.cin / 32, wc, rpw),
            "conv 3x3 ring32: bad configuration");
  ConvArgs a = a0;
  const int th = 2 * rpw * (4 / wc);
  const int64_t ntiles = int64_t((a.Wo + 15) / 16) * ((a.Ho + th - 1) / th) * a.N;
  FCE_CHECK(ntiles < (int64_t(1) << 30), "conv 3x3 ring32: too many tiles");
  a.gy = (a.cout + 32 * wc - 1) / (32 * wc);
  const int nch = a.cin / 32;
  if (stride == 1)
    nch == 1 ? launch_ring32_s<1, 1>(a, wc, rpw, int(ntiles), s) : launch_ring32_s<1, 2>(a, wc, rpw, int(ntiles), s);
  else
    nch == 1 ? launch_ring32_s<2, 1>(a, wc, rpw, int(ntiles), s) : launch_ring32_s<2, 2>(a, wc, rpw, int(ntiles), s);
  return launch_status("conv3x3_ring32_kernel");
}

// pd: tiles of staged input in flight ahead of the LDS store (1, or 2: two register sets)
static int launch_ring3(const ConvArgs& a0, int rp, int pd, int stride, hipStream_t s) {
  FCE_CHECK((a0.cin == 32 || a0.cin == 64) && (rp == 1 || rp == 2 || rp == 4), "conv 3x3 ring: bad configuration");
  ConvArgs a = a0;
  const int nch = a.cin / 32;
  const int64_t ntiles = int64_t((a.Wo + 15) / 16) * ((a.Ho + rp - 1) / rp) * a.N;
  FCE_CHECK(ntiles < (int64_t(1) << 30), "conv 3x3 ring: too many tiles");
  a.gy = ((a.cout + 15) / 16 + 3) / 4;
  const int nslot = int(ntiles);  // the leaf launcher turns the tile count into slots (occupancy)
  const dim3 grid(1);
  if (stride == 1)
    nch == 1 ? launch_ring3_s<1, 1>(a, rp, pd, grid, nslot, s) : launch_ring3_s<1, 2>(a, rp, pd, grid, nslot, s);
  else
    nch == 1 ? launch_ring3_s<2, 1>(a, rp, pd, grid, nslot, s) : launch_ring3_s<2, 2>(a, rp, pd, grid, nslot, s);
  return launch_status("conv3x3_ring_kernel");
}

int conv2d_impl(const fce_conv_desc& d, const fce_tensor& x, const void* w, const float* bias, const fce_tensor* res,
                const fce_tensor& y, const fce_detect_epi* det, hipStream_t s, int tile, const fce_tensor* dup = nullptr,
                int duplo = 0) {
  FCE_CHECK(d.k == 1 || d.k == 3 || (is_stem(d) && d.k <= 7), "conv: kernel size must be 1 or 3");
  FCE_CHECK(d.stride >= 1 && d.stride <= 2, "conv: stride must be 1 or 2");
  FCE_CHECK(x.n == y.n && x.c == d.cin && y.c == d.cout, "conv: channel/batch mismatch");
  const int Hin = x.h << d.up, Win = x.w << d.up;
  const int pad = d.k / 2;
  const int Ho = (Hin + 2 * pad - d.k) / d.stride + 1, Wo = (Win + 2 * pad - d.k) / d.stride + 1;
  FCE_CHECK(y.h == Ho && y.w == Wo, "conv: output spatial size mismatch");
  FCE_CHECK(y.layout == FCE_NHWC, "conv: output must be NHWC");
  if (int64_t(y.n) * Ho * Wo == 0) return FCE_OK;

  if (is_stem(d)) {
    FCE_CHECK(x.layout == FCE_NCHW && y.dtype == FCE_F16 && d.up == 0, "stem conv: NCHW input, f16 NHWC output");
    FCE_CHECK(d.epilogue == FCE_EPI_STORE && res == nullptr, "stem conv: plain store only");
    FCE_CHECK(y.cstride % 8 == 0 && y.coff % 8 == 0 && d.cout % 8 == 0, "stem conv: output slice must be 8-aligned");
    StemArgs a{x.data, x.dtype, x.n, x.c, x.h, x.w, d.stride, d.k, Ho, Wo, d.cout, static_cast<const float*>(w),
               bias, static_cast<_Float16*>(y.data) + y.coff, y.cstride, d.act};
    const int64_t P = int64_t(x.n) * Ho * Wo;
    const int blocks = grid_cap((P + 255) / 256);
    int coutT = d.cout <= 16 ? 16 : d.cout <= 32 ? 32 : d.cout <= 64 ? 64 : d.cout <= 96 ? 96 : 0;
    FCE_CHECK(coutT > 0, "stem conv: cout > 96 unsupported");
    const size_t shm = size_t(x.c) * d.k * d.k * coutT * sizeof(float);
    const int PX = coutT <= 32 ? 2 : 1;  // measured: PX 2 beats 4 (occupancy) and 1 (reuse) at cout 16
    const char* sv = getenv("FCE_STEM_VALU");  // diagnostics: the fp32 VALU stem instead of MFMA
    // the staged rows exceed 64 KiB above W = 1168 (imgsz 1280: 70 KiB): gfx950 LDS opt-in up to 160 KiB
    static const int SRE = [] {  // output rows per block (FCE_STEM_SR = 2 / 4 / 8; measured default 4)
      const char* e = getenv("FCE_STEM_SR");
      const int v = e ? atoi(e) : 4;
      return v == 2 || v == 8 ? v : 4;
    }();
    int SR = SRE;
    if (size_t(x.c) * (2 * SR + 1) * (x.w + 16) * 2 + 16 > 160 * 1024) SR = 4;
    if (stem_mfma_ok(d) && d.stride == 2 && x.c == d.cin && d.cout % 16 == 0 && x.w % 8 == 0 &&
        size_t(x.c) * (2 * SR + 1) * (x.w + 16) * 2 + 16 <= 160 * 1024 && !(sv && atoi(sv))) {
      // + the dummy staging slot
      const size_t lds = size_t(x.c) * (2 * SR + 1) * (x.w + 16) * sizeof(_Float16) + 16;
      const int64_t blocks2 = int64_t(x.n) * ((Ho + SR - 1) / SR);
      FCE_CHECK(blocks2 < (int64_t(1) << 31), "stem conv: input too large");
      const _Float16* wfr = reinterpret_cast<const _Float16*>(static_cast<const char*>(w) + stem_fp32_bytes(d));
      const int rc = d.cout / 16;
#define STEMM_SR(T, RC, SRC)                                                                                  \
  do {                                                                                                        \
    static const bool big = hipFuncSetAttribute(reinterpret_cast<const void*>(&stem_mfma_kernel<T, RC, SRC>), \
                                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) ==    \
                            hipSuccess;                                                                       \
    if (!big && lds > 64 * 1024) return fail(FCE_ERR_HIP, "stem conv: cannot opt in to >64 KiB LDS");        \
    FCE_LAUNCH((stem_mfma_kernel<T, RC, SRC>), dim3(unsigned(blocks2)), dim3(256), lds, s, a, wfr);           \
  } while (0)
#define STEMM(T, RC)          \
  do {                        \
    if (SR == 2)              \
      STEMM_SR(T, RC, 2);     \
    else if (SR == 8)         \
      STEMM_SR(T, RC, 8);     \
    else                      \
      STEMM_SR(T, RC, 4);     \
  } while (0)
#define STEMM_T(T)          \
  do {                      \
    if (rc == 1)            \
      STEMM(T, 1);          \
    else if (rc == 2)       \
      STEMM(T, 2);          \
    else if (rc == 3)       \
      STEMM(T, 3);          \
    else                    \
      STEMM(T, 4);          \
  } while (0)
      if (x.dtype == FCE_F16)
        STEMM_T(_Float16);
      else if (x.dtype == FCE_F32)
        STEMM_T(float);
      else
        STEMM_T(uint8_t);
#undef STEMM_T
#undef STEMM
#undef STEMM_SR
      return launch_status("stem_mfma_kernel");
    }
    if (d.k == 3 && d.stride == 2 && x.c == 3 && x.w % (2 * PX) == 0) {
      const int64_t threads = int64_t(x.n) * Ho * ((Wo + PX - 1) / PX);
      FCE_CHECK(threads < (int64_t(1) << 31), "stem conv: input too large");
      const dim3 grid(unsigned((threads + 255) / 256));
#define STEM2_LAUNCH(CT, P, T)                                                                       \
  FCE_LAUNCH((stem_s2_kernel<CT, P, T>), grid, dim3(256), shm + size_t(256) * P * CT * 2, s, a)
#define STEM2_DT(CT, P)                  \
  do {                                   \
    if (x.dtype == FCE_F16)              \
      STEM2_LAUNCH(CT, P, _Float16);     \
    else if (x.dtype == FCE_F32)         \
      STEM2_LAUNCH(CT, P, float);        \
    else                                 \
      STEM2_LAUNCH(CT, P, uint8_t);      \
  } while (0)
      if (coutT == 16)
        STEM2_DT(16, 2);
      else if (coutT == 32)
        STEM2_DT(32, 2);
      else if (coutT == 64)
        STEM2_DT(64, 1);
      else
        STEM2_DT(96, 1);
#undef STEM2_DT
#undef STEM2_LAUNCH
      return launch_status("stem_s2_kernel");
    }
#define STEM_LAUNCH(CT, T) FCE_LAUNCH((stem_kernel<CT, T>), dim3(blocks), dim3(256), shm, s, a)
#define STEM_DT(CT)                      \
  do {                                   \
    if (x.dtype == FCE_F16)              \
      STEM_LAUNCH(CT, _Float16);         \
    else if (x.dtype == FCE_F32)         \
      STEM_LAUNCH(CT, float);            \
    else                                 \
      STEM_LAUNCH(CT, uint8_t);          \
  } while (0)
    if (coutT == 16)
      STEM_DT(16);
    else if (coutT == 32)
      STEM_DT(32);
    else if (coutT == 64)
      STEM_DT(64);
    else
      STEM_DT(96);
#undef STEM_DT
#undef STEM_LAUNCH
    return launch_status("stem_kernel");
  }

  FCE_CHECK(x.layout == FCE_NHWC && x.dtype == FCE_F16, "conv: input must be NHWC f16");
  FCE_CHECK(x.cstride % 8 == 0 && x.coff % 8 == 0, "conv: input slice must be 8-channel aligned");

  if (is_dw(d)) {
    FCE_CHECK(d.groups == d.cin && d.cin == d.cout && d.cin % 8 == 0, "dwconv: groups == cin == cout, cin % 8 == 0");
    FCE_CHECK(y.dtype == FCE_F16 && d.up == 0 && res == nullptr && d.epilogue == FCE_EPI_STORE && d.k == 3,
              "dwconv: 3x3, plain f16 store only");
    return dwconv3x3(x, d.stride, static_cast<const float*>(w), d.cin, bias, d.act, y, s, tile >= 100 ? tile - 100 : -1);
  }

  FCE_CHECK(d.cin % 8 == 0, "conv: cin must be a multiple of 8");
  int out_kind;
  if (det) {
    FCE_CHECK(det->pred && det->part >= 0 && det->part <= 1 && d.k == 1 && d.up == 0 && res == nullptr,
              "conv detect epilogue: 1x1 conv into pred");
    FCE_CHECK(det->part == 1 || (d.cout == 4 * det->reg_max && det->reg_max == 16),
              "conv detect epilogue: box branch needs 4 x reg_max(16) outputs");
    FCE_CHECK(det->part == 0 || d.cout == det->nc, "conv detect epilogue: cls branch needs nc outputs");
    out_kind = det->part == 0 ? OUT_DFL : OUT_CLS;
  } else if (y.dtype == FCE_F32) {
    FCE_CHECK(d.epilogue == FCE_EPI_STORE && res == nullptr, "conv: f32 output supports plain store only");
    out_kind = OUT_F32;
  } else {
    out_kind = d.epilogue == FCE_EPI_WSTORE ? OUT_WSTORE : d.epilogue == FCE_EPI_ACCUM ? OUT_ACCUM : OUT_F16;
  }
  if (res) {
    FCE_CHECK(res->layout == FCE_NHWC && res->dtype == FCE_F16 && res->c == d.cout && res->h == Ho && res->w == Wo,
              "conv: residual must match the output view");
  }
  DenseGeom g = dense_geom(d);
  ConvArgs a;
  a.x = static_cast<const _Float16*>(x.data) + x.coff;
  a.N = x.n;
  a.Hs = x.h;
  a.Ws = x.w;
  a.xcs = x.cstride;
  a.Hin = Hin;
  a.Win = Win;
  a.up = d.up;
  a.cin = d.cin;
  a.cout = d.cout;
  a.stride = d.stride;
  a.Ho = Ho;
  a.Wo = Wo;
  a.P = y.n * Ho * Wo;
  a.w = static_cast<const _Float16*>(w);
  a.bias = bias;
  a.res = res ? static_cast<const _Float16*>(res->data) + res->coff : nullptr;
  a.rcs = res ? res->cstride : 0;
  a.ycs = y.cstride;
  a.y = y.dtype == FCE_F32 ? static_cast<void*>(static_cast<float*>(y.data) + y.coff)
                           : static_cast<void*>(static_cast<_Float16*>(y.data) + y.coff);
  a.act = d.act;
  a.fw = d.fusion_w;
  a.fn = d.fusion_n;
  a.fi = d.fusion_i;
  a.cpt = g.cpt;
  a.nchunk = g.nchunk;
  a.nsteps = g.nsteps;
  a.nalloc = g.nalloc;
  a.cmagic = g.cpt > 1 ? unsigned(0xFFFFFFFFull / unsigned(g.cpt) + 1ull) : 0u;
  FCE_CHECK(g.nalloc >= ((g.nsteps + 7) & ~7) + 8 && g.nchunk + 64 < 65536, "conv: K too large for the chunk cursor");
  a.vec_ok = (y.cstride % 4 == 0 && y.coff % 4 == 0 && (!res || (res->cstride % 4 == 0 && res->coff % 4 == 0))) ? 1 : 0;
  static const bool no_stg = [] {
    const char* e = getenv("FCE_NO_STG");
    return e && atoi(e) != 0;
  }();
  a.stg = !no_stg && (out_kind == OUT_F16 || out_kind == OUT_WSTORE) && y.dtype == FCE_F16 && d.cout % 8 == 0 &&
          y.cstride % 8 == 0 && y.coff % 8 == 0 && a.vec_ok;
  if (out_kind == OUT_WSTORE || out_kind == OUT_ACCUM) FCE_CHECK(d.fusion_w && d.fusion_n > d.fusion_i, "conv: fusion weights");
  a.pred = det ? det->pred : nullptr;
  a.det_A = det ? det->anchors : 0;
  a.det_a0 = det ? det->anchor_offset : 0;
  a.det_nc = det ? det->nc : 0;
  a.det_hw = Ho * Wo;
  a.det_w = Wo;
  a.det_stride = det ? det->stride : 0.f;
  a.det_best = det ? det->best : nullptr;
  a.dup = nullptr;
  a.dupcs = a.duplo = a.dupn = 0;
  if (dup) {
    FCE_CHECK(d.k == 1 && !is_dw(d) && out_kind == OUT_F16 && dup->layout == FCE_NHWC && dup->dtype == FCE_F16 &&
                  dup->n == y.n && dup->h == Ho && dup->w == Wo && duplo >= 0 && duplo % 8 == 0 && dup->c % 8 == 0 &&
                  duplo + dup->c <= d.cout && dup->cstride % 8 == 0 && dup->coff % 8 == 0 && a.vec_ok,
              "conv: duplicate store needs a 1x1 fp16 plain store and 8-aligned channel ranges");
    a.dup = static_cast<_Float16*>(dup->data) + dup->coff;
    a.dupcs = dup->cstride;
    a.duplo = duplo;
    a.dupn = dup->c;
  }
  const bool fast = d.cin % 32 == 0;
  int rc, rp;
  const int kind = tile >= 0 ? (tile >> 8) & 15 : -1;
  if (kind == 5) {  // persistent LDS ring 1x1 kernel
    rc = tile & 15;
    rp = (tile >> 4) & 15;
    const int wp = 1 << ((tile >> 12) & 3);
    FCE_CHECK(d.k == 1 && d.stride == 1 && ring_ok(g.nsteps, rc, rp, wp), "conv: bad 1x1 ring hint");
    if (out_kind == OUT_DFL) FCE_CHECK(rc == 4 && wp == 4 && g.cotiles == 4, "conv detect epilogue: one wave must own all 64 bins");
    return launch_ring(a, out_kind, rc, rp, wp, s);
  }
  if (kind == 7) {  // big-tile K-pipelined 1x1 kernel
    const int wp = 1 << ((tile >> 12) & 3);
    FCE_CHECK(pipe1_ok(d, out_kind == OUT_DFL) && (tile & 0xFF) == 0 && wp <= 4, "conv: bad big-tile 1x1 hint");
    return launch_pipe1(a, out_kind, wp, s);
  }
  if (kind == 4) {  // LDS-staged 1x1 kernel
    rc = tile & 15;
    rp = (tile >> 4) & 15;
    const int wp = 1 << ((tile >> 12) & 3);
    FCE_CHECK(d.k == 1 && d.stride == 1 && lds1_cfg_ok(rc, rp, wp), "conv: bad LDS 1x1 hint");
    if (out_kind == OUT_DFL) FCE_CHECK(rc == 4 && wp == 4 && g.cotiles == 4, "conv detect epilogue: one wave must own all 64 bins");
    return launch_lds1(a, out_kind, rc, rp, wp, s);
  }
  if (kind == 3) {  // streaming 1x1 kernel
    rc = tile & 15;
    rp = (tile >> 4) & 15;
    FCE_CHECK(d.k == 1 && fast && (rc == 1 || rc == 2 || rc == 4) && (rp == 1 || rp == 2), "conv: bad stream hint");
    if (out_kind == OUT_DFL) FCE_CHECK(rc == 4 && g.cotiles == 4, "conv detect epilogue: one wave must own all 64 bins");
    return launch_stream(a, out_kind, rc, rp, s);
  }
  if (kind == 2) {  // small-cin LDS tile 3x3 kernel
    rc = tile & 15;
    rp = (tile >> 4) & 15;
    FCE_CHECK(d.k == 3 && !fast && d.cin <= 64 && out_kind == OUT_F16 && d.up == 0 && (rc == 1 || rc == 2 || rc == 4) &&
                  (rp == 1 || rp == 2 || rp == 4),
              "conv: bad small-cin LDS-tile hint");
    return launch_small3(a, rc, rp, d.stride, x.n, s);
  }
  if (kind == 6) {  // persistent 3x3 ring, A in registers
    rp = (tile >> 4) & 15;
    FCE_CHECK(d.k == 3 && (d.cin == 32 || d.cin == 64) && out_kind == OUT_F16 && d.up == 0 && (tile & 14) == 0,
              "conv: bad 3x3 ring hint");
    return launch_ring3(a, rp, (tile & 1) ? 2 : 1, d.stride, s);  // 0x601: two tiles of input in flight
  }
  if (kind == 13) {  // persistent 3x3 ring fed by LDS-DMA
    rp = (tile >> 4) & 15;
    const int nbuf = (tile & 3) + 2, sub = ((tile >> 2) & 1) + 1, cpw = ((tile >> 3) & 1) + 1;
    FCE_CHECK(d.k == 3 && (d.cin == 32 || d.cin == 64 || d.cin == 128) && d.cout % (16 * cpw) == 0 &&
                  out_kind == OUT_F16 && d.up == 0 && (rp == 1 || rp == 2 || rp == 4 || (rp == 8 && cpw == 1)) &&
                  nbuf >= 2 && nbuf <= 4 && dring3_offer(d.stride, rp, d.cin / 32, nbuf, cpw, sub),
              "conv: bad 3x3 LDS-DMA ring hint");
    // the copies and the unconditional stores address input and output through buffer resources (byte offsets < 2^31),
    // the output as 8-byte pieces: other views take the register ring, which gives the same bits
    if (!a.vec_ok || int64_t(a.P) * a.ycs * 2 >= (int64_t(1) << 31) ||
        int64_t(a.N) * a.Hs * a.Ws * a.xcs * 2 >= (int64_t(1) << 31))  // cin 128: the implicit-GEMM kernel (same bits)
      return d.cin == 128 ? conv2d_impl(d, x, w, bias, res, y, det, s, -1, dup, duplo)
                          : launch_ring3(a, std::max(rp, 2) > 4 ? 4 : std::max(rp, 2), 1, d.stride, s);
    return launch_dring3(a, rp, nbuf, cpw, sub, d.stride, s);
  }
  if (kind == 9) {  // persistent 3x3 ring on 32x32x16 MFMAs
    const int rpw = (tile >> 4) & 15, wc = 1 << ((tile >> 12) & 3);
    FCE_CHECK(d.k == 3 && (d.cin == 32 || d.cin == 64) && d.cout % 32 == 0 && out_kind == OUT_F16 && d.up == 0 &&
                  (tile & 0xF) == 0,
              "conv: bad 3x3 ring32 hint");
    return launch_ring32(a, wc, rpw, d.stride, s);
  }
  if (kind == 8) {  // big-tile LDS-DMA 3x3 kernel
    const int wm = (tile >> 4) & 15, ab = ((tile >> 12) & 1) + 2, nw = 4;
    FCE_CHECK(d.k == 3 && fast && out_kind == OUT_F16 && d.up == 0 && (tile & 0xF) == 0 && (tile >> 13) == 0 &&
                  big3_ok(d.stride, wm, ab, nw),
              "conv: bad big-tile 3x3 hint");
    return launch_big3(a, wm, ab, nw, d.stride, x.n, s);
  }
  if (kind == 11) {  // 256-wide-tile 1x1 kernel
    const int wc = 1 << ((tile >> 4) & 1), nw = (tile >> 6) & 1 ? 4 : 8, wr = (tile >> 7) & 1 ? 4 : 8;
    FCE_CHECK(d.k == 1 && d.stride == 1 && (tile & 0x0F) == 0 && out_kind != OUT_DFL && big1_ok(wc) &&
                  (wr == 8 || nw == 4),
              "conv: bad big-tile 1x1 hint");
    return launch_big1(a, out_kind, wc, nw, wr, (tile >> 5) & 1, s);
  }
  if (kind == 12) {  // 256-wide-tile implicit-GEMM 3x3 kernel
    const int wc = 1 << ((tile >> 4) & 1), nw = (tile >> 6) & 1 ? 4 : 8, wr = (tile >> 7) & 1 ? 4 : 8;
    FCE_CHECK(d.k == 3 && fast && out_kind == OUT_F16 && d.up == 0 && (tile & 0x0F) == 0 && big1_ok(wc) &&
                  (wr == 8 || nw == 4),
              "conv: bad big-tile 3x3 (implicit GEMM) hint");
    return launch_big3g(a, wc, nw, wr, d.stride, (tile >> 5) & 1, s);
  }
  if (kind == 10) {  // wide-tile 3x3 kernel, per-K-step weight staging
    const int cw = 1 << ((tile >> 4) & 3);
    FCE_CHECK(d.k == 3 && fast && out_kind == OUT_F16 && d.up == 0 && (tile & 0xF) == 0 && (tile >> 6) == (0xA00 >> 6) &&
                  wide3_ok(d.stride, cw),
              "conv: bad wide-tile 3x3 hint");
    return launch_wide3(a, cw, d.stride, x.n, s);
  }
  if (kind == 1) {  // LDS halo-tile 3x3 kernel
    rc = tile & 15;
    rp = (tile >> 4) & 15;
    const int cw = 1 << ((tile >> 12) & 3), kp = ((tile >> 14) & 1) + 1;
    const bool al = (tile >> 15) & 1;
    FCE_CHECK(d.k == 3 && fast && out_kind == OUT_F16 && d.up == 0 &&
                  (al ? tile3al_ok(d.stride, rc, rp, cw, kp) : tile3_ok(d.stride, rc, rp, cw, kp)) &&
                  (kp == 1 || d.cin % 64 == 0),
              "conv: bad LDS-tile hint");
    return launch_tile3(a, rc, rp, cw, kp, al, d.stride, x.n, s);
  }
  FCE_CHECK(kind <= 0, "conv: unknown kernel variant");
  if (tile >= 0) {
    rc = tile & 15;
    rp = tile >> 4;
    FCE_CHECK((rc == 1 || rc == 2 || rc == 4) && (rp == 1 || rp == 2 || rp == 4), "conv: bad tile hint");
  } else {
    pick_tile(a.P, g.cotiles, out_kind == OUT_DFL, &rc, &rp);
  }
  if (out_kind == OUT_DFL) FCE_CHECK(rc == 4 && g.cotiles == 4, "conv detect epilogue: one wave must own all 64 bins");
  if (d.k == 3) FCE_CHECK(d.up == 0 && out_kind == OUT_F16, "conv 3x3: plain fp16 store, no fused upsampling");
  if (d.k == 1)
    launch_dense_rc<1>(a, out_kind, fast, rc, rp, s);
  else
    launch_dense_rc<3>(a, out_kind, fast, rc, rp, s);
  return launch_status("conv_mfma_kernel");
}

int conv2d(const fce_conv_desc& d, const fce_tensor& x, const void* w, const float* bias, const fce_tensor* res,
           const fce_tensor& y, hipStream_t s, int tile, const fce_tensor* dup, int duplo) {
  return conv2d_impl(d, x, w, bias, res, y, nullptr, s, tile, dup, duplo);
}

int conv2d_detect(const fce_conv_desc& d, const fce_tensor& x, const void* w, const float* bias,
                  const fce_detect_epi& e, hipStream_t s, int tile) {
  // the output view only carries the spatial geometry; results go to e.pred
  fce_tensor y{nullptr, FCE_F32, FCE_NHWC, x.n, d.cout, x.h, x.w, d.cout, 0};
  return conv2d_impl(d, x, w, bias, nullptr, y, &e, s, tile);
}

}  // namespace fce
