// Fused Bottleneck chain (reference ultralytics/nn/modules/block.py Bottleneck.forward :474-476, as C3k.m
// :1087-1108 runs two of them and C3k2(c3k = False).m :1064-1084 one):
//
//   for each of the NB bottlenecks:   h = SiLU(cv1(x))        3x3, ci -> cm
//                                      x = SiLU(cv2(h)) + x    3x3, cm -> ci   (shortcut)
//
// in ONE persistent kernel.  The n scale's C3k bottleneck pairs at 40^2 / 20^2 (n L7, L10, L24) and the C3k2
// bottlenecks of the 40^2 neck blocks (L15, L21) are 5-7 us launches of 0.9-1.9 GF each (latency-bound: launch,
// ramp, HBM round trip of every intermediate); here x is read once and only the chain's output is written.
//
// A block owns a run of full-width row bands (TH output rows x W columns of one image).  Per band the input
// (x over the band + 2 NB halo rows, rows outside the image zero) goes HBM -> registers (prefetched during the
// previous band) -> LDS, and every stage reads its B operands from the previous stage's LDS image: stage j computes
// its output over the band + (2 NB - j - 1) halo rows (zero outside the image: the next 3x3's padding), the last
// stage writes the band to HBM.  LDS images have one zero column either side of the W columns (the 3x3's column
// padding; a full-width band has no column halo), so only the ROW halos are recomputed.
//
// Unlike the fused C3k2 (weights resident in LDS, every wave all couts of its pixels), the stages' weights stream
// from L2: a wave owns one or two cout tiles of a stage and keeps their A fragments in 18 registers-sets (h8), each
// slot reloaded with the next stage's fragment as soon as its K-step is done, so a block reads the weights once per
// band and the LDS holds only activations.  Pixel fragments of a stage are dealt to the waves of a cout group round
// robin.  LDS images are 32-channel planes of positions with the conv tile kernels' XOR swizzle and a row stride of
// W + 8 (bn_slot): every B-fragment read is conflict-free (measured LDS conflict cycles 50 % -> 11-13 %, the rest
// stores).  Measured alternatives (profiles/r06_bneck_probe.txt): a fragment-outer K loop with each fragment's
// epilogue issued beside the next fragment's MFMAs ran 5-15 % slower (one B read in flight per MFMA instead of MF).
//
// Bitwise identical to the 2 NB unfused fce_conv2d calls: every stage walks the conv_pack K-steps (chunk-major:
// 32-channel chunk x 9 + tap, cin % 32 == 0) with v_mfma_f32_16x16x32_f16 from zero, the B values are the same
// fp16 values (each intermediate rounded to fp16 exactly where the unfused path stores it, zeros where it pads)
// and the epilogue is conv_epilogue's (bias, SiLU, residual add, fpin before every fp16 conversion).
#include <algorithm>

#include "mfma_stage.h"

namespace fce {

static __device__ __attribute__((aligned(16))) _Float16 g_bn_zero[8];

template <int CI, int CM, int NB, int W, int TH, int NW>
struct BnG {
  static_assert(CI % 32 == 0 && CM % 32 == 0, "bneck fused: chunk-major K order (cin % 32 == 0)");
  static_assert(NB == 1 || CI == CM, "bneck fused: a two-bottleneck chain reuses its buffers (ci == cm)");
  static constexpr int L = 2 * NB;  // halo rows of the input band
  // LDS row stride in positions: image column c at position c + 1, zero columns at 0 and W + 1; RS - W = 8 keeps the
  // XOR swizzle (bn_slot) of consecutive positions conflict-free across a row wrap (every B-fragment read of every
  // tap: 4 LDS cycles per ds_read_b128, checked exhaustively; the odd piece stride of the first version took 9-10)
  static constexpr int RS = W + 8;
  static constexpr int SI = CI / 8, SM = CM / 8;  // 16-byte pieces per position (CI / 32 planes of 4 pieces)
  // images (16-byte units): A = level L (the input, CI), B = level L - 1 (CM), C = level L - 2 (CI, NB = 2);
  // level L - 3 (NB = 2) goes back into A (same piece stride: ci == cm)
  static constexpr int PA = (TH + 2 * L) * RS, PB = (TH + 2 * L - 2) * RS, PC = (TH + 2 * L - 4) * RS;  // positions
  static constexpr int OA = 0, OB = OA + PA * SI, OC = OB + PB * SM;
  static constexpr int OBIAS = NB == 2 ? OC + PC * SI : OC;
  static constexpr int NBIAS = NB * (CM + CI);  // floats: stage j's biases at bias_off(j)
  static constexpr size_t LDS = size_t(OBIAS) * 16 + size_t(NBIAS) * 4;
  static constexpr int XP = CI / 8;                                        // 16-byte pieces per input pixel
  static constexpr int NE = (TH + 2 * L) * W * XP, NX = (NE + NW * 64 - 1) / (NW * 64);  // input pieces per thread
  static constexpr int NT = NW * 64;
};

// compile-time shape of stage J (0 .. 2 NB - 1): input level L - J, output level L - J - 1.  A wave owns CPW cout tiles
// (two for the 32-channel-input stages, whose 9 K-steps then fill the same 18 A-fragment registers as one tile of a
// 64-channel input's 18: every stage keeps NA = 18 fragments per wave) and deals the stage's pixel fragments with the
// other PG waves of its cout group
template <int CI, int CM, int NB, int W, int TH, int NW, int J>
struct BnStage {
  using G = BnG<CI, CM, NB, W, TH, NW>;
  static constexpr int CIN = J % 2 == 0 ? CI : CM, COUT = J % 2 == 0 ? CM : CI;
  static constexpr int KOUT = G::L - J - 1;                  // output halo rows
  static constexpr int ROWS = TH + 2 * KOUT, NP = ROWS * W;  // output rows / positions
  static constexpr int NF = (NP + 15) / 16;
  static constexpr int NS = 9 * CIN / 32;               // K-steps
  static constexpr int NALLOC = ((NS + 7) & ~7) + 8;  // fragments stored per cout tile (dense_geom / stage_nalloc)
  static constexpr int CT = COUT / 16, CPW = NS == 9 && CT % 2 == 0 ? 2 : 1, CG = CT / CPW, PG = NW / CG;
  static_assert(NW % CG == 0 && CPW * NS == 18, "bneck fused: wave layout (18 A fragments per wave)");
  static constexpr int MF = (NF + PG - 1) / PG;  // pixel fragments per wave
  static constexpr int SIN = J % 2 == 0 ? G::SI : G::SM, SOUT = J % 2 == 0 ? G::SM : G::SI;
  // image offsets: level k -> A (k == L), B (k == L - 1), C (k == L - 2, NB = 2), A (k == L - 3, NB = 2)
  static constexpr int img(int k) { return k == G::L || k == G::L - 3 ? G::OA : k == G::L - 1 ? G::OB : G::OC; }
  static constexpr int OIN = img(KOUT + 1), OOUT = img(KOUT), ORES = img(KOUT + 2);
  // positions of an image (its plane size): A and C hold CI channels, B CM; level L - 3 reuses A's planes
  static constexpr int npos(int k) { return k == G::L || k == G::L - 3 ? G::PA : k == G::L - 1 ? G::PB : G::PC; }
  static constexpr int PIN = npos(KOUT + 1), POUT = npos(KOUT), PRES = npos(KOUT + 2);
  static constexpr int BIAS = (J / 2) * (CM + CI) + (J % 2) * CM;  // float offset of this stage's biases
};

constexpr int kBnNA = 18;  // A fragments per wave and stage

// 16-byte slot of piece q of position u in an image of NQ pieces per position: the image is NQ / 4 planes (32-channel
// chunks) of NP positions x 4 pieces, piece q & 3 of plane q >> 2 at position u in slot (q & 3) ^ ((u >> 1) & 3) (the conv
// tile kernels' swizzle for 64-byte positions).  A 3x3 tap's ky then moves a slot by a constant (RS = W + 8: ky RS 4
// slots, with the swizzle flipped by 2 for odd ky when RS % 8 == 4), so a fragment's B address per kx is computed once
// per stage and every read is that base + an immediate offset (+ one XOR for odd ky at RS % 8 == 4).
template <int NQ, int NP>
__device__ __forceinline__ int bn_slot(int u, int q) {
  static_assert(NQ == 4 || NQ == 8, "bneck fused: 32 or 64 channels per image");
  return (q >> 2) * NP * 4 + u * 4 + ((q & 3) ^ ((u >> 1) & 3));
}

struct BneckArgs {
  const _Float16* x;
  int xcs;
  _Float16* y;
  int ycs;
  int H, ntiles, tiles_y;
  const h8* w[4];  // packed A fragments (conv_pack layout: [cout tile][nalloc][64 lanes]), stage order
  int nalloc[4];
  const float* b[4];
  int diag;  // FCE_BNECK_DIAG: block 0 prints its per-stage clocks
};

// Per-stage weight access: a buffer resource over the stage's packed fragments (SGPRs) and this wave's lane offset
// (one VGPR per stage); fragment (cout tile cg CPW + cl, K-step st) is then a constant soffset.  With 64-bit addresses
// hipcc kept every fragment's address live across the band loop (loop-invariant), ~150 VGPRs of them.
struct BnW {
  __amdgpu_buffer_rsrc_t r[4];
  uint32_t vo[4];
};

template <int CI, int CM, int NB, int W, int TH, int NW, int J>
__device__ __forceinline__ void bn_w_init(const BneckArgs& a, BnW& w) {
  using S = BnStage<CI, CM, NB, W, TH, NW, J>;
  const int lane = threadIdx.x & 63, cg = (threadIdx.x >> 6) % S::CG;
  w.r[J] = __builtin_amdgcn_make_buffer_rsrc(const_cast<h8*>(a.w[J]), 0, int(S::CT * S::NALLOC * 1024), 0x00020000);
  w.vo[J] = uint32_t((cg * S::CPW * S::NALLOC * 64 + lane) * 16);
}

// A fragment in register slot s of stage J for this wave: cout tile cg CPW + s / NS, K-step s % NS
template <int CI, int CM, int NB, int W, int TH, int NW, int J>
__device__ __forceinline__ h8 bn_a_frag(const BnW& w, int s) {
  using S = BnStage<CI, CM, NB, W, TH, NW, J>;
  const int cl = s / S::NS, st = s % S::NS;
  const u4 v = __builtin_amdgcn_raw_buffer_load_b128(w.r[J], int(w.vo[J]), (cl * S::NALLOC + st) * 1024, 0);
  return __builtin_bit_cast(h8, v);
}

template <int CI, int CM, int NB, int W, int TH, int NW, int J>
__device__ __forceinline__ void bn_load_a(const BnW& w, h8 (&av)[kBnNA]) {
#pragma unroll
  for (int s = 0; s < kBnNA; ++s) av[s] = bn_a_frag<CI, CM, NB, W, TH, NW, J>(w, s);
}

// epilogue of pixel fragment i, cout tile cl of this wave in stage J: bias, SiLU (+ the shortcut), fp16; into the next
// image (zeros outside the image) or, in the last stage, to HBM
template <int CI, int CM, int NB, int W, int TH, int NW, int J>
__device__ __forceinline__ void bn_epilogue(const BneckArgs& a, h8* sm, const f4& acc, int i, int cl, int n, int y0,
                                            __amdgpu_buffer_rsrc_t yr) {
  using G = BnG<CI, CM, NB, W, TH, NW>;
  using S = BnStage<CI, CM, NB, W, TH, NW, J>;
  int lane = int(threadIdx.x & 63);
  asm volatile("" : "+v"(lane));
  const int wave = threadIdx.x >> 6, col = lane & 15, grp = lane >> 4;
  const int cg = wave % S::CG, pg = wave / S::CG;
  const float* bias = reinterpret_cast<const float*>(sm + G::OBIAS) + S::BIAS;
  const int co0 = (cg * S::CPW + cl) * 16 + grp * 4;
  const int q = (pg + S::PG * i) * 16 + col;
  const int r = q / W, c = q - r * W;
  const int iy = y0 - S::KOUT + r;  // image row of this output position
  float v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = silu(acc[j] + bias[co0 + j]);
  if constexpr (J % 2 == 1) {  // shortcut: the bottleneck's input, two levels up (rows r + 2, same column)
    const int ur = (min(r, S::ROWS - 1) + 2) * G::RS + c + 1;
    const h4 rv = *reinterpret_cast<const h4*>(reinterpret_cast<const _Float16*>(sm + S::ORES + bn_slot<G::SI, S::PRES>(ur, co0 / 8)) +
                                               co0 % 8);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = fpin(v[j] + (float)rv[j]);
  }
  if constexpr (S::KOUT == 0) {  // the band's output rows -> HBM (every lane storing: rows past H are dropped)
    const bool ok = q < S::NP && iy < a.H;
    store_h4_or_drop(yr, ok, uint32_t((iy * W + c) * a.ycs + co0) * 2u, h4_of(v));
  } else {
    if (q >= S::NP) return;
    h4 o = h4_of(v);
    if (iy < 0 || iy >= a.H) o = h4{0, 0, 0, 0};  // outside the image: the next 3x3's zero padding
    *reinterpret_cast<h4*>(reinterpret_cast<_Float16*>(sm + S::OOUT + bn_slot<S::SOUT, S::POUT>(r * G::RS + c + 1, co0 / 8)) +
                           co0 % 8) = o;
  }
}

// one 3x3 stage of the band starting at image row y0 of image n.  av: this wave's A fragments of stage J; as each
// K-step's fragments are consumed their registers are reloaded with stage JN's (the next stage, or the next band's
// stage 0), so one 18-fragment register set serves every stage.  The B fragments of step st + 1 are read from LDS while
// step st's MFMAs run (two register sets, sched_barrier fences keep hipcc from hoisting every read of the stage).
template <int CI, int CM, int NB, int W, int TH, int NW, int J, int JN>
__device__ __forceinline__ void bn_stage(const BneckArgs& a, const BnW& w, h8* sm, h8 (&av)[kBnNA], int n, int y0,
                                         __amdgpu_buffer_rsrc_t yr) {
  using G = BnG<CI, CM, NB, W, TH, NW>;
  using S = BnStage<CI, CM, NB, W, TH, NW, J>;
  // the lane index through an opaque move: every address below is loop-invariant across bands, and hipcc otherwise
  // hoists all four stages' B / epilogue addresses out of the band loop (~80 VGPRs live, spills)
  int lane = int(threadIdx.x & 63);
  asm volatile("" : "+v"(lane));
  const int wave = threadIdx.x >> 6, col = lane & 15, grp = lane >> 4;
  const int cg = wave % S::CG, pg = wave / S::CG;
  const h8* in = sm + S::OIN;
  // B addresses: output (r, c) reads input rows r .. r + 2 (the input band starts one row higher) and image columns
  // c - 1 .. c + 1 = LDS columns c .. c + 2; per fragment the tap-(0, kx) byte address of each kx (lane piece grp of
  // plane 0), taps ky > 0 add ky RS 64 bytes (and flip the swizzle for odd ky when RS % 8 == 4)
  static_assert(G::RS % 4 == 0, "bneck fused: RS % 4 == 0");
  uint32_t ba[S::MF][3];
#pragma unroll
  for (int i = 0; i < S::MF; ++i) {
    const int q = min((pg + S::PG * i) * 16 + col, S::NP - 1);  // clamped: waves past the last fragment
    const int r = q / W, c = q - r * W;
#pragma unroll
    for (int kx = 0; kx < 3; ++kx)
      ba[i][kx] = uint32_t(reinterpret_cast<uintptr_t>(in + bn_slot<S::SIN, S::PIN>(r * G::RS + c + kx, grp)));
  }
  f4 acc[S::CPW][S::MF];
#pragma unroll
  for (int cl = 0; cl < S::CPW; ++cl)
#pragma unroll
    for (int i = 0; i < S::MF; ++i) acc[cl][i] = f4{0.f, 0.f, 0.f, 0.f};
  h8 bv[2][S::MF];
  auto read_b = [&](int st, h8 (&dst)[S::MF]) {
    const int tap = st % 9, c32 = st / 9, ky = tap / 3, kx = tap % 3;
    const uint32_t flip = (G::RS % 8 == 4 && (ky & 1)) ? 32u : 0u;  // slot ^ 2 (bytes ^ 32)
    const uint32_t off = uint32_t(c32 * S::PIN * 64 + ky * G::RS * 64);
#pragma unroll
    for (int i = 0; i < S::MF; ++i)
      dst[i] = *reinterpret_cast<const __attribute__((address_space(3))) h8*>(uintptr_t((ba[i][kx] ^ flip) + off));
  };
  read_b(0, bv[0]);
#pragma unroll
  for (int st = 0; st < S::NS; ++st) {
    if (st + 1 < S::NS) read_b(st + 1, bv[(st + 1) & 1]);
#pragma unroll
    for (int cl = 0; cl < S::CPW; ++cl)
#pragma unroll
      for (int i = 0; i < S::MF; ++i)
        acc[cl][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[cl * S::NS + st], bv[st & 1][i], acc[cl][i], 0, 0, 0);
    // this step's A registers are free: the next stage's fragments for those slots (the rest after the last step)
#pragma unroll
    for (int cl = 0; cl < S::CPW; ++cl) av[cl * S::NS + st] = bn_a_frag<CI, CM, NB, W, TH, NW, JN>(w, cl * S::NS + st);
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int i = 0; i < S::MF; ++i)
#pragma unroll
    for (int cl = 0; cl < S::CPW; ++cl) bn_epilogue<CI, CM, NB, W, TH, NW, J>(a, sm, acc[cl][i], i, cl, n, y0, yr);
#pragma unroll
  for (int s = S::CPW * S::NS; s < kBnNA; ++s) av[s] = bn_a_frag<CI, CM, NB, W, TH, NW, JN>(w, s);
}

template <int CI, int CM, int NB, int W, int TH, int NW>
__global__ __launch_bounds__(NW * 64, 1) void bneck_fused_kernel(BneckArgs a) {
  using G = BnG<CI, CM, NB, W, TH, NW>;
  extern __shared__ __attribute__((aligned(16))) h8 sm[];
  const int NGr = gridDim.x, bi = blockIdx.x;
  const int t_begin = int(int64_t(bi) * a.ntiles / NGr), t_end = int(int64_t(bi + 1) * a.ntiles / NGr);
  if (t_begin >= t_end) return;  // block-uniform

  // input band of tile t -> registers (rows outside the image: the zero line)
  h8 xv[G::NX];
  auto load_x = [&](int t) {
    const int n = t / a.tiles_y, y0 = (t - n * a.tiles_y) * TH;
#pragma unroll
    for (int i = 0; i < G::NX; ++i) {
      const int e = int(threadIdx.x) + G::NT * i;
      const int pos = e / G::XP, pc = e - pos * G::XP;
      const int r = pos / W, c = pos - r * W;
      const int iy = y0 - G::L + r;
      const bool ok = e < G::NE && iy >= 0 && iy < a.H;
      xv[i] = *reinterpret_cast<const h8*>(ok ? a.x + nhwc_off(n, iy, c, a.H, W, a.xcs) + pc * 8 : g_bn_zero);
    }
  };
  auto store_x = [&]() {
#pragma unroll
    for (int i = 0; i < G::NX; ++i) {
      const int e = int(threadIdx.x) + G::NT * i;
      const int pos = e / G::XP, pc = e - pos * G::XP;
      const int r = pos / W, c = pos - r * W;
      if (e < G::NE) sm[G::OA + bn_slot<G::SI, G::PA>(r * G::RS + c + 1, pc)] = xv[i];
    }
  };
  BnW wr;
  bn_w_init<CI, CM, NB, W, TH, NW, 0>(a, wr);
  bn_w_init<CI, CM, NB, W, TH, NW, 1>(a, wr);
  if constexpr (NB == 2) {
    bn_w_init<CI, CM, NB, W, TH, NW, 2>(a, wr);
    bn_w_init<CI, CM, NB, W, TH, NW, 3>(a, wr);
  }
  h8 av[kBnNA];
  bn_load_a<CI, CM, NB, W, TH, NW, 0>(wr, av);
  load_x(t_begin);
  // zero columns either side of every image row (never written again: stages and staging write columns 1 .. W),
  // and the stages' biases
  {
    const h8 z = h8{0, 0, 0, 0, 0, 0, 0, 0};
    constexpr int RA = TH + 2 * G::L, RB = TH + 2 * G::L - 2, RC = NB == 2 ? TH + 2 * G::L - 4 : 0;
    auto zero_cols = [&](int off, int rows, int np, int nq) {
      for (int e = int(threadIdx.x); e < 2 * rows * nq; e += G::NT) {
        const int r = e / (2 * nq), k = e - r * 2 * nq, side = k / nq, p = k - side * nq;
        sm[off + (p >> 2) * np * 4 + (r * G::RS + side * (W + 1)) * 4 + (p & 3)] = z;
      }
    };
    zero_cols(G::OA, RA, G::PA, G::SI);
    zero_cols(G::OB, RB, G::PB, G::SM);
    if constexpr (NB == 2) zero_cols(G::OC, RC, G::PC, G::SI);
    float* bias = reinterpret_cast<float*>(sm + G::OBIAS);
    for (int e = int(threadIdx.x); e < G::NBIAS; e += G::NT) {
      const int bk = e / (CM + CI), rem = e - bk * (CM + CI), j = 2 * bk + (rem >= CM ? 1 : 0);
      bias[e] = a.b[j][rem >= CM ? rem - CM : rem];
    }
  }

  const uint32_t img = uint32_t(a.H) * uint32_t(W) * uint32_t(a.ycs);
  // diagnostics (FCE_BNECK_DIAG=1): block 0, wave 0 sums s_memtime clocks per phase over its bands and prints them
  uint64_t clk[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, tprev = a.diag ? __builtin_amdgcn_s_memtime() : 0, t00 = tprev;
  auto tick = [&](int k) {
    if (a.diag) {
      const uint64_t tn = __builtin_amdgcn_s_memtime();
      clk[k] += tn - tprev;
      tprev = tn;
    }
  };
  for (int t = t_begin; t < t_end; ++t) {
    const int n = t / a.tiles_y, y0 = (t - n * a.tiles_y) * TH;
    const __amdgpu_buffer_rsrc_t yr = out_rsrc(a.y + int64_t(n) * img, img * 2u);
    // the previous band's last stage has read A / C (first time round: the zeroing is published)
    stage_barrier();
    tick(0);
    store_x();
    stage_barrier();
    tick(1);
    if constexpr (NB == 1) {
      bn_stage<CI, CM, NB, W, TH, NW, 0, 1>(a, wr, sm, av, n, y0, yr);
      tick(2);
      stage_barrier();
      tick(3);
      load_x(min(t + 1, t_end - 1));  // unconditional (clamped): the next band's input, in flight during the last stage
      bn_stage<CI, CM, NB, W, TH, NW, 1, 0>(a, wr, sm, av, n, y0, yr);
      tick(4);
    } else {
      bn_stage<CI, CM, NB, W, TH, NW, 0, 1>(a, wr, sm, av, n, y0, yr);
      tick(2);
      stage_barrier();
      tick(3);
      bn_stage<CI, CM, NB, W, TH, NW, 1, 2>(a, wr, sm, av, n, y0, yr);
      tick(4);
      stage_barrier();
      tick(5);
      bn_stage<CI, CM, NB, W, TH, NW, 2, 3>(a, wr, sm, av, n, y0, yr);
      tick(6);
      stage_barrier();
      tick(7);
      load_x(min(t + 1, t_end - 1));
      bn_stage<CI, CM, NB, W, TH, NW, 3, 0>(a, wr, sm, av, n, y0, yr);
      tick(8);
    }
  }
  if (a.diag && blockIdx.x == 0 && threadIdx.x == 0) {
    const unsigned long long nt = (unsigned long long)(t_end - t_begin);
    printf("bneck fused diag <%d,%d,%d,%d,%d>: %llu bands, total %llu clocks; per band: wait-x %llu, stage-x %llu, "
           "s0 %llu, b %llu, s1 %llu, b %llu, s2 %llu, b %llu, s3 %llu\n", CI, CM, NB, W, TH, nt,
           (unsigned long long)(tprev - t00), (unsigned long long)clk[0] / nt, (unsigned long long)clk[1] / nt,
           (unsigned long long)clk[2] / nt, (unsigned long long)clk[3] / nt, (unsigned long long)clk[4] / nt,
           (unsigned long long)clk[5] / nt, (unsigned long long)clk[6] / nt, (unsigned long long)clk[7] / nt,
           (unsigned long long)clk[8] / nt);
  }
}

// ============================================================================ host
// instantiated (ci, cm, nb, map width) with the band height: the n scale's C3k pairs (L7 at 40^2: 32 / 32, L10 and
// L24 at 20^2: 64 / 64) and its 40^2 neck C3k2 bottlenecks (L15, L21: 64 -> 32 -> 64), plus the 32-channel pair at
// 20^2 (n L7 at 320 input)
struct BnInst {
  int ci, cm, nb, w;
};
static constexpr BnInst kBnInsts[] = {{32, 32, 2, 40}, {32, 32, 2, 20}, {64, 64, 2, 20}, {64, 32, 1, 40}, {64, 32, 1, 20}};

template <int CI, int CM, int NB, int W, int TH, int NW>
static int bn_launch(const BneckArgs& a0, int N, hipStream_t s) {
  using G = BnG<CI, CM, NB, W, TH, NW>;
  static_assert(G::LDS <= 160 * 1024, "bneck fused: LDS over 160 KiB");
  auto k = bneck_fused_kernel<CI, CM, NB, W, TH, NW>;
  static const bool big = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
  if (!big && G::LDS > 64 * 1024) return fail(FCE_ERR_HIP, "bneck fused: cannot opt in to >64 KiB LDS");
  BneckArgs a = a0;
  a.tiles_y = (a.H + TH - 1) / TH;
  const int64_t tiles = int64_t(a.tiles_y) * N;
  if (tiles == 0) return FCE_OK;
  FCE_CHECK(tiles < (int64_t(1) << 30), "bneck fused: grid too large");
  a.ntiles = int(tiles);
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
  }
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k, NW * 64, G::LDS) != hipSuccess || occ < 1) occ = 1;
  const int grid = int(std::min<int64_t>(a.ntiles, int64_t(cus) * occ));
  FCE_LAUNCH(k, dim3(unsigned(grid)), dim3(NW * 64), G::LDS, s, a);
  return launch_status("bneck_fused_kernel");
}

static int bn_inst(const fce_bneck_desc& d, int w) {
  for (int i = 0; i < int(sizeof(kBnInsts) / sizeof(kBnInsts[0])); ++i)
    if (kBnInsts[i].ci == d.c && kBnInsts[i].cm == d.c_mid && kBnInsts[i].nb == d.n && (w < 0 || kBnInsts[i].w == w))
      return i;
  return -1;
}

bool bneck_fused_ok(const fce_bneck_desc& d) { return d.shortcut == 1 && bn_inst(d, -1) >= 0; }
bool bneck_fused_fits(const fce_bneck_desc& d, int h, int w) { return d.shortcut == 1 && h > 0 && bn_inst(d, w) >= 0; }

int bneck_fused(const fce_bneck_desc& d, const fce_tensor& x, const fce_tensor& y, hipStream_t s) {
  FCE_CHECK(d.shortcut == 1, "bneck fused: only the shortcut form");
  FCE_CHECK(x.layout == FCE_NHWC && y.layout == FCE_NHWC && x.dtype == FCE_F16 && y.dtype == FCE_F16,
            "bneck fused: NHWC f16 views");
  FCE_CHECK(x.c == d.c && y.c == d.c && x.n == y.n && x.h == y.h && x.w == y.w, "bneck fused: shape mismatch");
  FCE_CHECK(x.cstride % 8 == 0 && x.coff % 8 == 0 && y.cstride % 4 == 0 && y.coff % 4 == 0,
            "bneck fused: aligned channel slices");
  const int inst = bn_inst(d, x.w);
  FCE_CHECK(inst >= 0, "bneck fused: no instantiation for this channel configuration and map width");
  for (int i = 0; i < 2 * d.n; ++i) FCE_CHECK(d.w[i] && d.b[i], "bneck fused: null weights");
  BneckArgs a{};
  a.x = static_cast<const _Float16*>(x.data) + x.coff;
  a.xcs = x.cstride;
  a.y = static_cast<_Float16*>(y.data) + y.coff;
  a.ycs = y.cstride;
  a.H = x.h;
  for (int i = 0; i < 2 * d.n; ++i) {
    a.w[i] = static_cast<const h8*>(d.w[i]);
    a.b[i] = d.b[i];
    a.nalloc[i] = stage_nalloc(i % 2 == 0 ? d.c : d.c_mid, 3);
  }
  {
    const char* de = getenv("FCE_BNECK_DIAG");
    a.diag = de && atoi(de) != 0;
  }
  // band heights measured per instantiation (profiles/r06_bneck_probe.txt): L7 8 rows (4: 28.0, 10: 21.8 against 19.7
  // us), L10 / L24 3 rows (224 bands for 256 CUs; 5: 19.8, 4: 17.8 against 17.4 us), L15 / L21 6 rows (4: 17.5, 8: 14.8
  // against 13.0 us)
  switch (inst) {
    case 0: return bn_launch<32, 32, 2, 40, 8, 8>(a, x.n, s);
    case 1: return bn_launch<32, 32, 2, 20, 8, 8>(a, x.n, s);
    case 2: return bn_launch<64, 64, 2, 20, 3, 8>(a, x.n, s);
    case 3: return bn_launch<64, 32, 1, 40, 6, 8>(a, x.n, s);
    default: return bn_launch<64, 32, 1, 20, 8, 8>(a, x.n, s);
  }
}

}  // namespace fce
