// Two chained 1x1 convs in one kernel (the pairs of the n scale's C3k2(c3k = True) and C2PSA blocks, reference
// ultralytics/nn/modules/block.py C2f.forward :303-307, C3.forward :340, C2PSA.forward :1455-1464, PSABlock.forward
// :1345-1354, Attention.forward :1287-1304):
//
//   h = act1(W1 x + b1) (+ r1)                        op 1: cin1 -> cout1, its output view h
//   y = act2(W2 x2 + b2) (+ r2)                       op 2: cin2 -> cout2, where channels [ho, ho + hn) of its input
//                                                      view x2 ARE op 1's output channels [hs, hs + hn)
//
// e.g. C3k2 cv1 -> C3k's merged cv1 / cv2 on the b half (x2 = h[c : 2c]), C3k.cv3 -> C3k2.cv2 over [a | b | m]
// (x2 = [a | b | h]), Attention.proj (+ b) -> ffn[0], ffn[1] (+ x1) -> C2PSA.cv2 over [a | h].  At 40^2 / 20^2 each
// of these 1x1s is a 5-12 us launch, mostly latency (launch, ramp, a HBM round trip); here one persistent block per
// CU walks 64-pixel tiles: x (and the part of x2 that is not h) HBM -> registers (prefetched during the previous
// tile) -> LDS, op 1 from LDS into the x2 image's h channels (and to HBM where another op reads h), op 2 from the x2
// image to HBM.
//
// Waves split the couts (CPW cout tiles each, weights streamed from L2 into 24 rolling A-fragment registers as in
// bneck.hip) and the tile's four 16-pixel fragments.  LDS images are 32-channel planes of 64 positions with the conv
// tile kernels' XOR swizzle (conflict-free B-fragment reads).  Bitwise identical to the two fce_conv2d calls: the same
// packed K-steps (32-channel chunks in order, v_mfma_f32_16x16x32_f16 from zero) and conv_epilogue's arithmetic
// (bias, SiLU or none, residual add, fpin before every fp16 conversion; op 2's duplicate store).
#include <algorithm>

#include "mfma_stage.h"

namespace fce {

static __device__ __attribute__((aligned(16))) _Float16 g_pw_zero[8];

constexpr int kPwTP = 64;  // pixels per tile
constexpr int kPwNA = 24;  // A-fragment registers per wave

struct Pw2Args {
  const _Float16* x1;
  int x1cs;
  const _Float16* r1;  // op 1 residual or null
  int r1cs;
  _Float16* h;  // op 1 output view
  int hcs, h_store;
  const _Float16* x2;  // op 2 input view
  int x2cs, ho, hs, hn;
  const _Float16* r2;
  int r2cs;
  _Float16* y;
  int ycs;
  _Float16* dup;  // op 2 duplicate store: output channels [duplo, duplo + dupn) also to dup, or null
  int dupcs, duplo, dupn;
  int P, ntiles;
  const h8* w1;
  const h8* w2;
  const float* b1;
  const float* b2;
  int act1, act2;
  int epi1;         // op 1: FCE_EPI_STORE, _WSTORE (scaled by the BiFPN weight) or _ACCUM (added to h's contents)
  const float* fw;  // the BiFPN weights (epi1 != STORE)
  int fn, fi;
};

// stage geometry: COUT couts over the tile's 4 pixel fragments with NW waves
template <int CIN, int COUT, int NW>
struct PwStage {
  static constexpr int CT = COUT / 16, NS = CIN / 32;
  static constexpr int CG = CT < NW ? CT : NW, CPW = CT / CG, PG = NW / CG, MF = (kPwTP / 16) / PG;
  static constexpr int NALLOC = ((NS + 7) & ~7) + 8;  // fragments stored per cout tile (dense_geom)
  static_assert(CIN % 32 == 0 && COUT % 16 == 0 && CT % CG == 0 && NW % CG == 0 && (kPwTP / 16) % PG == 0,
                "pw2: wave layout");
  static_assert(CPW * NS <= kPwNA, "pw2: A fragments per wave");
};

// slot of piece q (8 channels) of tile pixel u in an image of 32-channel planes (kPwTP positions x 4 slots each)
__device__ __forceinline__ int pw_slot(int u, int q) { return (q >> 2) * kPwTP * 4 + u * 4 + ((q & 3) ^ ((u >> 1) & 3)); }

template <int CIN, int COUT, int NW>
__device__ __forceinline__ h8 pw_a(__amdgpu_buffer_rsrc_t r, uint32_t vo, int s) {
  using S = PwStage<CIN, COUT, NW>;
  const int cl = s / S::NS, st = s % S::NS;
  return __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(r, int(vo), (cl * S::NALLOC + st) * 1024, 0));
}

// one conv of the pair over the tile: B from the LDS image `img`, A rolling (slot s of this stage -> slot s of the
// next stage NXT once consumed); epi(cl, i, acc) per (cout tile, pixel fragment)
template <int CIN, int COUT, int NW, int CIN_N, int COUT_N, typename EPI>
__device__ __forceinline__ void pw_stage(const h8* img, h8 (&av)[kPwNA], __amdgpu_buffer_rsrc_t rn, uint32_t von, EPI epi) {
  using S = PwStage<CIN, COUT, NW>;
  using SN = PwStage<CIN_N, COUT_N, NW>;
  int lane = int(threadIdx.x & 63);
  asm volatile("" : "+v"(lane));  // keep the addresses out of the tile loop's hoisting (see bneck.hip)
  const int wave = threadIdx.x >> 6, col = lane & 15, grp = lane >> 4;
  const int pg = wave / S::CG;
  f4 acc[S::CPW][S::MF];
#pragma unroll
  for (int cl = 0; cl < S::CPW; ++cl)
#pragma unroll
    for (int i = 0; i < S::MF; ++i) acc[cl][i] = f4{0.f, 0.f, 0.f, 0.f};
  h8 bv[2][S::MF];
  auto read_b = [&](int st, h8 (&dst)[S::MF]) {
#pragma unroll
    for (int i = 0; i < S::MF; ++i) dst[i] = img[pw_slot((pg + S::PG * i) * 16 + col, st * 4 + grp)];
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
#pragma unroll
    for (int cl = 0; cl < S::CPW; ++cl) {
      const int s = cl * S::NS + st;
      if (s < SN::CPW * SN::NS) av[s] = pw_a<CIN_N, COUT_N, NW>(rn, von, s);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int s = S::CPW * S::NS; s < SN::CPW * SN::NS; ++s) av[s] = pw_a<CIN_N, COUT_N, NW>(rn, von, s);
#pragma unroll
  for (int cl = 0; cl < S::CPW; ++cl)
#pragma unroll
    for (int i = 0; i < S::MF; ++i) epi(cl, i, acc[cl][i]);
}

template <int CIN1, int COUT1, int CIN2, int COUT2, int NW>
__global__ __launch_bounds__(NW * 64, 1) void pw2_kernel(Pw2Args a) {
  using S1 = PwStage<CIN1, COUT1, NW>;
  using S2 = PwStage<CIN2, COUT2, NW>;
  constexpr int NT = NW * 64;
  constexpr int OX = 0, OE = OX + CIN1 / 32 * kPwTP * 4, OBIAS = OE + CIN2 / 32 * kPwTP * 4;
  constexpr int NX = (kPwTP * CIN1 / 8 + NT - 1) / NT, NE = (kPwTP * CIN2 / 8 + NT - 1) / NT;
  extern __shared__ __attribute__((aligned(16))) h8 sm[];
  const int NGr = gridDim.x, bi = blockIdx.x;
  const int t_begin = int(int64_t(bi) * a.ntiles / NGr), t_end = int(int64_t(bi + 1) * a.ntiles / NGr);
  if (t_begin >= t_end) return;  // block-uniform
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, col = lane & 15, grp = lane >> 4;

  // per-stage weight resources and this wave's lane offset (its cout group)
  const __amdgpu_buffer_rsrc_t wr1 = __builtin_amdgcn_make_buffer_rsrc(const_cast<h8*>(a.w1), 0,
                                                                       int(S1::CT * S1::NALLOC * 1024), 0x00020000);
  const __amdgpu_buffer_rsrc_t wr2 = __builtin_amdgcn_make_buffer_rsrc(const_cast<h8*>(a.w2), 0,
                                                                       int(S2::CT * S2::NALLOC * 1024), 0x00020000);
  const uint32_t vo1 = uint32_t(((wave % S1::CG) * S1::CPW * S1::NALLOC * 64 + lane) * 16);
  const uint32_t vo2 = uint32_t(((wave % S2::CG) * S2::CPW * S2::NALLOC * 64 + lane) * 16);

  // x (op 1's input) and op 2's input channels that are not op 1's output, tile t -> registers
  h8 xv[NX], ev[NE];
  auto load_in = [&](int t) {
    const int p0 = t * kPwTP;
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      const int e = int(threadIdx.x) + NT * i, u = e / (CIN1 / 8), q = e - u * (CIN1 / 8);
      const bool ok = e < kPwTP * CIN1 / 8 && p0 + u < a.P;
      xv[i] = *reinterpret_cast<const h8*>(ok ? a.x1 + int64_t(p0 + u) * a.x1cs + q * 8 : g_pw_zero);
    }
#pragma unroll
    for (int i = 0; i < NE; ++i) {
      const int e = int(threadIdx.x) + NT * i, u = e / (CIN2 / 8), q = e - u * (CIN2 / 8);
      const bool ok = e < kPwTP * CIN2 / 8 && p0 + u < a.P && !(q * 8 >= a.ho && q * 8 < a.ho + a.hn);
      ev[i] = *reinterpret_cast<const h8*>(ok ? a.x2 + int64_t(p0 + u) * a.x2cs + q * 8 : g_pw_zero);
    }
  };
  auto store_in = [&]() {
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      const int e = int(threadIdx.x) + NT * i, u = e / (CIN1 / 8), q = e - u * (CIN1 / 8);
      if (e < kPwTP * CIN1 / 8) sm[OX + pw_slot(u, q)] = xv[i];
    }
#pragma unroll
    for (int i = 0; i < NE; ++i) {
      const int e = int(threadIdx.x) + NT * i, u = e / (CIN2 / 8), q = e - u * (CIN2 / 8);
      if (e < kPwTP * CIN2 / 8 && !(q * 8 >= a.ho && q * 8 < a.ho + a.hn)) sm[OE + pw_slot(u, q)] = ev[i];
    }
  };
  h8 av[kPwNA];
#pragma unroll
  for (int s = 0; s < S1::CPW * S1::NS; ++s) av[s] = pw_a<CIN1, COUT1, NW>(wr1, vo1, s);
  load_in(t_begin);
  {
    float* bias = reinterpret_cast<float*>(sm + OBIAS);
    for (int e = int(threadIdx.x); e < COUT1 + COUT2; e += NT) bias[e] = e < COUT1 ? a.b1[e] : a.b2[e - COUT1];
  }
  const float* bias1 = reinterpret_cast<const float*>(sm + OBIAS);
  const float* bias2 = bias1 + COUT1;
  const float alpha1 = a.epi1 != FCE_EPI_STORE ? fusion_alpha(a.fw, a.fn, a.fi) : 1.f;  // conv_epilogue's weight
  _Float16* eimg = reinterpret_cast<_Float16*>(sm + OE);

  for (int t = t_begin; t < t_end; ++t) {
    const int p0 = t * kPwTP;
    stage_barrier();  // the previous tile's op 2 has read the images (first time round: the biases are published)
    store_in();
    stage_barrier();
    // ---- op 1: into the x2 image's h channels (and to HBM when another op reads h)
    {
      const int cg = wave % S1::CG, pg = wave / S1::CG;
      auto epi = [&](int cl, int i, const f4& acc) {
        const int co0 = (cg * S1::CPW + cl) * 16 + grp * 4;
        const int u = (pg + S1::PG * i) * 16 + col, pix = p0 + u;
        const int pc = min(pix, a.P - 1);
        h4 rv = h4{0, 0, 0, 0}, pv = h4{0, 0, 0, 0};
        if (a.r1) rv = *reinterpret_cast<const h4*>(a.r1 + int64_t(pc) * a.r1cs + co0);
        if (a.epi1 == FCE_EPI_ACCUM) pv = *reinterpret_cast<const h4*>(a.h + int64_t(pc) * a.hcs + co0);
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float tt = acc[j] + bias1[co0 + j];
          v[j] = a.act1 ? silu(tt) : tt;
        }
        if (a.r1) {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = fpin(v[j] + (float)rv[j]);
        }
        // the BiFPN weighted store / accumulate, in conv_epilogue's arithmetic
        if (a.epi1 == FCE_EPI_WSTORE) {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = fpin(v[j] * alpha1);
        } else if (a.epi1 == FCE_EPI_ACCUM) {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = fpin((float)pv[j] + fpin(alpha1 * v[j]));
        }
        const h4 hv = h4_of(v);
        if (co0 >= a.hs && co0 < a.hs + a.hn) {  // an op-2 input channel: into its image
          const int c2 = co0 - a.hs + a.ho;
          *reinterpret_cast<h4*>(eimg + pw_slot(u, c2 >> 3) * 8 + (c2 & 7)) = hv;
        }
        if (a.h_store && pix < a.P) *reinterpret_cast<h4*>(a.h + int64_t(pix) * a.hcs + co0) = hv;
      };
      pw_stage<CIN1, COUT1, NW, CIN2, COUT2>(sm + OX, av, wr2, vo2, epi);
    }
    stage_barrier();
    load_in(min(t + 1, t_end - 1));  // unconditional (clamped): the next tile's inputs, in flight during op 2
    // ---- op 2: to HBM
    {
      const int cg = wave % S2::CG, pg = wave / S2::CG;
      auto epi = [&](int cl, int i, const f4& acc) {
        const int co0 = (cg * S2::CPW + cl) * 16 + grp * 4;
        const int u = (pg + S2::PG * i) * 16 + col, pix = p0 + u;
        const int pc = min(pix, a.P - 1);
        h4 rv = h4{0, 0, 0, 0};
        if (a.r2) rv = *reinterpret_cast<const h4*>(a.r2 + int64_t(pc) * a.r2cs + co0);
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float tt = acc[j] + bias2[co0 + j];
          v[j] = a.act2 ? silu(tt) : tt;
        }
        if (a.r2) {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = fpin(v[j] + (float)rv[j]);
        }
        if (pix >= a.P) return;
        const h4 hv = h4_of(v);
        *reinterpret_cast<h4*>(a.y + int64_t(pix) * a.ycs + co0) = hv;
        if (a.dup && co0 >= a.duplo && co0 < a.duplo + a.dupn)
          *reinterpret_cast<h4*>(a.dup + int64_t(pix) * a.dupcs + (co0 - a.duplo)) = hv;
      };
      pw_stage<CIN2, COUT2, NW, CIN1, COUT1>(sm + OE, av, wr1, vo1, epi);
    }
  }
}

// ============================================================================ host
// instantiated (cin1, cout1, cin2, cout2): the n scale's C3k2(c3k = True) pairs (L7: c 64; L10 / L24: c 128), its
// C2PSA's three pairs (c 128) and two BiFPN realign -> C3k2 cv1 pairs of the neck
struct PwInst {
  int cin1, cout1, cin2, cout2;
};
static constexpr PwInst kPwInsts[] = {
    {128, 128, 64, 64},    // n L7 cv1 -> C3k cv1 / cv2 (merged)
    {64, 64, 192, 128},    // n L7 C3k cv3 -> cv2
    {256, 256, 128, 128},  // n L10 cv1 -> C3k cv1 / cv2 (and s L7)
    {64, 256, 128, 128},   // n L24 cv1 -> C3k cv1 / cv2 (its input is the 64-channel BiFPN_Concat)
    {128, 128, 384, 256},  // n L10 / L24 C3k cv3 -> cv2
    {256, 256, 128, 256},  // n L12 C2PSA cv1 -> attn.qkv
    {128, 128, 128, 256},  // n L12 attn.proj (+ b) -> ffn[0]
    {256, 128, 256, 256},  // n L12 ffn[1] (+ x1) -> cv2
    {128, 64, 64, 128},    // n L14 -> L15: BiFPN_Concat's realign of L8 (ACCUM) -> C3k2 cv1
    {128, 32, 32, 128},    // n L20 -> L21: the realign of L15 (ACCUM) -> C3k2 cv1
};

template <int CIN1, int COUT1, int CIN2, int COUT2>
static int pw_launch(const Pw2Args& a0, hipStream_t s) {
  constexpr int NW = 8;
  constexpr size_t LDS = size_t(CIN1 / 32 + CIN2 / 32) * kPwTP * 4 * 16 + size_t(COUT1 + COUT2) * 4;
  static_assert(LDS <= 160 * 1024, "pw2: LDS");
  auto k = pw2_kernel<CIN1, COUT1, CIN2, COUT2, NW>;
  static const bool big = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
  if (!big && LDS > 64 * 1024) return fail(FCE_ERR_HIP, "pw2: cannot opt in to >64 KiB LDS");
  Pw2Args a = a0;
  a.ntiles = (a.P + kPwTP - 1) / kPwTP;
  if (a.ntiles == 0) return FCE_OK;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
  }
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k, NW * 64, LDS) != hipSuccess || occ < 1) occ = 1;
  const int grid = int(std::min<int64_t>(a.ntiles, int64_t(cus) * occ));
  FCE_LAUNCH(k, dim3(unsigned(grid)), dim3(NW * 64), LDS, s, a);
  return launch_status("pw2_kernel");
}

template <int I>
static int pw_launch_i(const Pw2Args& a, hipStream_t s) {
  static_assert(I < int(sizeof(kPwInsts) / sizeof(kPwInsts[0])), "pw2: instance");
  return pw_launch<kPwInsts[I].cin1, kPwInsts[I].cout1, kPwInsts[I].cin2, kPwInsts[I].cout2>(a, s);
}

static int pw_inst(const fce_pw2_desc& d) {
  for (int i = 0; i < int(sizeof(kPwInsts) / sizeof(kPwInsts[0])); ++i)
    if (kPwInsts[i].cin1 == d.cin1 && kPwInsts[i].cout1 == d.cout1 && kPwInsts[i].cin2 == d.cin2 &&
        kPwInsts[i].cout2 == d.cout2)
      return i;
  return -1;
}

bool pw2_fused_ok(const fce_pw2_desc& d) { return pw_inst(d) >= 0; }

static bool same_map(const fce_tensor& a, const fce_tensor& b) { return a.n == b.n && a.h == b.h && a.w == b.w; }
static bool f16_nhwc(const fce_tensor& t) { return t.layout == FCE_NHWC && t.dtype == FCE_F16; }

int pw2_fused(const fce_pw2_desc& d, const fce_tensor& x1, const fce_tensor* r1, const fce_tensor& h, int h_store,
              const fce_tensor& x2, const fce_tensor* r2, const fce_tensor& y, const fce_tensor* dup, int dup_lo,
              hipStream_t s) {
  const int inst = pw_inst(d);
  FCE_CHECK(inst >= 0, "pw2: unsupported channel configuration");
  FCE_CHECK(f16_nhwc(x1) && f16_nhwc(h) && f16_nhwc(x2) && f16_nhwc(y) && (!r1 || f16_nhwc(*r1)) &&
                (!r2 || f16_nhwc(*r2)) && (!dup || f16_nhwc(*dup)),
            "pw2: NHWC f16 views");
  FCE_CHECK(x1.c == d.cin1 && h.c == d.cout1 && x2.c == d.cin2 && y.c == d.cout2 && (!r1 || r1->c == d.cout1) &&
                (!r2 || r2->c == d.cout2),
            "pw2: channel counts");
  FCE_CHECK(same_map(x1, h) && same_map(x1, x2) && same_map(x1, y) && (!r1 || same_map(x1, *r1)) &&
                (!r2 || same_map(x1, *r2)) && (!dup || same_map(x1, *dup)),
            "pw2: every view the same map");
  for (const fce_tensor* t : {&x1, &h, &x2, &y, r1, r2, dup})
    if (t) FCE_CHECK(t->cstride % 8 == 0 && t->coff % 8 == 0, "pw2: 8-aligned channel slices");
  // op 2's input overlaps op 1's output in one buffer: channels [ho, ho + hn) of x2 = [hs, hs + hn) of h
  FCE_CHECK(x2.data == h.data && x2.cstride == h.cstride, "pw2: op 2's input must share op 1's output buffer");
  const int lo = std::max(x2.coff, h.coff), hi = std::min(x2.coff + x2.c, h.coff + h.c);
  FCE_CHECK(hi > lo && (lo - x2.coff) % 32 == 0 && (lo - h.coff) % 16 == 0 && (hi - lo) % 16 == 0,
            "pw2: op 2's input must take aligned channels of op 1's output");
  FCE_CHECK(!dup || (dup_lo % 8 == 0 && dup->c % 8 == 0 && dup_lo + dup->c <= d.cout2), "pw2: duplicate store range");
  FCE_CHECK(d.w[0] && d.w[1] && d.b[0] && d.b[1], "pw2: null weights");
  FCE_CHECK(d.epi1 == FCE_EPI_STORE || ((d.epi1 == FCE_EPI_WSTORE || d.epi1 == FCE_EPI_ACCUM) && d.fw && d.fn > 0 &&
                                         d.fi >= 0 && d.fi < d.fn),
            "pw2: op 1's epilogue is a plain store or a BiFPN weighted store / accumulate with its weights");
  Pw2Args a{};
  a.x1 = static_cast<const _Float16*>(x1.data) + x1.coff;
  a.x1cs = x1.cstride;
  a.r1 = r1 ? static_cast<const _Float16*>(r1->data) + r1->coff : nullptr;
  a.r1cs = r1 ? r1->cstride : 0;
  a.h = static_cast<_Float16*>(h.data) + h.coff;
  a.hcs = h.cstride;
  a.h_store = h_store ? 1 : 0;
  a.x2 = static_cast<const _Float16*>(x2.data) + x2.coff;
  a.x2cs = x2.cstride;
  a.ho = lo - x2.coff;
  a.hs = lo - h.coff;
  a.hn = hi - lo;
  a.r2 = r2 ? static_cast<const _Float16*>(r2->data) + r2->coff : nullptr;
  a.r2cs = r2 ? r2->cstride : 0;
  a.y = static_cast<_Float16*>(y.data) + y.coff;
  a.ycs = y.cstride;
  a.dup = dup ? static_cast<_Float16*>(dup->data) + dup->coff : nullptr;
  a.dupcs = dup ? dup->cstride : 0;
  a.duplo = dup_lo;
  a.dupn = dup ? dup->c : 0;
  const int64_t P = int64_t(x1.n) * x1.h * x1.w;
  FCE_CHECK(P < (int64_t(1) << 30), "pw2: too many pixels");
  a.P = int(P);
  a.w1 = static_cast<const h8*>(d.w[0]);
  a.w2 = static_cast<const h8*>(d.w[1]);
  a.b1 = d.b[0];
  a.b2 = d.b[1];
  a.act1 = d.act[0] == FCE_ACT_SILU;
  a.act2 = d.act[1] == FCE_ACT_SILU;
  a.epi1 = d.epi1;
  a.fw = d.fw;
  a.fn = d.fn;
  a.fi = d.fi;
  static_assert(sizeof(kPwInsts) / sizeof(kPwInsts[0]) == 10, "pw2: one case per instance");
  switch (inst) {  // the template arguments are read from the table, so the two cannot disagree
    case 0: return pw_launch_i<0>(a, s);
    case 1: return pw_launch_i<1>(a, s);
    case 2: return pw_launch_i<2>(a, s);
    case 3: return pw_launch_i<3>(a, s);
    case 4: return pw_launch_i<4>(a, s);
    case 5: return pw_launch_i<5>(a, s);
    case 6: return pw_launch_i<6>(a, s);
    case 7: return pw_launch_i<7>(a, s);
    case 8: return pw_launch_i<8>(a, s);
    default: return pw_launch_i<9>(a, s);
  }
}

}  // namespace fce
