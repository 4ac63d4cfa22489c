// Big-tile implicit-GEMM convolution: the wide 1x1 and 3x3 convs of the m/l scales with 128-256-wide block tiles.
// Replaces (reference, ultralytics/): nn/modules/conv.py:39-89 Conv.forward_fuse (BN folded by
// utils/torch_utils.py:237-267) for 1x1 kernels -- the C2f / C3k / SPPF / C2PSA cv1 / cv2 / FFN pointwise convs, the
// BiFPN realign convs (fce_block.py:24-38), nn.Upsample feeding a 1x1 conv -- and for 3x3 kernels with cin % 32 == 0
// (the stride-2 downsampling convs and the wide bottleneck convs).  Variant codes 0xB00 (1x1) / 0xC00 (3x3) |
// log2(wc) << 4 | split << 5 | (nw == 4) << 6 | (wr == 4) << 7.
//
// Geometry: NW waves per block (8: one block per CU; 4: two per CU, so one block's prologue and staged epilogue run
// under the other's K loop), WC waves along the couts, each owning WR cout tiles (8: 128 couts; 4: 64, 4-wave blocks
// only), times NW / WC waves along the pixels, each owning 4 groups of 16 pixels (64 pixels).  With WR = 8 every wave
// runs 32 MFMAs per K-step from 8 A + 4 B fragment reads (0.375 KiB of LDS reads per MFMA, against 0.5 for 64 x 64
// wave tiles).  The copies go global -> LDS by LDS-DMA (global_load_lds) into a ring of K-step slots issued RING - 1
// steps ahead (5 slots for 8 waves x 256 couts, 4 for 8 x 128 and for 4 x 64-cout waves, 3 for 4 x 128-cout waves), or
// (split) into two rings: the weights, L2 hits, 2 steps ahead, the pixels in a deeper ring 3-5 steps ahead.  A
// register-staged version (one step ahead, 32 KiB in flight: measured ~2.6 TB/s effective, Little's law at HBM
// latency) could not keep enough bytes in flight without spilling.  One raw s_barrier per step behind a counted
// vmcnt: a __syncthreads() there makes hipcc wait vmcnt(0) first (a DMA is a pending LDS write), which drained the
// whole ring every step.  The next step's fragments are read into a second register set while this step's MFMAs run.
// 3x3 (implicit im2col): K-step j = (32-channel chunk j / 9, tap j % 9), the packed weights' chunk-major order;
// every B piece of a step is the lane's pixel shifted by the tap, or the zero line outside the image, so stride 2
// costs no more staging than stride 1.
// Same K order (32-channel steps, ascending), same fragments and the shared epilogue (bias, SiLU, residual,
// BiFPN weighted store / accumulate, Detect cls): bitwise identical to every other variant of the same conv.
#include <algorithm>

#include "conv_args.h"

namespace fce {

// Staged fp16 output (OUT_F16 / OUT_WSTORE with a.stg): the block's BP x BC*16 output tile is assembled in LDS
// (pixel rows of BC*16 halves, 16-byte slot sl of pixel px at sl ^ (px & (NSL - 1))) and written with 16-byte lane
// stores, whole pixel rows per NSL lanes.  The fragment-layout stores (8 bytes per lane, 16 pixels x 32 bytes per
// instruction) were the bound of this kernel: 512 -> 512 at 80^2, bs 32 ran 275 us with them and 132 us without
// any store (FCE_BIG1_DIAG=1).  Values exactly as conv_epilogue / conv_store_staged: bitwise the same.
template <int BC, int BP, int NT, int WR, int OUT>
__device__ __forceinline__ void big1_store_staged(const ConvArgs& a, f4 (&acc)[WR][4], int p0, int wc, int wp, int cbl0,
                                                  int col, int grp, _Float16* ot) {
  constexpr int ROW = BC * 16, NSL = 2 * BC;
  const int cotiles = (a.cout + 15) >> 4;
  float alpha = 1.f;
  if (OUT == OUT_WSTORE) alpha = fusion_alpha(a.fw, a.fn, a.fi);
#pragma unroll
  for (int r = 0; r < WR; ++r) {
    const int ctl = wc * WR + r;
    const int co0 = (cbl0 + ctl) * 16 + grp * 4;
    if (cbl0 + ctl >= cotiles) continue;
    float bz[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bz[j] = bias_or0(a.bias, co0 + j, a.cout);
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int px = wp * 64 + p * 16 + col, pix = p0 + px;
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
  constexpr int NP = BP * NSL;  // 16-byte pieces of the tile (a multiple of NT)
  static_assert(NP % NT == 0, "whole store rounds");
#pragma unroll 4
  for (int e = int(threadIdx.x); e < NP; e += NT) {
    const int px = e / NSL, sl = e - px * NSL;
    const int pix = p0 + px, co = cbl0 * 16 + sl * 8;
    if (pix < a.P && co < a.cout) {
      const h8 hv = *reinterpret_cast<const h8*>(ot + px * ROW + (sl ^ (px & (NSL - 1))) * 8);
      *reinterpret_cast<h8*>(static_cast<_Float16*>(a.y) + int64_t(pix) * a.ycs + co) = hv;
      if (OUT == OUT_F16 && a.dup && co >= a.duplo && co < a.duplo + a.dupn)
        *reinterpret_cast<h8*>(a.dup + int64_t(pix) * a.dupcs + (co - a.duplo)) = hv;
    }
  }
}

template <int WC, int NW, int RING_, int WR = 8, int RBD = 0>
struct Big1Geom {
  static constexpr int WP = NW / WC;
  static constexpr int BC = WC * WR;    // cout tiles per block (WR per wave)
  static constexpr int BP = WP * 64;    // pixels per block
  static constexpr int NA = BC * 64;    // A pieces (16 B) per K-step = BC DMA instructions (1 KiB each)
  static constexpr int NB = BP * 4;     // B pieces per K-step = NB / 64 DMA instructions
  static constexpr int IA = BC / NW, IB = NB / 64 / NW;  // DMA instructions per wave per K-step
  static constexpr int RING = RING_;    // K-step slots: the copies of step s + RING - 1 go out while step s computes
  // split rings (RBD > 0, the HBM-bound 1x1s): the weights (L2 hits) in a 3-slot ring issued 2 steps ahead, the
  // pixels (HBM) in an RBD-slot ring issued RBD - 1 steps ahead
  static constexpr int RA = RBD ? 3 : RING, RB = RBD ? RBD : RING;
  static constexpr size_t lds = RBD ? size_t(RA * NA + RB * NB) * 16 : size_t(RING) * (NA + NB) * 16;
  static_assert(BC % NW == 0 && (NB / 64) % NW == 0, "whole DMA rounds per wave");
  static_assert(RBD == 0 || RBD >= 4, "split rings: the pixel ring at least 4 deep");
};

// ring slots.  8-wave blocks (one per CU): 5 when a slot is 32 KiB (WC = 2), 4 for the 40 KiB slots of WC = 1
// (copies issued 4 / 3 steps ahead).  4-wave blocks (two per CU, 24 KiB slots): 3, so two blocks fit in the LDS and
// one block's prologue / staged epilogue overlaps the other's K loop; with 64-cout waves (16-20 KiB slots): 4
constexpr int big_ring(int wc, int nw, int wr = 8) { return nw == 4 ? (wr == 4 ? 4 : 3) : wc == 2 ? 5 : 4; }

__device__ __forceinline__ int b1_slot(int u, int q) { return u * 4 + (q ^ ((u >> 1) & 3)); }

__device__ __forceinline__ void b1_glds16(const void* src, h8* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                   (void __attribute__((address_space(3)))*)lds_wave_base, 16, 0, 0);
}

// DIAG (diagnostics only, FCE_BIG1_DIAG): 1 = no output stores (a guard that never fires keeps the MFMAs live),
// 2 = no copies after the prologue (MFMAs on stale slots), 3 = no MFMAs (copies + fragment reads only)
// K loop: the next step's fragments are read into a second register set while this step's MFMAs run, so the copies
// are waited for one step ahead of their use (4.5-8 % over reading them after the step's barrier, l/m shapes on one
// box; s_setprio 1 around the MFMAs measured slower)
// WR: cout tiles per wave, 8 (128 couts x 64 pixels) or, for 4-wave blocks, 4 (64 x 64: twice the blocks on the
// mid-size maps of the m/l scales, 0.5 KiB of fragment reads per MFMA)
template <int KS, int S, int WC, int NW, int OUT, int DIAG = 0, int WR = 8, int RBD = 0>
__global__ __launch_bounds__(NW * 64, NW == 4 ? 2 : 1) void conv_big_kernel(ConvArgs a) {
  static_assert(KS == 1 ? S == 1 : (KS == 3 && (S == 1 || S == 2)), "conv big tile: 1x1 s1 or 3x3 s1 / s2");
  static_assert(NW == 8 || NW == 4, "conv big tile: 8- or 4-wave blocks");
  static_assert(WR == 8 || (WR == 4 && NW == 4), "conv big tile: 64-cout waves in 4-wave blocks only");
  using G = Big1Geom<WC, NW, big_ring(WC, NW, WR), WR, RBD>;
  constexpr int WP = G::WP, BC = G::BC, BP = G::BP, NA = G::NA, NB = G::NB, IA = G::IA, IB = G::IB, RING = G::RING;
  constexpr int RA = G::RA, RB = G::RB;
  extern __shared__ __attribute__((aligned(16))) h8 big1_smem[];  // RING x [A | B]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 15, grp = lane >> 4;
  const int wc = wave / WP, wp = wave - wc * WP;
  // XCD-aware order (tile_block): the cout groups of one pixel tile (and, for 3x3, the neighbouring tiles that
  // share its halo rows) land on one XCD's L2
  int pt, cog;
  tile_block(a.gy, pt, cog);
  const int p0 = pt * BP;
  const int cotiles = (a.cout + 15) >> 4;
  const int ct_blk = cog * BC;
  const int nst = KS == 1 ? (a.cin + 31) >> 5 : (a.cin >> 5) * 9;
  const h8* wts = reinterpret_cast<const h8*>(a.w);

  // LDS-DMA copies (global_load_lds: no staging registers, no ds_write): this wave's instructions i = wave + 8 j.
  // A instruction i = block cout tile i, lane l -> LDS slot 64 i + l (the fragment-read layout).  B instruction i
  // covers LDS slots 64 i .. 64 i + 63 lane-linearly, so the XOR swizzle is applied to the SOURCE: slot e holds
  // piece (e & 3) ^ ((u >> 1) & 3) of pixel u = e >> 2 (b1_slot is an involution on the piece index).
  const h8* asrc[IA];
#pragma unroll
  for (int j = 0; j < IA; ++j) {
    const int ct = min(ct_blk + wave + NW * j, cotiles - 1);
    asrc[j] = wts + size_t(ct) * a.nalloc * 64 + lane;
  }
  // B sources.  1x1: the pixel's piece (through the x2^up upsampling), -1 past P.  3x3: the piece of input pixel
  // (oy S - 1, ox S - 1) (possibly outside the image) and bm = the valid kernel rows (bits 0-2) and columns
  // (bits 3-5) of the pixel, 0 past P.
  int64_t boff[IB];
  int bq[IB];
  unsigned bm[IB];
#pragma unroll
  for (int j = 0; j < IB; ++j) {
    const int e = (wave + NW * j) * 64 + lane;
    const int u = e >> 2, q = (e & 3) ^ ((u >> 1) & 3), pix = p0 + u;
    bq[j] = q * 8;
    if constexpr (KS == 1) {
      boff[j] = pix < a.P ? conv1x1_src(a, pix) + q * 8 : -1;
      bm[j] = 0;
    } else {
      const int hw = a.Ho * a.Wo;
      const int n = pix / hw, r = pix - n * hw, oy = r / a.Wo, ox = r - oy * a.Wo;
      const int iy0 = oy * S - 1, ix0 = ox * S - 1;
      unsigned m = 0;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        m |= unsigned(iy0 + k >= 0 && iy0 + k < a.Hs) << k;
        m |= unsigned(ix0 + k >= 0 && ix0 + k < a.Ws) << (3 + k);
      }
      bm[j] = pix < a.P ? m : 0u;
      boff[j] = ((int64_t(n) * a.Hs + iy0) * a.Ws + ix0) * a.xcs + q * 8;
    }
  }
  // the next K-step to issue (3x3: chunk, kernel row, kernel column), wave-uniform
  int ic = 0, iky = 0, ikx = 0;
  // the zero line's address, opaque to the compiler: otherwise it reloads it from the GOT (s_load) at every use
  // and waits lgkmcnt(0) for it, which also waits for the next step's fragment reads in flight
  const void* zl = g_zero_line;
  asm volatile("" : "+s"(zl));
  // ring slots of step t: one ring of (A | B) slots, or (RBD) an A ring and a deeper B ring
  auto slot_a = [&](int t) -> h8* { return RBD ? big1_smem + (t % RA) * NA : big1_smem + (t % RING) * (NA + NB); };
  auto slot_b = [&](int t) -> h8* {
    return RBD ? big1_smem + RA * NA + (t % RB) * NB : big1_smem + (t % RING) * (NA + NB) + NA;
  };
  auto issue_a = [&](int t) {  // step t's weight copies
    h8* slot = slot_a(t);
#pragma unroll
    for (int j = 0; j < IA; ++j) b1_glds16(asrc[j] + size_t(t) * 64, slot + (wave + NW * j) * 64);  // zero steps past nst
  };
  auto issue_b = [&](int t) {  // step t's pixel copies (called in step order: the 3x3 tap cursor advances)
    h8* slot = slot_b(t);
    if constexpr (KS == 1) {
#pragma unroll
      for (int j = 0; j < IB; ++j) {
        const bool ok = boff[j] >= 0 && t * 32 + bq[j] < a.cin;
        b1_glds16(ok ? static_cast<const void*>(a.x + boff[j] + t * 32) : zl, slot + (wave + NW * j) * 64);
      }
    } else {
      const int64_t toff = int64_t(iky * a.Ws + ikx) * a.xcs + ic * 32;
      const unsigned need = (1u << iky) | (8u << ikx);
      const bool live = t < nst;
#pragma unroll
      for (int j = 0; j < IB; ++j) {
        const bool ok = live && (bm[j] & need) == need;
        b1_glds16(ok ? static_cast<const void*>(a.x + boff[j] + toff) : zl, slot + (wave + NW * j) * 64);
      }
      if (++ikx == 3) {
        ikx = 0;
        if (++iky == 3) {
          iky = 0;
          ++ic;
        }
      }
    }
  };
  auto issue = [&](int t) {  // one ring: step t's copies, A then B
    issue_a(t);
    issue_b(t);
  };

  f4 acc[WR][4];
#pragma unroll
  for (int r = 0; r < WR; ++r)
#pragma unroll
    for (int p = 0; p < 4; ++p) acc[r][p] = f4{0.f, 0.f, 0.f, 0.f};

  // prologue: steps 0 .. RING - 2 in flight (copies past nst read zero weight steps / zero pixels: harmless).
  // Split rings: A(0), B(0), A(1), B(1), B(2) .. B(RB - 2)
  if constexpr (RBD) {
#pragma unroll
    for (int t = 0; t < RB - 1; ++t) {
      if (t < RA - 1) issue_a(t);
      issue_b(t);
    }
  } else {
#pragma unroll
    for (int t = 0; t < RING - 1; ++t) issue(t);
  }
  auto frags = [&](int t, h8(&fa)[WR], h8(&fb)[4]) {
    const h8* ca = slot_a(t);
    const h8* cb = slot_b(t);
#pragma unroll
    for (int p = 0; p < 4; ++p) fb[p] = cb[b1_slot(wp * 64 + p * 16 + col, grp)];
#pragma unroll
    for (int r = 0; r < WR; ++r) fa[r] = ca[(wc * WR + r) * 64 + lane];
  };
  // copies a wave may leave in flight at step s's wait (step s + 1's must have landed; vmcnt retires in issue
  // order).  One ring: the RING - 3 later steps.  Split rings: A(s + 1) went out at step s - 1 followed only by
  // B(s + RB - 2); early steps wait for more than needed (their later copies are all B's of the prologue)
  constexpr int ALLOW = RBD ? IB : (RING - 3) * (IA + IB);
  constexpr int ALLOW0 = RBD ? IA + (RB - 2) * IB : (RING - 2) * (IA + IB);  // before step 0
  // step s: step s + 1's copies landed (steps s + 2 .. s + RING - 2 may stay in flight) and published; step
  // s + RING - 1 issued into the slot step s - 1 used (its fragments were read during step s - 2 and consumed by
  // step s - 1's MFMAs, which every wave finished before this barrier); step s + 1's fragments read into the
  // other register set while step s's MFMAs run from this one
  auto step = [&](int s, h8(&ca)[WR], h8(&cb)[4], h8(&na)[WR], h8(&nb)[4]) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(ALLOW) : "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (DIAG != 2) {
      if constexpr (RBD) {
        issue_a(s + RA - 1);
        issue_b(s + RB - 1);
      } else {
        issue(s + RING - 1);
      }
    }
    frags(s + 1, na, nb);
#pragma unroll
    for (int r = 0; r < WR; ++r) {
      if (DIAG == 3) {
#pragma unroll
        for (int p = 0; p < 4; ++p) acc[r][p][0] += (float)ca[r][p] + (float)cb[p][r];
        continue;
      }
#pragma unroll
      for (int p = 0; p < 4; ++p) acc[r][p] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ca[r], cb[p], acc[r][p], 0, 0, 0);
    }
  };
  h8 a0[WR], b0[4], a1[WR], b1[4];
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(ALLOW0) : "memory");  // step 0 landed
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  frags(0, a0, b0);
  int s = 0;
  for (; s + 1 < nst; s += 2) {
    step(s, a0, b0, a1, b1);
    step(s + 1, a1, b1, a0, b0);
  }
  if (s < nst) step(s, a0, b0, a1, b1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no copy may land after the block exits (or in the staged tile)
  if (DIAG == 1) {
    float t = 0.f;
#pragma unroll
    for (int r = 0; r < WR; ++r)
#pragma unroll
      for (int p = 0; p < 4; ++p) t += acc[r][p][0] + acc[r][p][1] + acc[r][p][2] + acc[r][p][3];
    if (t == 1234.5678f) static_cast<_Float16*>(a.y)[tid] = (_Float16)t;
    return;
  }
  if constexpr (OUT == OUT_F16 || OUT == OUT_WSTORE) {
    if (a.stg) {  // the ring is free once every wave is past its last step (BP x BC*16 halves fit in it)
      static_assert(size_t(BP) * BC * 16 * 2 <= G::lds, "staged output tile exceeds the rings");
      __syncthreads();
      big1_store_staged<BC, BP, NW * 64, WR, OUT>(a, acc, p0, wc, wp, ct_blk, col, grp, reinterpret_cast<_Float16*>(big1_smem));
      return;
    }
  }
  conv_epilogue<WR, 4, OUT>(a, acc, p0 + wp * 64, ct_blk + wc * WR, col, grp);
}

bool big1_ok(int wc) { return wc == 1 || wc == 2; }

template <int KS, int S, int WC, int NW, int OUT, int DIAG, int WR = 8, int RBD = 0>
static int launch_big_d(const ConvArgs& a, dim3 grid, hipStream_t s) {
  constexpr size_t lds = Big1Geom<WC, NW, big_ring(WC, NW, WR), WR, RBD>::lds;
  static_assert(lds * (NW == 4 ? 2 : 1) <= 160 * 1024, "big tile: LDS over 160 KiB per CU");
  static const bool big =
      hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_big_kernel<KS, S, WC, NW, OUT, DIAG, WR, RBD>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
  if (!big) return fail(FCE_ERR_HIP, "conv big tile: cannot opt in to >64 KiB LDS");
  FCE_LAUNCH((conv_big_kernel<KS, S, WC, NW, OUT, DIAG, WR, RBD>), grid, dim3(NW * 64), lds, s, a);
  return FCE_OK;
}

template <int KS, int S, int WC, int NW, int OUT, int WR = 8, int RBD = 0>
static int launch_big_k(const ConvArgs& a, dim3 grid, hipStream_t s) {
  if constexpr (WR == 4 || RBD) return launch_big_d<KS, S, WC, NW, OUT, 0, WR, RBD>(a, grid, s);
  static const int diag = [] {
    const char* e = getenv("FCE_BIG1_DIAG");
    return e ? atoi(e) : 0;
  }();
  if constexpr (OUT == OUT_F16) {
    if (diag == 1) return launch_big_d<KS, S, WC, NW, OUT, 1>(a, grid, s);
    if (diag == 2) return launch_big_d<KS, S, WC, NW, OUT, 2>(a, grid, s);
    if (diag == 3) return launch_big_d<KS, S, WC, NW, OUT, 3>(a, grid, s);
  }
  return launch_big_d<KS, S, WC, NW, OUT, 0>(a, grid, s);
}

template <int WC, int NW, int WR = 8, int RBD = 0>
static int launch_big1_w(const ConvArgs& a, int out_kind, dim3 grid, hipStream_t s) {
  switch (out_kind) {
    case OUT_F16: return launch_big_k<1, 1, WC, NW, OUT_F16, WR, RBD>(a, grid, s);
    case OUT_F32: return launch_big_k<1, 1, WC, NW, OUT_F32, WR, RBD>(a, grid, s);
    case OUT_WSTORE: return launch_big_k<1, 1, WC, NW, OUT_WSTORE, WR, RBD>(a, grid, s);
    case OUT_ACCUM: return launch_big_k<1, 1, WC, NW, OUT_ACCUM, WR, RBD>(a, grid, s);
    case OUT_CLS: return launch_big_k<1, 1, WC, NW, OUT_CLS, WR, RBD>(a, grid, s);
    default: return fail(FCE_ERR_INVALID, "conv 1x1 big tile: unsupported epilogue");
  }
}

static ConvArgs big_grid(const ConvArgs& a0, int wc, int nw, int wr, dim3& grid) {
  ConvArgs a = a0;
  const int bp = (nw / wc) * 64, bc = wc * wr;
  a.gy = ((a.cout + 15) / 16 + bc - 1) / bc;
  const int64_t tiles = (int64_t(a.P) + bp - 1) / bp;
  grid = dim3(unsigned(std::min<int64_t>(tiles * a.gy, int64_t(1) << 31)));
  return a;
}

// the deep pixel ring (split rings) of each 1x1 configuration: as deep as the LDS allows (one block per CU for 8
// waves, two for 4), 0 = one ring
static constexpr int big1_rbd(int wc, int nw, int wr) {
  return nw == 8 ? (wc == 2 ? 6 : 4) : wr == 4 ? (wc == 2 ? 6 : 4) : (wc == 2 ? 4 : 0);
}
bool big1_split_ok(int wc, int nw, int wr) { return big1_rbd(wc, nw, wr) > 0; }

int launch_big1(const ConvArgs& a0, int out_kind, int wc, int nw, int wr, bool split, hipStream_t s) {
  FCE_CHECK(big1_ok(wc) && (nw == 8 || nw == 4) && (wr == 8 || (wr == 4 && nw == 4)) && a0.cin % 8 == 0 &&
                out_kind != OUT_DFL,
            "conv 1x1 big tile: bad configuration");
  dim3 grid;
  const ConvArgs a = big_grid(a0, wc, nw, wr, grid);
  FCE_CHECK(int64_t(grid.x) < (int64_t(1) << 31), "conv 1x1 big tile: grid too large");
  int rc;
  if (split) {
    if (nw == 8)
      rc = wc == 1 ? launch_big1_w<1, 8, 8, big1_rbd(1, 8, 8)>(a, out_kind, grid, s)
                   : launch_big1_w<2, 8, 8, big1_rbd(2, 8, 8)>(a, out_kind, grid, s);
    else if (wr == 8)
      rc = wc == 1 ? fail(FCE_ERR_INVALID, "conv 1x1 big tile: no split rings for 4 waves x 128 couts, wc 1")
                   : launch_big1_w<2, 4, 8, big1_rbd(2, 4, 8)>(a, out_kind, grid, s);
    else
      rc = wc == 1 ? launch_big1_w<1, 4, 4, big1_rbd(1, 4, 4)>(a, out_kind, grid, s)
                   : launch_big1_w<2, 4, 4, big1_rbd(2, 4, 4)>(a, out_kind, grid, s);
  } else if (nw == 8)
    rc = wc == 1 ? launch_big1_w<1, 8>(a, out_kind, grid, s) : launch_big1_w<2, 8>(a, out_kind, grid, s);
  else if (wr == 8)
    rc = wc == 1 ? launch_big1_w<1, 4>(a, out_kind, grid, s) : launch_big1_w<2, 4>(a, out_kind, grid, s);
  else
    rc = wc == 1 ? launch_big1_w<1, 4, 4>(a, out_kind, grid, s) : launch_big1_w<2, 4, 4>(a, out_kind, grid, s);
  if (rc != FCE_OK) return rc;
  return launch_status("conv_big_kernel");
}

template <int S, int NW, int WR>
static int launch_big3g_s(const ConvArgs& a, int wc, bool split, dim3 grid, hipStream_t s) {
  if (split)  // split rings for the 3x3s: wc 2 only (256 / 128-cout blocks)
    return wc == 2 ? launch_big_k<3, S, 2, NW, OUT_F16, WR, big1_rbd(2, NW, WR)>(a, grid, s)
                   : fail(FCE_ERR_INVALID, "conv 3x3 big tile: split rings need wc 2");
  return wc == 1 ? launch_big_k<3, S, 1, NW, OUT_F16, WR>(a, grid, s)
                 : launch_big_k<3, S, 2, NW, OUT_F16, WR>(a, grid, s);
}

int launch_big3g(const ConvArgs& a0, int wc, int nw, int wr, int stride, bool split, hipStream_t s) {
  FCE_CHECK(big1_ok(wc) && (nw == 8 || nw == 4) && (wr == 8 || (wr == 4 && nw == 4)) && a0.cin % 32 == 0 &&
                a0.up == 0 && (stride == 1 || stride == 2),
            "conv 3x3 big tile: bad configuration");
  dim3 grid;
  const ConvArgs a = big_grid(a0, wc, nw, wr, grid);
  FCE_CHECK(int64_t(grid.x) < (int64_t(1) << 31), "conv 3x3 big tile: grid too large");
  int rc;
  if (stride == 1)
    rc = nw == 8 ? launch_big3g_s<1, 8, 8>(a, wc, split, grid, s)
         : wr == 8 ? launch_big3g_s<1, 4, 8>(a, wc, split, grid, s)
                   : launch_big3g_s<1, 4, 4>(a, wc, split, grid, s);
  else
    rc = nw == 8 ? launch_big3g_s<2, 8, 8>(a, wc, split, grid, s)
         : wr == 8 ? launch_big3g_s<2, 4, 8>(a, wc, split, grid, s)
                   : launch_big3g_s<2, 4, 4>(a, wc, split, grid, s);
  if (rc != FCE_OK) return rc;
  return launch_status("conv_big_kernel");
}

}  // namespace fce
