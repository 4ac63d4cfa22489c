// Persistent 3x3 convolution ring fed by LDS-DMA (variant code 0xD00 | rp << 4 | (cpw - 1) << 3 | (sub - 1) << 2 |
// (nbuf - 2) of fce_conv2d_variant).
// Replaces (reference, ultralytics/): nn/modules/conv.py:39-89 Conv.forward_fuse (3x3, BN folded by
// utils/torch_utils.py:237-267) for cin 32 / 64, like conv3x3_ring_kernel (csrc/conv.hip), bitwise identical to it.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "conv_args.h"

namespace fce {

// slot swizzle of the tile kernels (conv.hip tile_slot): an involution of the 4 * KP pieces of position u
template <int KP>
__device__ __forceinline__ int dr_slot(int u, int q) {
  // KP 4 (16 pieces, 256 bytes per position: every position starts on bank 0): q ^ 2 (u & 7).  The lanes of a
  // ds_read_b128 group read two pieces q0, q0 ^ 1 (their lane groups) at 8 consecutive positions each, so the XOR term
  // takes all 8 even values per piece: 16 distinct 16-byte slots for any first position
  return KP == 1 ? (q ^ ((u >> 1) & 3)) : KP == 2 ? (q ^ (u & 6)) : (q ^ ((u & 7) << 1));
}

static bool dr_timing() {
  static const bool v = [] {
    const char* e = getenv("FCE_DRING_TIMING");
    return e && atoi(e) != 0;
  }();
  return v;
}

static int dr_blocks_per_cu(const void* kernel, size_t lds) {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kernel, 256, lds) != hipSuccess) {
    (void)hipGetLastError();
    n = 1;
  }
  return std::max(1, n);
}

// persistent slots per XCD (conv.hip ring_slots: tiles / 8 at most, the resident blocks of one XCD's CUs)
static int dr_slots(int units, int gy, int occ) {
  static const int cus = [] {
    int d = 0, n = 0;
    if (hipGetDevice(&d) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess) {
      (void)hipGetLastError();
      n = 256;
    }
    return std::max(1, n / 8);
  }();
  return std::max(1, std::min((units + 7) / 8, cus * occ / std::max(1, gy)));
}

// ============================================================================ 3x3, persistent, LDS-DMA ring
// conv3x3_ring_kernel (conv.hip: one cout tile per wave, its 9 * NCH A fragments in registers, TH = RP row x 16
// column tiles, the same K order, so bitwise identical) with the staged input copied global -> LDS by LDS-DMA
// (buffer_load_dwordx4 ... lds) into a ring of NBUF tile buffers, NBUF - 1 tiles ahead of the MFMAs, instead of one
// tile ahead through registers.  The register ring keeps ~16-21 KiB per block in flight for ~0.5 us of MFMAs; against
// an HBM round trip of 1-2 us under load that starves the stride-2 convs (n L3: 131 MB at 4.1 TB/s) and the 80^2 box
// convs.  Every wave issues the same number of copies per tile (the last ones fill a padding region with zeros: their
// offsets lie past the input resource's end, as do the out-of-image pieces), and its residual loads and output stores
// are unconditional (clamped loads, buffer stores past the output resource's end for lanes with nothing to write), so
// the vm ops issued after a tile's copies are a fixed count: each wave waits for exactly its own copies of the coming
// tile with a counted vmcnt, and a raw barrier then publishes every wave's.  The DMA destination is lane-linear, so
// the swizzled image (tile_slot) is kept by permuting the SOURCE pieces: LDS slot (u, s) holds piece dr_slot(u, s)
// (an involution) of position u.
// s_waitcnt vmcnt(n) for a wave-uniform n <= 63 (the instruction takes an immediate)
__device__ __forceinline__ void dr_vm_wait(int n) {
  switch (n) {
#define FCE_DRW(k)                                        \
  case k:                                                 \
    asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); \
    break;
#define FCE_DRW8(b) FCE_DRW(b) FCE_DRW(b + 1) FCE_DRW(b + 2) FCE_DRW(b + 3) FCE_DRW(b + 4) FCE_DRW(b + 5) FCE_DRW(b + 6) FCE_DRW(b + 7)
    FCE_DRW8(1) FCE_DRW8(9) FCE_DRW8(17) FCE_DRW8(25) FCE_DRW8(33) FCE_DRW8(41) FCE_DRW8(49) FCE_DRW(57) FCE_DRW(58)
    FCE_DRW(59) FCE_DRW(60) FCE_DRW(61) FCE_DRW(62) FCE_DRW(63)
#undef FCE_DRW8
#undef FCE_DRW
    default:
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

// CPW cout tiles per wave: 1 -- four waves along the couts, one B fragment read per MFMA (the register ring's ratio);
// 2 -- two waves along the couts x two along the rows, each B fragment feeding two MFMAs (half the LDS reads per
// MFMA: the bound of the 64 -> 64 stride-1 convs), the A fragments of both cout tiles in registers (no staging
// registers to make room for: the copies go straight to LDS).
// TM (diagnostics, FCE_DRING_TIMING=1): per wave, the clocks of each tile's phases summed over its tiles -- the wait for
// its copies plus the barrier, the residual loads and copy issue, the MFMA loop, the epilogue -- for the first 4096 blocks
template <int S, int RP, int NCH, int NBUF, int CPW, int SUB = 1, bool TM = false>
__global__ __launch_bounds__(256, 2) void conv3x3_dring_kernel(ConvArgs a, int nslot, unsigned long long* tm) {
  constexpr int WC = CPW == 1 ? 4 : 2, WRW = 4 / WC, RPT = RP * SUB;  // RPT rows per wave and tile
  using G = Dring3Geom<S, RPT, NCH, WRW>;
  constexpr int TW = G::TW, TH = G::TH, CI = G::CI, NQ = G::NQ, NE = G::NE, DPW = G::DPW, BUF = G::BUF;
  constexpr int KP = NCH;
  extern __shared__ __attribute__((aligned(16))) h8 dring_smem[];  // NBUF x BUF pieces
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = lane & 15, grp = lane >> 4;
  const int wc = wave % WC, wr = wave / WC;
  const int xcd = blockIdx.x & 7, loc = blockIdx.x >> 3;
  const int by = loc % a.gy, slot = loc / a.gy;
  const int tiles_x = (a.Wo + TW - 1) / TW, tiles_y = (a.Ho + TH - 1) / TH;
  const int ntiles = tiles_x * tiles_y * a.N;
  const int chunk = (ntiles + 7) >> 3, tbeg = xcd * chunk + slot, tend = min(ntiles, (xcd + 1) * chunk);
  if (tbeg >= tend) return;  // block-uniform
  const int step = nslot, count = (tend - tbeg + step - 1) / step;
  const int cotiles = (a.cout + 15) >> 4;
  int co0[CPW];
  bool cok[CPW];
  h8 af[CPW][NCH * 9];
  float bz[CPW][4];
#pragma unroll
  for (int cl = 0; cl < CPW; ++cl) {
    const int ct = (by * WC + wc) * CPW + cl;
    cok[cl] = ct < cotiles;
    co0[cl] = min(ct, cotiles - 1) * 16 + grp * 4;  // clamped: a tile past the couts is computed and dropped
    const h8* wf = reinterpret_cast<const h8*>(a.w) + (size_t(min(ct, cotiles - 1)) * a.nalloc) * 64 + lane;
#pragma unroll
    for (int k = 0; k < NCH * 9; ++k) af[cl][k] = wf[k * 64];
#pragma unroll
    for (int j = 0; j < 4; ++j) bz[cl][j] = bias_or0(a.bias, co0[cl] + j, a.cout);
  }
  const __amdgpu_buffer_rsrc_t yr = out_rsrc(a.y, uint32_t(a.P) * uint32_t(a.ycs) * 2u);
  // residual source: the view, or the zero line read at offset 0 (one load path: a branch around the load would leave
  // the compiler's wait at its use at vmcnt(0), i.e. also for the copies issued after it)
  const _Float16* const rbase = a.res ? a.res : g_zero_line;
  const int rcs = a.res ? a.rcs : 0;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<_Float16*>(a.x), 0, int(uint32_t(a.N) * uint32_t(a.Hs) * uint32_t(a.Ws) * uint32_t(a.xcs) * 2u), 0x00020000);
  // the copy pieces of this lane, tile-invariant: LDS slot e = (wave + 4 j) * 64 + lane holds piece dr_slot(u, s) of
  // staged position u = (row r, column c); its element offset from the tile's origin, and r / c for the bounds test
  // (padding slots past NE get a row that never passes it)
  int crow[DPW], ccol[DPW], crel[DPW];
#pragma unroll
  for (int j = 0; j < DPW; ++j) {
    const int e = (wave + 4 * j) * 64 + lane;
    const int u = e / NQ, sq = e - u * NQ;
    const int r = u / CI, cc = u - r * CI;
    const int c = S == 1 ? cc : (cc < (CI + 1) / 2 ? 2 * cc : 2 * (cc - (CI + 1) / 2) + 1);
    crow[j] = e < NE ? r : -(1 << 20);
    ccol[j] = c;
    crel[j] = (r * a.Ws + c) * a.xcs + dr_slot<KP>(u, sq) * 8;
  }
  // copies of the k-th tile of this block (clamped to its last: the look-ahead past the end re-copies it) into buffer b
  auto issue = [&](int k, int b) {
    const int tt = tbeg + min(k, count - 1) * step;
    const int tx = tt % tiles_x, r0 = tt / tiles_x, ty = r0 % tiles_y, n = r0 / tiles_y;
    const int iy0 = ty * TH * S - 1, ix0 = tx * TW * S - 1;
    const int org = ((n * a.Hs + iy0) * a.Ws + ix0) * a.xcs;  // element offset of the staged origin (< 2^30)
    h8* const dst = dring_smem + b * BUF;
#pragma unroll
    for (int j = 0; j < DPW; ++j) {
      const bool ok = unsigned(iy0 + crow[j]) < unsigned(a.Hs) && unsigned(ix0 + ccol[j]) < unsigned(a.Ws);
      // out of the image / padding: an offset past the resource's end, which reads zeros (no branch, no zero line)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (void __attribute__((address_space(3)))*)(dst + (wave + 4 * j) * 64),
                                               16, ok ? uint32_t(org + crel[j]) * 2u : 0x80000000u, 0, 0, 0);
    }
  };
#pragma unroll
  for (int k = 0; k < NBUF - 1; ++k) issue(k, k);
  // the A fragments and biases landed (with the prologue's copies) before the tile loop: otherwise hipcc's waitcnt
  // pass, merging the loop's back edge with the entry, kept a counted vmcnt wait before nearly every MFMA of every tile
  // (satisfied at once after the first tile: no time change measured, `profiles/r06_dring_probe.txt`)
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  // vm ops per tile after its copies: CPW x RPT residual loads, DPW copies, CPW x RPT stores
  constexpr int NO = CPW * RPT, PER = NO + DPW + NO;
  unsigned long long ph[4] = {0, 0, 0, 0}, tprev = 0;
  auto tick = [&](int i) {
    if constexpr (TM) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      ph[i] += t - tprev;
      tprev = t;
    }
  };
  if constexpr (TM) tprev = __builtin_amdgcn_s_memtime();
  for (int k = 0; k < count; ++k) {
    // this wave's copies of tile k are older than: the prologue's later copies and k earlier tiles (k < NBUF - 1), or
    // the stores of the tile that issued them and NBUF - 2 whole tiles since
    const int newer = k < NBUF - 1 ? (NBUF - 2 - k) * DPW + k * PER : NO + (NBUF - 2) * PER;
    dr_vm_wait(newer);
    __builtin_amdgcn_s_barrier();  // every wave's copies of tile k landed; tile k - 1's reads are done
    asm volatile("" ::: "memory");
    tick(3);
    const int tt = tbeg + k * step;
    const int tx = tt % tiles_x, r0 = tt / tiles_x, ty = r0 % tiles_y, n = r0 / tiles_y;
    const int oy0 = ty * TH + wr * RPT, ox = tx * TW + col;  // the wave's first output row (SUB sub-tiles of RP rows)
    const int pix0 = (n * a.Ho + oy0) * a.Wo + ox;  // output pixel of row q: pix0 + q Wo (< 2^30: the output < 2 GiB)
    // residuals first (clamped, unconditional: the zero line without one), then the copies of tile k + NBUF - 1 into
    // the buffer tile k - 1 used: the epilogue's wait for the residuals leaves those copies in flight
    h4 rres[CPW][RPT];
#pragma unroll
    for (int cl = 0; cl < CPW; ++cl)
#pragma unroll
      for (int q = 0; q < RPT; ++q) {
        const int pix = (n * a.Ho + min(oy0 + q, a.Ho - 1)) * a.Wo + min(ox, a.Wo - 1);
        rres[cl][q] = *reinterpret_cast<const h4*>(rbase + int64_t(pix) * rcs + (a.res ? co0[cl] : 0));
      }
    issue(k + NBUF - 1, (k + NBUF - 1) % NBUF);
    tick(0);
    const h8* const img = dring_smem + (k % NBUF) * BUF;
#pragma unroll
    for (int sb = 0; sb < SUB; ++sb) {  // sub-tiles: more MFMAs per barrier and copy wait, the same registers
      f4 acc[CPW][RP];
#pragma unroll
      for (int cl = 0; cl < CPW; ++cl)
#pragma unroll
        for (int p = 0; p < RP; ++p) acc[cl][p] = f4{0.f, 0.f, 0.f, 0.f};
      // K-steps (chunk, tap) in the ring's order; the B fragments of step s + 1 are read while step s's MFMAs run (a
      // register double buffer: without it hipcc waited lgkmcnt(0) before nearly every MFMA group)
      // a sub-tile RP S CI positions on (a multiple of 8: the same swizzle) reads at a constant offset from the first's
      // addresses, which the ds reads take as an immediate (recomputed addresses per sub-tile spilled)
      constexpr bool SHIFT = (RP * S * CI) % 8 == 0;
      auto read_b = [&](int st, h8 (&bv)[RP]) {
        const int kc = st / 9, tap = st - kc * 9, ky = tap / 3, kx = tap - ky * 3;
#pragma unroll
        for (int p = 0; p < RP; ++p) {
          const int u = ((wr * RPT + (SHIFT ? 0 : sb * RP) + p) * S + ky) * CI + tile_col<S, CI>(col * S + kx);
          bv[p] = img[(SHIFT ? sb * RP * S * CI * NQ : 0) + u * NQ + dr_slot<KP>(u, kc * 4 + grp)];
        }
      };
      h8 bb[2][RP];
      read_b(0, bb[0]);
#pragma unroll
      for (int st = 0; st < NCH * 9; ++st) {
        if (st + 1 < NCH * 9) read_b(st + 1, bb[(st + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);  // the next step's reads ahead of this step's MFMAs
#pragma unroll
        for (int p = 0; p < RP; ++p)
#pragma unroll
          for (int cl = 0; cl < CPW; ++cl)
            acc[cl][p] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[cl][st], bb[st & 1][p], acc[cl][p], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
      // epilogue: tile3_post's arithmetic (bias, SiLU, residual, fp16), every lane storing (dropped past the edges)
      if (sb == 0) {
        tick(1);
        dr_vm_wait(DPW);  // the residuals (older than this tile's copies)
      }
#pragma unroll
      for (int cl = 0; cl < CPW; ++cl)
#pragma unroll
        for (int p = 0; p < RP; ++p) {
          const int q = sb * RP + p, oy = oy0 + q;
          float v[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float t = acc[cl][p][j] + bz[cl][j];
            v[j] = a.act ? silu(t) : t;
          }
          if (a.res) {
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = fpin(v[j] + (float)rres[cl][q][j]);
          }
          const bool ok = cok[cl] && oy < a.Ho && ox < a.Wo;
          const uint32_t off = uint32_t((pix0 + q * a.Wo) * a.ycs + co0[cl]) * 2u;
          store_h4_or_drop(yr, ok, off,
                           h4{(_Float16)fpin(v[0]), (_Float16)fpin(v[1]), (_Float16)fpin(v[2]), (_Float16)fpin(v[3])});
        }
      // one sub-tile's accumulators live at a time (interleaving the next one's MFMAs with this epilogue spilled)
      if (SUB > 1) __builtin_amdgcn_sched_barrier(0);
    }
    tick(2);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no copy may land in LDS after the block is gone
  if constexpr (TM) {
    tick(3);
    if (lane == 0 && blockIdx.x < 4096) {
      unsigned long long* o = tm + (size_t(blockIdx.x) * 4 + wave) * 5;
      for (int i = 0; i < 4; ++i) o[i] = ph[i];
      o[4] = count;
    }
  }
}

template <int S, int RP, int NCH, int NBUF, int CPW, int SUB>
static int launch_dring3_k(const ConvArgs& a, int ntiles, hipStream_t s) {
  if constexpr (!dring3_offer(S, RP, NCH, NBUF, CPW, SUB)) {
    return fail(FCE_ERR_INVALID, "conv 3x3 LDS-DMA ring: configuration not instantiated");  // launch_dring3 checks first
  } else {
    constexpr size_t lds = size_t(NBUF) * Dring3Geom<S, RP * SUB, NCH, CPW == 1 ? 1 : 2>::BUF * 16;
    auto k = conv3x3_dring_kernel<S, RP, NCH, NBUF, CPW, SUB>;
    static const bool big = lds <= 64 * 1024 || hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                                                     160 * 1024) == hipSuccess;
    if (!big) return fail(FCE_ERR_HIP, "conv 3x3 LDS-DMA ring: cannot opt in to >64 KiB LDS");
    static const int occ = dr_blocks_per_cu(reinterpret_cast<const void*>(k), lds);
    const int nslot = dr_slots(ntiles, a.gy, occ);
    const unsigned grid = unsigned(8 * a.gy * nslot);
    if (!dr_timing()) {
      FCE_LAUNCH(k, dim3(grid), dim3(256), lds, s, a, nslot, nullptr);
      return launch_status("conv3x3_dring_kernel");
    }
    // diagnostics: one timed launch, synchronised, the per-tile phase clocks (averaged over waves) on stderr
    auto kt = conv3x3_dring_kernel<S, RP, NCH, NBUF, CPW, SUB, true>;
    if (lds > 64 * 1024)
      FCE_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kt), hipFuncAttributeMaxDynamicSharedMemorySize,
                                        160 * 1024));
    static unsigned long long* tm = nullptr;
    const size_t nrec = size_t(4096) * 4 * 5;
    if (!tm) FCE_HIP_CHECK(hipMalloc(&tm, nrec * 8));
    FCE_HIP_CHECK(hipMemsetAsync(tm, 0, nrec * 8, s));
    hipLaunchKernelGGL(kt, dim3(grid), dim3(256), lds, s, a, nslot, tm);
    FCE_HIP_CHECK(hipStreamSynchronize(s));
    std::vector<unsigned long long> h(nrec);
    FCE_HIP_CHECK(hipMemcpy(h.data(), tm, nrec * 8, hipMemcpyDeviceToHost));
    double ph[4] = {0, 0, 0, 0}, tiles = 0;
    for (size_t i = 0; i < nrec / 5; ++i) {
      for (int j = 0; j < 4; ++j) ph[j] += double(h[i * 5 + j]);
      tiles += double(h[i * 5 + 4]);
    }
    if (tiles > 0)
      fprintf(stderr, "dring<S%d,RP%d,NCH%d,NBUF%d,CPW%d,SUB%d> grid %u, %.2f tiles per wave; clocks per tile: res+copy issue %.0f, "
              "mfma %.0f, epilogue %.0f, wait+barrier %.0f\n", S, RP, NCH, NBUF, CPW, SUB, grid, tiles / (nrec / 5 > grid * 4 ? grid * 4 : nrec / 5),
              ph[0] / tiles, ph[1] / tiles, ph[2] / tiles, ph[3] / tiles);
    return launch_status("conv3x3_dring_kernel");
  }
}

template <int S, int RP, int NCH, int CPW, int SUB>
static int launch_dring3_u(const ConvArgs& a, int nbuf, int ntiles, hipStream_t s) {
  return nbuf == 2 ? launch_dring3_k<S, RP, NCH, 2, CPW, SUB>(a, ntiles, s)
                   : nbuf == 3 ? launch_dring3_k<S, RP, NCH, 3, CPW, SUB>(a, ntiles, s)
                               : launch_dring3_k<S, RP, NCH, 4, CPW, SUB>(a, ntiles, s);
}

template <int S, int RP, int NCH, int CPW>
static int launch_dring3_b(const ConvArgs& a, int nbuf, int sub, int ntiles, hipStream_t s) {
  return sub == 1 ? launch_dring3_u<S, RP, NCH, CPW, 1>(a, nbuf, ntiles, s)
                  : launch_dring3_u<S, RP, NCH, CPW, 2>(a, nbuf, ntiles, s);
}

template <int S, int NCH, int CPW>
static int launch_dring3_s(const ConvArgs& a, int rp, int nbuf, int sub, int ntiles, hipStream_t s) {
  if (rp == 1) return launch_dring3_b<S, 1, NCH, CPW>(a, nbuf, sub, ntiles, s);
  if (rp == 2) return launch_dring3_b<S, 2, NCH, CPW>(a, nbuf, sub, ntiles, s);
  if (rp == 4) return launch_dring3_b<S, 4, NCH, CPW>(a, nbuf, sub, ntiles, s);
  if constexpr (CPW == 1) return launch_dring3_b<S, 8, NCH, 1>(a, nbuf, sub, ntiles, s);
  return fail(FCE_ERR_INVALID, "conv 3x3 LDS-DMA ring: 8-row tiles need one cout tile per wave");
}

template <int S, int NCH>
static int launch_dring3_c(const ConvArgs& a, int rp, int nbuf, int cpw, int sub, int ntiles, hipStream_t s) {
  return cpw == 1 ? launch_dring3_s<S, NCH, 1>(a, rp, nbuf, sub, ntiles, s)
                  : launch_dring3_s<S, NCH, 2>(a, rp, nbuf, sub, ntiles, s);
}

// nbuf: tile buffers of the LDS-DMA ring (nbuf - 1 tiles of input in flight ahead of the MFMAs); cpw: cout tiles per wave
int launch_dring3(const ConvArgs& a0, int rp, int nbuf, int cpw, int sub, int stride, hipStream_t s) {
  FCE_CHECK((a0.cin == 32 || a0.cin == 64 || a0.cin == 128) && a0.cout % (16 * cpw) == 0 &&
                (rp == 1 || rp == 2 || rp == 4 || (rp == 8 && cpw == 1)) && nbuf >= 2 && nbuf <= 4 &&
                (cpw == 1 || cpw == 2) && (sub == 1 || sub == 2) && (stride == 1 || stride == 2) &&
                dring3_offer(stride, rp, a0.cin / 32, nbuf, cpw, sub),
            "conv 3x3 LDS-DMA ring: bad configuration");
  FCE_CHECK(a0.vec_ok && int64_t(a0.P) * a0.ycs * 2 < (int64_t(1) << 31) &&
                int64_t(a0.N) * a0.Hs * a0.Ws * a0.xcs * 2 < (int64_t(1) << 31),
            "conv 3x3 LDS-DMA ring: 8-byte aligned output, input and output below 2 GiB (the caller takes the register ring otherwise)");
  ConvArgs a = a0;
  const int th = rp * cpw * sub;  // cpw 2: two waves along the rows
  const int64_t ntiles = int64_t((a.Wo + 15) / 16) * ((a.Ho + th - 1) / th) * a.N;
  FCE_CHECK(ntiles < (int64_t(1) << 30), "conv 3x3 LDS-DMA ring: too many tiles");
  a.gy = ((a.cout + 15) / 16 + 3) / 4;  // 4 cout tiles per block either way
  const int nch = a.cin / 32;
  if (stride == 1)
    return nch == 1 ? launch_dring3_c<1, 1>(a, rp, nbuf, cpw, sub, int(ntiles), s)
                    : nch == 2 ? launch_dring3_c<1, 2>(a, rp, nbuf, cpw, sub, int(ntiles), s)
                               : launch_dring3_c<1, 4>(a, rp, nbuf, cpw, sub, int(ntiles), s);
  return nch == 1 ? launch_dring3_c<2, 1>(a, rp, nbuf, cpw, sub, int(ntiles), s)
                  : nch == 2 ? launch_dring3_c<2, 2>(a, rp, nbuf, cpw, sub, int(ntiles), s)
                             : launch_dring3_c<2, 4>(a, rp, nbuf, cpw, sub, int(ntiles), s);
}

}  // namespace fce
