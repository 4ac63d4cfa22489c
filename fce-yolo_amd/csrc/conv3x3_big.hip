// Big-tile 3x3 convolution fed by LDS-DMA (gfx950 global_load_lds_dwordx4); the m/l-scale 3x3 convs.
// Replaces (reference, ultralytics/): nn/modules/conv.py:39-89 Conv.forward_fuse (3x3, BN folded by
// utils/torch_utils.py:237-267) for cin % 32 == 0.  Variant code 0x800 | wm << 4 of fce_conv2d_variant.
#include <vector>

#include "conv_args.h"

namespace fce {

// For the wide 3x3 convs of the m/l scales (cin % 32 == 0, cin >= 128).  Every wave owns 64 couts x 64 output
// pixels (4 cout tiles x 4 output rows of 16 columns: 16 MFMAs per 4 A + 4 B fragment reads, half the LDS
// bytes per flop of the 32 x 64 tiles above); the block is WM x (4 / WM) such waves.  The K loop runs in
// stages of (32-channel chunk, kernel row ky): per stage the block's A fragments (WM * 4 cout tiles x 3 taps,
// 1 KiB each, contiguous in the packed weights) and, at ky = 0, the chunk's input halo tile are copied
// global -> LDS with global_load_lds_dwordx4 (no registers, no staging writes) into the other of two LDS
// buffers while this stage's MFMAs run: one barrier per stage.  The glds destination is lane-linear, so the
// input image keeps the tile kernels' XOR swizzle by permuting the SOURCE pieces (slot q of pixel u holds
// channel piece q ^ ((u >> 1) & 3); the read side applies the same involution).  Out-of-image pixels and the
// padding of the last instruction read the zero line.  K order (chunk, tap) and the fragment layouts are the
// implicit-GEMM kernel's: bitwise identical to every other variant.
template <int S, int WM, int AB, int NW = 4>
struct Big3Geom {
  static constexpr int WN = NW / WM, TW = 16, TH = WN * 4;
  static constexpr int RI = (TH - 1) * S + 3, CI = (TW - 1) * S + 3;
  static constexpr int NPX = RI * CI;                   // staged input pixels per chunk (64 B each)
  static constexpr int BINS = (NPX * 4 + 63) / 64;      // 1 KiB DMA instructions for the input tile
  static constexpr int AINS = WM * 4 * 3;               // 1 KiB DMA instructions for a stage's weights
  static constexpr int AH8 = AINS * 64, BH8 = BINS * 64;  // buffer sizes in 16-byte pieces
  static constexpr size_t lds = size_t(AB * AH8 + 2 * BH8) * 16;
};

__device__ __forceinline__ void glds16(const void* src, h8* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                   (void __attribute__((address_space(3)))*)lds_wave_base, 16, 0, 0);
}

// s_waitcnt vmcnt(n) for a wave-uniform n (the instruction takes an immediate)
__device__ __forceinline__ void vm_wait(int n) {
  switch (n) {
#define FCE_VMW(k)                                        \
  case k:                                                 \
    asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); \
    break;
    FCE_VMW(1) FCE_VMW(2) FCE_VMW(3) FCE_VMW(4) FCE_VMW(5) FCE_VMW(6) FCE_VMW(7) FCE_VMW(8)
    FCE_VMW(9) FCE_VMW(10) FCE_VMW(11) FCE_VMW(12) FCE_VMW(13) FCE_VMW(14) FCE_VMW(15)
#undef FCE_VMW
    default:
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

// AB = weight-stage buffers.  AB 2: stage s's weights are issued at stage s - 1, the input tile of chunk c + 1
// at stage (c, 0) (two stages ahead of its use).  AB 3: weights two stages ahead, the next input tile at
// (c, 1).  Each wave waits with a counted vmcnt for exactly the copies the coming stage reads (its own
// copies are retired in issue order; the raw barrier then publishes every wave's), so the copies issued
// later stay in flight across the barrier.
// TM (diagnostics, FCE_BIG3_TIMING=1): per wave, the clocks spent waiting for a stage (vmcnt + barrier) and
// computing it, summed over the stages, for the first 4096 blocks.
template <int S, int WM, int AB, int NW, bool TM>
__global__ __launch_bounds__(NW * 64, 2) void conv3x3_big_kernel(ConvArgs a, unsigned long long* tm) {
  using G = Big3Geom<S, WM, AB, NW>;
  constexpr int WN = G::WN, TW = G::TW, TH = G::TH, CI = G::CI, NPX = G::NPX;
  constexpr int BINS = G::BINS, AINS = G::AINS, AH8 = G::AH8, BH8 = G::BH8;
  extern __shared__ __attribute__((aligned(16))) h8 big3_smem[];  // [A0 | A1 (| A2) | B0 | B1], one array
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = lane & 15, grp = lane >> 4;
  const int wc = wave / WN, wr = wave - wc * WN;
  const int tiles_x = (a.Wo + TW - 1) / TW, tiles_y = (a.Ho + TH - 1) / TH;
  int t, cog;
  tile_block(a.gy, t, cog);
  const int tx = t % tiles_x;
  t /= tiles_x;
  const int ty = t % tiles_y;
  const int n = t / tiles_y;
  const int ox0 = tx * TW, oy0 = ty * TH;
  const int cotiles = (a.cout + 15) >> 4;
  const int ct_blk = cog * WM * 4;
  const int spt = a.cin >> 5;
  const int nst = spt * 3;
  const _Float16* xn = a.x + int64_t(n) * a.Hs * a.Ws * a.xcs;
  const h8* wts = reinterpret_cast<const h8*>(a.w);
  const int iy0 = oy0 * S - 1, ix0 = ox0 * S - 1;
  h8* const bbase = big3_smem + AB * AH8;

  // input-tile pieces this lane copies (fixed over chunks): pixel offset in the image, or -1 (zero line)
  constexpr int BPW = (BINS + NW - 1) / NW;  // DMA instructions per wave for the input tile (some waves one fewer)
  const int nb = wave + NW * (BPW - 1) < BINS ? BPW : BPW - 1;
  int64_t boff[BPW];
#pragma unroll
  for (int j = 0; j < BPW; ++j) {
    const int e = (wave + NW * j) * 64 + lane;
    const int u = e >> 2, slot = e & 3;
    boff[j] = -1;
    if (u < NPX) {
      const int r = u / CI, cc = u - r * CI;
      const int c = S == 1 ? cc : (cc < (CI + 1) / 2 ? 2 * cc : 2 * (cc - (CI + 1) / 2) + 1);
      const int iy = iy0 + r, ix = ix0 + c;
      const int q = slot ^ ((u >> 1) & 3);
      if (iy >= 0 && iy < a.Hs && ix >= 0 && ix < a.Ws) boff[j] = (int64_t(iy) * a.Ws + ix) * a.xcs + q * 8;
    }
  }
  // weight rows this lane copies: instruction i = wave + NW j -> cout tile i / 3, tap i % 3
  constexpr int APW = (AINS + NW - 1) / NW;
  const int na = wave + NW * (APW - 1) < AINS ? APW : APW - 1;
  const h8* asrc[APW];
#pragma unroll
  for (int j = 0; j < APW; ++j) {
    const int i = min(wave + NW * j, AINS - 1), r = i / 3, kx = i - r * 3;
    const int ct = min(ct_blk + r, cotiles - 1);
    asrc[j] = wts + (size_t(ct) * a.nalloc + kx) * 64 + lane;
  }
  auto issue_a = [&](int s) {
    const int c = s / 3, ky = s - c * 3;
    h8* ab = big3_smem + (s % AB) * AH8;
#pragma unroll
    for (int j = 0; j < APW; ++j)
      if (wave + NW * j < AINS) glds16(asrc[j] + (c * 9 + ky * 3) * 64, ab + (wave + NW * j) * 64);
  };
  auto issue_b = [&](int c) {
    h8* bb = bbase + (c & 1) * BH8;
#pragma unroll
    for (int j = 0; j < BPW; ++j) {
      if (wave + NW * j < BINS) {
        const void* src = boff[j] >= 0 ? static_cast<const void*>(xn + boff[j] + c * 32)
                                       : static_cast<const void*>(g_zero_line);
        glds16(src, bb + (wave + NW * j) * 64);
      }
    }
  };

  f4 acc[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int p = 0; p < 4; ++p) acc[r][p] = f4{0.f, 0.f, 0.f, 0.f};
  issue_a(0);
  issue_b(0);
  if (AB == 3 && nst > 1) issue_a(1);
  unsigned long long t_start = 0, t_wait = 0, t_comp = 0, t0 = 0;
  if constexpr (TM) t_start = __builtin_amdgcn_s_memtime();
  for (int s = 0; s < nst; ++s) {
    if constexpr (TM) t0 = __builtin_amdgcn_s_memtime();
    const int c = s / 3, ky = s - c * 3;
    // copies this wave may leave in flight: those issued after the last one stage s reads
    int allow;
    if (AB == 2) {
      allow = (ky == 1 && c + 1 < spt) ? nb : 0;  // the next input tile, issued at (c, 0) after A(s)
    } else {
      allow = s + 1 < nst ? na : 0;                   // A(s + 1)
      if (ky == 2 && c + 1 < spt) allow += nb;        // + the next input tile, issued at (c, 1)
    }
    vm_wait(allow);
    __builtin_amdgcn_s_barrier();  // every wave's copies for stage s landed; stage s - 1's reads are done
    asm volatile("" ::: "memory");
    if constexpr (TM) {
      const unsigned long long t1 = __builtin_amdgcn_s_memtime();
      t_wait += t1 - t0;
      t0 = t1;
    }
    // this stage's copies (weights of stage s + AB - 1, and the next input tile at ky == AB - 2) are issued
    // one at a time between the MFMA groups below, where their issue cost hides under the matrix work
    const int sa = s + AB - 1;
    const bool do_a = sa < nst, do_b = ky == AB - 2 && c + 1 < spt;
    const int ca = sa / 3, kya = sa - ca * 3;
    h8* const abw = big3_smem + (sa % AB) * AH8;
    h8* const bbw = bbase + ((c + 1) & 1) * BH8;
    auto piece = [&](int i) {
      if (i < APW) {
        if (do_a && wave + NW * i < AINS) glds16(asrc[i] + (ca * 9 + kya * 3) * 64, abw + (wave + NW * i) * 64);
      } else if (i < APW + BPW) {
        const int j = i - APW;
        if (do_b && wave + NW * j < BINS) {
          const void* src = boff[j] >= 0 ? static_cast<const void*>(xn + boff[j] + (c + 1) * 32)
                                         : static_cast<const void*>(g_zero_line);
          glds16(src, bbw + (wave + NW * j) * 64);
        }
      }
    };
    const h8* ab = big3_smem + (s % AB) * AH8 + (wc * 4) * 3 * 64 + lane;
    const h8* bb = bbase + (c & 1) * BH8;
    // fragments of tap kx + 1 are read while tap kx's 16 MFMAs run (register double buffer)
    h8 fr[2][8];
    auto load = [&](int kx, h8(&f)[8]) {
#pragma unroll
      for (int r = 0; r < 4; ++r) f[r] = ab[(r * 3 + kx) * 64];
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const int u = ((wr * 4 + p) * S + ky) * CI + tile_col<S, CI>(col * S + kx);
        f[4 + p] = bb[u * 4 + (grp ^ ((u >> 1) & 3))];
      }
    };
    load(0, fr[0]);
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      if (kx < 2) load(kx + 1, fr[(kx + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);  // keep the next tap's reads ahead of this tap's MFMAs
#pragma unroll
      for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int p = 0; p < 4; ++p)
          acc[r][p] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fr[kx & 1][r], fr[kx & 1][4 + p], acc[r][p], 0, 0, 0);
        piece(kx * 4 + r);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#pragma unroll
    for (int i = 12; i < APW + BPW; ++i) piece(i);  // stride 2: more copies than MFMA groups
    if constexpr (TM) t_comp += __builtin_amdgcn_s_memtime() - t0;
  }
  if constexpr (TM) {
    if (lane == 0 && blockIdx.x < 4096) {
      unsigned long long* o = tm + (size_t(blockIdx.x) * 8 + wave) * 4;
      o[0] = t_wait;
      o[1] = t_comp;
      o[2] = __builtin_amdgcn_s_memtime() - t_start;
      o[3] = nst;
    }
  }
  tile3_store<4, 4>(a, acc, n, oy0 + wr * 4, ox0, ct_blk + wc * 4, col, grp);
}

static bool big3_timing() {
  static const bool v = [] {
    const char* e = getenv("FCE_BIG3_TIMING");
    return e && atoi(e) != 0;
  }();
  return v;
}

template <int S, int WM, int AB, int NW>
static int launch_big3_k(const ConvArgs& a, dim3 grid, hipStream_t s) {
  constexpr size_t lds = Big3Geom<S, WM, AB, NW>::lds;
  if constexpr (lds <= 160 * 1024) {
    static const bool big =
        hipFuncSetAttribute(reinterpret_cast<const void*>(&conv3x3_big_kernel<S, WM, AB, NW, false>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess &&
        hipFuncSetAttribute(reinterpret_cast<const void*>(&conv3x3_big_kernel<S, WM, AB, NW, true>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
    if (!big) return fail(FCE_ERR_HIP, "conv 3x3 big tile: cannot opt in to >64 KiB LDS");
    if (!big3_timing()) {
      FCE_LAUNCH((conv3x3_big_kernel<S, WM, AB, NW, false>), grid, dim3(NW * 64), lds, s, a, nullptr);
      return FCE_OK;
    }
    // diagnostics: one timed launch, synchronised, summary on stderr
    static unsigned long long* tm = nullptr;
    const size_t nrec = size_t(4096) * 8 * 4;
    if (!tm) FCE_HIP_CHECK(hipMalloc(&tm, nrec * 8));
    FCE_HIP_CHECK(hipMemsetAsync(tm, 0, nrec * 8, s));
    hipLaunchKernelGGL((conv3x3_big_kernel<S, WM, AB, NW, true>), grid, dim3(NW * 64), lds, s, a, tm);
    FCE_HIP_CHECK(hipStreamSynchronize(s));
    std::vector<unsigned long long> h(nrec);
    FCE_HIP_CHECK(hipMemcpy(h.data(), tm, nrec * 8, hipMemcpyDeviceToHost));
    double w = 0, c = 0, t = 0;
    int nw = 0, nst = 0;
    for (size_t i = 0; i < nrec / 4; ++i)
      if (h[i * 4 + 3]) {
        w += h[i * 4];
        c += h[i * 4 + 1];
        t += h[i * 4 + 2];
        nst = int(h[i * 4 + 3]);
        ++nw;
      }
    if (nw)
      fprintf(stderr, "big3<S%d,WM%d,AB%d,NW%d> waves %d stages %d: per stage wait %.0f compute %.0f clocks; lifetime %.0f\n",
              S, WM, AB, NW, nw, nst, w / nw / nst, c / nw / nst, t / nw);
  }
  return FCE_OK;
}

int launch_big3(const ConvArgs& a, int wm, int ab, int nw, int stride, int n, hipStream_t s) {
  FCE_CHECK(big3_ok(stride, wm, ab, nw) && a.cin % 32 == 0 && a.up == 0, "conv 3x3 big tile: bad configuration");
  const int th = (nw / wm) * 4;
  const int64_t tiles = int64_t((a.Wo + 15) / 16) * ((a.Ho + th - 1) / th) * n;
  ConvArgs b = a;
  b.gy = ((a.cout + 15) / 16 + wm * 4 - 1) / (wm * 4);
  FCE_CHECK(tiles * b.gy < (int64_t(1) << 31), "conv 3x3 big tile: grid too large");
  const dim3 grid(unsigned(tiles * b.gy));
  int rc;
  if (stride == 1) {
    if (wm == 1)
      rc = ab == 2 ? launch_big3_k<1, 1, 2, 4>(b, grid, s) : launch_big3_k<1, 1, 3, 4>(b, grid, s);
    else
      rc = ab == 2 ? launch_big3_k<1, 2, 2, 4>(b, grid, s) : launch_big3_k<1, 2, 3, 4>(b, grid, s);
  } else {
    rc = ab == 2 ? launch_big3_k<2, 2, 2, 4>(b, grid, s) : launch_big3_k<2, 2, 3, 4>(b, grid, s);
  }
  if (rc != FCE_OK) return rc;
  return launch_status("conv3x3_big_kernel");
}

}  // namespace fce
